// Grouped Pippenger MSM for the random-linear-combination batch check (gfx950).
#include "kcommon.hpp"

namespace dh {

// ---------------------------------------------------------------- grouped Pippenger MSM
DH_DEV uint32_t scalar_digit(const uint4& s, int bit, int c) {
  // bits [bit, bit + c) of the 128-bit little-endian scalar, zero beyond bit 127
  const uint32_t w[4] = {s.x, s.y, s.z, s.w};
  int wi = bit >> 5, sh = bit & 31;
  uint64_t lo = wi < 4 ? w[wi] : 0;
  uint64_t hi = wi + 1 < 4 ? w[wi + 1] : 0;
  uint64_t v = (lo | (hi << 32)) >> sh;
  return (uint32_t)v & ((1u << c) - 1);
}

// Signed window digits (scalars < 2^127, or < 2^63 per half with the endomorphism split; k_scalars): window w
// holds d_w = v_w + carry_w, mapped to
// [-2^(c-1), 2^(c-1)) with a carry into the next window; the top window needs no mapping (nwin * c >= 128, or
// >= 64, leaves it at least one spare bit, so its digit is at most 2^(c-1)). Bucket |d| in [1, 2^(c-1)], the sign
// travels in bit 31 of the sorted-list entry and the bucket pass negates the point: half the buckets of
// unsigned digits, so half the bucket-reduction work, for the same accumulation count.
constexpr uint32_t NEG_BIT = 0x80000000u;
DH_DEV int32_t signed_digit(const uint4& s, int w, const msm_geom& g, uint32_t& carry) {
  const uint32_t v = scalar_digit(s, w * g.c, g.c) + carry;
  const uint32_t half = 1u << (g.c - 1);
  if (w + 1 < g.nwin && v >= half) {
    carry = 1;
    return (int32_t)v - (int32_t)(1u << g.c);
  }
  carry = 0;
  return (int32_t)v;
}

// Entry e refers to point pidx[e] with scalar scal[sidx ? sidx[e] : pidx[e]] and belongs to group
// grp ? grp[e] : e / gsize. The sorted list stores point indices (| NEG_BIT for a negative digit), bucket by bucket.
DH_DEV size_t entry_group(const uint32_t* grp, size_t e, uint32_t gsize) { return grp ? grp[e] : e / gsize; }

// the scalar of half h of an entry: the whole 127-bit scalar, or with the endomorphism split a = (x, y), b = (z, w),
// or with the G2 psi split the 31-bit part in word h
DH_DEV uint4 half_scalar(const uint4& s, uint32_t h, const msm_geom& g) {
  if (g.halves == 1) return s;
  if (g.halves == 4) return make_uint4(h == 0 ? s.x : h == 1 ? s.y : h == 2 ? s.z : s.w, 0, 0, 0);
  return h ? make_uint4(s.z, s.w, 0, 0) : make_uint4(s.x, s.y, 0, 0);
}
// the round of a point index: the endomorphism images follow the n points (parts of half_stride = nround points)
DH_DEV uint32_t round_of(uint32_t idx, uint32_t nround) { return idx < nround ? idx : idx % nround; }

__global__ void k_msm_hist(const uint32_t* __restrict__ pidx, const uint32_t* __restrict__ sidx,
                           const uint32_t* __restrict__ grp, size_t m, const uint4* __restrict__ scal, msm_geom g,
                           uint32_t* __restrict__ cnt) {
  size_t e = gtid();
  if (e >= m) return;
  const uint4 s = scal[sidx ? sidx[e] : pidx[e]];
  const size_t gi = entry_group(grp, e, g.gsize);
  for (uint32_t h = 0; h < g.halves; h++) {
    const uint4 sh = half_scalar(s, h, g);
    uint32_t carry = 0;
    for (int w = 0; w < g.nwin; w++) {
      const int32_t d = signed_digit(sh, w, g, carry);
      if (d) atomicAdd(&cnt[(gi * g.nwin + w) * g.nbuck + (uint32_t)(d < 0 ? -d : d)], 1u);
    }
  }
}

__global__ void k_msm_scatter(const uint32_t* __restrict__ pidx, const uint32_t* __restrict__ sidx,
                              const uint32_t* __restrict__ grp, size_t m, const uint4* __restrict__ scal, msm_geom g,
                              uint32_t* __restrict__ cursor, uint32_t* __restrict__ list) {
  size_t e = gtid();
  if (e >= m) return;
  const uint32_t idx0 = pidx[e];
  const uint4 s = scal[sidx ? sidx[e] : idx0];
  const size_t gi = entry_group(grp, e, g.gsize);
  for (uint32_t h = 0; h < g.halves; h++) {
    const uint4 sh = half_scalar(s, h, g);
    const uint32_t idx = idx0 + h * g.half_stride;  // endo(P) sits half_stride points after P
    uint32_t carry = 0;
    for (int w = 0; w < g.nwin; w++) {
      const int32_t d = signed_digit(sh, w, g, carry);
      if (d) {
        uint32_t pos = atomicAdd(&cursor[(gi * g.nwin + w) * g.nbuck + (uint32_t)(d < 0 ? -d : d)], 1u);
        list[pos] = d < 0 ? (idx | NEG_BIT) : idx;
      }
    }
  }
}

// The counting sort through LDS. A workgroup takes a tile of consecutive entries and one slab of the key space (at
// most SLAB_MAX consecutive keys: one window's 32,769 buckets at c = 16, or the windows of the tile's groups at the
// bisection's small c), and counts its entries' digits that fall in the slab into an LDS histogram (ds_add: no
// global traffic per entry). The histogram pass flushes the nonzero LDS counts into the global counts; the scatter
// pass claims each nonzero (tile, key)'s range of the sorted list with ONE global atomic and then places the tile's
// entries by LDS atomics on the claimed bases. Tiles hold enough entries that the digits outnumber the slab's keys
// several times over (sort_plan), so the global atomics fall from one per digit to about one per key and tile.
constexpr uint32_t SORT_T = 1024, SLAB_MAX = 36864;  // 144 KiB of counters: one workgroup per CU

template <bool SCATTER>
__global__ __launch_bounds__(SORT_T) void k_msm_sort_lds(const uint32_t* __restrict__ pidx, const uint32_t* __restrict__ sidx,
                                                         const uint32_t* __restrict__ grp, size_t m, const uint4* __restrict__ scal,
                                                         msm_geom g, size_t nk, uint32_t tile, uint32_t slab,
                                                         uint32_t* __restrict__ gcnt, uint32_t* __restrict__ list) {
  extern __shared__ uint32_t h[];  // slab counters (dynamic: slab x 4 bytes)
  const size_t e0 = (size_t)blockIdx.x * tile, e1 = min(m, e0 + tile);
  const size_t rowkeys = (size_t)g.nwin * g.nbuck;
  // the tile's key span: its groups' rows (entries of a group are consecutive without grp), else every key
  const size_t kb = grp ? 0 : (e0 / g.gsize) * rowkeys, ke = grp ? nk : min(nk, ((e1 - 1) / g.gsize + 1) * rowkeys);
  const size_t K0 = kb + (size_t)blockIdx.y * slab;
  if (K0 >= ke) return;  // workgroup-uniform, before any barrier
  const uint32_t ns = (uint32_t)min((size_t)slab, ke - K0);
  for (uint32_t k = threadIdx.x; k < ns; k += SORT_T) h[k] = 0;
  __syncthreads();
  // f(key in the slab, point index | sign) for every digit of the tile's entries
  auto each = [&](auto&& f) {
    for (size_t e = e0 + threadIdx.x; e < e1; e += SORT_T) {
      const uint32_t idx0 = pidx[e];
      const uint4 s = scal[sidx ? sidx[e] : idx0];
      const size_t gi = entry_group(grp, e, g.gsize);
      for (uint32_t hh = 0; hh < g.halves; hh++) {
        const uint4 sh = half_scalar(s, hh, g);
        const uint32_t idx = idx0 + hh * g.half_stride;
        uint32_t carry = 0;
        for (int w = 0; w < g.nwin; w++) {
          const int32_t d = signed_digit(sh, w, g, carry);
          const size_t key = (gi * g.nwin + w) * g.nbuck + (uint32_t)(d < 0 ? -d : d);
          if (d && key - K0 < ns) f((uint32_t)(key - K0), d < 0 ? (idx | NEG_BIT) : idx);
        }
      }
    }
  };
  each([&](uint32_t k, uint32_t) { atomicAdd(&h[k], 1u); });
  __syncthreads();
  if constexpr (!SCATTER) {
    for (uint32_t k = threadIdx.x; k < ns; k += SORT_T)
      if (h[k]) atomicAdd(&gcnt[K0 + k], h[k]);
  } else {
    for (uint32_t k = threadIdx.x; k < ns; k += SORT_T)
      if (h[k]) h[k] = atomicAdd(&gcnt[K0 + k], h[k]);  // this tile's base in the key's range of the list
    __syncthreads();
    each([&](uint32_t k, uint32_t v) { list[atomicAdd(&h[k], 1u)] = v; });
  }
}

// exclusive scan, 3 phases: per-block totals, scan of totals (one block), final per-block scan
constexpr int SCAN_T = 256, SCAN_I = 16, SCAN_B = SCAN_T * SCAN_I;

__global__ __launch_bounds__(SCAN_T) void k_scan_reduce(const uint32_t* __restrict__ in, size_t n,
                                                        uint32_t* __restrict__ block_sums) {
  __shared__ uint32_t sh[SCAN_T];
  size_t base = (size_t)blockIdx.x * SCAN_B + threadIdx.x * SCAN_I;
  uint32_t s = 0;
  for (int k = 0; k < SCAN_I; k++)
    if (base + k < n) s += in[base + k];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int off = SCAN_T / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off) sh[threadIdx.x] += sh[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) block_sums[blockIdx.x] = sh[0];
}

// in-place exclusive scan of a[0..n) with n <= SCAN_B, single block; also writes the total to *total
__global__ __launch_bounds__(SCAN_T) void k_scan_small(uint32_t* __restrict__ a, size_t n, uint32_t* __restrict__ total) {
  __shared__ uint32_t sh[SCAN_T];
  uint32_t v[SCAN_I];
  size_t base = threadIdx.x * SCAN_I;
  uint32_t s = 0;
  for (int k = 0; k < SCAN_I; k++) {
    v[k] = base + k < n ? a[base + k] : 0;
    s += v[k];
  }
  sh[threadIdx.x] = s;
  __syncthreads();
  // Hillis-Steele inclusive scan of the per-thread sums
  for (int off = 1; off < SCAN_T; off <<= 1) {
    uint32_t t = threadIdx.x >= off ? sh[threadIdx.x - off] : 0;
    __syncthreads();
    sh[threadIdx.x] += t;
    __syncthreads();
  }
  uint32_t run = sh[threadIdx.x] - s;
  for (int k = 0; k < SCAN_I; k++) {
    if (base + k < n) a[base + k] = run;
    run += v[k];
  }
  if (threadIdx.x == SCAN_T - 1 && total) *total = sh[SCAN_T - 1];
}

__global__ __launch_bounds__(SCAN_T) void k_scan_final(const uint32_t* __restrict__ in, size_t n,
                                                       const uint32_t* __restrict__ block_off, uint32_t* __restrict__ out) {
  __shared__ uint32_t sh[SCAN_T];
  size_t base = (size_t)blockIdx.x * SCAN_B + threadIdx.x * SCAN_I;
  uint32_t v[SCAN_I];
  uint32_t s = 0;
  for (int k = 0; k < SCAN_I; k++) {
    v[k] = base + k < n ? in[base + k] : 0;
    s += v[k];
  }
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < SCAN_T; off <<= 1) {
    uint32_t t = threadIdx.x >= off ? sh[threadIdx.x - off] : 0;
    __syncthreads();
    sh[threadIdx.x] += t;
    __syncthreads();
  }
  uint32_t run = block_off[blockIdx.x] + sh[threadIdx.x] - s;
  for (int k = 0; k < SCAN_I; k++) {
    if (base + k < n) out[base + k] = run;
    run += v[k];
  }
}

// Bucket accumulation, load-balanced: the sorted list (bucket by bucket, all keys back to back) is cut
// into chunks of L consecutive entries, one thread per chunk, so every lane does the same number of point
// additions whatever the bucket sizes (one thread per bucket left the wave waiting for its fullest
// bucket: Poisson(16) sizes at c = 16). A key that lies wholly inside a chunk is written to its bucket
// directly; a key cut by chunk boundaries leaves partial sums: the chunk where it starts keeps a "tail"
// partial, each later chunk it covers a "head" partial (kind 1: the key ends in that chunk, kind 2: it
// covers the whole chunk), and k_msm_bucket_fix28 adds them up. A bucket whose key holds no entry is never read
// (the reduction tests the key's count).
constexpr uint32_t NO_KEY = 0xffffffffu;

template <class F>
__global__ __launch_bounds__(64) void k_sum_partials(const uint32_t* __restrict__ parts, size_t k, size_t rec_words,
                                                     uint32_t* __restrict__ outA, uint32_t* __restrict__ outB,
                                                     uint8_t* __restrict__ flag) {
  const int t = threadIdx.x;
  constexpr size_t JW = 3 * npw<F>::N;  // Jacobian words
  if (t == 2) {
    uint32_t any = 0;
    for (size_t i = 0; i < k; i++) any |= parts[i * rec_words + 2 * JW];
    if (flag) flag[0] = any ? 1 : 0;
  }
  if (t > 1) return;
  jac<F> acc = jac_inf<F>();
  for (size_t i = 0; i < k; i++) acc = jac_add(acc, ld_jac_aos<F>(parts + i * rec_words, t));
  st_jac_aos<F>(t ? outB : outA, 0, acc);
}

hipError_t launch_sum_partials(int sig_g2, const uint32_t* parts, size_t k, size_t rec_words, uint32_t* outA, uint32_t* outB,
                               uint8_t* flag, hipStream_t st) {
  if (sig_g2) hipLaunchKernelGGL(k_sum_partials<fp2>, dim3(1), dim3(64), 0, st, parts, k, rec_words, outA, outB, flag);
  else hipLaunchKernelGGL(k_sum_partials<fp>, dim3(1), dim3(64), 0, st, parts, k, rec_words, outA, outB, flag);
  return hipGetLastError();
}

// the node-wide verdict of one batch, on the device (no host round trip): res[2] = 2 when some rank abandoned the batch
// (res[0]), else the pairing check's res[1]; when it passed, every decoded round of the batch is valid
__global__ void k_node_mark(size_t n, uint8_t* __restrict__ res, const uint8_t* __restrict__ status,
                            uint8_t* __restrict__ verdict) {
  const size_t i = gtid();
  const uint8_t r = res[0] ? 2 : (res[1] == 1 ? 1 : 0);
  if (i == 0) res[2] = r;
  if (i < n && r == 1) verdict[i] = status[i] == DEC_OK ? 1 : 0;
}

hipError_t launch_node_mark(size_t n, uint8_t* res, const uint8_t* status, uint8_t* verdict, hipStream_t st) {
  hipLaunchKernelGGL(k_node_mark, dim3(nblk(n ? n : 1, 256)), dim3(256), 0, st, n, res, status, verdict);
  return hipGetLastError();
}

__global__ void k_mark_groups(const uint32_t* __restrict__ entries, size_t m, size_t gsize, const uint8_t* __restrict__ pass,
                              const uint8_t* __restrict__ status, uint8_t* __restrict__ verdict) {
  size_t e = gtid();
  if (e >= m) return;
  uint32_t i = entries[e];
  if (pass[e / gsize]) verdict[i] = status[i] == DEC_OK ? 1 : 0;
}

__global__ void k_iota(uint32_t* __restrict__ v, size_t n) {
  size_t i = gtid();
  if (i < n) v[i] = (uint32_t)i;
}


hipError_t launch_iota(uint32_t* v, size_t n, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_iota, dim3(nblk(n, 256)), dim3(256), 0, st, v, n);
  return hipGetLastError();
}

// exclusive scan of cnt[0..nk) into off[0..nk], off[nk] = total; tmp needs nblk(nk, SCAN_B) words

hipError_t launch_scan(const uint32_t* cnt, size_t nk, uint32_t* off, uint32_t* tmp, hipStream_t st) {
  size_t nb = (nk + SCAN_B - 1) / SCAN_B;
  if (nb > (size_t)SCAN_B) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)nb), dim3(SCAN_T), 0, st, cnt, nk, tmp);
  hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(SCAN_T), 0, st, tmp, nb, off + nk);
  hipLaunchKernelGGL(k_scan_final, dim3((unsigned)nb), dim3(SCAN_T), 0, st, cnt, nk, tmp, off);
  return hipGetLastError();
}


hipError_t launch_msm_sort(const msm_geom& g, const uint32_t* pidx, const uint32_t* sidx, const uint32_t* grp, size_t m,
                           size_t ngroups, const uint4* scal, msm_ws& ws, hipStream_t st) {
  size_t nk = ngroups * g.nwin * (size_t)g.nbuck;
  ws.max_entries = msm_entries(g, m);
  hipError_t e = hipMemsetAsync(ws.cnt, 0, nk * sizeof(uint32_t), st);
  if (e != hipSuccess) return e;
  // DRANDHIP_SORT_GLOBAL=1 (experiments): the one-global-atomic-per-digit sort
  static const bool global_env = [] {
    const char* v = getenv("DRANDHIP_SORT_GLOBAL");
    return v && atoi(v) == 1;
  }();
  // a tile whose keys span more than 16 slabs (a grouping by grp over many groups: the tbls per-signer sums at c = 16,
  // 64 groups x 2 windows x 32,769 keys = 114 slabs) would be read once per slab: there the one-atomic-per-digit sort wins
  // (k_msm_hist + k_msm_scatter 7.0 ms against 14.4 for the LDS sort, gpurun_out r05w)
  const bool global_sort = global_env || (grp && nk > 16 * (size_t)SLAB_MAX);
  // the LDS sort's plan: tiles of about density x the slab's keys in digits (DRANDHIP_SORT_DENSITY), slabs of at
  // most SLAB_MAX keys over the keys a tile can touch
  dim3 grid;
  uint32_t tile = 0, slab = 0;
  if (m && !global_sort) {
    static const size_t density = [] {
      const char* v = getenv("DRANDHIP_SORT_DENSITY");
      const long d = v ? atol(v) : 0;
      return (size_t)(d >= 1 && d <= 256 ? d : 8);
    }();
    const size_t digits = (size_t)g.halves * g.nwin, rowkeys = (size_t)g.nwin * g.nbuck;
    // DRANDHIP_SORT_SLAB: the LDS slab in keys (smaller slabs let the workgroups share a CU with the kernels beside them)
    static const size_t slab_max = [] {
      const char* v = getenv("DRANDHIP_SORT_SLAB");
      const long d = v ? atol(v) : 0;
      return (size_t)(d >= 1024 && d <= SLAB_MAX ? d : SLAB_MAX);
    }();
    static const hipError_t lds_attr = [] {  // dynamic LDS beyond 64 KiB
      hipError_t a = hipFuncSetAttribute((const void*)k_msm_sort_lds<false>, hipFuncAttributeMaxDynamicSharedMemorySize, SLAB_MAX * 4);
      hipError_t b = hipFuncSetAttribute((const void*)k_msm_sort_lds<true>, hipFuncAttributeMaxDynamicSharedMemorySize, SLAB_MAX * 4);
      return a != hipSuccess ? a : b;
    }();
    if (lds_attr != hipSuccess) return lds_attr;
    const size_t t = std::min(m, std::max<size_t>(SORT_T, density * std::min<size_t>(nk, slab_max) / digits));
    // keys one tile can touch: every key with grp, else the rows of at most t / gsize + 2 consecutive groups
    const size_t span = grp ? nk : std::min(nk, std::min<size_t>(ngroups, (t - 1) / g.gsize + 2) * rowkeys);
    const size_t nslab = (span + slab_max - 1) / slab_max;
    tile = (uint32_t)t;
    slab = (uint32_t)((span + nslab - 1) / nslab);
    grid = dim3((unsigned)((m + t - 1) / t), (unsigned)nslab);
  }
  if (m && global_sort) hipLaunchKernelGGL(k_msm_hist, dim3(nblk(m, 256)), dim3(256), 0, st, pidx, sidx, grp, m, scal, g, ws.cnt);
  if (m && !global_sort)
    hipLaunchKernelGGL(k_msm_sort_lds<false>, grid, dim3(SORT_T), slab * 4, st, pidx, sidx, grp, m, scal, g, nk, tile, slab, ws.cnt, ws.list);
  if ((e = launch_scan(ws.cnt, nk, ws.off, ws.scan_tmp, st)) != hipSuccess) return e;
  if ((e = hipMemcpyAsync(ws.cnt, ws.off, nk * sizeof(uint32_t), hipMemcpyDeviceToDevice, st)) != hipSuccess) return e;
  if (m && global_sort)
    hipLaunchKernelGGL(k_msm_scatter, dim3(nblk(m, 256)), dim3(256), 0, st, pidx, sidx, grp, m, scal, g, ws.cnt, ws.list);
  if (m && !global_sort)
    hipLaunchKernelGGL(k_msm_sort_lds<true>, grid, dim3(SORT_T), slab * 4, st, pidx, sidx, grp, m, scal, g, nk, tile, slab, ws.cnt, ws.list);
  return hipGetLastError();
}

// ================================================================ the RLC MSM in the lazily reduced 28-bit form
// Points enter once in the 28-bit form (k_msm_prep28: sigma affine, the hash points Jacobian, each with its
// endomorphism image at index n + i) and every addition of the bucket pass, the fix-up, the bucket reduction and the
// window Horner runs on lazy values (fp28.hpp for G1, fp2_28.hpp for G2): no 12 <-> 14 limb slicing or final
// subtraction per product, no modular reduction per sum. The bucket pass uses the formulas without exceptional-case
// tests and one zero test of Z per run (poisoned); the rare poisoned run is recomputed with the exact formulas.
// Stored Fp elements take 16 words (14 limbs + 2 pad: four 16-byte loads), a Jacobian point 3 elements, infinity
// stored as Z = 0 (all limbs zero: a finite point's Z is never 0 mod p). The window sums leave in the 12 x 32-bit
// Montgomery Jacobian form the pairing checks read.
constexpr int W28 = 16;
DH_DEV f28 ld28(const uint32_t* p) {
  const uint4* q = (const uint4*)p;
  f28 a;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint4 t = q[i];
    a.l[4 * i] = t.x;
    a.l[4 * i + 1] = t.y;
    if (4 * i + 2 < 14) a.l[4 * i + 2] = t.z;
    if (4 * i + 3 < 14) a.l[4 * i + 3] = t.w;
  }
  return a;
}
DH_DEV void st28(uint32_t* p, const f28& a) {
  uint4* q = (uint4*)p;
#pragma unroll
  for (int i = 0; i < 4; i++)
    q[i] = make_uint4(a.l[4 * i], a.l[4 * i + 1], 4 * i + 2 < 14 ? a.l[4 * i + 2] : 0u, 4 * i + 3 < 14 ? a.l[4 * i + 3] : 0u);
}
DH_DEV void ld28(f28& a, const uint32_t* p) { a = ld28(p); }
DH_DEV void st28(uint32_t* p, const f28& a, int) { st28(p, a); }
DH_DEV void ld28(f228& a, const uint32_t* p) {
  a.c0 = ld28(p);
  a.c1 = ld28(p + W28);
}
DH_DEV void st28(uint32_t* p, const f228& a, int) {
  st28(p, a.c0);
  st28(p + W28, a.c1);
}
DH_DEV bool z_all_zero(const f28& z) {
  uint32_t nz = 0;
#pragma unroll
  for (int k = 0; k < 14; k++) nz |= z.l[k];
  return nz == 0;
}
DH_DEV bool z_all_zero(const f228& z) { return z_all_zero(z.c0) && z_all_zero(z.c1); }
DH_DEV void set_zero(f28& z) {
#pragma unroll
  for (int k = 0; k < 14; k++) z.l[k] = 0;
}
DH_DEV void set_zero(f228& z) {
  set_zero(z.c0);
  set_zero(z.c1);
}

// the lazy-form curve of each signature group: element / point types and the formulas the MSM needs
struct c28_g1 {
  static constexpr int OCC = 2;  // waves per SIMD the bucket pass is compiled for
  static constexpr int PARTS = 2;  // P, phi(P): two 63-bit scalar halves
  static constexpr size_t LCAP = 32;  // longest bucket-pass chunk
  using E = f28;
  using P = j28;
  using F = fp;  // 12 x 32-bit form of the outputs
  static constexpr int EW = W28;
  DH_DEV static P inf() { return j28_inf(); }
  DH_DEV static P madd_fast(const P& a, const E& x, const E& y) { return j28_madd_fast(a, x, y); }
  DH_DEV static P madd(const P& a, const E& x, const E& y) { return j28_madd(a, x, y); }
  DH_DEV static P add_fast(const P& a, const P& b) { return j28_add_fast(a, b); }
  DH_DEV static P add(const P& a, const P& b) { return j28_add(a, b); }
  template <bool EXACT>
  DH_DEV static P add_mem(const P& a, const uint32_t* q) {  // a + the Jacobian point stored at q
    j28 b;
    b.x = ld28(q);
    b.y = ld28(q + W28);
    b.z = ld28(q + 2 * W28);
    b.inf = z_all_zero(b.z);
    return EXACT ? j28_add(a, b) : j28_add_fast(a, b);
  }
  template <bool EXACT>
  DH_DEV static P addx(const P& a, const P& b) { return EXACT ? j28_add(a, b) : j28_add_fast(a, b); }
  DH_DEV static P dbl(const P& a) { return j28_dbl(a); }
  DH_DEV static bool poisoned(const P& a) { return j28_poisoned(a); }
  DH_DEV static E neg(const E& y) { return f28_neg2(y); }  // y < 2
  DH_DEV static fp out(const E& a) { return f28_to_fp(a); }
  // prep (k_msm_prep28): conversion, products kept < 2, inversion of a public value, the endomorphism phi
  DH_DEV static E in(const fp& a) { return f28_from_fp(a); }
  DH_DEV static E mulr(const E& a, const E& b) { return f28_mul(a, b); }
  DH_DEV static E sqrr(const E& a) { return f28_sqr(a); }
  DH_DEV static E one() { return f28_one(); }
  DH_DEV static E inv(const E& a) { return f28_from_fp(fp_inv_vt(f28_to_fp(a))); }
  DH_DEV static bool is_zero(const fp& a) { return fp_is_zero(a); }
  DH_DEV static E endo_x(const E& x);
  DH_DEV static E endo_y(const E& y) { return y; }
};
struct c28_g2 {
  static constexpr int OCC = 1;  // 512 registers: the G2 mixed addition's values fit VGPRs + AGPRs, no scratch
  static constexpr int PARTS = 4;  // P, psi(P), psi^2(P), psi^3(P): four 31-bit scalar parts
  static constexpr size_t LCAP = 64;
  using E = f228;
  using P = j228;
  using F = fp2;
  static constexpr int EW = 2 * W28;
  DH_DEV static P inf() { return j228_inf(); }
  // the bucket pass's additions take carry-free product operands (fp2_28.hpp NC); the reduction kernels' do not
  DH_DEV static P madd_fast(const P& a, const E& x, const E& y) { return j228_madd<false, true>(a, x, y); }
  DH_DEV static P madd(const P& a, const E& x, const E& y) { return j228_madd<true>(a, x, y); }
  DH_DEV static P add_fast(const P& a, const P& b) { return j228_add<false>(a, b); }
  DH_DEV static P add(const P& a, const P& b) { return j228_add<true>(a, b); }
  template <bool EXACT>
  DH_DEV static P add_mem(const P& a, const uint32_t* q) {  // coordinates loaded where the formula uses them
    f228 z;
    ld28(z, q + 2 * EW);
    return j228_add_ld<EXACT>(a, z_all_zero(z), [&](int k) { f228 c; ld28(c, q + k * EW); return c; });
  }
  template <bool EXACT>
  DH_DEV static P addx(const P& a, const P& b) { return j228_add<EXACT>(a, b); }
  DH_DEV static P dbl(const P& a) { return j228_dbl(a); }
  DH_DEV static bool poisoned(const P& a) { return j228_poisoned(a); }
  DH_DEV static E neg(const E& y) { return f2_neg3(y); }  // y < 2
  DH_DEV static fp2 out(const E& a) { return f2_to_fp2(a); }
  DH_DEV static E in(const fp2& a) { return f2_from_fp2(a); }
  DH_DEV static E mulr(const E& a, const E& b) { return f2_red(f2_mul(a, b)); }
  DH_DEV static E sqrr(const E& a) { return f2_red(f2_sqr<2>(a)); }
  DH_DEV static E one() { return f2_one(); }
  DH_DEV static E inv(const E& a) { return f2_from_fp2(fp2_inv_vt(f2_to_fp2(a))); }
  DH_DEV static bool is_zero(const fp2& a) { return fp2_is_zero(a); }
  // psi(x, y) = (conj(x) PSI_X, conj(y) PSI_Y), reduced back to < 2
  DH_DEV static E endo_x(const E& x) { return f2_red(f2_mul(f2_conj(x), f2_c28(PSI_X28))); }
  DH_DEV static E endo_y(const E& y) { return f2_red(f2_mul(f2_conj(y), f2_c28(PSI_Y28))); }
  // psi^2(x, y) = (x PSI2_X, y PSI2_Y) with constants in Fp
  DH_DEV static E psi2_x(const E& x) { return f2_red({f28_mul(x.c0, f28_c(PSI2_X28)), f28_mul(x.c1, f28_c(PSI2_X28))}); }
  DH_DEV static E psi2_y(const E& y) { return f2_red({f28_mul(y.c0, f28_c(PSI2_Y28)), f28_mul(y.c1, f28_c(PSI2_Y28))}); }
};

template <class C>
DH_DEV typename C::P ldj28(const uint32_t* base, size_t i) {
  const uint32_t* p = base + (size_t)3 * C::EW * i;
  typename C::P r;
  ld28(r.x, p);
  ld28(r.y, p + C::EW);
  ld28(r.z, p + 2 * C::EW);
  r.inf = z_all_zero(r.z);
  return r;
}
template <class C>
DH_DEV void stj28(uint32_t* base, size_t i, const typename C::P& a) {
  uint32_t* p = base + (size_t)3 * C::EW * i;
  st28(p, a.x, 0);
  st28(p + C::EW, a.y, 0);
  typename C::E z = a.z;
  if (a.inf) set_zero(z);
  st28(p + 2 * C::EW, z, 0);
}

// beta (phi(x, y) = (beta x, y) on G1) as a 28-bit Montgomery constant (beta R' mod p)
__device__ __constant__ uint32_t BETA28[14] = {0xa75929au, 0x681b798u, 0x22a3e9du, 0xabc02bfu, 0x4e5bb45u, 0x55e6e7eu, 0x4814117u,
                                               0x6d04f1bu, 0xae3387du, 0x54acb0cu, 0x0a4c74bu, 0x56138b5u, 0xb64e066u, 0x00076f2u};

DH_DEV f28 c28_g1::endo_x(const f28& x) { return f28_mul(x, f28_c(BETA28)); }

// The batch's points in the lazy affine form, each followed (index n + i) by its endomorphism image (phi on G1,
// psi on G2; G2 also psi^2 and psi^3 at 2n + i and 3n + i, the four parts of its scalars): S from the decoded
// signatures; Q from the Jacobian hash points, made affine with ONE variable-time inversion per workgroup (Montgomery's
// trick at two levels: each lane multiplies the Z's of its K rounds, storing the prefix products in Q's x slots; the
// workgroup's 256 lane products are combined by a prefix and a suffix product scan through LDS, lane 0 inverts the
// total, and each lane's inverse is total^-1 x (the other lanes' product); each 1/Z then comes out on the lane's way
// back). The bucket pass takes mixed additions for both point sets: 7M + 4S per entry instead of 11M + 5S for the hash
// points. A hash point at infinity (Z = 0, probability ~2^-255) cannot be the message of a valid signature: its round
// is marked DEC_BAD, which is its VerifyBeacon verdict. K (rounds per lane) follows the batch size so that the launch
// fills the chip's 2-wave residency (131,072 lanes): 8 at 1M rounds, 1 at a 131k shard (prep28_k). r04 inverted once
// per lane: at a 131k shard (K = 1) that was one ~64k-instruction inversion per round, as much work per batch as a 1M
// batch's, ~12% of the pipelined 131k shape's GPU time (profiles/r05/node_131072_trace_r05l).
constexpr uint32_t PREP28_KMAX = 16;
// the endomorphism images of affine point i at part * n + i
template <class C>
DH_DEV void prep28_images(uint32_t* __restrict__ out, size_t n, size_t i, const typename C::E& x, const typename C::E& y) {
  constexpr int EW = C::EW;
  st28(out + 2 * EW * (n + i), C::endo_x(x), 0);
  st28(out + 2 * EW * (n + i) + EW, C::endo_y(y), 0);
  if constexpr (C::PARTS == 4) {
    const typename C::E x2 = C::psi2_x(x), y2 = C::psi2_y(y);
    st28(out + 2 * EW * (2 * n + i), x2, 0);
    st28(out + 2 * EW * (2 * n + i) + EW, y2, 0);
    st28(out + 2 * EW * (3 * n + i), C::endo_x(x2), 0);
    st28(out + 2 * EW * (3 * n + i) + EW, C::endo_y(y2), 0);
  }
}
static uint32_t prep28_k(size_t n) {
  uint32_t k = 1;
  while (k < PREP28_KMAX && n / (2 * k) >= 131072) k *= 2;
  return k;
}
// inclusive product scan of v over the workgroup's 256 lanes, forwards (lane t: v_0 ... v_t) or backwards (v_t ... v_255)
template <class C, bool BACK>
DH_DEV typename C::E block_product_scan(typename C::E v, typename C::E* sh) {
  const int t = threadIdx.x;
#pragma unroll 1
  for (int off = 1; off < 256; off <<= 1) {
    sh[t] = v;
    __syncthreads();
    const int src = BACK ? t + off : t - off;
    const bool has = BACK ? src < 256 : src >= 0;
    typename C::E o;
    if (has) o = sh[src];
    __syncthreads();
    if (has) v = C::mulr(v, o);
  }
  return v;
}
// sets: bit 0 converts S (sig_aff), bit 1 Q (q_pts); tbls Recover converts its partials and its round hash points
// separately (different counts)
template <class C>
__global__ __launch_bounds__(256, 2) void k_msm_prep28(size_t n, uint32_t K, uint8_t* __restrict__ status,
                                                       const uint32_t* __restrict__ sig_aff, const uint32_t* __restrict__ q_pts,
                                                       uint32_t* __restrict__ S, uint32_t* __restrict__ Q, uint32_t sets) {
  using E = typename C::E;
  using F = typename C::F;
  constexpr int EW = C::EW, FW = npw<F>::N;
  __shared__ E sh[256];
  const size_t lo = gtid() * K;
  const size_t hi = lo < n ? min(n, lo + K) : lo;  // lanes past n take part in the workgroup's scans only
#pragma unroll 1
  for (size_t i = lo; i < hi && (sets & 1); i++) {
    if (status[i] != DEC_OK) continue;
    const aff<F> a = ld_aff_aos<F>(sig_aff, i);
    const E x = C::in(a.x), y = C::in(a.y);
    st28(S + 2 * EW * i, x, 0);
    st28(S + 2 * EW * i + EW, y, 0);
    prep28_images<C>(S, n, i, x, y);
  }
  if (!(sets & 2)) return;  // a kernel argument: uniform, before the barriers
  E acc = C::one();
#pragma unroll 1
  for (size_t i = lo; i < hi; i++) {
    if (status[i] != DEC_OK) continue;
    F z;
    ld_f<F>(z, q_pts + 3 * FW * i + 2 * FW);
    if (C::is_zero(z)) {
      status[i] = DEC_BAD;
      continue;
    }
    st28(Q + 2 * EW * i, acc, 0);  // prefix product, read back below
    acc = C::mulr(acc, C::in(z));
  }
  // acc^-1 = total^-1 x (product of the other lanes' acc): exclusive prefix x exclusive suffix
  const int t = threadIdx.x;
  const E pre = block_product_scan<C, false>(acc, sh);
  sh[t] = pre;
  __syncthreads();
  const E pre_x = t ? sh[t - 1] : C::one();
  __syncthreads();
  if (t == 255) sh[0] = C::inv(pre);  // the workgroup's one inversion (every factor is a nonzero Z or one)
  __syncthreads();
  const E tinv = sh[0];
  __syncthreads();
  const E suf = block_product_scan<C, true>(acc, sh);
  sh[t] = suf;
  __syncthreads();
  const E suf_x = t < 255 ? sh[t + 1] : C::one();
  E inv = C::mulr(C::mulr(tinv, pre_x), suf_x);
#pragma unroll 1
  for (size_t k = hi; k-- > lo;) {
    if (status[k] != DEC_OK) continue;
    E pr;
    ld28(pr, Q + 2 * EW * k);
    const jac<F> q = ld_jac_aos<F>(q_pts, k);
    const E zi = C::mulr(inv, pr);
    inv = C::mulr(inv, C::in(q.z));
    const E zi2 = C::sqrr(zi);
    const E x = C::mulr(C::in(q.x), zi2);
    const E y = C::mulr(C::in(q.y), C::mulr(zi2, zi));
    st28(Q + 2 * EW * k, x, 0);
    st28(Q + 2 * EW * k + EW, y, 0);
    prep28_images<C>(Q, n, k, x, y);
  }
}

// one affine / Jacobian point of a sorted-list entry, negated for a negative digit
template <class C, bool AFFINE>
DH_DEV typename C::P bucket_add(const typename C::P& acc, const uint32_t* __restrict__ pts, uint32_t raw, bool exact) {
  const uint32_t idx = raw & ~NEG_BIT;
  if constexpr (AFFINE) {
    typename C::E x, y;
    ld28(x, pts + 2 * C::EW * idx);
    ld28(y, pts + 2 * C::EW * idx + C::EW);
    if (raw & NEG_BIT) y = C::neg(y);
    return exact ? C::madd(acc, x, y) : C::madd_fast(acc, x, y);
  } else {
    typename C::P q = ldj28<C>(pts, idx);
    if (raw & NEG_BIT) q.y = C::neg(q.y);
    return exact ? C::add(acc, q) : C::add_fast(acc, q);
  }
}

// the balanced bucket pass (chunks of the sorted list, head / tail partials and their metadata, above) on 28-bit
// points. skip (optional): per-round status; an entry whose round (point index mod nround: the endomorphism images
// follow the points) is not DEC_OK adds nothing — the batch check sorts before the rounds are decoded (verify_core),
// so such rounds carry nonzero scalars
template <class C, bool AFFINE>
__global__ __launch_bounds__(256, C::OCC) void k_msm_bucket28(const uint32_t* __restrict__ off, const uint32_t* __restrict__ list,
                                                         size_t nkeys, uint32_t L, const uint32_t* __restrict__ pts,
                                                         uint32_t* __restrict__ buckets, uint32_t* __restrict__ part,
                                                         uint32_t* __restrict__ meta, const uint8_t* __restrict__ skip,
                                                         uint32_t nround) {
  const size_t t = gtid();
  const uint32_t total = off[nkeys];
  const size_t s = t * (size_t)L;
  if (s >= total) return;
  const uint32_t e = (uint32_t)min(s + L, (size_t)total);
  size_t lo = 0, hi = nkeys;
  while (hi - lo > 1) {
    size_t mid = (lo + hi) >> 1;
    if (off[mid] <= s) lo = mid;
    else hi = mid;
  }
  size_t key = lo;
  uint32_t kend = off[key + 1];
  const bool starts_before = off[key] < s;
  bool first = true;
  uint32_t head_kind = 0, tail_key = NO_KEY, run0 = (uint32_t)s;
  typename C::P acc = C::inf();
#pragma unroll 1
  for (uint32_t j = (uint32_t)s; j < e; j++) {
    const uint32_t raw = list[j];
    const uint32_t idx = raw & ~NEG_BIT;
    if (!skip || skip[round_of(idx, nround)] == DEC_OK) acc = bucket_add<C, AFFINE>(acc, pts, raw, false);
    const bool ends = j + 1 == kend;
    if (ends || j + 1 == e) {
      if (C::poisoned(acc)) {  // an exceptional case somewhere in the run: again with the exact formulas
        acc = C::inf();
#pragma unroll 1
        for (uint32_t k = run0; k <= j; k++) {
          const uint32_t r2 = list[k];
          const uint32_t i2 = r2 & ~NEG_BIT;
          if (!skip || skip[round_of(i2, nround)] == DEC_OK) acc = bucket_add<C, AFFINE>(acc, pts, r2, true);
        }
      }
      if (first && starts_before) {
        stj28<C>(part, 2 * t, acc);
        head_kind = ends ? 1 : 2;
      } else if (ends) {
        stj28<C>(buckets, key, acc);
      } else {
        stj28<C>(part, 2 * t + 1, acc);
        tail_key = (uint32_t)key;
      }
      first = false;
      run0 = j + 1;
      if (ends && j + 1 < e) {
        do {
          key++;
        } while (off[key + 1] <= j + 1);
        kend = off[key + 1];
        acc = C::inf();
      }
    }
  }
  if (meta) {
    meta[2 * t] = head_kind;
    meta[2 * t + 1] = tail_key;
  }
}

// The reduction kernels below compute with the formulas without exceptional-case tests, test the result for the
// poison those cases leave (Z = 0 mod p, fp28.hpp j28_madd_fast) and only then, rarely, recompute with the exact
// formulas: every stored point is exact (infinity stored as Z = 0), so no poison crosses a kernel boundary.
template <class C, bool EXACT>
DH_DEV typename C::P fix_run(const uint32_t* __restrict__ part, const uint32_t* __restrict__ meta, size_t t, size_t nch) {
  typename C::P acc = ldj28<C>(part, 2 * t + 1);
#pragma unroll 1
  for (size_t u = t + 1; u < nch; u++) {
    acc = C::template add_mem<EXACT>(acc, part + (size_t)3 * C::EW * (2 * u));
    if (meta[2 * u] == 1) break;
  }
  return acc;
}
template <class C>
__global__ __launch_bounds__(256, C::OCC) void k_msm_bucket_fix28(const uint32_t* __restrict__ off, size_t nkeys, uint32_t L,
                                                                  const uint32_t* __restrict__ meta, const uint32_t* __restrict__ part,
                                                                  uint32_t* __restrict__ buckets) {
  const size_t t = gtid();
  const uint32_t total = off[nkeys];
  const size_t nch = (total + L - 1) / L;
  if (t >= nch) return;
  const uint32_t key = meta[2 * t + 1];
  if (key == NO_KEY) return;
  typename C::P acc = fix_run<C, false>(part, meta, t, nch);
  if (C::poisoned(acc)) acc = fix_run<C, true>(part, meta, t, nch);
  stj28<C>(buckets, key, acc);
}

// per (set, group, window, segment): sum_{d in seg} d B_d in two passes (fewer live points per thread): the segment's
// running sums give tot = sum (d - a + 1) B_d and run = sum B_d (segsum28), then tot + (a - 1) run (segoff28). A bucket
// whose key holds no entry is the identity and is not read (the bucket array is never cleared). Rows of both point
// sets share the keys: row gw -> key row gw % rows_per_set.
template <class C, bool EXACT>
DH_DEV void seg_run(const uint32_t* __restrict__ buckets, const uint32_t* __restrict__ off, size_t krow, size_t brow, uint32_t a,
                    uint32_t last, typename C::P& run, typename C::P& tot) {
  run = C::inf();
  tot = C::inf();
#pragma unroll 1
  for (int d = (int)last - 1; d >= (int)a; d--) {
    if (off[krow + d + 1] != off[krow + d]) run = C::template add_mem<EXACT>(run, buckets + (size_t)3 * C::EW * (brow + d));
    tot = C::template addx<EXACT>(tot, run);
  }
}
// points through LDS for the wave-level trees: word-major (word k of thread i at buf[k * nthr + i]: one ds_read_b32
// per word across the wave, conflict-free); infinity travels as Z = 0, like stj28
DH_DEV void lds_put(uint32_t* buf, int nthr, int i, int k0, const f28& a) {
#pragma unroll
  for (int k = 0; k < 14; k++) buf[(k0 + k) * nthr + i] = a.l[k];
}
DH_DEV void lds_get(const uint32_t* buf, int nthr, int i, int k0, f28& a) {
#pragma unroll
  for (int k = 0; k < 14; k++) a.l[k] = buf[(k0 + k) * nthr + i];
}
DH_DEV void lds_put(uint32_t* buf, int nthr, int i, int k0, const f228& a) {
  lds_put(buf, nthr, i, k0, a.c0);
  lds_put(buf, nthr, i, k0 + 14, a.c1);
}
DH_DEV void lds_get(const uint32_t* buf, int nthr, int i, int k0, f228& a) {
  lds_get(buf, nthr, i, k0, a.c0);
  lds_get(buf, nthr, i, k0 + 14, a.c1);
}
template <class C>
constexpr int lds_words() { return 3 * 14 * (C::EW / W28); }
template <class C>
DH_DEV void lds_put_pt(uint32_t* buf, int nthr, int i, const typename C::P& a) {
  constexpr int EL = 14 * (C::EW / W28);
  lds_put(buf, nthr, i, 0, a.x);
  lds_put(buf, nthr, i, EL, a.y);
  typename C::E z = a.z;
  if (a.inf) set_zero(z);
  lds_put(buf, nthr, i, 2 * EL, z);
}
template <class C>
DH_DEV typename C::P lds_get_pt(const uint32_t* buf, int nthr, int i) {
  constexpr int EL = 14 * (C::EW / W28);
  typename C::P r;
  lds_get(buf, nthr, i, 0, r.x);
  lds_get(buf, nthr, i, EL, r.y);
  lds_get(buf, nthr, i, 2 * EL, r.z);
  r.inf = z_all_zero(r.z);
  return r;
}
// a + the point in LDS slot i, its coordinates read where the formula uses them (G2: fewer values live)
template <class C, bool EXACT>
DH_DEV typename C::P add_lds(const typename C::P& a, const uint32_t* buf, int nthr, int i) {
  if constexpr (C::PARTS == 4) {
    constexpr int EL = 28;
    f228 z;
    lds_get(buf, nthr, i, 2 * EL, z);
    return j228_add_ld<EXACT>(a, z_all_zero(z), [&](int k) { f228 c; lds_get(buf, nthr, i, k * EL, c); return c; });
  } else {
    return C::template addx<EXACT>(a, lds_get_pt<C>(buf, nthr, i));
  }
}
// The sum of cnt stored points p[0 .. cnt) (rowtree: a lane's serial run of G segment values), or, with three
// arguments, of the points first + k for k = lane, lane + 64, ... < parts (rowred: a row's wave partials). EXACT = false
// takes the additions without their exceptional-case tests; a poisoned result (Z = 0 without the infinity flag, which
// every later fast addition keeps) is recomputed with the exact formulas by the caller, so the loop body holds one
// formula (r05 checked and redid each addition in the loop: both formulas and the old sum live at once, the G2 row tree
// ~2,500 scratch instructions per step)
template <class C, bool EXACT>
DH_DEV typename C::P run_mem(const uint32_t* __restrict__ p, uint32_t cnt) {
  typename C::P acc = C::inf();
#pragma unroll 1
  for (uint32_t k = 0; k < cnt; k++) acc = C::template add_mem<EXACT>(acc, p + (size_t)3 * C::EW * k);
  return acc;
}
template <class C, bool EXACT>
DH_DEV typename C::P run_mem(const uint32_t* __restrict__ base, size_t first, uint32_t parts) {
  typename C::P acc = C::inf();
#pragma unroll 1
  for (uint32_t k = threadIdx.x; k < parts; k += 64) acc = C::template add_mem<EXACT>(acc, base + (size_t)3 * C::EW * (first + k));
  return acc;
}
// the exact sum of the two points parked in LDS slots i and j, out of line: the fast tree step that calls it on a
// poisoned sum (never for honest inputs) keeps none of its registers
template <class C>
__attribute__((noinline)) DH_DEV typename C::P add_lds_exact(const uint32_t* buf, int nthr, int i, int j) {
  return add_lds<C, true>(lds_get_pt<C>(buf, nthr, i), buf, nthr, j);
}
// the tree over aligned runs of `span` lanes (a power of two <= 64) of each wave: lane l, l % span == 0, ends with the
// sum of lanes [l, l + span). Every thread of the workgroup calls it (barriers); buf: lds_words<C>() x blockDim words.
// The inputs are exact (stored points), so a poisoned sum is recomputed with the exact formulas on the spot.
template <class C>
DH_DEV typename C::P wave_tree(typename C::P acc, uint32_t* buf, uint32_t span) {
  const int nthr = blockDim.x, i = threadIdx.x, lane = i & 63;
#pragma unroll 1
  for (uint32_t step = 1; step < span; step <<= 1) {
    // every lane still holding a partial sum parks it: its partner reads it, and a poisoned sum is redone from the
    // two parked operands, so the lane's own sum is not live across the fast addition
    if ((lane & (step - 1)) == 0) lds_put_pt<C>(buf, nthr, i, acc);
    __syncthreads();
    if ((lane & (2 * step - 1)) == 0) {
      typename C::P s = add_lds<C, false>(acc, buf, nthr, i + (int)step);
      if (C::poisoned(s)) {
        if constexpr (C::PARTS == 4) s = add_lds_exact<C>(buf, nthr, i, i + (int)step);
        else s = add_lds<C, true>(lds_get_pt<C>(buf, nthr, i), buf, nthr, i + (int)step);  // G1: a call would cost
      }                                                                                        // the second wave/SIMD
      acc = s;
    }
    __syncthreads();
  }
  return acc;
}

template <class C>
__global__ __launch_bounds__(256, C::OCC) void k_msm_segsum28(const uint32_t* __restrict__ buckets, const uint32_t* __restrict__ off,
                                                              msm_geom g, size_t ngw, size_t rows_per_set, uint32_t* __restrict__ segs,
                                                              uint32_t* __restrict__ runs) {
  const size_t t = gtid();
  if (t >= ngw * g.nseg) return;
  const size_t gw = t / g.nseg;
  const uint32_t s = t % g.nseg;
  const uint32_t a = 1 + s * g.seglen;
  uint32_t last = a + g.seglen;
  if (last > g.nbuck) last = g.nbuck;
  const size_t krow = (gw % rows_per_set) * g.nbuck, brow = gw * g.nbuck;
  typename C::P run, tot;
  seg_run<C, false>(buckets, off, krow, brow, a, last, run, tot);
  if (C::poisoned(run) || C::poisoned(tot)) seg_run<C, true>(buckets, off, krow, brow, a, last, run, tot);
  stj28<C>(segs, t, tot);
  stj28<C>(runs, t, run);
}
// [k] run + tot, run and tot read from memory where the additions use them: the addend is not held in registers
// across the doublings (G2: 84 fewer live registers; the addition's spills went from ~1,350 scratch instructions per
// step to none)
template <class C, bool EXACT>
DH_DEV typename C::P seg_off(const uint32_t* __restrict__ run, uint32_t k, const uint32_t* __restrict__ tot) {
  typename C::P acc = C::inf();
#pragma unroll 1
  for (int bit = 31 - __builtin_clz(k); bit >= 0; bit--) {
    acc = C::dbl(acc);
    if ((k >> bit) & 1) acc = C::template add_mem<EXACT>(acc, run);
  }
  return C::template add_mem<EXACT>(acc, tot);
}
template <class C>
__global__ __launch_bounds__(256, C::OCC) void k_msm_segoff28(msm_geom g, size_t ngw, uint32_t* __restrict__ segs,
                                                              const uint32_t* __restrict__ runs) {
  const size_t t = gtid();
  if (t >= ngw * g.nseg) return;
  const uint32_t k = (t % g.nseg) * g.seglen;  // a - 1
  if (!k) return;
  const uint32_t* run = runs + (size_t)3 * C::EW * t;
  if (ldj28<C>(runs, t).inf) return;  // run at infinity: the segment's value is tot as stored
  uint32_t* tot = segs + (size_t)3 * C::EW * t;
  typename C::P r = seg_off<C, false>(run, k, tot);
  if (C::poisoned(r)) r = seg_off<C, true>(run, k, tot);
  stj28<C>(segs, t, r);
}

// The segment values of a (set, group, window) row summed by wave-level trees through LDS (r04: a tree of log2(nseg)
// launches of one addition per thread, 12 at level 0). A tree inside a wave keeps few lanes busy (63 additions over 6
// steps of 64 lanes), so k_msm_rowtree28 first has each lane add G consecutive segment values in a serial run (G = 8
// for many rows of more than 64 segments: 7/8 of the additions at full lane use; 2 for level 0's few rows, whose
// latency the one call waits on), then the wave tree sums the lanes: a
// row's lanes (lpr = nseg / G, rounded up to a power of two <= 64 with the extra lanes holding the identity) leave the
// row sum in its first lane, or, for more than 64 lanes (a multiple of 64: fit_segments), one partial per wave that
// k_msm_rowred28 (one wave per row) sums the same way. Measured against r04's launch tree on the tbls MSMs (64 groups of
// 2 windows of 2,048 segments, gpurun_out r05w): the pure wave tree was 8.2 ms against 4.4.
template <class C>
__global__ __launch_bounds__(256, C::OCC) void k_msm_rowtree28(const uint32_t* __restrict__ segs, uint32_t nseg, uint32_t G,
                                                               size_t ngw, uint32_t lpr, uint32_t span, uint32_t* __restrict__ out) {
  __shared__ uint32_t buf[lds_words<C>() * 256];
  const size_t t = gtid();
  typename C::P acc = C::inf();
  if (t < ngw * lpr) {
    const size_t row = t / lpr;
    const uint32_t s0 = (uint32_t)(t % lpr) * G;
    const uint32_t* p = segs + (size_t)3 * C::EW * (row * nseg + s0);
    const uint32_t cnt = s0 >= nseg ? 0 : min(G, nseg - s0);
    acc = run_mem<C, false>(p, cnt);
    if (C::poisoned(acc)) acc = run_mem<C, true>(p, cnt);
  }
  acc = wave_tree<C>(acc, buf, span);
  if (t < ngw * lpr && (t & (span - 1)) == 0) stj28<C>(out, t / span, acc);
}
template <class C>
__global__ __launch_bounds__(64) void k_msm_rowred28(const uint32_t* __restrict__ parts_in, uint32_t parts, uint32_t span,
                                                     uint32_t* __restrict__ rowsum) {
  __shared__ uint32_t buf[lds_words<C>() * 64];
  const size_t row = blockIdx.x;
  typename C::P acc = run_mem<C, false>(parts_in, row * parts, parts);
  if (C::poisoned(acc)) acc = run_mem<C, true>(parts_in, row * parts, parts);
  acc = wave_tree<C>(acc, buf, span);
  if (threadIdx.x == 0) stj28<C>(rowsum, row, acc);
}

template <class C, bool EXACT>
DH_DEV typename C::P horner28(const uint32_t* __restrict__ rowsum, const msm_geom& g, size_t t) {
  typename C::P acc = ldj28<C>(rowsum, t * g.nwin + g.nwin - 1);
#pragma unroll 1
  for (int w = g.nwin - 2; w >= 0; w--) {
#pragma unroll 1
    for (int k = 0; k < g.c; k++) acc = C::dbl(acc);
    acc = C::template add_mem<EXACT>(acc, rowsum + (size_t)3 * C::EW * (t * g.nwin + w));
  }
  return acc;
}

// per (set, group): Horner over the windows' row sums, out = 12 x 32-bit Montgomery Jacobian (jac_inf for the identity)
template <class C>
__global__ __launch_bounds__(64) void k_msm_windows28(const uint32_t* __restrict__ rowsum, msm_geom g, size_t ngroups,
                                                      uint32_t* __restrict__ out) {
  const size_t t = gtid();
  if (t >= ngroups) return;
  typename C::P acc = horner28<C, false>(rowsum, g, t);
  if (C::poisoned(acc)) acc = horner28<C, true>(rowsum, g, t);
  jac<typename C::F> r = jac_inf<typename C::F>();
  if (!acc.inf) {
    r.x = C::out(acc.x);
    r.y = C::out(acc.y);
    r.z = C::out(acc.z);
  }
  st_jac_aos<typename C::F>(out, t, r);
}

hipError_t launch_msm_prep28(int sig_g2, size_t n, uint8_t* status, const uint32_t* sig_aff, const uint32_t* q_pts,
                             uint32_t* S, uint32_t* Q, hipStream_t st, uint32_t sets) {
  if (!n) return hipSuccess;
  const uint32_t K = prep28_k(n);
  const size_t nt = (n + K - 1) / K;
  if (sig_g2)
    hipLaunchKernelGGL(k_msm_prep28<c28_g2>, dim3(nblk(nt, 256)), dim3(256), 0, st, n, K, status, sig_aff, q_pts, S, Q, sets);
  else
    hipLaunchKernelGGL(k_msm_prep28<c28_g1>, dim3(nblk(nt, 256)), dim3(256), 0, st, n, K, status, sig_aff, q_pts, S, Q, sets);
  return hipGetLastError();
}

// Block size of the reduction kernels: 64 threads when the launch holds at most one wave per CU (level 0's few rows),
// so its waves land on separate CUs instead of four to a CU. These kernels spill (G2: ~1 KB per lane) and run one wave
// per SIMD, so their time is the latency of scratch round trips through the CU's vector cache, which four waves on one
// CU share: the G2 level-0 row tree took 1.13 ms in 256-thread blocks and 0.58 ms in 64-thread blocks (rocprofv3
// single-stream batches, profiles/r05/rocprof_unchained_rowtree_blk*_r05x2.csv). Launches with more waves keep
// 256-thread blocks (the row tree's LDS buffer is sized for 256 lanes: one 64-lane block per CU would cap the many-row
// launches at 256 waves).
static unsigned few_waves_block(size_t nthreads) { return nthreads <= 256 * 64 ? 64u : 256u; }

// nsets = 2: the sigma points S and the hash points Q share the sorted lists (the batch check); 1: S only
template <class C>
static hipError_t msm28(const msm_geom& g, size_t ngroups, const uint32_t* S, const uint32_t* Q, msm_ws& ws, hipStream_t st,
                        const uint8_t* skip, int nsets = 2) {
  const size_t nk = ngroups * g.nwin * (size_t)g.nbuck;
  constexpr size_t jw = 3 * C::EW;
  uint32_t* bB = ws.buckets + nk * jw;
  uint32_t* pB = ws.part + msm_nchunks(ws.max_entries) * 2 * jw;
  if (ws.max_entries) {
    // chunks of up to LCAP entries (G2: 64, so half as many keys cut by chunk boundaries for k_msm_bucket_fix28),
    // about two per lane the chip holds at the pass's occupancy (G1 2 waves/SIMD: 262,144 chunks; G2 1: 131,072)
    const uint32_t L = msm_chunk_len(ws.max_entries, C::LCAP, (size_t)C::OCC * 131072);
    const size_t nch = (ws.max_entries + L - 1) / L;
    hipLaunchKernelGGL((k_msm_bucket28<C, true>), dim3(nblk(nch, 256)), dim3(256), 0, st, ws.off, ws.list, nk, L, S, ws.buckets,
                       ws.part, ws.meta, skip, g.half_stride);
    hipLaunchKernelGGL(k_msm_bucket_fix28<C>, dim3(nblk(nch, 256)), dim3(256), 0, st, ws.off, nk, L, ws.meta, ws.part, ws.buckets);
    if (nsets == 2) {
      hipLaunchKernelGGL((k_msm_bucket28<C, true>), dim3(nblk(nch, 256)), dim3(256), 0, st, ws.off, ws.list, nk, L, Q, bB, pB,
                         ws.meta, skip, g.half_stride);
      hipLaunchKernelGGL(k_msm_bucket_fix28<C>, dim3(nblk(nch, 256)), dim3(256), 0, st, ws.off, nk, L, ws.meta, pB, bB);
    }
  }
  const size_t rows = ngroups * g.nwin, ngw = (size_t)nsets * rows;
  const unsigned sb = few_waves_block(ngw * g.nseg);
  hipLaunchKernelGGL(k_msm_segsum28<C>, dim3(nblk(ngw * g.nseg, sb)), dim3(sb), 0, st, ws.buckets, ws.off, g, ngw, rows, ws.segs,
                     ws.runs);
  if (g.nseg > 1)
    hipLaunchKernelGGL(k_msm_segoff28<C>, dim3(nblk(ngw * g.nseg, sb)), dim3(sb), 0, st, g, ngw, ws.segs, ws.runs);
  // row sums: ws.runs (free after the offsets) when a row's lanes fit one wave; else the waves' partials go to ws.runs
  // and the row sums to ws.segs
  // G: 8 when the rows' segments are many (the additions' count matters: the bisection's and the tbls per-signer
  // levels), 2 when they are few (level 0: 4-8 rows, where the serial run lengthens the one call's latency path)
  uint32_t G = g.nseg <= 64 ? 1 : (ngw * g.nseg >= ((size_t)1 << 17) ? 8 : 2);
  if (G == 2 && g.nseg / 2 > 64 && (g.nseg / 2) % 64) G = 8;
  uint32_t lpr = (g.nseg + G - 1) / G, span = 64;
  if (lpr <= 64) {
    for (span = 1; span < lpr;) span *= 2;
    lpr = span;
  } else if (lpr % 64) {
    // whole waves per row (fit_segments keeps rows of more than 512 segments at a multiple of 512, but the recover and
    // tbls callers do not run it): the extra lanes start past nseg and add the identity
    lpr = (lpr + 63) / 64 * 64;
  }
  const uint32_t* rowsum = ws.runs;
  if (g.nseg > 1)
    hipLaunchKernelGGL(k_msm_rowtree28<C>, dim3(nblk(ngw * lpr, few_waves_block(ngw * lpr))), dim3(few_waves_block(ngw * lpr)), 0,
                       st, ws.segs, g.nseg, G, ngw, lpr, span, ws.runs);
  else
    rowsum = ws.segs;  // one segment per row: its value is the row sum
  if (lpr > 64) {
    const uint32_t parts = lpr / 64;
    uint32_t pspan = 1;
    while (pspan < parts) pspan *= 2;
    hipLaunchKernelGGL(k_msm_rowred28<C>, dim3((unsigned)ngw), dim3(64), 0, st, ws.runs, parts, pspan, ws.segs);
    rowsum = ws.segs;
  }
  hipLaunchKernelGGL(k_msm_windows28<C>, dim3(nblk(nsets * ngroups, 64)), dim3(64), 0, st, rowsum, g, nsets * ngroups, ws.out2);
  return hipGetLastError();
}

// the RLC MSM on the 28-bit points of launch_msm_prep28: both point sets, one reduction pass over 2 x ngroups
hipError_t launch_msm28(int sig_g2, const msm_geom& g, const uint32_t* entries, size_t m, size_t ngroups, const uint4* scal,
                        const uint32_t* S, const uint32_t* Q, msm_ws& ws, uint32_t* outA, uint32_t* outB, hipStream_t st,
                        const uint8_t* skip, bool presorted) {
  hipError_t e = hipSuccess;
  if (!presorted && (e = launch_msm_sort(g, entries, nullptr, nullptr, m, ngroups, scal, ws, st)) != hipSuccess) return e;
  e = sig_g2 ? msm28<c28_g2>(g, ngroups, S, Q, ws, st, skip) : msm28<c28_g1>(g, ngroups, S, Q, ws, st, skip);
  if (e != hipSuccess) return e;
  const size_t ow = sig_g2 ? 72 : 36, bytes = ngroups * ow * 4;
  if ((e = hipMemcpyAsync(outA, ws.out2, bytes, hipMemcpyDeviceToDevice, st)) != hipSuccess) return e;
  return hipMemcpyAsync(outB, ws.out2 + ngroups * ow, bytes, hipMemcpyDeviceToDevice, st);
}

// one point set of 28-bit points (launch_msm_prep28): entry e is point pidx[e] (+ its endomorphism images at
// g.half_stride steps) with scalar scal[sidx ? sidx[e] : pidx[e]] in group grp ? grp[e] : e / g.gsize; out: ngroups
// 12 x 32-bit Jacobian sums (the tbls Recover's VerifyPartial batch: all partials' sigmas, the hash points per signer)
hipError_t launch_msm28_set(int sig_g2, const msm_geom& g, const uint32_t* pidx, const uint32_t* sidx, const uint32_t* grp,
                            size_t m, size_t ngroups, const uint4* scal, const uint32_t* P, msm_ws& ws, uint32_t* out,
                            hipStream_t st) {
  hipError_t e = launch_msm_sort(g, pidx, sidx, grp, m, ngroups, scal, ws, st);
  if (e != hipSuccess) return e;
  e = sig_g2 ? msm28<c28_g2>(g, ngroups, P, nullptr, ws, st, nullptr, 1) : msm28<c28_g1>(g, ngroups, P, nullptr, ws, st, nullptr, 1);
  if (e != hipSuccess) return e;
  return hipMemcpyAsync(out, ws.out2, ngroups * (sig_g2 ? 72 : 36) * 4, hipMemcpyDeviceToDevice, st);
}

// bisection: the entries of the failing groups, in order, on the device (groups are runs of gsize consecutive entries,
// only the last one partial, so a failing group's entries land at rank(group) * gsize + their offset in the group)
__global__ void k_fail_flags(const uint8_t* __restrict__ pass, size_t ngroups, uint32_t* __restrict__ flags) {
  const size_t g = gtid();
  if (g < ngroups) flags[g] = pass[g] ? 0u : 1u;
}
__global__ void k_compact_failing(const uint32_t* __restrict__ entries, size_t m, size_t gsize, const uint8_t* __restrict__ pass,
                                  const uint32_t* __restrict__ rank, uint32_t* __restrict__ out) {
  const size_t e = gtid();
  if (e >= m) return;
  const size_t g = e / gsize;
  if (!pass[g]) out[(size_t)rank[g] * gsize + (e - g * gsize)] = entries[e];
}
hipError_t launch_compact_failing(const uint32_t* entries, size_t m, size_t gsize, size_t ngroups, const uint8_t* pass,
                                  uint32_t* flags, uint32_t* rank, uint32_t* scan_tmp, uint32_t* out, hipStream_t st) {
  if (!m) return hipSuccess;
  hipLaunchKernelGGL(k_fail_flags, dim3(nblk(ngroups, 256)), dim3(256), 0, st, pass, ngroups, flags);
  hipError_t e = launch_scan(flags, ngroups, rank, scan_tmp, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_compact_failing, dim3(nblk(m, 256)), dim3(256), 0, st, entries, m, gsize, pass, rank, out);
  return hipGetLastError();
}

hipError_t launch_mark_groups(const uint32_t* entries, size_t m, size_t gsize, const uint8_t* pass, const uint8_t* status,
                              uint8_t* verdict, hipStream_t st) {
  if (!m) return hipSuccess;
  hipLaunchKernelGGL(k_mark_groups, dim3(nblk(m, 256)), dim3(256), 0, st, entries, m, gsize, pass, status, verdict);
  return hipGetLastError();
}


DH_COUNTER_ACCESSOR(msm)

}  // namespace dh
