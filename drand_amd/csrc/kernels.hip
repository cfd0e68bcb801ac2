// Batch beacon-verification kernels for gfx950.
//
// Path (one call of dh_verify_batch, see drandhip.cpp):
//   k_prep_sig     decode + subgroup-check every signature, randomness = SHA-256(sig)    [A4a, A5]
//   k_prep_msg     DigestBeacon + hash_to_curve without cofactor clearing               [A2, A3, A4b]
//   k_scalars      128-bit random-linear-combination scalars r_i = SHA-256(seed || i)   [batching, new]
//   MSM (grouped Pippenger, shared sort for both point sets):
//     k_msm_hist -> scan -> k_msm_scatter -> k_msm_bucket<S>, k_msm_bucket<Q> -> k_msm_segsum -> k_msm_tree
//     -> k_msm_windows       per group g:  A_g = sum r_i sigma_i,  B_g = sum r_i Q_i
//   k_group_check  e(A_g, g2) == e([h_eff] B_g, pk)  (or the G2-signature mirror), one lane per group [A4c]
//   k_leaf_check   per-round 2-pairing check for rounds left in failing groups (bisection leaves)
// All scheme semantics follow /root/reference/crypto/schemes.go:70-72 (VerifyBeacon) and the kyber /
// kilic behaviour restated in oracle/bls_oracle.c.
#include <hip/hip_runtime.h>
#include "pairing.hpp"
#include "h2c.hpp"
#include "codec.hpp"
#include "kernels.hpp"

namespace dh {

// ---------------------------------------------------------------- point <-> AoS global memory (16-B aligned)
template <class F>
struct npw {  // words per field element
  static constexpr int N = limbs_of<F>::N;
};

template <class F>
DH_DEV void ld_f(F& a, const uint32_t* p);
template <>
DH_DEV void ld_f<fp>(fp& a, const uint32_t* p) {
  const uint4* q = (const uint4*)p;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    uint4 t = q[i];
    a.v[4 * i] = t.x; a.v[4 * i + 1] = t.y; a.v[4 * i + 2] = t.z; a.v[4 * i + 3] = t.w;
  }
}
template <>
DH_DEV void ld_f<fp2>(fp2& a, const uint32_t* p) {
  ld_f<fp>(a.c0, p);
  ld_f<fp>(a.c1, p + 12);
}
template <class F>
DH_DEV void st_f(uint32_t* p, const F& a);
template <>
DH_DEV void st_f<fp>(uint32_t* p, const fp& a) {
  uint4* q = (uint4*)p;
#pragma unroll
  for (int i = 0; i < 3; i++) q[i] = make_uint4(a.v[4 * i], a.v[4 * i + 1], a.v[4 * i + 2], a.v[4 * i + 3]);
}
template <>
DH_DEV void st_f<fp2>(uint32_t* p, const fp2& a) {
  st_f<fp>(p, a.c0);
  st_f<fp>(p + 12, a.c1);
}
template <class F>
DH_DEV jac<F> ld_jac_aos(const uint32_t* base, size_t i) {
  constexpr int N = npw<F>::N;
  const uint32_t* p = base + (size_t)3 * N * i;
  jac<F> r;
  ld_f<F>(r.x, p);
  ld_f<F>(r.y, p + N);
  ld_f<F>(r.z, p + 2 * N);
  return r;
}
template <class F>
DH_DEV void st_jac_aos(uint32_t* base, size_t i, const jac<F>& a) {
  constexpr int N = npw<F>::N;
  uint32_t* p = base + (size_t)3 * N * i;
  st_f<F>(p, a.x);
  st_f<F>(p + N, a.y);
  st_f<F>(p + 2 * N, a.z);
}
template <class F>
DH_DEV aff<F> ld_aff_aos(const uint32_t* base, size_t i) {
  constexpr int N = npw<F>::N;
  const uint32_t* p = base + (size_t)2 * N * i;
  aff<F> r;
  ld_f<F>(r.x, p);
  ld_f<F>(r.y, p + N);
  return r;
}
template <class F>
DH_DEV void st_aff_aos(uint32_t* base, size_t i, const aff<F>& a) {
  constexpr int N = npw<F>::N;
  uint32_t* p = base + (size_t)2 * N * i;
  st_f<F>(p, a.x);
  st_f<F>(p + N, a.y);
}

// the other group of the pairing
template <class F>
struct other;
template <>
struct other<fp> {
  using T = fp2;
};
template <>
struct other<fp2> {
  using T = fp;
};

DH_DEV size_t gtid() { return (size_t)blockIdx.x * blockDim.x + threadIdx.x; }

// ---------------------------------------------------------------- prep: signatures
template <class F>
__global__ __launch_bounds__(256, 4) void k_prep_sig(const uint8_t* __restrict__ sigs, size_t stride, size_t n,
                                                  uint8_t* __restrict__ status, uint32_t* __restrict__ sig_aff,
                                                  uint8_t* __restrict__ rand_out) {
  size_t i = gtid();
  if (i >= n) return;
  const uint8_t* s = sigs + i * stride;
  aff<F> a;
  uint8_t st;
  if constexpr (sizeof(F) == sizeof(fp)) {
    st = g1_decompress(a, s, true);
    if (rand_out) st_digest(rand_out + 32 * i, sha256_aligned<48>(s));
  } else {
    st = g2_decompress(a, s, true);
    if (rand_out) st_digest(rand_out + 32 * i, sha256_aligned<96>(s));
  }
  if (st != DEC_OK) {
    a.x = F{};
    a.y = F{};
    st = DEC_BAD;  // infinity signatures are rejected like kilic's engine + kyber's verify
  }
  status[i] = st;
  st_aff_aos<F>(sig_aff, i, a);
}

// ---------------------------------------------------------------- prep: messages -> hash points (no cofactor)
template <class F>
__global__ __launch_bounds__(256, 4) void k_prep_msg(const uint64_t* __restrict__ rounds, const uint8_t* __restrict__ prevs,
                                                  size_t prev_stride, const uint32_t* __restrict__ prev_lens, size_t n,
                                                  int chained, int dst_id, uint32_t* __restrict__ q_out) {
  size_t i = gtid();
  if (i >= n) return;
  sha_h d;
  if (chained) {
    uint32_t pl = prev_lens ? prev_lens[i] : (uint32_t)prev_stride;
    d = digest_chained(prevs + i * prev_stride, pl, rounds[i]);
  } else {
    d = digest_unchained(rounds[i]);
  }
  if constexpr (sizeof(F) == sizeof(fp)) {
    st_jac_aos<fp>(q_out, i, h2c_g1_noclear(d, dst_id));
  } else {
    st_jac_aos<fp2>(q_out, i, h2c_g2_noclear(d, dst_id));
  }
}

// ---------------------------------------------------------------- RLC scalars
// r_i = first 16 bytes of SHA-256(seed[32] || i_be64), 0 for rounds that failed decoding.
__global__ __launch_bounds__(256) void k_scalars(const uint32_t* __restrict__ seed_words, size_t n,
                                                 const uint8_t* __restrict__ status, uint4* __restrict__ scal) {
  size_t i = gtid();
  if (i >= n) return;
  uint32_t w[16];
#pragma unroll
  for (int j = 0; j < 8; j++) w[j] = seed_words[j];
  w[8] = (uint32_t)((uint64_t)i >> 32);
  w[9] = (uint32_t)i;
  w[10] = 0x80000000u;
#pragma unroll
  for (int j = 11; j < 15; j++) w[j] = 0;
  w[15] = 40 * 8;
  sha_h s = sha_iv();
  sha_compress(s, w);
  uint4 r = make_uint4(s.h[3], s.h[2], s.h[1], s.h[0]);  // little-endian words of a 128-bit integer
  if (status[i] != DEC_OK) r = make_uint4(0, 0, 0, 0);
  scal[i] = r;
}

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

__global__ void k_msm_hist(const uint32_t* __restrict__ entries, size_t m, const uint4* __restrict__ scal, msm_geom g,
                           uint32_t* __restrict__ cnt) {
  size_t e = gtid();
  if (e >= m) return;
  const uint4 s = scal[entries[e]];
  const size_t grp = e / g.gsize;
  for (int w = 0; w < g.nwin; w++) {
    uint32_t d = scalar_digit(s, w * g.c, g.c);
    if (d) atomicAdd(&cnt[(grp * g.nwin + w) * g.nbuck + d], 1u);
  }
}

__global__ void k_msm_scatter(const uint32_t* __restrict__ entries, size_t m, const uint4* __restrict__ scal,
                              msm_geom g, uint32_t* __restrict__ cursor, uint32_t* __restrict__ list) {
  size_t e = gtid();
  if (e >= m) return;
  const uint32_t idx = entries[e];
  const uint4 s = scal[idx];
  const size_t grp = e / g.gsize;
  for (int w = 0; w < g.nwin; w++) {
    uint32_t d = scalar_digit(s, w * g.c, g.c);
    if (d) {
      uint32_t pos = atomicAdd(&cursor[(grp * g.nwin + w) * g.nbuck + d], 1u);
      list[pos] = idx;
    }
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

// bucket accumulation: one thread per (group, window, digit) key. P = affine (madd) or Jacobian (add) inputs.
template <class F, bool AFFINE>
__global__ __launch_bounds__(256, 4) void k_msm_bucket(const uint32_t* __restrict__ off, const uint32_t* __restrict__ list,
                                                    size_t nkeys, const uint32_t* __restrict__ pts,
                                                    uint32_t* __restrict__ buckets) {
  size_t k = gtid();
  if (k >= nkeys) return;
  uint32_t b = off[k], e = off[k + 1];
  jac<F> acc = jac_inf<F>();
  for (uint32_t j = b; j < e; j++) {
    uint32_t idx = list[j];
    if constexpr (AFFINE) {
      acc = jac_add_aff(acc, ld_aff_aos<F>(pts, idx));
    } else {
      acc = jac_add(acc, ld_jac_aos<F>(pts, idx));
    }
  }
  st_jac_aos<F>(buckets, k, acc);
}

// per (group, window, segment): sum_{d in seg} d * B_d via running sums; seg covers digits [a, a + len)
template <class F>
__global__ __launch_bounds__(256, 4) void k_msm_segsum(const uint32_t* __restrict__ buckets, msm_geom g, size_t ngw,
                                                    uint32_t* __restrict__ segs) {
  size_t t = gtid();
  if (t >= ngw * g.nseg) return;
  const size_t gw = t / g.nseg;
  const uint32_t s = t % g.nseg;
  const uint32_t a = 1 + s * g.seglen;  // first digit of the segment
  uint32_t last = a + g.seglen;         // exclusive
  if (last > g.nbuck) last = g.nbuck;
  jac<F> run = jac_inf<F>(), tot = jac_inf<F>();
  for (int d = (int)last - 1; d >= (int)a; d--) {
    run = jac_add(run, ld_jac_aos<F>(buckets, gw * g.nbuck + d));
    tot = jac_add(tot, run);
  }
  // tot = sum (d - a + 1) B_d ; add (a - 1) * run
  uint32_t k = a - 1;
  if (k && !jac_is_inf(run)) {
    jac<F> acc = jac_inf<F>();
    for (int bit = 31 - __builtin_clz(k); bit >= 0; bit--) {
      acc = jac_dbl(acc);
      if ((k >> bit) & 1) acc = jac_add(acc, run);
    }
    tot = jac_add(tot, acc);
  }
  st_jac_aos<F>(segs, t, tot);
}

// pairwise tree reduction in place over rows of `stride` points whose first `width` are live:
// v[r][c] += v[r][c + half] for c + half < width
template <class F>
__global__ __launch_bounds__(256, 4) void k_msm_tree(uint32_t* __restrict__ v, size_t rows, uint32_t stride, uint32_t width,
                                                  uint32_t half) {
  size_t t = gtid();
  if (t >= rows * half) return;
  size_t r = t / half, c = t % half;
  if (c + half >= width) return;
  size_t i = r * stride + c;
  st_jac_aos<F>(v, i, jac_add(ld_jac_aos<F>(v, i), ld_jac_aos<F>(v, i + half)));
}

// per group: Horner over windows, result[g] = sum_w 2^(c w) W_{g,w}; W_{g,w} = segs[(g*nwin + w) * nseg]
template <class F>
__global__ __launch_bounds__(64) void k_msm_windows(const uint32_t* __restrict__ segs, msm_geom g, size_t ngroups,
                                                    uint32_t* __restrict__ out) {
  size_t t = gtid();
  if (t >= ngroups) return;
  jac<F> acc = ld_jac_aos<F>(segs, (t * g.nwin + g.nwin - 1) * g.nseg);
  for (int w = g.nwin - 2; w >= 0; w--) {
    for (int k = 0; k < g.c; k++) acc = jac_dbl(acc);
    acc = jac_add(acc, ld_jac_aos<F>(segs, (t * g.nwin + w) * g.nseg));
  }
  st_jac_aos<F>(out, t, acc);
}

// ---------------------------------------------------------------- key decode (one thread)
template <class K>
__global__ void k_decode_key(const uint8_t* __restrict__ pk, uint32_t* __restrict__ key_aff, uint8_t* __restrict__ ok) {
  if (gtid() != 0) return;
  aff<K> a;
  uint8_t st;
  if constexpr (sizeof(K) == sizeof(fp)) st = g1_decompress(a, pk, true);
  else st = g2_decompress(a, pk, true);
  *ok = st;
  if (st != DEC_OK) {
    a.x = K{};
    a.y = K{};
  }
  st_aff_aos<K>(key_aff, 0, a);
}

DH_DEV jac<fp> g1_gen() { return {fp_c(cst::G1X), fp_c(cst::G1Y), fp_one()}; }
DH_DEV jac<fp2> g2_gen() { return {fp2_c(cst::G2X), fp2_c(cst::G2Y), fp2_one()}; }

// the verification equation for signature sum S and (cofactor-cleared) hash sum H:
//   G1 signatures: e(H, pk) * e(-S, g2) == 1       G2 signatures: e(pk, H) * e(-g1, S) == 1
// (kyber-bls12381 ValidatePairing(p1,p2,p3,p4) = AddPair(p1,p2), AddPairInv(p3,p4), Check())
DH_DEV bool check_g1sig(const jac<fp>& S, const jac<fp>& H, const aff<fp2>& pk) {
  jac<fp> P[2] = {H, jac_neg(S)};
  jac<fp2> Q[2] = {jac_from_aff(pk), g2_gen()};
  return pairing_check<2>(P, Q);
}
DH_DEV bool check_g2sig(const jac<fp2>& S, const jac<fp2>& H, const aff<fp>& pk) {
  jac<fp> P[2] = {jac_from_aff(pk), jac_neg(g1_gen())};
  jac<fp2> Q[2] = {H, S};
  return pairing_check<2>(P, Q);
}

// one lane per group: A = sum r sigma, B = sum r Q (pre-cofactor)
template <class F>
__global__ __launch_bounds__(64) void k_group_check(const uint32_t* __restrict__ A, const uint32_t* __restrict__ B,
                                                    size_t ngroups, const uint32_t* __restrict__ key_aff,
                                                    uint8_t* __restrict__ pass) {
  size_t t = gtid();
  if (t >= ngroups) return;
  jac<F> S = ld_jac_aos<F>(A, t);
  jac<F> Hq = ld_jac_aos<F>(B, t);
  bool ok;
  if constexpr (sizeof(F) == sizeof(fp)) {
    ok = check_g1sig(S, h2c_clear_g1(Hq), ld_aff_aos<fp2>(key_aff, 0));
  } else {
    ok = check_g2sig(S, h2c_clear_g2(Hq), ld_aff_aos<fp>(key_aff, 0));
  }
  pass[t] = ok ? 1 : 0;
}

// bisection leaves: full per-round verification of the listed rounds
template <class F>
__global__ __launch_bounds__(64) void k_leaf_check(const uint32_t* __restrict__ entries, size_t m,
                                                   const uint32_t* __restrict__ sig_aff, const uint32_t* __restrict__ q_pts,
                                                   const uint32_t* __restrict__ key_aff, const uint8_t* __restrict__ status,
                                                   uint8_t* __restrict__ verdict) {
  size_t t = gtid();
  if (t >= m) return;
  uint32_t i = entries[t];
  if (status[i] != DEC_OK) {
    verdict[i] = 0;
    return;
  }
  jac<F> S = jac_from_aff(ld_aff_aos<F>(sig_aff, i));
  jac<F> Hq = ld_jac_aos<F>(q_pts, i);
  bool ok;
  if constexpr (sizeof(F) == sizeof(fp)) {
    ok = check_g1sig(S, h2c_clear_g1(Hq), ld_aff_aos<fp2>(key_aff, 0));
  } else {
    ok = check_g2sig(S, h2c_clear_g2(Hq), ld_aff_aos<fp>(key_aff, 0));
  }
  verdict[i] = ok ? 1 : 0;
}

// verdict for every entry of a passing group: status == OK
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

// ---------------------------------------------------------------- synthetic-chain signer (tests / bench data)
// sig_i = [sk] H(DigestBeacon(round_i, prev_i)), compressed. Not on the verification path.
template <class F>
__global__ __launch_bounds__(256, 4) void k_sign(const uint32_t* __restrict__ sk, const uint64_t* __restrict__ rounds,
                                                 const uint8_t* __restrict__ prevs, size_t prev_stride,
                                                 const uint32_t* __restrict__ prev_lens, size_t n, int chained, int dst_id,
                                                 uint8_t* __restrict__ out) {
  size_t i = gtid();
  if (i >= n) return;
  sha_h d;
  if (chained) {
    uint32_t pl = prev_lens ? prev_lens[i] : (uint32_t)prev_stride;
    d = digest_chained(prevs + i * prev_stride, pl, rounds[i]);
  } else {
    d = digest_unchained(rounds[i]);
  }
  if constexpr (sizeof(F) == sizeof(fp)) {
    jac<fp> h = h2c_clear_g1(h2c_g1_noclear(d, dst_id));
    g1_compress(out + 48 * i, jac_mul_words(h, sk, 256));
  } else {
    jac<fp2> h = h2c_clear_g2(h2c_g2_noclear(d, dst_id));
    g2_compress(out + 96 * i, jac_mul_words(h, sk, 256));
  }
}

// public key [sk] g in the key group
template <class K>
__global__ void k_pubkey(const uint32_t* __restrict__ sk, uint8_t* __restrict__ out) {
  if (gtid() != 0) return;
  if constexpr (sizeof(K) == sizeof(fp)) {
    g1_compress(out, jac_mul_words(g1_gen(), sk, 256));
  } else {
    g2_compress(out, jac_mul_words(g2_gen(), sk, 256));
  }
}

// ---------------------------------------------------------------- host launchers
static inline unsigned nblk(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

hipError_t launch_prep(int sig_g2, const uint8_t* sigs, size_t stride, size_t n, uint8_t* status, uint32_t* sig_aff,
                       uint8_t* rand_out, hipStream_t st) {
  if (!n) return hipSuccess;
  if (sig_g2)
    hipLaunchKernelGGL(k_prep_sig<fp2>, dim3(nblk(n, 256)), dim3(256), 0, st, sigs, stride, n, status, sig_aff, rand_out);
  else
    hipLaunchKernelGGL(k_prep_sig<fp>, dim3(nblk(n, 256)), dim3(256), 0, st, sigs, stride, n, status, sig_aff, rand_out);
  return hipGetLastError();
}

hipError_t launch_msg(int sig_g2, const uint64_t* rounds, const uint8_t* prevs, size_t prev_stride, const uint32_t* prev_lens,
                      size_t n, int chained, int dst_id, uint32_t* q_out, hipStream_t st) {
  if (!n) return hipSuccess;
  if (sig_g2)
    hipLaunchKernelGGL(k_prep_msg<fp2>, dim3(nblk(n, 256)), dim3(256), 0, st, rounds, prevs, prev_stride, prev_lens, n,
                       chained, dst_id, q_out);
  else
    hipLaunchKernelGGL(k_prep_msg<fp>, dim3(nblk(n, 256)), dim3(256), 0, st, rounds, prevs, prev_stride, prev_lens, n,
                       chained, dst_id, q_out);
  return hipGetLastError();
}

hipError_t launch_scalars(const uint32_t* seed_words, size_t n, const uint8_t* status, uint4* scal, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_scalars, dim3(nblk(n, 256)), dim3(256), 0, st, seed_words, n, status, scal);
  return hipGetLastError();
}

hipError_t launch_decode_key(int key_g2, const uint8_t* pk, uint32_t* key_aff, uint8_t* ok, hipStream_t st) {
  if (key_g2) hipLaunchKernelGGL(k_decode_key<fp2>, dim3(1), dim3(64), 0, st, pk, key_aff, ok);
  else hipLaunchKernelGGL(k_decode_key<fp>, dim3(1), dim3(64), 0, st, pk, key_aff, ok);
  return hipGetLastError();
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

template <class F>
static hipError_t msm_reduce(const msm_geom& g, size_t ngroups, uint32_t* buckets, uint32_t* segs, uint32_t* out,
                             hipStream_t st) {
  size_t ngw = ngroups * g.nwin;
  hipLaunchKernelGGL(k_msm_segsum<F>, dim3(nblk(ngw * g.nseg, 256)), dim3(256), 0, st, buckets, g, ngw, segs);
  for (uint32_t width = g.nseg; width > 1;) {
    uint32_t half = (width + 1) / 2;
    hipLaunchKernelGGL(k_msm_tree<F>, dim3(nblk(ngw * half, 256)), dim3(256), 0, st, segs, ngw, g.nseg, width, half);
    width = half;  // live prefix of each row; the row stride stays nseg
  }
  hipLaunchKernelGGL(k_msm_windows<F>, dim3(nblk(ngroups, 64)), dim3(64), 0, st, segs, g, ngroups, out);
  return hipGetLastError();
}

hipError_t launch_msm(int sig_g2, const msm_geom& g, const uint32_t* entries, size_t m, size_t ngroups, const uint4* scal,
                      const uint32_t* sig_aff, const uint32_t* q_pts, msm_ws& ws, uint32_t* outA, uint32_t* outB,
                      hipStream_t st) {
  size_t nk = ngroups * g.nwin * (size_t)g.nbuck;
  hipError_t e = hipMemsetAsync(ws.cnt, 0, nk * sizeof(uint32_t), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_msm_hist, dim3(nblk(m, 256)), dim3(256), 0, st, entries, m, scal, g, ws.cnt);
  if ((e = launch_scan(ws.cnt, nk, ws.off, ws.scan_tmp, st)) != hipSuccess) return e;
  if ((e = hipMemcpyAsync(ws.cnt, ws.off, nk * sizeof(uint32_t), hipMemcpyDeviceToDevice, st)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_msm_scatter, dim3(nblk(m, 256)), dim3(256), 0, st, entries, m, scal, g, ws.cnt, ws.list);
  if (sig_g2) {
    hipLaunchKernelGGL((k_msm_bucket<fp2, true>), dim3(nblk(nk, 256)), dim3(256), 0, st, ws.off, ws.list, nk, sig_aff,
                       ws.buckets);
    if ((e = msm_reduce<fp2>(g, ngroups, ws.buckets, ws.segs, outA, st)) != hipSuccess) return e;
    hipLaunchKernelGGL((k_msm_bucket<fp2, false>), dim3(nblk(nk, 256)), dim3(256), 0, st, ws.off, ws.list, nk, q_pts,
                       ws.buckets);
    if ((e = msm_reduce<fp2>(g, ngroups, ws.buckets, ws.segs, outB, st)) != hipSuccess) return e;
  } else {
    hipLaunchKernelGGL((k_msm_bucket<fp, true>), dim3(nblk(nk, 256)), dim3(256), 0, st, ws.off, ws.list, nk, sig_aff,
                       ws.buckets);
    if ((e = msm_reduce<fp>(g, ngroups, ws.buckets, ws.segs, outA, st)) != hipSuccess) return e;
    hipLaunchKernelGGL((k_msm_bucket<fp, false>), dim3(nblk(nk, 256)), dim3(256), 0, st, ws.off, ws.list, nk, q_pts,
                       ws.buckets);
    if ((e = msm_reduce<fp>(g, ngroups, ws.buckets, ws.segs, outB, st)) != hipSuccess) return e;
  }
  return hipGetLastError();
}

hipError_t launch_group_check(int sig_g2, const uint32_t* A, const uint32_t* B, size_t ngroups, const uint32_t* key_aff,
                              uint8_t* pass, hipStream_t st) {
  if (sig_g2)
    hipLaunchKernelGGL(k_group_check<fp2>, dim3(nblk(ngroups, 64)), dim3(64), 0, st, A, B, ngroups, key_aff, pass);
  else
    hipLaunchKernelGGL(k_group_check<fp>, dim3(nblk(ngroups, 64)), dim3(64), 0, st, A, B, ngroups, key_aff, pass);
  return hipGetLastError();
}

hipError_t launch_mark_groups(const uint32_t* entries, size_t m, size_t gsize, const uint8_t* pass, const uint8_t* status,
                              uint8_t* verdict, hipStream_t st) {
  if (!m) return hipSuccess;
  hipLaunchKernelGGL(k_mark_groups, dim3(nblk(m, 256)), dim3(256), 0, st, entries, m, gsize, pass, status, verdict);
  return hipGetLastError();
}

hipError_t launch_leaf_check(int sig_g2, const uint32_t* entries, size_t m, const uint32_t* sig_aff, const uint32_t* q_pts,
                             const uint32_t* key_aff, const uint8_t* status, uint8_t* verdict, hipStream_t st) {
  if (!m) return hipSuccess;
  if (sig_g2)
    hipLaunchKernelGGL(k_leaf_check<fp2>, dim3(nblk(m, 64)), dim3(64), 0, st, entries, m, sig_aff, q_pts, key_aff, status,
                       verdict);
  else
    hipLaunchKernelGGL(k_leaf_check<fp>, dim3(nblk(m, 64)), dim3(64), 0, st, entries, m, sig_aff, q_pts, key_aff, status,
                       verdict);
  return hipGetLastError();
}

hipError_t launch_sign(int sig_g2, const uint32_t* sk, const uint64_t* rounds, const uint8_t* prevs, size_t prev_stride,
                       const uint32_t* prev_lens, size_t n, int chained, int dst_id, uint8_t* out, hipStream_t st) {
  if (!n) return hipSuccess;
  if (sig_g2)
    hipLaunchKernelGGL(k_sign<fp2>, dim3(nblk(n, 256)), dim3(256), 0, st, sk, rounds, prevs, prev_stride, prev_lens, n,
                       chained, dst_id, out);
  else
    hipLaunchKernelGGL(k_sign<fp>, dim3(nblk(n, 256)), dim3(256), 0, st, sk, rounds, prevs, prev_stride, prev_lens, n,
                       chained, dst_id, out);
  return hipGetLastError();
}

hipError_t launch_pubkey(int key_g2, const uint32_t* sk, uint8_t* out, hipStream_t st) {
  if (key_g2) hipLaunchKernelGGL(k_pubkey<fp2>, dim3(1), dim3(64), 0, st, sk, out);
  else hipLaunchKernelGGL(k_pubkey<fp>, dim3(1), dim3(64), 0, st, sk, out);
  return hipGetLastError();
}

}  // namespace dh
