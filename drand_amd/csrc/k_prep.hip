// Batch beacon-verification kernels for gfx950 — per-round preparation (this file), see also
// k_msm.hip, k_check.hip, k_sign.hip.
//
// Path (one call of dh_verify_batch, see drandhip.cpp):
//   k_prep_sig     decode + subgroup-check every signature, randomness = SHA-256(sig)    [A4a, A5]
//   k_prep_msg     DigestBeacon + hash_to_curve without cofactor clearing               [A2, A3, A4b]
//   k_scalars      128-bit random-linear-combination scalars r_i = SHA-256(seed || i)   [batching, new]
//   MSM (grouped Pippenger, shared sort for both point sets):
//     k_msm_hist -> scan -> k_msm_scatter -> k_msm_bucket28<S>, k_msm_bucket28<Q> -> k_msm_segsum28 -> k_msm_tree28
//     -> k_msm_windows       per group g:  A_g = sum r_i sigma_i,  B_g = sum r_i Q_i
//   k_group_check  e(A_g, g2) == e([h_eff] B_g, pk)  (or the G2-signature mirror), one lane per group [A4c]
//   k_leaf_check   per-round 2-pairing check for rounds left in failing groups (bisection leaves)
// All scheme semantics follow /root/reference/crypto/schemes.go:70-72 (VerifyBeacon) and the kyber /
// kilic behaviour restated in oracle/bls_oracle.c.
#include "kcommon.hpp"

namespace dh {

// ---------------------------------------------------------------- prep: signatures
template <class F>
__global__ __launch_bounds__(256, occ<F>::W) void k_prep_sig(const uint8_t* __restrict__ sigs, size_t stride, size_t n,
                                                  uint8_t* __restrict__ status, uint32_t* __restrict__ sig_aff,
                                                  uint8_t* __restrict__ rand_out) {
  size_t i = gtid();
  if (i >= n) return;
  const uint8_t* s = sigs + i * stride;
  aff<F> a;
  uint8_t st;
  if constexpr (sizeof(F) == sizeof(fp)) {
    // the point goes to HBM first and the subgroup test reloads it when it needs it (fp28.hpp g1_in_subgroup28)
    st = g1_decompress(a, s, false);
    if (st == DEC_OK) st_aff_aos<F>(sig_aff, i, a);
    if (rand_out) st_digest(rand_out + 32 * i, sha256_aligned<48>(s));
    if (st == DEC_OK && !g1_in_subgroup28([&] { return ld_aff_aos<fp>(sig_aff, i); })) st = DEC_BAD;
    if (st == DEC_OK) {
      status[i] = st;
      return;
    }
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

// G2 signatures in two passes: decompression (Fp2 square root) and the psi subgroup test each fit one lane's
// registers, the fused kernel spilled 1.1 KB per lane. The affine point and status go through HBM between them
// (96 + 1 B per round, written and read once).
__global__ __launch_bounds__(256, occ<fp2>::W) void k_dec_sig_g2(const uint8_t* __restrict__ sigs, size_t stride, size_t n,
                                                             uint8_t* __restrict__ status, uint32_t* __restrict__ sig_aff,
                                                             uint8_t* __restrict__ rand_out) {
  size_t i = gtid();
  if (i >= n) return;
  const uint8_t* s = sigs + i * stride;
  aff<fp2> a;
  uint8_t st = g2_decompress(a, s, false);
  if (rand_out) st_digest(rand_out + 32 * i, sha256_aligned<96>(s));
  if (st != DEC_OK) {
    a.x = fp2{};
    a.y = fp2{};
    st = DEC_BAD;  // infinity signatures are rejected like kilic's engine + kyber's verify
  }
  status[i] = st;
  st_aff_aos<fp2>(sig_aff, i, a);
}

// two waves per SIMD (some scratch) measured 5% faster over the whole unchained batch than one wave with the
// lazy-form test's values in VGPRs + AGPRs and no scratch (gpurun_out r03g: 80.1 against 84.1 ms per 1M rounds)
__global__ __launch_bounds__(256, 2) void k_sub_sig_g2(size_t n, uint8_t* __restrict__ status, uint32_t* __restrict__ sig_aff) {
  size_t i = gtid();
  if (i >= n || status[i] != DEC_OK) return;
  // P stays in HBM: the lazy-form test reloads it where it needs its coordinates (fp2_28.hpp g2_in_subgroup28)
  if (!g2_in_subgroup28([&] { return ld_aff_aos<fp2>(sig_aff, i); })) {
    status[i] = DEC_BAD;
    st_aff_aos<fp2>(sig_aff, i, aff<fp2>{fp2{}, fp2{}});
  }
}

// ---------------------------------------------------------------- small-batch path (drandhip.cpp verify_small)
// The signature pass split at the decoded point: the per-round pairing check needs only the point, so it starts as soon
// as the decode finishes and runs beside the subgroup test, whose result is ANDed into the verdict at the end
// (k_and_subgroup). A G1 round's decode is a fraction of k_prep_sig<fp> (one square root); the test (two [|u|] chains)
// is the rest. The subgroup kernels write only sub_bad (the point and status stay as the pairing check reads them).
__global__ __launch_bounds__(64) void k_dec_sig_g1(const uint8_t* __restrict__ sigs, size_t stride, size_t n,
                                                   uint8_t* __restrict__ status, uint32_t* __restrict__ sig_aff,
                                                   uint8_t* __restrict__ rand_out) {
  size_t i = gtid();
  if (i >= n) return;
  const uint8_t* s = sigs + i * stride;
  aff<fp> a;
  uint8_t st = g1_decompress(a, s, false);
  if (rand_out) st_digest(rand_out + 32 * i, sha256_aligned<48>(s));
  if (st != DEC_OK) {
    a.x = fp{};
    a.y = fp{};
    st = DEC_BAD;  // infinity signatures are rejected like kilic's engine + kyber's verify
  }
  status[i] = st;
  st_aff_aos<fp>(sig_aff, i, a);
}

template <class F>
__global__ __launch_bounds__(64) void k_sub_flag(size_t n, const uint8_t* __restrict__ status, const uint32_t* __restrict__ sig_aff,
                                                 uint8_t* __restrict__ sub_bad) {
  size_t i = gtid();
  if (i >= n) return;
  bool bad = false;
  if (status[i] == DEC_OK) {
    if constexpr (sizeof(F) == sizeof(fp)) bad = !g1_in_subgroup28([&] { return ld_aff_aos<fp>(sig_aff, i); });
    else bad = !g2_in_subgroup28([&] { return ld_aff_aos<fp2>(sig_aff, i); });
  }
  sub_bad[i] = bad ? 1 : 0;
}

__global__ __launch_bounds__(64) void k_and_subgroup(size_t n, const uint8_t* __restrict__ sub_bad, uint8_t* __restrict__ verdict) {
  size_t i = gtid();
  if (i >= n) return;
  if (sub_bad[i]) verdict[i] = 0;
}

// small-batch path, G1 hash in three launches, as the G2 hash runs (k_h2f_g2 -> k_sswu_g2 -> k_add_iso_g2): the
// round's two SSWU maps (each a square-root exponentiation, the bulk of the hash) run in two workgroups of their own,
// so on two SIMDs side by side, instead of one after the other on one lane (k_prep_msg_g1). Two waves of ONE
// workgroup measured no faster (1.24 ms against 1.1: they shared a SIMD, and a dependent MAD chain needs one SIMD's
// issue slots to itself). The hash is the small path's critical step for G1 signatures (decode 0.44-0.57 ms beside it).
// tmp: per round u0, u1 (2 x 12 words), then the two SSWU points (2 x 36 words) — hash_small_tmp_bytes.
__global__ __launch_bounds__(64) void k_h2f_g1_small(const uint64_t* __restrict__ rounds, const uint8_t* __restrict__ prevs,
                                                     size_t prev_stride, const uint32_t* __restrict__ prev_lens,
                                                     const uint8_t* __restrict__ msgs32, size_t n, int chained, int dst_id,
                                                     uint8_t* __restrict__ status, uint32_t* __restrict__ u_out) {
  const size_t i = gtid();
  if (i >= n) return;
  const sha_h d = message_of(rounds, prevs, prev_stride, prev_lens, msgs32, chained, i, status);
  uint32_t b[4][8];
  xmd32<4>(b, d, dst_id);
  st_f<fp>(u_out + 24 * i, fp_from_be512(b[0], b[1]));
  st_f<fp>(u_out + 24 * i + 12, fp_from_be512(b[2], b[3]));
}

// one SSWU map per workgroup (lane 0): map j of round j / 2
__global__ __launch_bounds__(64) void k_sswu_g1_small(const uint32_t* __restrict__ u, size_t m, uint32_t* __restrict__ pts) {
  const size_t j = blockIdx.x;
  if (j >= m || threadIdx.x) return;
  fp x;
  ld_f<fp>(x, u + 12 * j);
  st_jac_aos<fp>(pts, j, swu_jac(sswu_g1(x)));
}

__global__ __launch_bounds__(64) void k_add_iso_g1_small(const uint32_t* __restrict__ pts, size_t n, uint32_t* __restrict__ q_out) {
  const size_t i = gtid();
  if (i >= n) return;
  const jac<fp> p0 = ld_jac_aos<fp>(pts, 2 * i), p1 = ld_jac_aos<fp>(pts, 2 * i + 1);
  jac<fp> s;
  const jac<fp> q = jac_add_distinct(s, p0, p1) ? iso11_jac(s) : jac_add(iso11_jac(p0), iso11_jac(p1));
  st_jac_aos<fp>(q_out, i, q);
}

size_t hash_small_tmp_bytes(int sig_g2, size_t n) {
  return sig_g2 ? hash_tmp_bytes(1, n) : n * (24 + 72) * 4;
}

hipError_t launch_hash_small(int sig_g2, const uint64_t* rounds, const uint8_t* prevs, size_t prev_stride, const uint32_t* prev_lens,
                             const uint8_t* msgs32, size_t n, int chained, int dst_id, uint8_t* status, uint32_t* q_out,
                             uint32_t* tmp, hipStream_t st) {
  if (!n) return hipSuccess;
  if (sig_g2) return launch_hash(1, rounds, prevs, prev_stride, prev_lens, msgs32, n, chained, dst_id, status, q_out, tmp, st);
  uint32_t* pts = tmp + 24 * n;
  hipLaunchKernelGGL(k_h2f_g1_small, dim3(nblk(n, 64)), dim3(64), 0, st, rounds, prevs, prev_stride, prev_lens, msgs32, n,
                     chained, dst_id, status, tmp);
  hipLaunchKernelGGL(k_sswu_g1_small, dim3((unsigned)(2 * n)), dim3(64), 0, st, (const uint32_t*)tmp, 2 * n, pts);
  hipLaunchKernelGGL(k_add_iso_g1_small, dim3(nblk(n, 64)), dim3(64), 0, st, (const uint32_t*)pts, n, q_out);
  return hipGetLastError();
}

hipError_t launch_dec_sig(int sig_g2, const uint8_t* sigs, size_t stride, size_t n, uint8_t* status, uint32_t* sig_aff,
                          uint8_t* rand_out, hipStream_t st) {
  if (!n) return hipSuccess;
  if (sig_g2)
    hipLaunchKernelGGL(k_dec_sig_g2, dim3(nblk(n, 256)), dim3(256), 0, st, sigs, stride, n, status, sig_aff, rand_out);
  else
    hipLaunchKernelGGL(k_dec_sig_g1, dim3(nblk(n, 64)), dim3(64), 0, st, sigs, stride, n, status, sig_aff, rand_out);
  return hipGetLastError();
}

hipError_t launch_sub_flag(int sig_g2, size_t n, const uint8_t* status, const uint32_t* sig_aff, uint8_t* sub_bad, hipStream_t st) {
  if (!n) return hipSuccess;
  if (sig_g2) hipLaunchKernelGGL(k_sub_flag<fp2>, dim3(nblk(n, 64)), dim3(64), 0, st, n, status, sig_aff, sub_bad);
  else hipLaunchKernelGGL(k_sub_flag<fp>, dim3(nblk(n, 64)), dim3(64), 0, st, n, status, sig_aff, sub_bad);
  return hipGetLastError();
}

hipError_t launch_and_subgroup(size_t n, const uint8_t* sub_bad, uint8_t* verdict, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_and_subgroup, dim3(nblk(n, 64)), dim3(64), 0, st, n, sub_bad, verdict);
  return hipGetLastError();
}

// ---------------------------------------------------------------- prep: messages -> hash points (no cofactor)
// G1 (fused): hash_to_curve without clear_cofactor, one round per lane
__global__ __launch_bounds__(256, occ<fp>::W) void k_prep_msg_g1(const uint64_t* __restrict__ rounds, const uint8_t* __restrict__ prevs,
                                                            size_t prev_stride, const uint32_t* __restrict__ prev_lens,
                                                            const uint8_t* __restrict__ msgs32, size_t n, int chained, int dst_id,
                                                            uint8_t* __restrict__ status, uint32_t* __restrict__ q_out) {
  size_t i = gtid();
  if (i >= n) return;
  const sha_h d = message_of(rounds, prevs, prev_stride, prev_lens, msgs32, chained, i, status);
  st_jac_aos<fp>(q_out, i, h2c_g1_noclear(d, dst_id));
}

// G2 in three passes. The G2 map keeps more Fp2 values live than one lane's 256 VGPRs hold (fused, the kernel
// needed 19.3 KB of scratch per lane, and 8 such 1M-round dispatches in flight failed to launch), so the state
// between the passes goes through HBM: u0, u1 (192 B per round) and the two SSWU points on E2' (576 B per
// round), each written and read once (~1.5 KB per round against ~1.3 M integer products of work).
// pass 1: message -> expand_message_xmd -> hash_to_field: u0, u1 (Montgomery Fp2), 48 words per round
__global__ __launch_bounds__(256) void k_h2f_g2(const uint64_t* __restrict__ rounds, const uint8_t* __restrict__ prevs,
                                                size_t prev_stride, const uint32_t* __restrict__ prev_lens,
                                                const uint8_t* __restrict__ msgs32, size_t n, int chained, int dst_id,
                                                uint8_t* __restrict__ status, uint32_t* __restrict__ u_out) {
  size_t i = gtid();
  if (i >= n) return;
  const sha_h d = message_of(rounds, prevs, prev_stride, prev_lens, msgs32, chained, i, status);
  uint32_t b[8][8];
  xmd32<8>(b, d, dst_id);
  const fp2 u0 = {fp_from_be512(b[0], b[1]), fp_from_be512(b[2], b[3])};
  const fp2 u1 = {fp_from_be512(b[4], b[5]), fp_from_be512(b[6], b[7])};
  st_f<fp2>(u_out + 48 * i, u0);
  st_f<fp2>(u_out + 48 * i + 24, u1);
}

// pass 2: one SSWU map per lane (2 per round), the point on E2' as Jacobian (Z = xd)
__global__ __launch_bounds__(256, 2) void k_sswu_g2(const uint32_t* __restrict__ u, size_t m, uint32_t* __restrict__ pts) {
  size_t j = gtid();
  if (j >= m) return;
  fp2 x;
  ld_f<fp2>(x, u + 24 * j);
  st_jac_aos<fp2>(pts, j, swu_jac(sswu_g2(x)));
}

// pass 3: Q = iso3(P0 + P1) (h2c_g2_noclear's order: one isogeny after the addition on E2'). When the two SSWU
// points share x (never for honest inputs) the round is listed in exc[] and k_add_iso_g2_exc takes the textbook
// order, two isogenies then the addition on E2, on a small grid.
__global__ __launch_bounds__(256, 2) void k_add_iso_g2(const uint32_t* __restrict__ pts, size_t n, uint32_t* __restrict__ q_out,
                                                       uint32_t* __restrict__ exc) {
  size_t i = gtid();
  if (i >= n) return;
  jac<fp2> s;
  if (!jac_add_distinct_mem(s, pts + 144 * i, pts + 144 * i + 72)) {
    exc[1 + atomicAdd(exc, 1u)] = (uint32_t)i;
    return;
  }
  st_jac_aos<fp2>(q_out, i, iso3_jac_lean(s));
}

constexpr unsigned EXC_THREADS = 64;
__global__ __launch_bounds__(EXC_THREADS, 1) void k_add_iso_g2_exc(const uint32_t* __restrict__ pts, const uint32_t* __restrict__ exc,
                                                                   uint32_t* __restrict__ q_out) {
  const uint32_t cnt = exc[0];
  for (uint32_t k = threadIdx.x; k < cnt; k += EXC_THREADS) {
    const uint32_t i = exc[1 + k];
    const jac<fp2> p0 = ld_jac_aos<fp2>(pts, 2 * (size_t)i), p1 = ld_jac_aos<fp2>(pts, 2 * (size_t)i + 1);
    st_jac_aos<fp2>(q_out, i, jac_add(iso3_jac(p0), iso3_jac(p1)));
  }
}

// ---------------------------------------------------------------- RLC scalars
// r_i = first 16 bytes of SHA-256(seed[32] || i_be64), 0 for rounds that failed decoding.
__global__ __launch_bounds__(256) void k_scalars(const uint32_t* __restrict__ seed_words, size_t n,
                                                 const uint8_t* __restrict__ status, int parts, uint4* __restrict__ scal) {
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
  // little-endian words of a 127-bit integer (top bit cleared: the MSM's signed window digits need one spare
  // bit; the batch check's soundness error is 2^-127 per group), or with the endomorphism split two 63-bit
  // halves a, b: the round's scalar is a + b*mu mod r (mu = the endomorphism's eigenvalue, -z^2 on G1 or z on
  // G2, |mu| > 2^63, so distinct (a, b) give distinct scalars: soundness error 2^-126 per group), or on G2 four
  // 31-bit parts a, b, c, d: the scalar a + b z + c z^2 + d z^3 (psi = [z] on G2), |value| < 2^31 (1 + 2^64 +
  // 2^128 + 2^192) < r / 2, so distinct parts give distinct scalars: soundness error 2^-124 per group
  uint4 r = parts == 4   ? make_uint4(s.h[3] & 0x7fffffffu, s.h[2] & 0x7fffffffu, s.h[1] & 0x7fffffffu, s.h[0] & 0x7fffffffu)
            : parts == 2 ? make_uint4(s.h[3], s.h[2] & 0x7fffffffu, s.h[1], s.h[0] & 0x7fffffffu)
                         : make_uint4(s.h[3], s.h[2], s.h[1], s.h[0] & 0x7fffffffu);
  if (status && status[i] != DEC_OK) r = make_uint4(0, 0, 0, 0);
  scal[i] = r;
}

// ---------------------------------------------------------------- key decode
// Thread 0 decodes the point (square root, no subgroup test), then two waves run side by side: wave 0's first lane the
// subgroup test, wave 1's first lane (G2 keys: the G1-signature schemes) [h_eff] pk, so the batch check can read
// e([h_eff] B, pk) as e(B, [h_eff] pk) and skip the per-check cofactor clearing (k_vm_prep_groups). One lane did all
// three in a row: 6.8 ms for a G2 key (k_decode_key<fp2>, profiles/r06/rocprof_single_beacon_r06d.csv), the cost
// of a key-cache miss.
template <class K>
__global__ __launch_bounds__(128) void k_decode_key(const uint8_t* __restrict__ pk, uint32_t* __restrict__ key_aff,
                                                    uint8_t* __restrict__ ok) {
  __shared__ int st_sh, sub_sh;
  const int t = threadIdx.x;
  if (t == 0) {
    aff<K> a;
    uint8_t st;
    if constexpr (sizeof(K) == sizeof(fp)) st = g1_decompress(a, pk, false);
    else st = g2_decompress(a, pk, false);
    if (st != DEC_OK) {
      a.x = K{};
      a.y = K{};
    }
    st_aff_aos<K>(key_aff, 0, a);
    st_sh = st;
    sub_sh = 1;
  }
  __syncthreads();
  const bool dec_ok = st_sh == DEC_OK;
  if (t == 0 && dec_ok) {
    bool in;
    if constexpr (sizeof(K) == sizeof(fp)) in = g1_in_subgroup28([&] { return ld_aff_aos<fp>(key_aff, 0); });
    else in = g2_in_subgroup28([&] { return ld_aff_aos<fp2>(key_aff, 0); });
    sub_sh = in ? 1 : 0;
  }
  if constexpr (sizeof(K) == sizeof(fp2)) {
    if (t == 64) {
      aff<fp2> h{fp2{}, fp2{}};
      if (dec_ok) {
        const aff<fp2> a = ld_aff_aos<fp2>(key_aff, 0);
        h = jac_to_aff(jac_add(jac_mul_uabs(a), jac_from_aff(a)));  // G1's h_eff = 1 - z = |z| + 1, applied to pk
      }
      st_aff_aos<fp2>(key_aff, 1, h);
    }
  }
  __syncthreads();
  if (t == 0) {
    const uint8_t st = (uint8_t)st_sh == DEC_OK && !sub_sh ? (uint8_t)DEC_BAD : (uint8_t)st_sh;
    *ok = st;
    if (st != DEC_OK) st_aff_aos<K>(key_aff, 0, aff<K>{K{}, K{}});
  }
}


hipError_t launch_prep(int sig_g2, const uint8_t* sigs, size_t stride, size_t n, uint8_t* status, uint32_t* sig_aff,
                       uint8_t* rand_out, hipStream_t st) {
  if (!n) return hipSuccess;
  if (sig_g2) {
    hipLaunchKernelGGL(k_dec_sig_g2, dim3(nblk(n, 256)), dim3(256), 0, st, sigs, stride, n, status, sig_aff, rand_out);
    hipLaunchKernelGGL(k_sub_sig_g2, dim3(nblk(n, 256)), dim3(256), 0, st, n, status, sig_aff);
  } else
    hipLaunchKernelGGL(k_prep_sig<fp>, dim3(nblk(n, 256)), dim3(256), 0, st, sigs, stride, n, status, sig_aff, rand_out);
  return hipGetLastError();
}


hipError_t launch_scalars(const uint32_t* seed_words, size_t n, const uint8_t* status, uint4* scal, int parts, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_scalars, dim3(nblk(n, 256)), dim3(256), 0, st, seed_words, n, status, parts, scal);
  return hipGetLastError();
}

hipError_t launch_decode_key(int key_g2, const uint8_t* pk, uint32_t* key_aff, uint8_t* ok, hipStream_t st) {
  if (key_g2) hipLaunchKernelGGL(k_decode_key<fp2>, dim3(1), dim3(128), 0, st, pk, key_aff, ok);
  else hipLaunchKernelGGL(k_decode_key<fp>, dim3(1), dim3(128), 0, st, pk, key_aff, ok);
  return hipGetLastError();
}


// G2: the SSWU points (2 x 72 words per round), then the exceptional-round list (count + n indices)
size_t hash_tmp_bytes(int sig_g2, size_t n) { return sig_g2 ? n * 2 * 72 * 4 + (n + 1) * 4 : 0; }

hipError_t launch_hash(int sig_g2, const uint64_t* rounds, const uint8_t* prevs, size_t prev_stride, const uint32_t* prev_lens,
                       const uint8_t* msgs32, size_t n, int chained, int dst_id, uint8_t* status, uint32_t* q_out, uint32_t* tmp,
                       hipStream_t st) {
  if (!n) return hipSuccess;
  if (!sig_g2) {
    hipLaunchKernelGGL(k_prep_msg_g1, dim3(nblk(n, 256)), dim3(256), 0, st, rounds, prevs, prev_stride, prev_lens, msgs32, n,
                       chained, dst_id, status, q_out);
    return hipGetLastError();
  }
  // u0, u1 of round i go to q_out (48 of its 72 words per round), the SSWU points to tmp
  hipLaunchKernelGGL(k_h2f_g2, dim3(nblk(n, 256)), dim3(256), 0, st, rounds, prevs, prev_stride, prev_lens, msgs32, n, chained,
                     dst_id, status, q_out);
  hipLaunchKernelGGL(k_sswu_g2, dim3(nblk(2 * n, 256)), dim3(256), 0, st, (const uint32_t*)q_out, 2 * n, tmp);
  uint32_t* exc = tmp + n * 2 * 72;
  hipError_t e = hipMemsetAsync(exc, 0, 4, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_add_iso_g2, dim3(nblk(n, 256)), dim3(256), 0, st, (const uint32_t*)tmp, n, q_out, exc);
  hipLaunchKernelGGL(k_add_iso_g2_exc, dim3(1), dim3(EXC_THREADS), 0, st, (const uint32_t*)tmp, (const uint32_t*)exc, q_out);
  return hipGetLastError();
}

DH_COUNTER_ACCESSOR(prep)

}  // namespace dh
