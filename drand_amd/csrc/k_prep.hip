// Batch beacon-verification kernels for gfx950 — per-round preparation (this file), see also
// k_msm.hip, k_check.hip, k_sign.hip.
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
__global__ __launch_bounds__(256, occ<F>::W) void k_prep_msg(const uint64_t* __restrict__ rounds, const uint8_t* __restrict__ prevs,
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

// hash points for caller-given 32-byte messages (tbls: the DigestBeacon of each round)
template <class F>
__global__ __launch_bounds__(256, occ<F>::W) void k_prep_msg32(const uint8_t* __restrict__ msgs, size_t n, int dst_id,
                                                       uint32_t* __restrict__ q_out) {
  size_t i = gtid();
  if (i >= n) return;
  sha_h d;
#pragma unroll
  for (int j = 0; j < 8; j++) d.h[j] = ld_be32a(msgs + 32 * i + 4 * j);
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
  // little-endian words of a 127-bit integer (top bit cleared: the MSM's signed window digits need one spare
  // bit; the batch check's soundness error is 2^-127 per group)
  uint4 r = make_uint4(s.h[3], s.h[2], s.h[1], s.h[0] & 0x7fffffffu);
  if (status[i] != DEC_OK) r = make_uint4(0, 0, 0, 0);
  scal[i] = r;
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


hipError_t launch_msg32(int sig_g2, const uint8_t* msgs, size_t n, int dst_id, uint32_t* q_out, hipStream_t st) {
  if (!n) return hipSuccess;
  if (sig_g2) hipLaunchKernelGGL(k_prep_msg32<fp2>, dim3(nblk(n, 256)), dim3(256), 0, st, msgs, n, dst_id, q_out);
  else hipLaunchKernelGGL(k_prep_msg32<fp>, dim3(nblk(n, 256)), dim3(256), 0, st, msgs, n, dst_id, q_out);
  return hipGetLastError();
}

}  // namespace dh
