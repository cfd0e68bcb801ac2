// Synthetic-chain signer and public-key derivation (tests / bench inputs; not on the verification path).
#include "kcommon.hpp"

namespace dh {

// ---------------------------------------------------------------- synthetic-chain signer (tests / bench data)
// sig_i = [sk] H(DigestBeacon(round_i, prev_i)) (or [sk] H(msgs32_i)), compressed. Not on the verification path.
// G1: one fused kernel. G2: the hash points come from launch_hash's three passes (k_prep.hip), then k_sign_g2.
__global__ __launch_bounds__(256, occ<fp>::W) void k_sign_g1(const uint32_t* __restrict__ sk, const uint64_t* __restrict__ rounds,
                                                        const uint8_t* __restrict__ prevs, size_t prev_stride,
                                                        const uint32_t* __restrict__ prev_lens, const uint8_t* __restrict__ msgs32,
                                                        size_t n, int chained, int dst_id, uint8_t* __restrict__ out) {
  size_t i = gtid();
  if (i >= n) return;
  const sha_h d = message_of(rounds, prevs, prev_stride, prev_lens, msgs32, chained, i, nullptr);
  jac<fp> h = h2c_clear_g1(h2c_g1_noclear(d, dst_id));
  g1_compress(out + 48 * i, jac_mul_words(h, sk, 256));
}

__global__ __launch_bounds__(256, 2) void k_sign_g2(const uint32_t* __restrict__ sk, const uint32_t* __restrict__ q, size_t n,
                                                    uint8_t* __restrict__ out) {
  size_t i = gtid();
  if (i >= n) return;
  const jac<fp2> h = h2c_clear_g2(ld_jac_aos<fp2>(q, i));
  g2_compress(out + 96 * i, jac_mul_words(h, sk, 256));
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


hipError_t launch_sign(int sig_g2, const uint32_t* sk, const uint64_t* rounds, const uint8_t* prevs, size_t prev_stride,
                       const uint32_t* prev_lens, const uint8_t* msgs32, size_t n, int chained, int dst_id, uint8_t* out,
                       uint32_t* q_tmp, uint32_t* h_tmp, hipStream_t st) {
  if (!n) return hipSuccess;
  if (!sig_g2) {
    hipLaunchKernelGGL(k_sign_g1, dim3(nblk(n, 256)), dim3(256), 0, st, sk, rounds, prevs, prev_stride, prev_lens, msgs32, n,
                       chained, dst_id, out);
    return hipGetLastError();
  }
  hipError_t e = launch_hash(1, rounds, prevs, prev_stride, prev_lens, msgs32, n, chained, dst_id, nullptr, q_tmp, h_tmp, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_sign_g2, dim3(nblk(n, 256)), dim3(256), 0, st, sk, (const uint32_t*)q_tmp, n, out);
  return hipGetLastError();
}


hipError_t launch_pubkey(int key_g2, const uint32_t* sk, uint8_t* out, hipStream_t st) {
  if (key_g2) hipLaunchKernelGGL(k_pubkey<fp2>, dim3(1), dim3(64), 0, st, sk, out);
  else hipLaunchKernelGGL(k_pubkey<fp>, dim3(1), dim3(64), 0, st, sk, out);
  return hipGetLastError();
}

}  // namespace dh
