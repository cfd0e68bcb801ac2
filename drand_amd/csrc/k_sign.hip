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

// RFC 9380 hash_to_curve (RO) of arbitrary messages under an arbitrary DST (<= 255 bytes), compressed: the general
// form of the fixed-shape hashing in the verification kernels (32-byte digest, two fixed DSTs), for known-answer
// tests (RFC 9380 J.9.1 / J.10.1) and callers hashing other messages. Each lane builds its expand_message_xmd
// preimages in its own scratch row (>= 64 + msg + dst + 4 bytes). Not on the batch path.
template <class F>
__global__ __launch_bounds__(64, 1) void k_h2c_generic(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ off, size_t n,
                                                       const uint8_t* __restrict__ dst, uint32_t dlen, uint8_t* __restrict__ scratch,
                                                       size_t sstride, uint8_t* __restrict__ out) {
  size_t i = gtid();
  if (i >= n) return;
  constexpr bool G1 = sizeof(F) == sizeof(fp);
  constexpr uint32_t L = G1 ? 128 : 256;  // len_in_bytes: 2 (G1) or 2 x 2 (G2) field elements of 64 bytes
  const uint8_t* m = msgs + off[i];
  const uint32_t mlen = off[i + 1] - off[i];
  uint8_t* s = scratch + i * sstride;
  uint64_t k = 0;
  for (int j = 0; j < 64; j++) s[k++] = 0;  // Z_pad
  for (uint32_t j = 0; j < mlen; j++) s[k++] = m[j];
  s[k++] = (uint8_t)(L >> 8);
  s[k++] = (uint8_t)L;
  s[k++] = 0;
  for (uint32_t j = 0; j < dlen; j++) s[k++] = dst[j];
  s[k++] = (uint8_t)dlen;
  const sha_h b0 = sha256_bytes(s, k);
  uint32_t uni[L / 4];
  sha_h prev;
  for (int j = 0; j < 8; j++) prev.h[j] = 0;
  for (uint32_t bi = 1; bi <= L / 32; bi++) {
    k = 0;
    for (int j = 0; j < 8; j++) {
      const uint32_t wv = b0.h[j] ^ prev.h[j];
      s[k++] = (uint8_t)(wv >> 24);
      s[k++] = (uint8_t)(wv >> 16);
      s[k++] = (uint8_t)(wv >> 8);
      s[k++] = (uint8_t)wv;
    }
    s[k++] = (uint8_t)bi;
    for (uint32_t j = 0; j < dlen; j++) s[k++] = dst[j];
    s[k++] = (uint8_t)dlen;
    prev = sha256_bytes(s, k);
    for (int j = 0; j < 8; j++) uni[8 * (bi - 1) + j] = prev.h[j];
  }
  if constexpr (G1) {
    const jac<fp> q = h2c_g1_map(fp_from_be512(uni, uni + 8), fp_from_be512(uni + 16, uni + 24));
    g1_compress(out + 48 * i, h2c_clear_g1(q));
  } else {
    const fp2 u0 = {fp_from_be512(uni, uni + 8), fp_from_be512(uni + 16, uni + 24)};
    const fp2 u1 = {fp_from_be512(uni + 32, uni + 40), fp_from_be512(uni + 48, uni + 56)};
    g2_compress(out + 96 * i, h2c_clear_g2(h2c_g2_map(u0, u1)));
  }
}

hipError_t launch_h2c_generic(int g2, const uint8_t* msgs, const uint32_t* off, size_t n, const uint8_t* dst, uint32_t dlen,
                              uint8_t* scratch, size_t sstride, uint8_t* out, hipStream_t st) {
  if (!n) return hipSuccess;
  if (g2)
    hipLaunchKernelGGL(k_h2c_generic<fp2>, dim3(nblk(n, 64)), dim3(64), 0, st, msgs, off, n, dst, dlen, scratch, sstride, out);
  else
    hipLaunchKernelGGL(k_h2c_generic<fp>, dim3(nblk(n, 64)), dim3(64), 0, st, msgs, off, n, dst, dlen, scratch, sstride, out);
  return hipGetLastError();
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

DH_COUNTER_ACCESSOR(sign)

}  // namespace dh
