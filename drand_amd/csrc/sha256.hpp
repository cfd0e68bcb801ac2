// SHA-256 (FIPS 180-4) per lane, plus the fixed-shape messages of the beacon path:
//   DigestBeacon  unchained / on-g1 : SHA-256(round_be64)              /root/reference/crypto/schemes.go:147-151,187-191
//   DigestBeacon  chained           : SHA-256(prev || round_be64)      /root/reference/crypto/schemes.go:106-114
//   RandomnessFromSignature         : SHA-256(sig)                     /root/reference/crypto/schemes.go:249-252
//   expand_message_xmd (RFC 9380 5.3.1) of a 32-byte digest, used by hash-to-curve [kilic/bls12-381 v0.1.0
//   HashToCurve, DSTs from kyber-bls12381 v0.2.5]; the DST-dependent blocks are precomputed in consts.hpp.
// Every loop is fully unrolled so the 16-word message schedule lives in registers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "consts.hpp"

namespace dh {

#ifndef DH_DEV
#define DH_DEV __device__ __forceinline__
#endif

__device__ __constant__ uint32_t SHA_K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

struct sha_h {
  uint32_t h[8];
};

DH_DEV sha_h sha_iv() {
  return {{0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au, 0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u}};
}

DH_DEV uint32_t ror32(uint32_t x, int n) { return __builtin_rotateright32(x, n); }

// one compression; w = 16 big-endian message words (consumed)
DH_DEV void sha_compress(sha_h& s, uint32_t w[16]) {
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      uint32_t s0 = ror32(w15, 7) ^ ror32(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = ror32(w2, 17) ^ ror32(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t t1 = h + (ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25)) + ((e & f) ^ (~e & g)) + SHA_K[i] + wi;
    uint32_t t2 = (ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
  s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

DH_DEV uint32_t ld_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
// 4-byte aligned big-endian word load
DH_DEV uint32_t ld_be32a(const uint8_t* p) { return __builtin_bswap32(*(const uint32_t*)p); }

DH_DEV void st_digest(uint8_t* out, const sha_h& s) {
#pragma unroll
  for (int i = 0; i < 8; i++) *(uint32_t*)(out + 4 * i) = __builtin_bswap32(s.h[i]);
}

// SHA-256 of nwords big-endian words loaded from p (4-byte aligned), nwords*4 <= 119 bytes
// compile-time sized; used for randomness (48 or 96 bytes) and the RLC scalar PRF.
template <int NBYTES>
DH_DEV sha_h sha256_aligned(const uint8_t* p) {
  static_assert(NBYTES % 4 == 0 && NBYTES <= 119, "shape");
  constexpr int NB = (NBYTES + 9 + 63) / 64;
  sha_h s = sha_iv();
#pragma unroll
  for (int blk = 0; blk < NB; blk++) {
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      const int pos = blk * 16 + j;  // word index in the padded message
      uint32_t v = 0;
      if (pos < NBYTES / 4) v = ld_be32a(p + 4 * pos);
      if (pos == NBYTES / 4) v = 0x80000000u;
      if (blk == NB - 1 && j == 15) v = (uint32_t)(NBYTES * 8);
      w[j] = v;
    }
    sha_compress(s, w);
  }
  return s;
}

// DigestBeacon for unchained / on-g1 schemes: SHA-256(round as 8 big-endian bytes)
DH_DEV sha_h digest_unchained(uint64_t round) {
  uint32_t w[16];
#pragma unroll
  for (int j = 0; j < 16; j++) w[j] = 0;
  w[0] = (uint32_t)(round >> 32);
  w[1] = (uint32_t)round;
  w[2] = 0x80000000u;
  w[15] = 64;
  sha_h s = sha_iv();
  sha_compress(s, w);
  return s;
}

// DigestBeacon for the chained scheme: SHA-256(prev || round_be64), prevlen a multiple of 4, <= 96.
// prevlen == 0 is the "no previous signature" case (crypto/schemes.go:108-110 skips it).
DH_DEV sha_h digest_chained(const uint8_t* prev, uint32_t prevlen, uint64_t round) {
  const uint32_t pw = prevlen >> 2;
  const uint32_t total = prevlen + 8;
  const uint32_t nb = (total + 9 + 63) >> 6;  // 1 or 2
  sha_h s = sha_iv();
#pragma unroll
  for (int blk = 0; blk < 2; blk++) {
    if ((uint32_t)blk < nb) {
      uint32_t w[16];
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const uint32_t pos = blk * 16 + j;
        uint32_t v = 0;
        if (pos < pw) v = ld_be32a(prev + 4 * pos);
        if (pos == pw) v = (uint32_t)(round >> 32);
        if (pos == pw + 1) v = (uint32_t)round;
        if (pos == pw + 2) v = 0x80000000u;
        if ((uint32_t)blk == nb - 1 && j == 15) v = total * 8;
        w[j] = v;
      }
      sha_compress(s, w);
    }
  }
  return s;
}

// DigestBeacon for the chained scheme with a previous signature of ANY length and alignment: the reference
// hashes whatever the store holds (crypto/schemes.go:106-114, chain/boltdb/trimmed.go:183-189), so a
// corrupted 31-, 97- or 100-byte record is hashed too and simply fails verification. Byte loads, one
// compression per 64 bytes; the stored-signature shape (4-byte aligned, <= 96 bytes) takes digest_chained.
DH_DEV sha_h digest_chained_any(const uint8_t* prev, uint32_t prevlen, uint64_t round) {
  const uint64_t total = (uint64_t)prevlen + 8;
  const uint64_t nb = (total + 9 + 63) >> 6;
  sha_h s = sha_iv();
#pragma unroll 1
  for (uint64_t blk = 0; blk < nb; blk++) {
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      uint32_t v = 0;
#pragma unroll
      for (int b = 0; b < 4; b++) {
        const uint64_t pos = blk * 64 + (uint64_t)(4 * j + b);
        uint32_t byte = 0;
        if (pos < prevlen) byte = prev[pos];
        else if (pos < total) byte = (uint32_t)(round >> (8 * (7 - (pos - prevlen)))) & 0xffu;
        else if (pos == total) byte = 0x80u;
        v = (v << 8) | byte;
      }
      if (blk == nb - 1 && j == 14) v = (uint32_t)((total * 8) >> 32);
      if (blk == nb - 1 && j == 15) v = (uint32_t)(total * 8);
      w[j] = v;
    }
    sha_compress(s, w);
  }
  return s;
}

// SHA-256 of len bytes at p (any alignment), one compression per 64 bytes
DH_DEV sha_h sha256_bytes(const uint8_t* p, uint64_t len) {
  const uint64_t nb = (len + 9 + 63) >> 6;
  sha_h s = sha_iv();
#pragma unroll 1
  for (uint64_t blk = 0; blk < nb; blk++) {
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
      uint32_t v = 0;
#pragma unroll
      for (int b = 0; b < 4; b++) {
        const uint64_t pos = blk * 64 + (uint64_t)(4 * j + b);
        const uint32_t byte = pos < len ? p[pos] : (pos == len ? 0x80u : 0u);
        v = (v << 8) | byte;
      }
      if (blk == nb - 1 && j == 14) v = (uint32_t)((len * 8) >> 32);
      if (blk == nb - 1 && j == 15) v = (uint32_t)(len * 8);
      w[j] = v;
    }
    sha_compress(s, w);
  }
  return s;
}

// expand_message_xmd(SHA-256, msg = 32-byte digest, DST = 43 bytes, len = 32*NOUT):
// writes NOUT 32-byte blocks b_1..b_NOUT (as big-endian words) into out[NOUT][8].
// dst_id 0 = G2 DST, 1 = G1 DST; len_id 0 = 128 bytes (hash to G1), 1 = 256 bytes (G2).
template <int NOUT>
DH_DEV void xmd32(uint32_t out[NOUT][8], const sha_h& msg, int dst_id) {
  constexpr int len_id = NOUT == 4 ? 0 : 1;
  static_assert(NOUT == 4 || NOUT == 8, "xmd shape");
  sha_h b0;
#pragma unroll
  for (int i = 0; i < 8; i++) b0.h[i] = cst::XMD_ZPAD_H[i];
  {
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = msg.h[j];
#pragma unroll
    for (int j = 0; j < 8; j++) w[8 + j] = cst::XMD_B0A[dst_id][len_id][j];
    sha_compress(b0, w);
#pragma unroll
    for (int j = 0; j < 16; j++) w[j] = cst::XMD_B0B[dst_id][j];
    sha_compress(b0, w);
  }
  uint32_t prev[8];
#pragma unroll
  for (int j = 0; j < 8; j++) prev[j] = 0;
#pragma unroll
  for (int i = 1; i <= NOUT; i++) {
    sha_h bi = sha_iv();
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 8; j++) w[j] = b0.h[j] ^ prev[j];
#pragma unroll
    for (int j = 0; j < 8; j++) w[8 + j] = cst::XMD_BIA[dst_id][j];
    w[8] |= (uint32_t)i << 24;
    sha_compress(bi, w);
#pragma unroll
    for (int j = 0; j < 16; j++) w[j] = cst::XMD_BIB[dst_id][j];
    sha_compress(bi, w);
#pragma unroll
    for (int j = 0; j < 8; j++) {
      prev[j] = bi.h[j];
      out[i - 1][j] = bi.h[j];
    }
  }
}

}  // namespace dh
