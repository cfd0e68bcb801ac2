// Scalar field F_r of BLS12-381 (r = 0x73eda753...00000001, 255 bits) on gfx950, per lane: 8 x 32-bit limbs,
// Montgomery form with R = 2^256. Used for the tbls Lagrange coefficients at 0 (kyber v1.1.18 share.RecoverCommit,
// lagrangeBasis; called through /root/reference/chain/beacon/chainstore.go:202), computed per round on the device:
// ~t^2 products for t = 33, under 1% of the interpolation they feed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dh {

#ifndef DH_DEV
#define DH_DEV __device__ __forceinline__
#endif

struct fr {
  uint32_t v[8];
};

__device__ __constant__ uint32_t FR_MOD[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                                              0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
__device__ __constant__ uint32_t FR_R2[8] = {0xf3f29c6du, 0xc999e990u, 0x87925c23u, 0x2b6cedcbu,
                                             0x7254398fu, 0x05d31496u, 0x9f59ff11u, 0x0748d9d9u};  // 2^512 mod r
__device__ __constant__ uint32_t FR_MOD_M2[8] = {0xffffffffu, 0xfffffffeu, 0xfffe5bfeu, 0x53bda402u,
                                                 0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};  // r - 2
constexpr uint32_t FR_N0 = 0xffffffffu;  // -r^-1 mod 2^32 (r = 1 mod 2^32)

DH_DEV void fr_sub_mod_if(uint32_t t[8], uint32_t hi) {  // t (+ hi * 2^256) < 2r  ->  t mod r
  uint32_t d[8];
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d[i] = __builtin_subc(t[i], FR_MOD[i], br, &br);
  const bool take = hi || !br;
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = take ? d[i] : t[i];
}

// Montgomery product (CIOS), inputs < r, output < r
DH_DEV fr fr_mul(const fr& a, const fr& b) {
  uint32_t t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t t8 = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      c += (uint64_t)a.v[j] * b.v[i] + t[j];
      t[j] = (uint32_t)c;
      c >>= 32;
    }
    uint64_t s = (uint64_t)t8 + c;
    t8 = (uint32_t)s;
    const uint32_t t9 = (uint32_t)(s >> 32);
    const uint32_t m = t[0] * FR_N0;
    c = ((uint64_t)m * FR_MOD[0] + t[0]) >> 32;
#pragma unroll
    for (int j = 1; j < 8; j++) {
      c += (uint64_t)m * FR_MOD[j] + t[j];
      t[j - 1] = (uint32_t)c;
      c >>= 32;
    }
    s = (uint64_t)t8 + c;
    t[7] = (uint32_t)s;
    t8 = t9 + (uint32_t)(s >> 32);
  }
  fr_sub_mod_if(t, t8);
  fr r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
  return r;
}

DH_DEV fr fr_sub(const fr& a, const fr& b) {
  fr r;
  unsigned br = 0, c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
  const uint32_t mask = 0u - br;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = __builtin_addc(r.v[i], FR_MOD[i] & mask, c, &c);
  return r;
}

// Montgomery form of a small integer x < r
DH_DEV fr fr_from_u32(uint32_t x) {
  fr a, r2;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a.v[i] = i ? 0u : x;
    r2.v[i] = FR_R2[i];
  }
  return fr_mul(a, r2);
}

DH_DEV fr fr_one() { return fr_from_u32(1); }

// a^(r-2) (Fermat), square-and-multiply over the fixed public exponent
DH_DEV fr fr_inv(const fr& a) {
  fr acc = fr_one();
#pragma unroll 1
  for (int i = 254; i >= 0; i--) {
    acc = fr_mul(acc, acc);
    if ((FR_MOD_M2[i >> 5] >> (i & 31)) & 1) acc = fr_mul(acc, a);
  }
  return acc;
}

// out of Montgomery form: canonical little-endian words
DH_DEV void fr_to_words(const fr& a, uint32_t out[8]) {
  fr one;
#pragma unroll
  for (int i = 0; i < 8; i++) one.v[i] = i ? 0u : 1u;
  const fr c = fr_mul(a, one);
#pragma unroll
  for (int i = 0; i < 8; i++) out[i] = c.v[i];
}

// the shorter of w and r - w (little-endian words) into k; true when it is r - w, whose digits the caller negates
// ([-(r - w)] P = [w] P on the order-r subgroup). A Lagrange coefficient of the first t signers is +-C(t, k) mod r: half
// of them sit just below r, and their recoding as r - w is a ~31-bit number instead of a 255-bit one.
DH_DEV bool fr_short(const uint32_t w[8], uint32_t k[8]) {
  uint32_t n[8];
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) n[i] = __builtin_subc(FR_MOD[i], w[i], br, &br);
  bool less = false, eq = true;  // n < w, from the top word
#pragma unroll
  for (int i = 7; i >= 0; i--) {
    if (eq && n[i] != w[i]) {
      less = n[i] < w[i];
      eq = false;
    }
  }
#pragma unroll
  for (int i = 0; i < 8; i++) k[i] = less ? n[i] : w[i];
  return less;
}

// non-adjacent form of k < 2^255 (little-endian words) as positive / negative digit masks over 256 positions
// width-4 NAF of a scalar w < 2^255 (little-endian words): digit b in nibble b (word b / 8, bits 4 (b % 8)), 0 = zero,
// v in 1..4 = +(2v - 1), v in 9..12 = -(2(v - 8) - 1): odd digits in [-7, 7], each followed by at least three zeros
// (k_lagrange's table holds P, 3P, 5P, 7P); 256 positions suffice for w < 2^255
DH_DEV void fr_wnaf4(const uint32_t w[8], uint32_t* nib) {
  uint32_t k[9];
#pragma unroll
  for (int i = 0; i < 8; i++) k[i] = w[i];
  k[8] = 0;
  uint32_t acc = 0;
#pragma unroll 1
  for (int b = 0; b < 256; b++) {
    uint32_t v = 0;
    if (k[0] & 1) {
      int d = (int)(k[0] & 15);
      if (d >= 8) d -= 16;
      if (d > 0) {  // k -= d: clears the low four bits, no borrow
        k[0] -= (uint32_t)d;
        v = (uint32_t)(d + 1) / 2;
      } else {  // k += -d: the low four bits carry out
        unsigned c = (unsigned)(-d);
#pragma unroll
        for (int i = 0; i < 9; i++) k[i] = __builtin_addc(k[i], 0u, c, &c);
        v = 8 + (uint32_t)(1 - d) / 2;
      }
    }
#pragma unroll
    for (int i = 0; i < 8; i++) k[i] = (k[i] >> 1) | (k[i + 1] << 31);
    k[8] >>= 1;
    acc |= v << (4 * (b & 7));
    if ((b & 7) == 7) {
      nib[b >> 3] = acc;
      acc = 0;
    }
  }
}

// Regular signed 4-bit windows of a scalar 0 < w < r (little-endian words): 64 digits, every one odd and nonzero,
// sum d_i 16^i = w, so a Straus chain adds at every window with no digit-dependent branch (k_lagrange's path for waves
// whose rounds do not share one Lagrange basis). An even w is recoded as r - w (odd) with every digit negated
// ([-(r - w)] P = [w] P on the order-r subgroup). Digit i in nibble i (word i / 8, bits 4 (i % 8)): (|d| - 1) / 2 in
// bits 0-2 (table entry P, 3P, ..., 15P), bit 3 the sign. Steps: d = (k mod 32) - 16 (odd, |d| <= 15), k = (k - d) / 16
// stays odd; after 63 steps k <= 2^255 / 2^252 + 16 / 15 is the last digit (1 .. 9).
DH_DEV void fr_reg4(const uint32_t w[8], uint32_t* nib) {
  uint32_t k[8];
  const bool flip = !(w[0] & 1);
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) k[i] = flip ? __builtin_subc(FR_MOD[i], w[i], br, &br) : w[i];
  uint32_t acc = 0;
#pragma unroll 1
  for (int i = 0; i < 64; i++) {
    int d;
    if (i < 63) {
      d = (int)(k[0] & 31) - 16;
      // k -= d (k - d = 16 mod 32), then k >>= 4
      if (d < 0) {
        unsigned c = (unsigned)(-d);
#pragma unroll
        for (int m = 0; m < 8; m++) k[m] = __builtin_addc(k[m], 0u, c, &c);
      } else {
        unsigned b = (unsigned)d;
#pragma unroll
        for (int m = 0; m < 8; m++) k[m] = __builtin_subc(k[m], 0u, b, &b);
      }
#pragma unroll
      for (int m = 0; m < 7; m++) k[m] = (k[m] >> 4) | (k[m + 1] << 28);
      k[7] >>= 4;
    } else {
      d = (int)k[0];
    }
    if (flip) d = -d;
    const uint32_t v = (uint32_t)((d < 0 ? -d : d) - 1) / 2 | (d < 0 ? 8u : 0u);
    acc |= v << (4 * (i & 7));
    if ((i & 7) == 7) {
      nib[i >> 3] = acc;
      acc = 0;
    }
  }
}

DH_DEV void fr_naf_masks(const uint32_t w[8], uint32_t* pos, uint32_t* neg) {
  uint32_t k[9];
#pragma unroll
  for (int i = 0; i < 8; i++) k[i] = w[i];
  k[8] = 0;
  uint32_t p = 0, n = 0;
#pragma unroll 1
  for (int b = 0; b < 256; b++) {
    if (k[0] & 1) {
      if ((k[0] & 3) == 3) {  // digit -1: k += 1
        n |= 1u << (b & 31);
        unsigned c = 1;
#pragma unroll
        for (int i = 0; i < 9; i++) k[i] = __builtin_addc(k[i], 0u, c, &c);
      } else {  // digit +1: k -= 1
        p |= 1u << (b & 31);
        k[0] -= 1;
      }
    }
#pragma unroll
    for (int i = 0; i < 8; i++) k[i] = (k[i] >> 1) | (k[i + 1] << 31);
    k[8] >>= 1;
    if ((b & 31) == 31) {
      pos[b >> 5] = p;
      neg[b >> 5] = n;
      p = n = 0;
    }
  }
}

}  // namespace dh
