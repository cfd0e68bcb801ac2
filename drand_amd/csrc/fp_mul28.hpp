// Fp Montgomery product and squaring on 14 x 28-bit limbs behind the 12 x 32-bit interface of fp.hpp.
// These are the bodies of the library's out-of-line field products (fp.hpp dh_fp_mul_vec / dh_fp_sqr_vec; call
// clobbers v0-v39, v48-v53, s0-s17, checked at build time by drand_amd/tools/check_fp_abi.py) and of the pairing
// VM's inlined products (k_vm.hip); bench/microbench_fp28.hip measures them against the 32-bit form.
//
// Why 28 bits: on gfx950 the 32-bit product-scanning step is a v_mad_u64_u32 PLUS a v_addc_co_u32 for the carry
// into the column's third word, and the carry add issues as slowly as the multiply (~19 T MAC/s either way against
// 37 T/s for the bare MAD, profiles/microbench_carry_r02.txt). A 28x28-bit product is < 2^56, so one 64-bit
// accumulator absorbs a whole column (<= 28 products + the carry-in < 2^61) with ONE v_mad_u64_u32 per product
// and no carry add: 392 MADs for a product, 301 for a squaring, plus ~25 column normalisations (mask, 64-bit
// shift, one 28-bit v_mul_lo for the Montgomery quotient digit) and the 12 <-> 14 limb slicing.
// Measured (bench/microbench_fp28.hip, profiles/microbench_fp28_r02.txt): 69.96 vs 59.65 G products/s, 80.74 vs
// 67.91 G squarings/s, bit-identical results over 2^28 chained products.
//
// Same values as the 32-bit form: inputs < p, output < p, x*y / 2^384 mod p. The product slices y * 2^8 and the
// squaring slices x * 2^4 (both < 2^392), so the 28-bit Montgomery division by R' = 2^392 leaves x*y / 2^384; the
// result before the final subtraction is < 2p (x*y*2^8 + m*p < 2^392 * 2p).
#pragma once
#include <stdint.h>

namespace dh {
namespace m28 {
constexpr uint32_t MASK = 0x0fffffffu;
constexpr uint32_t N0 = 0x0ffcfffdu;  // -p^-1 mod 2^28
// p as 12 x 32-bit words (the final conditional subtraction works on the joined words)
__device__ constexpr uint32_t P32[12] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u,
                                         0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
__device__ constexpr uint32_t P[14] = {0xfffaaabu, 0xfefffffu, 0x3ffffb9u, 0xfffeb15u, 0x6241eabu, 0xa0f6b0fu, 0xf6730d2u,
                                       0xf38512bu, 0x4774b84u, 0x4bacd76u, 0xba7b643u, 0xe69a4b1u, 0x1ea397fu, 0x001a011u};

// limb i = bits [28 i - s, 28 i - s + 28) of the 384-bit x (s = 0, or 8 for x * 2^8)
template <int S>
__device__ __forceinline__ void split(uint32_t L[14], const uint32_t x[12]) {
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const int b = 28 * i - S;
    uint32_t v;
    if (b < 0) {
      v = x[0] << (-b);
    } else {
      const int w = b >> 5, o = b & 31;
      const uint64_t two = (uint64_t)x[w] | ((w + 1 < 12) ? ((uint64_t)x[w + 1] << 32) : 0);
      v = (uint32_t)(two >> o);
    }
    L[i] = v & MASK;
  }
}

// 14 x 28-bit limbs (value < 2^384) -> 12 x 32-bit words
__device__ __forceinline__ void join(uint32_t r[12], const uint32_t L[14]) {
#pragma unroll
  for (int j = 0; j < 12; j++) {
    const int b = 32 * j, i = b / 28, o = b % 28;
    uint64_t v = (uint64_t)L[i] >> o;
    if (i + 1 < 14) v |= (uint64_t)L[i + 1] << (28 - o);
    if (i + 2 < 14 && 56 - o < 32) v |= (uint64_t)L[i + 2] << (56 - o);
    r[j] = (uint32_t)v;
  }
}

// product-scanning Montgomery reduction over the column sums given by COL(k, acc)
#define M28_BODY(COL)                                                   \
  uint32_t Mq[14], R[14];                                               \
  uint64_t acc = 0;                                                     \
  _Pragma("unroll") for (int k = 0; k < 14; k++) {                      \
    COL(k, acc);                                                        \
    _Pragma("unroll") for (int i = 0; i < k; i++) acc += (uint64_t)Mq[i] * P[k - i]; \
    Mq[k] = ((uint32_t)acc * N0) & MASK;                                \
    acc += (uint64_t)Mq[k] * P[0];                                      \
    acc >>= 28;                                                         \
  }                                                                     \
  _Pragma("unroll") for (int k = 14; k < 27; k++) {                     \
    COL(k, acc);                                                        \
    _Pragma("unroll") for (int i = k - 13; i < 14; i++) acc += (uint64_t)Mq[i] * P[k - i]; \
    R[k - 14] = (uint32_t)acc & MASK;                                   \
    acc >>= 28;                                                         \
  }                                                                     \
  R[13] = (uint32_t)acc;

__device__ __forceinline__ void mul(uint32_t r[12], const uint32_t x[12], const uint32_t y[12]) {
  uint32_t X[14], Y[14];
  split<0>(X, x);
  split<8>(Y, y);
#define COLM(k, acc)                                                                         \
  _Pragma("unroll") for (int i = ((k) > 13 ? (k) - 13 : 0); i <= ((k) < 13 ? (k) : 13); i++) \
      acc += (uint64_t)X[i] * Y[(k) - i];
  M28_BODY(COLM)
#undef COLM
  join(r, R);
  // < 2p: one conditional subtraction, as fp_mul (fips_final_sub form)
  uint32_t t[12];
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) t[i] = __builtin_subc(r[i], P32[i], br, &br);
#pragma unroll
  for (int i = 0; i < 12; i++) r[i] = br ? r[i] : t[i];
}

// x^2 / 2^384 = (x 2^4)^2 / 2^392: square the limbs of x 2^4 (< 2^385) symmetrically, 105 products instead of 196
__device__ __forceinline__ void sqr(uint32_t r[12], const uint32_t x[12]) {
  uint32_t X[14], X2[14];
  split<4>(X, x);
#pragma unroll
  for (int i = 0; i < 14; i++) X2[i] = X[i] << 1;
#define COLS(k, acc)                                                                                  \
  _Pragma("unroll") for (int i = ((k) > 13 ? (k) - 13 : 0); 2 * i < (k); i++) acc += (uint64_t)X[i] * X2[(k) - i]; \
  if (((k) & 1) == 0) acc += (uint64_t)X[(k) / 2] * X[(k) / 2];
  M28_BODY(COLS)
#undef COLS
  join(r, R);
  uint32_t t[12];
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) t[i] = __builtin_subc(r[i], P32[i], br, &br);
#pragma unroll
  for (int i = 0; i < 12; i++) r[i] = br ? r[i] : t[i];
}
// The same product with each column's sum split off the critical path: the Montgomery quotient digit Mq[k] waits only
// for the previous digit's term Mq[k-1] * P[1] and the carry; every other term of column k (the x*y products and the
// older digits' products) goes into two independent accumulators that the scheduler can interleave with the previous
// column. Same terms, same bound (< 2^61), same result.
#define M28_ILP_BODY(COL2)                                                                  \
  uint32_t Mq[14], R[14];                                                                   \
  uint64_t acc = 0;                                                                         \
  _Pragma("unroll") for (int k = 0; k < 27; k++) {                                          \
    uint64_t s0 = 0, s1 = 0;                                                                \
    COL2(k, s0, s1);                                                                        \
    _Pragma("unroll") for (int i = (k > 13 ? k - 13 : 0); i <= (k < 14 ? k - 2 : 13); i++) \
      if (i & 1) s1 += (uint64_t)Mq[i] * P[k - i];                                          \
      else s0 += (uint64_t)Mq[i] * P[k - i];                                                \
    acc = (acc >> 28) + (s0 + s1);                                                          \
    if (k < 14) {                                                                           \
      if (k >= 1) acc += (uint64_t)Mq[k - 1] * P[1];                                        \
      Mq[k] = ((uint32_t)acc * N0) & MASK;                                                  \
      acc += (uint64_t)Mq[k] * P[0];                                                        \
    } else {                                                                                \
      R[k - 14] = (uint32_t)acc & MASK;                                                     \
    }                                                                                       \
  }                                                                                         \
  R[13] = (uint32_t)(acc >> 28);

__device__ __forceinline__ void final_sub(uint32_t r[12]) {
  uint32_t t[12];
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) t[i] = __builtin_subc(r[i], P32[i], br, &br);
#pragma unroll
  for (int i = 0; i < 12; i++) r[i] = br ? r[i] : t[i];
}

__device__ __forceinline__ void mul_ilp(uint32_t r[12], const uint32_t x[12], const uint32_t y[12]) {
  uint32_t X[14], Y[14];
  split<0>(X, x);
  split<8>(Y, y);
#define COLM2(k, s0, s1)                                                                     \
  _Pragma("unroll") for (int i = ((k) > 13 ? (k) - 13 : 0); i <= ((k) < 13 ? (k) : 13); i++) \
      if (i & 1) s1 += (uint64_t)X[i] * Y[(k) - i];                                          \
      else s0 += (uint64_t)X[i] * Y[(k) - i];
  M28_ILP_BODY(COLM2)
#undef COLM2
  join(r, R);
  final_sub(r);
}

__device__ __forceinline__ void sqr_ilp(uint32_t r[12], const uint32_t x[12]) {
  uint32_t X[14], X2[14];
  split<4>(X, x);
#pragma unroll
  for (int i = 0; i < 14; i++) X2[i] = X[i] << 1;
#define COLS2(k, s0, s1)                                                                                  \
  _Pragma("unroll") for (int i = ((k) > 13 ? (k) - 13 : 0); 2 * i < (k); i++)                              \
      if (i & 1) s1 += (uint64_t)X[i] * X2[(k) - i];                                                      \
      else s0 += (uint64_t)X[i] * X2[(k) - i];                                                            \
  if (((k) & 1) == 0) s1 += (uint64_t)X[(k) / 2] * X[(k) / 2];
  M28_ILP_BODY(COLS2)
#undef COLS2
  join(r, R);
  final_sub(r);
}
}  // namespace m28
}  // namespace dh
