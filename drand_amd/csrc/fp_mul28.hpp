// Fp Montgomery product and squaring on 14 x 28-bit limbs.
//   * mul / sqr: behind the 12 x 32-bit interface of fp.hpp — the bodies of the library's out-of-line field products
//     (fp.hpp dh_fp_mul_vec / dh_fp_sqr_vec; call clobbers v0-v39, v48-v53, s0-s17, checked at build time by
//     drand_amd/tools/check_fp_abi.py);
//   * mont_mul / mont_sqr: the same reduction on values already held as 28-bit limbs, Montgomery radix R' = 2^392
//     — the pairing VM's own representation (k_vm.hip), which skips the 12 <-> 14 limb slicing and the final
//     subtraction.
//
// Why 28 bits: on gfx950 the 32-bit product-scanning step is a v_mad_u64_u32 PLUS a v_addc_co_u32 for the carry
// into the column's third word, and the carry add issues as slowly as the multiply (~19 T MAC/s either way against
// 37 T/s for the bare MAD, profiles/microbench_carry_r02.txt). A 28x28-bit product is < 2^56, so one 64-bit
// accumulator absorbs a whole column (<= 28 products + the carry-in < 2^61) with ONE v_mad_u64_u32 per product
// and no carry add: 392 MADs for a product, 301 for a squaring, plus ~25 column normalisations (mask, 64-bit
// shift, one 28-bit v_mul_lo for the Montgomery quotient digit).
// Measured at one dependent chain per lane (bench/microbench_fp28.hip, profiles/microbench_fp28_r02b.txt): +5%
// products and +11% squarings over the 12 x 32-bit form at 8 waves/SIMD, +7% / +22% at 1 wave/SIMD; splitting
// each column's sum over two accumulators (more ILP) measured only +1.5-2% and was not kept.
//
// mont_mul(X, Y) = X Y / 2^392 + m p / 2^392 with m < 2^392: for X, Y < 2p the result is < 4p^2/2^392 + p
// < 1.002 p, limbs normalised (R[13] < 2^19).
// mul(x, y) (12 x 32-bit, x, y < p): the product slices y * 2^8 and the squaring slices x * 2^4 (both < 2^392), so
// the division by 2^392 leaves x y / 2^384, the value of the 32-bit form; one conditional subtraction gives < p.
#pragma once
#include <stdint.h>

namespace dh {

// Counting build (make -C drand_amd count -> libdrandhip_count.so): every field product or squaring a lane executes
// bumps a per-translation-unit device counter, read back by the host after each profiled launch
// (dh_profile_read "products"; bench/count_products.py -> bench/workmodel.json). The regular build compiles nothing.
#ifdef DH_COUNT_PRODUCTS
static __device__ unsigned long long dh_nprod;
#define DH_COUNT_PROD() atomicAdd(&dh_nprod, 1ull)
#define DH_COUNTER_ACCESSOR(tu)                                                  \
  hipError_t count_take_##tu(unsigned long long* v) {                            \
    hipError_t e = hipMemcpyFromSymbol(v, HIP_SYMBOL(dh_nprod), sizeof *v);      \
    if (e != hipSuccess) return e;                                               \
    const unsigned long long z = 0;                                              \
    return hipMemcpyToSymbol(HIP_SYMBOL(dh_nprod), &z, sizeof z);                \
  }
#else
#define DH_COUNT_PROD() ((void)0)
#define DH_COUNTER_ACCESSOR(tu)
#endif

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
  uint32_t Mq[14];                                                      \
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

// R = X Y / 2^392 (mod p, < X Y / 2^392 + p)
__device__ __forceinline__ void mont_mul(uint32_t R[14], const uint32_t X[14], const uint32_t Y[14]) {
#define COLM(k, acc)                                                                         \
  _Pragma("unroll") for (int i = ((k) > 13 ? (k) - 13 : 0); i <= ((k) < 13 ? (k) : 13); i++) \
      acc += (uint64_t)X[i] * Y[(k) - i];
  M28_BODY(COLM)
#undef COLM
}

// R = X^2 / 2^392, the off-diagonal products once against the doubled limbs: 105 products instead of 196
__device__ __forceinline__ void mont_sqr(uint32_t R[14], const uint32_t X[14]) {
  uint32_t X2[14];
#pragma unroll
  for (int i = 0; i < 14; i++) X2[i] = X[i] << 1;
#define COLS(k, acc)                                                                                  \
  _Pragma("unroll") for (int i = ((k) > 13 ? (k) - 13 : 0); 2 * i < (k); i++) acc += (uint64_t)X[i] * X2[(k) - i]; \
  if (((k) & 1) == 0) acc += (uint64_t)X[(k) / 2] * X[(k) / 2];
  M28_BODY(COLS)
#undef COLS
}

// r < 2p -> r < p (12 x 32-bit words)
__device__ __forceinline__ void final_sub(uint32_t r[12]) {
  uint32_t t[12];
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) t[i] = __builtin_subc(r[i], P32[i], br, &br);
#pragma unroll
  for (int i = 0; i < 12; i++) r[i] = br ? r[i] : t[i];
}

__device__ __forceinline__ void mul(uint32_t r[12], const uint32_t x[12], const uint32_t y[12]) {
  uint32_t X[14], Y[14], R[14];
  split<0>(X, x);
  split<8>(Y, y);
  mont_mul(R, X, Y);
  join(r, R);
  final_sub(r);
}

// x^2 / 2^384 = (x 2^4)^2 / 2^392 (x 2^4 < 2^385)
__device__ __forceinline__ void sqr(uint32_t r[12], const uint32_t x[12]) {
  uint32_t X[14], R[14];
  split<4>(X, x);
  mont_sqr(R, X);
  join(r, R);
  final_sub(r);
}
}  // namespace m28
}  // namespace dh
