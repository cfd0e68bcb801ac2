// Montgomery multiplication / squaring for the BLS12-381 base field on gfx950, product scanning (FIPS).
//
// Column k of the 2x12-limb product accumulates a_i b_{k-i} and m_i p_{k-i} into a 96-bit accumulator
// (acc = 64-bit VGPR pair + a 32-bit top word). Each partial product is ONE v_mad_u64_u32 whose 64-bit
// addend is the accumulator pair itself and whose carry-out goes straight into the top word with one
// v_addc_co_u32 — no 64-bit add emulation and no register shuffling, which is what the compiler emits
// for the textbook CIOS loop (fp.hpp: fp_mul_cios), ~2x more VALU issue for the same 288 products.
// Output is fully reduced (< p); inputs must be < p.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dh {

// acc(64) += x*y, carry into hi32. The carry-out lane mask goes through an SGPR pair the compiler
// allocates (an early-clobber output), never VCC: a "vcc" clobber is not a reliable way to keep the
// compiler from holding a live branch condition in VCC across the statement (seen on ROCm 7.2 in the
// scalar-branch exponentiation loop).
#define DH_MAC(acc, hi, x, y)                                                                       \
  do {                                                                                              \
    uint64_t c_;                                                                                    \
    asm volatile("v_mad_u64_u32 %0, %2, %3, %4, %0\n\tv_addc_co_u32_e64 %1, %2, 0, %1, %2"          \
                 : "+v"(acc), "+v"(hi), "=&s"(c_)                                                   \
                 : "v"(x), "v"(y));                                                                 \
  } while (0)

__device__ __forceinline__ void fips_mont_mul(uint32_t r[12], const uint32_t a[12], const uint32_t b[12]) {
  constexpr uint32_t P[12] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u,
                              0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
  constexpr uint32_t NP0 = 0xfffcfffdu;
  uint32_t m[12];
  uint64_t acc = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int k = 0; k < 12; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) DH_MAC(acc, hi, a[i], b[k - i]);
#pragma unroll
    for (int i = 0; i < k; i++) DH_MAC(acc, hi, m[i], P[k - i]);
    m[k] = (uint32_t)acc * NP0;
    DH_MAC(acc, hi, m[k], P[0]);  // low word becomes 0
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
#pragma unroll
  for (int k = 12; k < 23; k++) {
#pragma unroll
    for (int i = k - 11; i < 12; i++) DH_MAC(acc, hi, a[i], b[k - i]);
#pragma unroll
    for (int i = k - 11; i < 12; i++) DH_MAC(acc, hi, m[i], P[k - i]);
    r[k - 12] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  r[11] = (uint32_t)acc;  // < 2p < 2^382: no further carry
  // conditional subtraction of p
  uint32_t d[12];
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t t = (uint64_t)r[i] - P[i] - br;
    d[i] = (uint32_t)t;
    br = (t >> 63) & 1;
  }
#pragma unroll
  for (int i = 0; i < 12; i++) r[i] = br ? r[i] : d[i];
}

// squaring: off-diagonal products once, doubled, plus the diagonal (222 instead of 288 partial products)
__device__ __forceinline__ void fips_mont_sqr(uint32_t r[12], const uint32_t a[12]) {
  constexpr uint32_t P[12] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u,
                              0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
  constexpr uint32_t NP0 = 0xfffcfffdu;
  uint32_t m[12];
  uint64_t acc = 0;  // accumulator of the Montgomery part + carried column value
  uint32_t hi = 0;
#pragma unroll
  for (int k = 0; k < 23; k++) {
    // s = sum_{i<j, i+j=k} a_i a_j  (96-bit), then acc += 2 s + [k even] a_{k/2}^2
    uint64_t s = 0;
    uint32_t sh = 0;
#pragma unroll
    for (int i = (k > 11 ? k - 11 : 0); i < k - i; i++) DH_MAC(s, sh, a[i], a[k - i]);
    // double s (sh:s is < 2^96)
    sh = (sh << 1) | (uint32_t)(s >> 63);
    s <<= 1;
    if ((k & 1) == 0) DH_MAC(s, sh, a[k >> 1], a[k >> 1]);
    // acc += s
    {
      uint32_t slo = (uint32_t)s, shi = (uint32_t)(s >> 32);
      uint32_t alo = (uint32_t)acc, ahi = (uint32_t)(acc >> 32);
      uint64_t c_;
      asm volatile(
          "v_add_co_u32_e64 %0, %3, %0, %4\n\t"
          "v_addc_co_u32_e64 %1, %3, %1, %5, %3\n\t"
          "v_addc_co_u32_e64 %2, %3, %2, %6, %3"
          : "+v"(alo), "+v"(ahi), "+v"(hi), "=&s"(c_)
          : "v"(slo), "v"(shi), "v"(sh));
      acc = (uint64_t)alo | ((uint64_t)ahi << 32);
    }
    if (k < 12) {
#pragma unroll
      for (int i = 0; i < k; i++) DH_MAC(acc, hi, m[i], P[k - i]);
      m[k] = (uint32_t)acc * NP0;
      DH_MAC(acc, hi, m[k], P[0]);
    } else {
#pragma unroll
      for (int i = k - 11; i < 12; i++) DH_MAC(acc, hi, m[i], P[k - i]);
      r[k - 12] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  r[11] = (uint32_t)acc;
  uint32_t d[12];
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t t = (uint64_t)r[i] - P[i] - br;
    d[i] = (uint32_t)t;
    br = (t >> 63) & 1;
  }
#pragma unroll
  for (int i = 0; i < 12; i++) r[i] = br ? r[i] : d[i];
}

#undef DH_MAC

// The same product-scanning schedule in plain C (no inline asm): the carry-out of each 64-bit
// accumulation is recovered with a compare, which the compiler fuses into v_cmp + v_addc. Kept as the
// hazard-free reference for the asm version (bench/microbench_fp.hip compares both).
#define DH_MACC(acc, hi, x, y)                             \
  do {                                                     \
    uint64_t t_ = (uint64_t)(x) * (uint64_t)(y) + (acc);   \
    hi += t_ < (acc) ? 1u : 0u;                            \
    acc = t_;                                              \
  } while (0)

__device__ __forceinline__ void fips_mont_mul_c(uint32_t r[12], const uint32_t a[12], const uint32_t b[12]) {
  constexpr uint32_t P[12] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u,
                              0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
  constexpr uint32_t NP0 = 0xfffcfffdu;
  uint32_t m[12];
  uint64_t acc = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int k = 0; k < 12; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) DH_MACC(acc, hi, a[i], b[k - i]);
#pragma unroll
    for (int i = 0; i < k; i++) DH_MACC(acc, hi, m[i], P[k - i]);
    m[k] = (uint32_t)acc * NP0;
    DH_MACC(acc, hi, m[k], P[0]);
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
#pragma unroll
  for (int k = 12; k < 23; k++) {
#pragma unroll
    for (int i = k - 11; i < 12; i++) DH_MACC(acc, hi, a[i], b[k - i]);
#pragma unroll
    for (int i = k - 11; i < 12; i++) DH_MACC(acc, hi, m[i], P[k - i]);
    r[k - 12] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  r[11] = (uint32_t)acc;
  uint32_t d[12];
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t t = (uint64_t)r[i] - P[i] - br;
    d[i] = (uint32_t)t;
    br = (t >> 63) & 1;
  }
#pragma unroll
  for (int i = 0; i < 12; i++) r[i] = br ? r[i] : d[i];
}
#undef DH_MACC
}  // namespace dh
