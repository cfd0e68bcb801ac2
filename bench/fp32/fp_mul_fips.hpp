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

#include <utility>

#include "fp_mac_g.hpp"
#include "fp_mac_n.hpp"

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

__device__ __forceinline__ void fips_mont_mul1(uint32_t r[12], const uint32_t a[12], const uint32_t b[12]) {
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
__device__ __forceinline__ void fips_mont_sqr1(uint32_t r[12], const uint32_t a[12]) {
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

// Column-statement form (the one used): every column's partial products are ONE inline-asm statement
// (fp_mac_n.hpp, generated). The hazard recognizer assumes a one-wait-state dst-forwarding hazard between
// two inline-asm statements that share a register (gfx940+), so one MAC per statement costs an s_nop 0 per
// partial product (252 of them in fips_mont_mul1); one statement per column leaves ~1 per column. Inside a
// statement, v_mad_u64_u32 (carry-out to an SGPR pair) followed by v_addc_co_u32 reading it is the
// ordinary VALU-writes-SGPR / VALU-reads-carry sequence of the compiler's own 64-bit adds.
#define DH_P_LIMBS                                                                                      \
  {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u,                        \
   0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau}

template <int K>
__device__ __forceinline__ void mul_col(uint64_t& acc, uint32_t& hi, uint32_t m[12], uint32_t r[12],
                                        const uint32_t a[12], const uint32_t b[12], const uint32_t P[12]) {
  constexpr uint32_t NP0 = 0xfffcfffdu;
  constexpr int LO = K > 11 ? K - 11 : 0, UP = K < 12 ? K : 11, MUP = K < 12 ? K - 1 : 11;
  constexpr int C = (UP - LO + 1) + (MUP >= LO ? MUP - LO + 1 : 0);
  constexpr int C1 = UP - LO + 1, C2 = C - C1;
  uint32_t xs[C1], ys[C1], ms[C2 > 0 ? C2 : 1], ps[C2 > 0 ? C2 : 1];
#pragma unroll
  for (int i = LO; i <= UP; i++) { xs[i - LO] = a[i]; ys[i - LO] = b[K - i]; }
#pragma unroll
  for (int i = LO; i <= MUP; i++) { ms[i - LO] = m[i]; ps[i - LO] = P[K - i]; }
  mac_g<C1, C2, 1>(acc, hi, xs, ys, ms, ps);  // the column's carry word starts here (hi not read)
  if constexpr (K < 12) {
    m[K] = (uint32_t)acc * NP0;
    uint32_t p0 = P[0];
    mac_g<0, 1, 0>(acc, hi, xs, ys, &m[K], &p0);  // low word becomes 0
  } else {
    r[K - 12] = (uint32_t)acc;
  }
  acc = (acc >> 32) | ((uint64_t)hi << 32);
}

template <int K>
__device__ __forceinline__ void sqr_col(uint64_t& acc, uint32_t& hi, uint32_t m[12], uint32_t r[12],
                                        const uint32_t a[12], const uint32_t P[12]) {
  constexpr uint32_t NP0 = 0xfffcfffdu;
  constexpr int LO = K > 11 ? K - 11 : 0, MUP = K < 12 ? K - 1 : 11;
  constexpr int D = (K + 1) / 2 - LO > 0 ? (K + 1) / 2 - LO : 0;  // pairs i < K-i, i >= LO
  constexpr int CM = MUP >= LO ? MUP - LO + 1 : 0;
  uint64_t s = 0;
  uint32_t sh = 0;
  if constexpr (D > 0) {
    uint32_t xs[D], ys[D];
#pragma unroll
    for (int j = 0; j < D; j++) { xs[j] = a[LO + j]; ys[j] = a[K - LO - j]; }
    mac_n<D>(s, sh, xs, ys);
    sh = (sh << 1) | (uint32_t)(s >> 63);
    s <<= 1;
  }
  if constexpr ((K & 1) == 0) mac_n<1>(s, sh, &a[K >> 1], &a[K >> 1]);
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
  if constexpr (CM > 0) {
    uint32_t xs[CM], ys[CM];
#pragma unroll
    for (int j = 0; j < CM; j++) { xs[j] = m[LO + j]; ys[j] = P[K - LO - j]; }
    mac_n<CM>(acc, hi, xs, ys);
  }
  if constexpr (K < 12) {
    m[K] = (uint32_t)acc * NP0;
    uint32_t p0 = P[0];
    mac_n<1>(acc, hi, &m[K], &p0);
  } else {
    r[K - 12] = (uint32_t)acc;
  }
  acc = (acc >> 32) | ((uint64_t)hi << 32);
  hi = 0;
}

template <int... K>
__device__ __forceinline__ void mul_cols(std::integer_sequence<int, K...>, uint64_t& acc, uint32_t& hi, uint32_t m[12],
                                         uint32_t r[12], const uint32_t a[12], const uint32_t b[12], const uint32_t P[12]) {
  (mul_col<K>(acc, hi, m, r, a, b, P), ...);
}
template <int... K>
__device__ __forceinline__ void sqr_cols(std::integer_sequence<int, K...>, uint64_t& acc, uint32_t& hi, uint32_t m[12],
                                         uint32_t r[12], const uint32_t a[12], const uint32_t P[12]) {
  (sqr_col<K>(acc, hi, m, r, a, P), ...);
}

__device__ __forceinline__ void fips_final_sub(uint32_t r[12], uint64_t acc, const uint32_t P[12]) {
  r[11] = (uint32_t)acc;  // < 2p < 2^382: no further carry
  uint32_t d[12];
  unsigned br = 0;  // one v_sub_co / v_subb_co per limb (see fp.hpp: fp_reduce_once)
#pragma unroll
  for (int i = 0; i < 12; i++) d[i] = __builtin_subc(r[i], P[i], br, &br);
#pragma unroll
  for (int i = 0; i < 12; i++) r[i] = br ? r[i] : d[i];
}

__device__ __forceinline__ void fips_mont_mul(uint32_t r[12], const uint32_t a[12], const uint32_t b[12]) {
  const uint32_t P[12] = DH_P_LIMBS;
  uint32_t m[12];
  uint64_t acc = 0;
  uint32_t hi = 0;
  mul_cols(std::make_integer_sequence<int, 23>{}, acc, hi, m, r, a, b, P);
  fips_final_sub(r, acc, P);
}

__device__ __forceinline__ void fips_mont_sqr_col(uint32_t r[12], const uint32_t a[12]) {
  const uint32_t P[12] = DH_P_LIMBS;
  uint32_t m[12];
  uint64_t acc = 0;
  uint32_t hi = 0;
  sqr_cols(std::make_integer_sequence<int, 23>{}, acc, hi, m, r, a, P);
  fips_final_sub(r, acc, P);
}
// Squaring, three phases: (1) the off-diagonal triangle T = sum_{i<j} a_i a_j 2^(32(i+j)) by product scanning
// (66 products, no per-column doubling), (2) 2T word by word with one v_alignbit each, (3) Montgomery
// product scanning over 2T + the diagonal squares, where each column's incoming word is added in the same
// two instructions that shift the accumulator (no separate 96-bit add). 222 products as in fips_mont_sqr_col,
// ~25% fewer other instructions.
template <int K>
__device__ __forceinline__ void sqr_tri_col(uint64_t& acc, uint32_t& hi, uint32_t t[24], const uint32_t a[12]) {
  constexpr int LO = K > 11 ? K - 11 : 0;
  constexpr int D = (K + 1) / 2 - LO > 0 ? (K + 1) / 2 - LO : 0;  // pairs i < K-i, i >= LO
  if constexpr (D > 0) {
    uint32_t xs[D], ys[D];
#pragma unroll
    for (int j = 0; j < D; j++) { xs[j] = a[LO + j]; ys[j] = a[K - LO - j]; }
    mac_g<D, 0, 1>(acc, hi, xs, ys, xs, ys);  // new carry word (hi not read)
  } else {
    hi = 0;
  }
  t[K] = (uint32_t)acc;
  acc = (acc >> 32) | ((uint64_t)hi << 32);
}

// acc <- (hi:acc_hi) + w, i.e. shift the 96-bit column accumulator down one word and add the next input word
__device__ __forceinline__ void acc_shift_add(uint64_t& acc, uint32_t& hi, uint32_t w) {
  uint32_t lo = (uint32_t)(acc >> 32), h = hi;
  uint64_t c_;
  asm volatile("v_add_co_u32_e64 %0, %2, %0, %3\n\tv_addc_co_u32_e64 %1, %2, %1, 0, %2"
               : "+v"(lo), "+v"(h), "=&s"(c_)
               : "v"(w));
  acc = (uint64_t)lo | ((uint64_t)h << 32);
}

template <int K>
__device__ __forceinline__ void sqr_red_col(uint64_t& acc, uint32_t& hi, uint32_t m[12], uint32_t r[12], const uint32_t t[24],
                                            const uint32_t a[12], const uint32_t P[12]) {
  constexpr uint32_t NP0 = 0xfffcfffdu;
  constexpr int LO = K > 11 ? K - 11 : 0, MUP = K < 12 ? K - 1 : 11;
  constexpr int CM = MUP >= LO ? MUP - LO + 1 : 0;
  constexpr int C = CM + ((K & 1) == 0 ? 1 : 0);
  // word K of 2T
  uint32_t u = K == 0 ? t[0] << 1 : __builtin_amdgcn_alignbit(t[K], t[K > 0 ? K - 1 : 0], 31);
  if constexpr (K == 0) {
    acc = u;
  } else {
    acc_shift_add(acc, hi, u);
  }
  {
    constexpr int C1 = C - CM;  // the diagonal square a_{K/2}^2 on even columns
    uint32_t xs[1], ys[1], ms[CM > 0 ? CM : 1], ps[CM > 0 ? CM : 1];
    if constexpr (C1) { xs[0] = a[K >> 1]; ys[0] = a[K >> 1]; }
#pragma unroll
    for (int j = 0; j < CM; j++) { ms[j] = m[LO + j]; ps[j] = P[K - LO - j]; }
    mac_g<C1, CM, 1>(acc, hi, xs, ys, ms, ps);  // new carry word (hi not read; C = 0 sets it to 0)
  }
  if constexpr (K < 12) {
    m[K] = (uint32_t)acc * NP0;
    uint32_t p0 = P[0];
    mac_g<0, 1, 0>(acc, hi, m, m, &m[K], &p0);
  } else {
    r[K - 12] = (uint32_t)acc;
  }
}

template <int... K>
__device__ __forceinline__ void sqr_tri_cols(std::integer_sequence<int, K...>, uint64_t& acc, uint32_t& hi, uint32_t t[24],
                                             const uint32_t a[12]) {
  (sqr_tri_col<K>(acc, hi, t, a), ...);
}
template <int... K>
__device__ __forceinline__ void sqr_red_cols(std::integer_sequence<int, K...>, uint64_t& acc, uint32_t& hi, uint32_t m[12],
                                             uint32_t r[12], const uint32_t t[24], const uint32_t a[12], const uint32_t P[12]) {
  (sqr_red_col<K>(acc, hi, m, r, t, a, P), ...);
}

__device__ __forceinline__ void fips_mont_sqr(uint32_t r[12], const uint32_t a[12]) {
  const uint32_t P[12] = DH_P_LIMBS;
  uint32_t t[24], m[12];
  uint64_t acc = 0;
  uint32_t hi = 0;
  t[0] = 0;
  sqr_tri_cols(std::integer_sequence<int, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21>{},
               acc, hi, t, a);
  t[22] = (uint32_t)acc;
  t[23] = (uint32_t)(acc >> 32);
  acc = 0;
  hi = 0;
  sqr_red_cols(std::make_integer_sequence<int, 23>{}, acc, hi, m, r, t, a, P);
  acc_shift_add(acc, hi, __builtin_amdgcn_alignbit(t[23], t[22], 31));
  fips_final_sub(r, acc, P);
}
#undef DH_P_LIMBS

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
