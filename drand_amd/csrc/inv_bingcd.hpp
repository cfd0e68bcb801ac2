// Variable-time inverse modulo p by the optimized binary GCD of T. Pornin ("Optimized Binary GCD for Modular
// Inversion", IACR ePrint 2020/972, Algorithm 2): 25 outer rounds of 31 divsteps, each round's steps run on 64-bit
// approximations of a and b (their low 31 and top 33 bits) and their effect is then applied to the full 384-bit
// values as one linear combination with 32-bit factors, so the 12-word arithmetic runs 25 times instead of once per
// divstep (~450 times in the plain binary GCD it replaces, fp.hpp inv_vt_int's former body: one lane's inversion was
// 0.19 ms, 7% of a pairing check, profiles/r06/vm_phase_profile_r06z.txt). 25 x 31 >= 2 len(p) - 1 = 761 divsteps
// bring b to gcd = 1. The cofactors u, v are divided by 2^31 each round (Montgomery: add q p, q = -t p^-1 mod 2^31),
// which keeps a = u y and b = v y (mod p) exact, so v is the inverse with no correction factor.
// Plain integer code with a qualifier macro: the library compiles it for the device, tests/test_inv_bingcd.py compiles
// the same source for the host and checks it against Python's pow(y, -1, p) (edge cases and random inputs); the
// algorithm is prototyped line by line in that test.
#pragma once
#include <stdint.h>

#ifndef DH_HD
#define DH_HD __device__ __forceinline__
#endif

namespace dh {
namespace bgcd {

// p, little-endian 32-bit words
DH_HD uint32_t P(int i) {
  const uint32_t t[12] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u,
                          0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
  return t[i];
}
constexpr uint32_t NP31 = 0x7ffcfffdu;  // -p^-1 mod 2^31
constexpr int K = 31;                  // divsteps per round
constexpr int ROUNDS = 25;             // ceil((2 * 381 - 1) / 31)

DH_HD int clz32(uint32_t w) { return __builtin_clz(w); }  // w != 0

// An empty asm on the device hides the value from the optimiser: a chain of selects on one index is otherwise turned
// into an array in scratch indexed at run time (the word pick in approx() below); a no-op in the host build
DH_HD void dh_opaque64(uint64_t& v) {
#if defined(__AMDGCN__)
  asm volatile("" : "+v"(v));
#else
  (void)v;
#endif
}

// out (13 words) = x (12 words) * m
DH_HD void mul_small(uint32_t out[13], const uint32_t x[12], uint32_t m) {
  uint64_t c = 0;
  #pragma unroll
  for (int i = 0; i < 12; i++) {
    c = (uint64_t)x[i] * m + (c >> 32);
    out[i] = (uint32_t)c;
  }
  out[12] = (uint32_t)(c >> 32);
}

DH_HD uint32_t mag(int64_t f) { return (uint32_t)(f < 0 ? -f : f); }  // |f| <= 2^31

// r = |x fx + y fy| / 2^31 (the division is exact); returns true when x fx + y fy < 0
DH_HD bool lin_div(uint32_t r[12], const uint32_t x[12], int64_t fx, const uint32_t y[12], int64_t fy) {
  uint32_t s[13], t[13];
  mul_small(s, x, mag(fx));
  mul_small(t, y, mag(fy));
  bool neg;
  if ((fx < 0) == (fy < 0)) {
    uint64_t c = 0;
    #pragma unroll
    for (int i = 0; i < 13; i++) {
      c = (uint64_t)s[i] + t[i] + (c >> 32);
      s[i] = (uint32_t)c;
    }
    neg = fx < 0;
  } else {
    int64_t c = 0;  // s - t, two's complement over 13 words
    #pragma unroll
    for (int i = 0; i < 13; i++) {
      c += (int64_t)s[i] - (int64_t)t[i];
      s[i] = (uint32_t)c;
      c >>= 32;  // arithmetic: 0 or -1
    }
    neg = (fx < 0) != (c < 0);
    if (c < 0) {  // |s - t| = -(s - t)
      uint64_t d = 1;
      #pragma unroll
      for (int i = 0; i < 13; i++) {
        d += (uint64_t)(uint32_t)~s[i];
        s[i] = (uint32_t)d;
        d >>= 32;
      }
    }
  }
  #pragma unroll
  for (int i = 0; i < 12; i++) r[i] = (s[i] >> K) | (s[i + 1] << (32 - K));
  return neg;
}

// r = (x fx + y fy) / 2^31 mod p for x, y in [0, p): a negative factor takes p - x, the division adds q p with
// q = -t p^-1 mod 2^31, the result (< 3p) is reduced by at most two subtractions
DH_HD void lin_mod(uint32_t r[12], const uint32_t x[12], int64_t fx, const uint32_t y[12], int64_t fy) {
  uint32_t xs[12], ys[12];
  uint64_t bx = 0, by = 0;
  #pragma unroll
  for (int i = 0; i < 12; i++) {  // p - x, p - y (borrow chains)
    const uint64_t dx = (uint64_t)P(i) - x[i] - bx, dy = (uint64_t)P(i) - y[i] - by;
    xs[i] = fx < 0 ? (uint32_t)dx : x[i];
    ys[i] = fy < 0 ? (uint32_t)dy : y[i];
    bx = (dx >> 32) & 1;
    by = (dy >> 32) & 1;
  }
  uint32_t s[13], t[13], w[14];
  mul_small(s, xs, mag(fx));
  mul_small(t, ys, mag(fy));
  uint64_t c = 0;
  #pragma unroll
  for (int i = 0; i < 13; i++) {
    c = (uint64_t)s[i] + t[i] + (c >> 32);
    w[i] = (uint32_t)c;
  }
  w[13] = (uint32_t)(c >> 32);
  const uint32_t q = (w[0] * NP31) & 0x7fffffffu;
  c = 0;
  #pragma unroll
  for (int i = 0; i < 14; i++) {
    c = (uint64_t)(i < 12 ? P(i) : 0u) * q + w[i] + (c >> 32);
    w[i] = (uint32_t)c;
  }
  #pragma unroll
  for (int i = 0; i < 12; i++) r[i] = (w[i] >> K) | (w[i + 1] << (32 - K));
  #pragma unroll
  for (int k = 0; k < 2; k++) {  // r < 3p -> [0, p)
    uint32_t d[12];
    uint64_t b = 0;
    #pragma unroll
    for (int i = 0; i < 12; i++) {
      const uint64_t e = (uint64_t)r[i] - P(i) - b;
      d[i] = (uint32_t)e;
      b = (e >> 32) & 1;
    }
    if (!b)
      #pragma unroll
      for (int i = 0; i < 12; i++) r[i] = d[i];
  }
}

// the low 31 bits and the top 33 bits of x (< 2^n, n >= 64) as one 64-bit approximation; the words are picked by
// selects over a fully unrolled loop (a register array indexed at run time would live in scratch on the device)
DH_HD uint64_t approx(const uint32_t x[12], int n) {
  const int s = n - 33, w = s >> 5, o = s & 31;
  uint64_t two = 0;  // words w + 1 : w
#pragma unroll
  for (int j = 0; j < 11; j++) {
    uint64_t pj = ((uint64_t)x[j + 1] << 32) | x[j];
    dh_opaque64(pj);
    two = j == w ? pj : two;
  }
  const uint64_t hi = (two >> o) & 0x1ffffffffull;
  return (x[0] & 0x7fffffffu) | (hi << 31);
}

// a = a^-1 mod p for a nonzero a < p (12 x 32-bit words)
DH_HD void inverse(uint32_t a_io[12]) {
  uint32_t a[12], b[12], u[12], v[12];
  #pragma unroll
  for (int i = 0; i < 12; i++) {
    a[i] = a_io[i];
    b[i] = P(i);
    u[i] = i == 0;
    v[i] = 0;
  }
#pragma unroll 1
  for (int r = 0; r < ROUNDS; r++) {
    int n = 64;  // max(bit length of a, of b, 64): the highest nonzero word of a | b, scanned upwards
#pragma unroll
    for (int i = 2; i < 12; i++) {
      const uint32_t w = a[i] | b[i];
      if (w) n = 32 * i + 32 - clz32(w);
    }
    uint64_t ab = approx(a, n), bb = approx(b, n);
    int64_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
#pragma unroll 1
    for (int i = 0; i < K; i++) {
      if (ab & 1) {
        if (ab < bb) {
          const uint64_t t = ab;
          ab = bb;
          bb = t;
          int64_t e = f0;
          f0 = f1;
          f1 = e;
          e = g0;
          g0 = g1;
          g1 = e;
        }
        ab -= bb;
        f0 -= f1;
        g0 -= g1;
      }
      ab >>= 1;
      f1 *= 2;
      g1 *= 2;
    }
    uint32_t na[12], nb[12];
    if (lin_div(na, a, f0, b, g0)) {
      f0 = -f0;
      g0 = -g0;
    }
    if (lin_div(nb, a, f1, b, g1)) {
      f1 = -f1;
      g1 = -g1;
    }
    uint32_t nu[12], nv[12];
    lin_mod(nu, u, f0, v, g0);
    lin_mod(nv, u, f1, v, g1);
    #pragma unroll
    for (int i = 0; i < 12; i++) {
      a[i] = na[i];
      b[i] = nb[i];
      u[i] = nu[i];
      v[i] = nv[i];
    }
  }
  #pragma unroll
  for (int i = 0; i < 12; i++) a_io[i] = v[i];
}

}  // namespace bgcd
}  // namespace dh
