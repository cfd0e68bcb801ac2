// Shared device helpers of the kernel translation units (AoS point I/O, generators, check equations).
#pragma once
#include <hip/hip_runtime.h>
#include "pairing.hpp"
#include "h2c.hpp"
#include "codec.hpp"
#include "kernels.hpp"

namespace dh {

// ---------------------------------------------------------------- point <-> AoS global memory (16-B aligned)
template <class F>
struct npw {  // words per field element
  static constexpr int N = limbs_of<F>::N;
};

template <class F>
DH_DEV void ld_f(F& a, const uint32_t* p);
template <>
DH_DEV void ld_f<fp>(fp& a, const uint32_t* p) {
  const uint4* q = (const uint4*)p;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    uint4 t = q[i];
    a.v[4 * i] = t.x; a.v[4 * i + 1] = t.y; a.v[4 * i + 2] = t.z; a.v[4 * i + 3] = t.w;
  }
}
template <>
DH_DEV void ld_f<fp2>(fp2& a, const uint32_t* p) {
  ld_f<fp>(a.c0, p);
  ld_f<fp>(a.c1, p + 12);
}
template <class F>
DH_DEV void st_f(uint32_t* p, const F& a);
template <>
DH_DEV void st_f<fp>(uint32_t* p, const fp& a) {
  uint4* q = (uint4*)p;
#pragma unroll
  for (int i = 0; i < 3; i++) q[i] = make_uint4(a.v[4 * i], a.v[4 * i + 1], a.v[4 * i + 2], a.v[4 * i + 3]);
}
template <>
DH_DEV void st_f<fp2>(uint32_t* p, const fp2& a) {
  st_f<fp>(p, a.c0);
  st_f<fp>(p + 12, a.c1);
}
template <class F>
DH_DEV jac<F> ld_jac_aos(const uint32_t* base, size_t i) {
  constexpr int N = npw<F>::N;
  const uint32_t* p = base + (size_t)3 * N * i;
  jac<F> r;
  ld_f<F>(r.x, p);
  ld_f<F>(r.y, p + N);
  ld_f<F>(r.z, p + 2 * N);
  return r;
}
template <class F>
DH_DEV void st_jac_aos(uint32_t* base, size_t i, const jac<F>& a) {
  constexpr int N = npw<F>::N;
  uint32_t* p = base + (size_t)3 * N * i;
  st_f<F>(p, a.x);
  st_f<F>(p + N, a.y);
  st_f<F>(p + 2 * N, a.z);
}
template <class F>
DH_DEV aff<F> ld_aff_aos(const uint32_t* base, size_t i) {
  constexpr int N = npw<F>::N;
  const uint32_t* p = base + (size_t)2 * N * i;
  aff<F> r;
  ld_f<F>(r.x, p);
  ld_f<F>(r.y, p + N);
  return r;
}
template <class F>
DH_DEV void st_aff_aos(uint32_t* base, size_t i, const aff<F>& a) {
  constexpr int N = npw<F>::N;
  uint32_t* p = base + (size_t)2 * N * i;
  st_f<F>(p, a.x);
  st_f<F>(p + N, a.y);
}

// add-2007-bl for two points held in memory (AoS Jacobian, 72 words each), coordinates loaded as they are needed;
// Z3 = 2 Z1 Z2 h (= ((Z1 + Z2)^2 - Z1^2 - Z2^2) h). false (r unset) when x1 == x2, as jac_add_distinct.
DH_DEV bool jac_add_distinct_mem(jac<fp2>& r, const uint32_t* P, const uint32_t* Q) {
  fp2 c1, c2, zz, u1, h;
  {
    fp2 z1, z2;
    ld_f<fp2>(z1, P + 48);
    ld_f<fp2>(z2, Q + 48);
    const fp2 z1z1 = fp2_sqr(z1), z2z2 = fp2_sqr(z2);
    c1 = fp2_mul(z1, z1z1);
    c2 = fp2_mul(z2, z2z2);
    zz = fp2_mul(z1, z2);
    fp2 x;
    ld_f<fp2>(x, P);
    u1 = fp2_mul(x, z2z2);
    ld_f<fp2>(x, Q);
    h = fp2_sub(fp2_mul(x, z1z1), u1);
  }
  if (fp2_is_zero(h)) return false;
  fp2 s1, rr;
  {
    fp2 y;
    ld_f<fp2>(y, P + 24);
    s1 = fp2_mul(y, c2);
    ld_f<fp2>(y, Q + 24);
    rr = fp2_dbl(fp2_sub(fp2_mul(y, c1), s1));
  }
  const fp2 i = fp2_sqr(fp2_dbl(h));
  const fp2 j = fp2_mul(h, i);
  const fp2 v = fp2_mul(u1, i);
  r.x = fp2_sub(fp2_sub(fp2_sqr(rr), j), fp2_dbl(v));
  r.y = fp2_sub(fp2_mul(rr, fp2_sub(v, r.x)), fp2_dbl(fp2_mul(s1, j)));
  r.z = fp2_dbl(fp2_mul(zz, h));
  return true;
}

// the other group of the pairing
template <class F>
struct other;
template <>
struct other<fp> {
  using T = fp2;
};
template <>
struct other<fp2> {
  using T = fp;
};

// minimum waves per SIMD for the per-round kernels: G1 point code fits 128 VGPRs (4 waves); G2 (Fp2)
// point code spills heavily at 128, so it gets 256 VGPRs (2 waves) instead
template <class F>
struct occ {
  static constexpr int W = 2;
};
template <>
struct occ<fp2> {
  static constexpr int W = 2;
};

DH_DEV size_t gtid() { return (size_t)blockIdx.x * blockDim.x + threadIdx.x; }

DH_DEV jac<fp> g1_gen() { return {fp_c(cst::G1X), fp_c(cst::G1Y), fp_one()}; }
DH_DEV jac<fp2> g2_gen() { return {fp2_c(cst::G2X), fp2_c(cst::G2Y), fp2_one()}; }

static inline unsigned nblk(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

// DigestBeacon of round i; false when the chained record is longer than its slot (a caller error on the
// device entry point: the round is rejected instead of reading past the record)
DH_DEV bool beacon_digest(sha_h& d, const uint64_t* __restrict__ rounds, const uint8_t* __restrict__ prevs, size_t prev_stride,
                          const uint32_t* __restrict__ prev_lens, int chained, size_t i) {
  if (!chained) {
    d = digest_unchained(rounds[i]);
    return true;
  }
  const uint64_t pl = prev_lens ? (uint64_t)prev_lens[i] : (uint64_t)prev_stride;
  if (pl > prev_stride) {
    d = digest_unchained(rounds[i]);
    return false;
  }
  const uint8_t* p = prevs + i * prev_stride;
  if (pl <= 96 && (pl & 3) == 0 && (((uintptr_t)p) & 3) == 0) d = digest_chained(p, (uint32_t)pl, rounds[i]);
  else d = digest_chained_any(p, (uint32_t)pl, rounds[i]);
  return true;
}

// message i: the beacon digest of (rounds, prevs) or, for VerifyRecovered / tbls, the given 32-byte msgs32[i]
DH_DEV sha_h message_of(const uint64_t* __restrict__ rounds, const uint8_t* __restrict__ prevs, size_t prev_stride,
                        const uint32_t* __restrict__ prev_lens, const uint8_t* __restrict__ msgs32, int chained, size_t i,
                        uint8_t* __restrict__ status) {
  sha_h d;
  if (msgs32) {
#pragma unroll
    for (int j = 0; j < 8; j++) d.h[j] = ld_be32a(msgs32 + 32 * i + 4 * j);
  } else if (!beacon_digest(d, rounds, prevs, prev_stride, prev_lens, chained, i) && status) {
    status[i] = DEC_BAD;
  }
  return d;
}


}  // namespace dh
