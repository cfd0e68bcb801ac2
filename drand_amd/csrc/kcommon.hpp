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

}  // namespace dh
