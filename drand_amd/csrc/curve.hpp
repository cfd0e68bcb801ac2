// Short-Weierstrass (a = 0) Jacobian point arithmetic, generic over the base field:
//   G1: y^2 = x^3 + 4        over Fp   (F = fp)
//   G2: y^2 = x^3 + 4(1+i)   over Fp2  (F = fp2)
// One point per lane. Infinity is z == 0. Formulas: dbl-2009-l, add-2007-bl, madd-2007-bl
// (Explicit-Formulas Database), with the exceptional cases (P == Q, P == -Q) branched: they
// never occur in the verification data flow except adversarially, so the branch is wave-uniform
// in practice and costs nothing when not taken.
//
// Replaces kilic/bls12-381 v0.1.0 g1.go / g2.go (PointG1/PointG2 Add, Double, MulScalar) as used
// through kyber-bls12381 v0.2.5 behind /root/reference/crypto/schemes.go:98,139,177.
#pragma once
#include "fp2.hpp"

namespace dh {

// ---- overload set so the point code below is written once for fp and fp2
DH_DEV fp f_add(const fp& a, const fp& b) { return fp_add(a, b); }
// sum that only feeds a product: unreduced (< 2p) over Fp, where the product is one Montgomery multiplication;
// reduced over Fp2, whose product adds and subtracts its operands' coordinates first (they must be < p there)
DH_DEV fp f_add_nr(const fp& a, const fp& b) { return fp_add_nr(a, b); }
DH_DEV fp f_sub(const fp& a, const fp& b) { return fp_sub(a, b); }
DH_DEV fp f_dbl(const fp& a) { return fp_dbl(a); }
DH_DEV fp f_neg(const fp& a) { return fp_neg(a); }
DH_DEV fp f_mul(const fp& a, const fp& b) { return fp_mul(a, b); }
DH_DEV fp f_sqr(const fp& a) { return fp_sqr(a); }
DH_DEV bool f_is_zero(const fp& a) { return fp_is_zero(a); }
DH_DEV bool f_eq(const fp& a, const fp& b) { return fp_eq(a, b); }
DH_DEV fp f_select(bool c, const fp& a, const fp& b) { return fp_select(c, a, b); }
DH_DEV void f_set_zero(fp& a) { a = fp_zero(); }
DH_DEV void f_set_one(fp& a) { a = fp_one(); }
DH_DEV fp f_inv(const fp& a) { return fp_inv(a); }
DH_DEV fp f_inv_vt(const fp& a) { return fp_inv_vt(a); }

DH_DEV fp2 f_add(const fp2& a, const fp2& b) { return fp2_add(a, b); }
DH_DEV fp2 f_add_nr(const fp2& a, const fp2& b) { return fp2_add(a, b); }
DH_DEV fp2 f_sub(const fp2& a, const fp2& b) { return fp2_sub(a, b); }
DH_DEV fp2 f_dbl(const fp2& a) { return fp2_dbl(a); }
DH_DEV fp2 f_neg(const fp2& a) { return fp2_neg(a); }
DH_DEV fp2 f_mul(const fp2& a, const fp2& b) { return fp2_mul(a, b); }
DH_DEV fp2 f_sqr(const fp2& a) { return fp2_sqr(a); }
DH_DEV bool f_is_zero(const fp2& a) { return fp2_is_zero(a); }
DH_DEV bool f_eq(const fp2& a, const fp2& b) { return fp2_eq(a, b); }
DH_DEV fp2 f_select(bool c, const fp2& a, const fp2& b) { return fp2_select(c, a, b); }
DH_DEV void f_set_zero(fp2& a) { a = fp2_zero(); }
DH_DEV void f_set_one(fp2& a) { a = fp2_one(); }
DH_DEV fp2 f_inv(const fp2& a) { return fp2_inv(a); }
DH_DEV fp2 f_inv_vt(const fp2& a) { return fp2_inv_vt(a); }

template <class F>
struct jac {
  F x, y, z;
};
template <class F>
struct aff {
  F x, y;
};

template <class F>
DH_DEV jac<F> jac_inf() {
  jac<F> r;
  f_set_one(r.x);
  f_set_one(r.y);
  f_set_zero(r.z);
  return r;
}
template <class F>
DH_DEV bool jac_is_inf(const jac<F>& p) { return f_is_zero(p.z); }

template <class F>
DH_DEV jac<F> jac_from_aff(const aff<F>& a) {
  jac<F> r;
  r.x = a.x;
  r.y = a.y;
  f_set_one(r.z);
  return r;
}

template <class F>
DH_DEV jac<F> jac_neg(const jac<F>& p) {
  return {p.x, f_neg(p.y), p.z};
}

// dbl-2009-l: 2M + 5S
template <class F>
DH_DEV jac<F> jac_dbl(const jac<F>& p) {
  F a = f_sqr(p.x);
  F b = f_sqr(p.y);
  F c = f_sqr(b);
  F d = f_sub(f_sub(f_sqr(f_add_nr(p.x, b)), a), c);
  d = f_dbl(d);
  F e = f_add_nr(f_dbl(a), a);  // 3a < 2p: only ever a product operand below
  F f = f_sqr(e);
  jac<F> r;
  r.x = f_sub(f, f_dbl(d));
  F c8 = f_dbl(f_dbl(f_dbl(c)));
  r.y = f_sub(f_mul(e, f_sub(d, r.x)), c8);
  r.z = f_dbl(f_mul(p.y, p.z));
  return r;  // z == 0 propagates infinity
}

// add-2007-bl: 11M + 5S, full special-case handling
template <class F>
DH_DEV jac<F> jac_add(const jac<F>& p, const jac<F>& q) {
  if (jac_is_inf(p)) return q;
  if (jac_is_inf(q)) return p;
  F z1z1 = f_sqr(p.z);
  F z2z2 = f_sqr(q.z);
  F u1 = f_mul(p.x, z2z2);
  F u2 = f_mul(q.x, z1z1);
  F s1 = f_mul(f_mul(p.y, q.z), z2z2);
  F s2 = f_mul(f_mul(q.y, p.z), z1z1);
  F h = f_sub(u2, u1);
  F rr = f_sub(s2, s1);
  if (f_is_zero(h)) {
    if (f_is_zero(rr)) return jac_dbl(p);
    return jac_inf<F>();
  }
  F i = f_sqr(f_dbl(h));
  F j = f_mul(h, i);
  rr = f_dbl(rr);
  F v = f_mul(u1, i);
  jac<F> r;
  r.x = f_sub(f_sub(f_sqr(rr), j), f_dbl(v));
  r.y = f_sub(f_mul(rr, f_sub(v, r.x)), f_dbl(f_mul(s1, j)));
  r.z = f_mul(f_sub(f_sub(f_sqr(f_add(p.z, q.z)), z1z1), z2z2), h);
  return r;
}

// madd-2007-bl (q affine, z2 = 1): 7M + 4S
template <class F>
DH_DEV jac<F> jac_add_aff(const jac<F>& p, const aff<F>& q) {
  if (jac_is_inf(p)) return jac_from_aff(q);
  F z1z1 = f_sqr(p.z);
  F u2 = f_mul(q.x, z1z1);
  F s2 = f_mul(f_mul(q.y, p.z), z1z1);
  F h = f_sub(u2, p.x);
  F rr = f_sub(s2, p.y);
  if (f_is_zero(h)) {
    if (f_is_zero(rr)) return jac_dbl(p);
    return jac_inf<F>();
  }
  F hh = f_sqr(h);
  F i = f_dbl(f_dbl(hh));
  F j = f_mul(h, i);
  rr = f_dbl(rr);
  F v = f_mul(p.x, i);
  jac<F> r;
  r.x = f_sub(f_sub(f_sqr(rr), j), f_dbl(v));
  r.y = f_sub(f_mul(rr, f_sub(v, r.x)), f_dbl(f_mul(p.y, j)));
  r.z = f_sub(f_sub(f_sqr(f_add(p.z, h)), z1z1), hh);
  return r;
}

// projective equality without normalisation
template <class F>
DH_DEV bool jac_eq(const jac<F>& a, const jac<F>& b) {
  bool ia = jac_is_inf(a), ib = jac_is_inf(b);
  if (ia || ib) return ia && ib;
  F z1 = f_sqr(a.z), z2 = f_sqr(b.z);
  if (!f_eq(f_mul(a.x, z2), f_mul(b.x, z1))) return false;
  return f_eq(f_mul(a.y, f_mul(z2, b.z)), f_mul(b.y, f_mul(z1, a.z)));
}

// [k] P for a public (wave-uniform) little-endian word scalar, MSB first
template <class F>
DH_DEV jac<F> jac_mul_words(const jac<F>& p, const uint32_t* k, int nbits) {
  jac<F> acc = jac_inf<F>();
  for (int b = nbits - 1; b >= 0; b--) {
    acc = jac_dbl(acc);
    if ((k[b >> 5] >> (b & 31)) & 1) acc = jac_add(acc, p);
  }
  return acc;
}

// [|u|] P, |u| = 0xd201000000010000 (bits 63,62,60,57,48,16): affine base, madd steps
template <class F>
DH_DEV jac<F> jac_mul_uabs(const aff<F>& p) {
  jac<F> acc = jac_from_aff(p);
  // remaining bits after the top one, MSB first
#pragma unroll 1
  for (int b = 62; b >= 0; b--) {
    acc = jac_dbl(acc);
    if ((cst::U_ABS >> b) & 1) acc = jac_add_aff(acc, p);
  }
  return acc;
}
template <class F>
DH_DEV jac<F> jac_mul_uabs_j(const jac<F>& p) {
  jac<F> acc = p;
#pragma unroll 1
  for (int b = 62; b >= 0; b--) {
    acc = jac_dbl(acc);
    if ((cst::U_ABS >> b) & 1) acc = jac_add(acc, p);
  }
  return acc;
}

template <class F>
DH_DEV aff<F> jac_to_aff(const jac<F>& p) {
  F zi = f_inv(p.z);
  F zi2 = f_sqr(zi);
  return {f_mul(p.x, zi2), f_mul(p.y, f_mul(zi2, zi))};
}
// the same for PUBLIC points (verification side: variable-time inversion)
template <class F>
DH_DEV aff<F> jac_to_aff_vt(const jac<F>& p) {
  F zi = f_inv_vt(p.z);
  F zi2 = f_sqr(zi);
  return {f_mul(p.x, zi2), f_mul(p.y, f_mul(zi2, zi))};
}

// ---- SoA global-memory layout: limb k of element i of an array of n elements at k*n + i
// (coalesced across lanes). Fp = 12 limbs, Fp2 = 24 limbs (c0 limbs then c1 limbs).
DH_DEV void ld(fp& a, const uint32_t* base, size_t n, size_t i) {
#pragma unroll
  for (int k = 0; k < 12; k++) a.v[k] = base[k * n + i];
}
DH_DEV void st(uint32_t* base, size_t n, size_t i, const fp& a) {
#pragma unroll
  for (int k = 0; k < 12; k++) base[k * n + i] = a.v[k];
}
DH_DEV void ld(fp2& a, const uint32_t* base, size_t n, size_t i) {
  ld(a.c0, base, n, i);
  ld(a.c1, base + 12 * n, n, i);
}
DH_DEV void st(uint32_t* base, size_t n, size_t i, const fp2& a) {
  st(base, n, i, a.c0);
  st(base + 12 * n, n, i, a.c1);
}
template <class F>
struct limbs_of;
template <>
struct limbs_of<fp> {
  static constexpr int N = 12;
};
template <>
struct limbs_of<fp2> {
  static constexpr int N = 24;
};

// a point array: x, y, z each an SoA block of limbs_of<F>::N * n words
template <class F>
DH_DEV void ld_jac(jac<F>& p, const uint32_t* base, size_t n, size_t i) {
  constexpr int L = limbs_of<F>::N;
  ld(p.x, base, n, i);
  ld(p.y, base + L * n, n, i);
  ld(p.z, base + 2 * L * n, n, i);
}
template <class F>
DH_DEV void st_jac(uint32_t* base, size_t n, size_t i, const jac<F>& p) {
  constexpr int L = limbs_of<F>::N;
  st(base, n, i, p.x);
  st(base + L * n, n, i, p.y);
  st(base + 2 * L * n, n, i, p.z);
}
template <class F>
DH_DEV void ld_aff(aff<F>& p, const uint32_t* base, size_t n, size_t i) {
  constexpr int L = limbs_of<F>::N;
  ld(p.x, base, n, i);
  ld(p.y, base + L * n, n, i);
}
template <class F>
DH_DEV void st_aff(uint32_t* base, size_t n, size_t i, const aff<F>& p) {
  constexpr int L = limbs_of<F>::N;
  st(base, n, i, p.x);
  st(base + L * n, n, i, p.y);
}

}  // namespace dh
