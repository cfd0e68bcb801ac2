// RFC 9380 hash_to_curve (BLS12381G1_XMD:SHA-256_SSWU_RO_ and BLS12381G2_XMD:SHA-256_SSWU_RO_), per lane.
// Replaces kilic/bls12-381 v0.1.0 HashToCurve (hash_to_field, swu.go, isogeny.go) used by kyber-bls12381
// v0.2.5 for every drand scheme (/root/reference/crypto/schemes.go:98-104,139-145,177-185).
//
// Deviation from the textbook pipeline, for speed, with identical results:
//  * SSWU's final division x = X / tv4 is not performed; the isogeny is evaluated on the projective x
//    (homogeneous Horner), so no field inversion is spent per map_to_curve.
//  * clear_cofactor is NOT applied per round. It is a group homomorphism, so the batch kernels apply it
//    once to the random linear combination sum_i r_i Q_i (see kernels.hip). The per-round path
//    (bisection leaves, single verify) applies it explicitly with h2c_clear_g1 / h2c_clear_g2.
#pragma once
#include "curve.hpp"
#include "sha256.hpp"
#include "fp28.hpp"

namespace dh {

// OS2IP(64 big-endian bytes given as two 8-word digests) mod p, in Montgomery form.
DH_DEV fp fp_from_be512(const uint32_t hi[8], const uint32_t lo[8]) {
  fp h, l;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    h.v[k] = hi[7 - k];
    l.v[k] = lo[7 - k];
  }
#pragma unroll
  for (int k = 8; k < 12; k++) h.v[k] = l.v[k] = 0;
  return fp_add(fp_mul(h, fp_c(cst::K256R)), fp_mul(l, fp_c(cst::R2)));
}

// ---------------------------------------------------------------- G1: SSWU on E1' (A', B', Z = 11)
// RFC 9380 F.2.1.2 sqrt_ratio for q = 3 mod 4: returns isQR, y = sqrt(u/v) or sqrt(Z u / v)
DH_DEV bool fp_sqrt_ratio(fp& y, const fp& u, const fp& v) {
  fp tv1 = fp_sqr(v);
  fp tv2 = fp_mul(u, v);
  tv1 = fp_mul(tv1, tv2);
  fp y1 = fp_pow_sched(tv1, cst::SCHED_SR1_C1, cst::SCHED_SR1_C1_LEN);
  y1 = fp_mul(y1, tv2);
  fp y2 = fp_mul(y1, fp_c(cst::SQRT_RATIO1_C2));
  fp tv3 = fp_mul(fp_sqr(y1), v);
  bool qr = fp_eq(tv3, u);
  y = fp_select(qr, y1, y2);
  return qr;
}

// map_to_curve_simple_swu (RFC 9380 6.6.2 straight-line), output x = xn / xd, y affine
template <class F>
struct swu_out {
  F xn, xd, y;
};

DH_DEV swu_out<fp> sswu_g1(const fp& u) {
  const fp A = fp_c(cst::SSWU1_A), B = fp_c(cst::SSWU1_B), Z = fp_c(cst::SSWU1_Z);
  fp tv1 = fp_mul(Z, fp_sqr(u));
  fp tv2 = fp_add(fp_sqr(tv1), tv1);
  fp tv3 = fp_mul(B, fp_add(tv2, fp_one()));
  fp tv4 = fp_mul(A, fp_select(fp_is_zero(tv2), Z, fp_neg(tv2)));
  fp t2 = fp_sqr(tv3);
  fp tv6 = fp_sqr(tv4);
  t2 = fp_add(t2, fp_mul(A, tv6));
  t2 = fp_mul(t2, tv3);
  tv6 = fp_mul(tv6, tv4);
  t2 = fp_add(t2, fp_mul(B, tv6));
  fp x = fp_mul(tv1, tv3);
  fp y1;
  bool gx1_sq = fp_sqrt_ratio(y1, t2, tv6);
  fp y = fp_mul(fp_mul(tv1, u), y1);
  x = fp_select(gx1_sq, tv3, x);
  y = fp_select(gx1_sq, y1, y);
  bool e1 = fp_sgn0(u) == fp_sgn0(y);
  y = fp_select(e1, y, fp_neg(y));
  return {x, tv4, y};
}

// 11-isogeny E1' -> E1 (RFC 9380 E.2) on a Jacobian point of E1' (x = X/Z^2, y = Y/Z^3), Jacobian output,
// Z' = 0 if a denominator vanishes (the point is in the isogeny's kernel: its image is the identity).
// Homogeneous Horner in x = X / D with D = Z^2: acc_d = acc_d * X + c_{d-j} * D^j, j = 1..deg.
// Evaluated on lazily reduced 28-bit limbs (fp28.hpp): the ~120 products skip the 12 <-> 14 limb slicing and the
// Horner sums skip their reductions (every accumulator stays < 4p, a product input up to ~50p); three conversion
// products in (X, Y, Z) and three out.
DH_DEV jac<fp> iso11_jac(const jac<fp>& p) {
  using namespace cst;
  const f28 X = f28_from_fp(p.x), Zp = f28_from_fp(p.z);
  const f28 D = f28_sqr(Zp);                                            // < 2
  f28 xn = f28_c(ISO11_XNUM_28[ISO11_XNUM_LEN - 1]);
  f28 xd = f28_c(ISO11_XDEN_28[ISO11_XDEN_LEN - 1]);
  f28 yn = f28_c(ISO11_YNUM_28[ISO11_YNUM_LEN - 1]);
  f28 yd = f28_c(ISO11_YDEN_28[ISO11_YDEN_LEN - 1]);
  f28 zp = D;
#pragma unroll 1
  for (int j = 1; j < ISO11_YNUM_LEN; j++) {
    if (j > 1) zp = f28_mul(zp, D);                                     // < 2
    yn = f28_add(f28_mul(yn, X), f28_mul(f28_c(ISO11_YNUM_28[ISO11_YNUM_LEN - 1 - j]), zp));  // < 4
    yd = f28_add(f28_mul(yd, X), f28_mul(f28_c(ISO11_YDEN_28[ISO11_YDEN_LEN - 1 - j]), zp));
    if (j < ISO11_XNUM_LEN) xn = f28_add(f28_mul(xn, X), f28_mul(f28_c(ISO11_XNUM_28[ISO11_XNUM_LEN - 1 - j]), zp));
    if (j < ISO11_XDEN_LEN) xd = f28_add(f28_mul(xd, X), f28_mul(f28_c(ISO11_XDEN_28[ISO11_XDEN_LEN - 1 - j]), zp));
  }
  // x' = xn / (xd D) = Nx / a, y' = (Y / Z^3) yn / yd = Ny / (Z^3 yd)   (deg xn = deg xd + 1, deg yn = deg yd)
  // Z' = a yd Z^3, X' = Nx yd Z^3 Z', Y' = Y yn a Z'^2
  const f28 a = f28_mul(xd, D);
  const f28 z3 = f28_mul(D, Zp);
  const f28 ydz3 = f28_mul(yd, z3);
  const f28 rz = f28_mul(a, ydz3);
  jac<fp> r;
  r.z = f28_to_fp(rz);
  r.x = f28_to_fp(f28_mul(f28_mul(xn, ydz3), rz));
  r.y = f28_to_fp(f28_mul(f28_mul(f28_mul(f28_from_fp(p.y), yn), a), f28_sqr(rz)));
  return r;
}

// SSWU output (x = xn / xd, y affine) as a Jacobian point of E': Z = xd, X = xn xd, Y = y xd^3
template <class F>
DH_DEV jac<F> swu_jac(const swu_out<F>& s) {
  jac<F> r;
  r.z = s.xd;
  r.x = f_mul(s.xn, s.xd);
  r.y = f_mul(s.y, f_mul(f_sqr(s.xd), s.xd));
  return r;
}

// add-2007-bl on Jacobian points (the addition law does not involve the curve's a, so it holds on E1' with
// A' != 0). Returns false, leaving r unset, when x0 == x1 (P == Q or P == -Q): the caller takes the
// exceptional path. Neither input may be the identity (SSWU outputs never are: xd = tv4 != 0).
template <class F>
DH_DEV bool jac_add_distinct(jac<F>& r, const jac<F>& p, const jac<F>& q) {
  F z1z1 = f_sqr(p.z);
  F z2z2 = f_sqr(q.z);
  F u1 = f_mul(p.x, z2z2);
  F u2 = f_mul(q.x, z1z1);
  F s1 = f_mul(f_mul(p.y, q.z), z2z2);
  F s2 = f_mul(f_mul(q.y, p.z), z1z1);
  F h = f_sub(u2, u1);
  if (f_is_zero(h)) return false;
  F rr = f_dbl(f_sub(s2, s1));
  F i = f_sqr(f_dbl(h));
  F j = f_mul(h, i);
  F v = f_mul(u1, i);
  r.x = f_sub(f_sub(f_sqr(rr), j), f_dbl(v));
  r.y = f_sub(f_mul(rr, f_sub(v, r.x)), f_dbl(f_mul(s1, j)));
  r.z = f_mul(f_sub(f_sub(f_sqr(f_add(p.z, q.z)), z1z1), z2z2), h);
  return true;
}

// hash_to_curve(G1) without clear_cofactor: Q = iso(swu(u0)) + iso(swu(u1)).
// The isogeny is a group homomorphism, so Q = iso(swu(u0) + swu(u1)): the two SSWU points are added on E1'
// and ONE isogeny is evaluated (~117 products saved per round). Same point, same bytes. When the two SSWU
// points share x (never for honest inputs) the textbook order is used: two isogenies, addition on E1.
// map_to_curve of two field elements, summed (hash_to_curve minus the hashing and the cofactor clearing)
DH_DEV jac<fp> h2c_g1_map(const fp& u0, const fp& u1) {
  const jac<fp> p0 = swu_jac(sswu_g1(u0));
  const jac<fp> p1 = swu_jac(sswu_g1(u1));
  jac<fp> s;
  if (jac_add_distinct(s, p0, p1)) return iso11_jac(s);
  return jac_add(iso11_jac(p0), iso11_jac(p1));
}

DH_DEV jac<fp> h2c_g1_noclear(const sha_h& digest, int dst_id) {
  uint32_t b[4][8];
  xmd32<4>(b, digest, dst_id);
  return h2c_g1_map(fp_from_be512(b[0], b[1]), fp_from_be512(b[2], b[3]));
}

// clear_cofactor(G1) = [h_eff] P, h_eff = 1 - u = 0xd201000000010001 = |u| + 1
DH_DEV jac<fp> h2c_clear_g1(const jac<fp>& p) { return jac_add(jac_mul_uabs_j(p), p); }

// ---------------------------------------------------------------- G2: SSWU on E2' (A' = 240i, B' = 1012(1+i), Z = -(2+i))
DH_DEV swu_out<fp2> sswu_g2(const fp2& u) {
  const fp2 A = fp2_c(cst::SSWU2_A), B = fp2_c(cst::SSWU2_B), Z = fp2_c(cst::SSWU2_Z);
  fp2 tv1 = fp2_mul(Z, fp2_sqr(u));
  fp2 tv2 = fp2_add(fp2_sqr(tv1), tv1);
  fp2 tv3 = fp2_mul(B, fp2_add(tv2, fp2_one()));
  fp2 tv4 = fp2_mul(A, fp2_select(fp2_is_zero(tv2), Z, fp2_neg(tv2)));
  fp2 t2 = fp2_sqr(tv3);
  fp2 tv6 = fp2_sqr(tv4);
  t2 = fp2_add(t2, fp2_mul(A, tv6));
  t2 = fp2_mul(t2, tv3);
  tv6 = fp2_mul(tv6, tv4);
  t2 = fp2_add(t2, fp2_mul(B, tv6));
  fp2 x = fp2_mul(tv1, tv3);
  fp2 y1;
  bool gx1_sq = fp2_sqrt_ratio_cm(y1, t2, tv6);
  fp2 y = fp2_mul(fp2_mul(tv1, u), y1);
  x = fp2_select(gx1_sq, tv3, x);
  y = fp2_select(gx1_sq, y1, y);
  bool e1 = fp2_sgn0(u) == fp2_sgn0(y);
  y = fp2_select(e1, y, fp2_neg(y));
  return {x, tv4, y};
}

// 3-isogeny E2' -> E2 (RFC 9380 E.3) on a Jacobian point of E2', same homogeneous evaluation as iso11_jac
DH_DEV jac<fp2> iso3_jac(const jac<fp2>& p) {
  using namespace cst;
  const fp2 D = fp2_sqr(p.z);
  fp2 xn = fp2_c(ISO3_XNUM[ISO3_XNUM_LEN - 1]);
  fp2 xd = fp2_c(ISO3_XDEN[ISO3_XDEN_LEN - 1]);
  fp2 yn = fp2_c(ISO3_YNUM[ISO3_YNUM_LEN - 1]);
  fp2 yd = fp2_c(ISO3_YDEN[ISO3_YDEN_LEN - 1]);
  fp2 zp = D;
#pragma unroll 1
  for (int j = 1; j < ISO3_YNUM_LEN; j++) {
    if (j > 1) zp = fp2_mul(zp, D);
    yn = fp2_add(fp2_mul(yn, p.x), fp2_mul(fp2_c(ISO3_YNUM[ISO3_YNUM_LEN - 1 - j]), zp));
    yd = fp2_add(fp2_mul(yd, p.x), fp2_mul(fp2_c(ISO3_YDEN[ISO3_YDEN_LEN - 1 - j]), zp));
    if (j < ISO3_XNUM_LEN) xn = fp2_add(fp2_mul(xn, p.x), fp2_mul(fp2_c(ISO3_XNUM[ISO3_XNUM_LEN - 1 - j]), zp));
    if (j < ISO3_XDEN_LEN) xd = fp2_add(fp2_mul(xd, p.x), fp2_mul(fp2_c(ISO3_XDEN[ISO3_XDEN_LEN - 1 - j]), zp));
  }
  const fp2 a = fp2_mul(xd, D);
  const fp2 z3 = fp2_mul(D, p.z);
  const fp2 ydz3 = fp2_mul(yd, z3);
  jac<fp2> r;
  r.z = fp2_mul(a, ydz3);
  r.x = fp2_mul(fp2_mul(xn, ydz3), r.z);
  r.y = fp2_mul(fp2_mul(fp2_mul(p.y, yn), a), fp2_sqr(r.z));
  return r;
}

// Register-lean forms for the G2 pass kernels (k_prep.hip): the same maps as iso3_jac / jac_add_distinct with
// the operations reordered so that at most ~7 Fp2 values are live at once (one lane holds ~10 in 256 VGPRs).
// Same points; the Jacobian representatives differ (Z scaled), which no consumer depends on.
//
// iso3 with the y-part first: Ny = Y yn and yd Z^3 collapse before the x-part's Horner runs.
DH_DEV jac<fp2> iso3_jac_lean(const jac<fp2>& p) {
  using namespace cst;
  const fp2 D = fp2_sqr(p.z);
  fp2 ydz3;
  fp2 ny;
  {
    fp2 yn = fp2_c(ISO3_YNUM[ISO3_YNUM_LEN - 1]);
    fp2 yd = fp2_c(ISO3_YDEN[ISO3_YDEN_LEN - 1]);
    fp2 zp = D;
#pragma unroll 1
    for (int j = 1; j < ISO3_YNUM_LEN; j++) {
      if (j > 1) zp = fp2_mul(zp, D);
      yn = fp2_add(fp2_mul(yn, p.x), fp2_mul(fp2_c(ISO3_YNUM[ISO3_YNUM_LEN - 1 - j]), zp));
      yd = fp2_add(fp2_mul(yd, p.x), fp2_mul(fp2_c(ISO3_YDEN[ISO3_YDEN_LEN - 1 - j]), zp));
    }
    ydz3 = fp2_mul(yd, fp2_mul(D, p.z));
    ny = fp2_mul(p.y, yn);
  }
  fp2 xn = fp2_c(ISO3_XNUM[ISO3_XNUM_LEN - 1]);
  fp2 xd = fp2_c(ISO3_XDEN[ISO3_XDEN_LEN - 1]);
  fp2 zp = D;
#pragma unroll 1
  for (int j = 1; j < ISO3_XNUM_LEN; j++) {
    if (j > 1) zp = fp2_mul(zp, D);
    xn = fp2_add(fp2_mul(xn, p.x), fp2_mul(fp2_c(ISO3_XNUM[ISO3_XNUM_LEN - 1 - j]), zp));
    if (j < ISO3_XDEN_LEN) xd = fp2_add(fp2_mul(xd, p.x), fp2_mul(fp2_c(ISO3_XDEN[ISO3_XDEN_LEN - 1 - j]), zp));
  }
  const fp2 a = fp2_mul(xd, D);
  jac<fp2> r;
  r.z = fp2_mul(a, ydz3);
  r.x = fp2_mul(fp2_mul(xn, ydz3), r.z);
  r.y = fp2_mul(fp2_mul(ny, a), fp2_sqr(r.z));
  return r;
}

// hash_to_curve(G2) without clear_cofactor, one isogeny after the addition on E2' (see h2c_g1_noclear)
DH_DEV jac<fp2> h2c_g2_map(const fp2& u0, const fp2& u1) {
  const jac<fp2> p0 = swu_jac(sswu_g2(u0));
  const jac<fp2> p1 = swu_jac(sswu_g2(u1));
  jac<fp2> s;
  if (jac_add_distinct(s, p0, p1)) return iso3_jac(s);
  return jac_add(iso3_jac(p0), iso3_jac(p1));
}

DH_DEV jac<fp2> h2c_g2_noclear(const sha_h& digest, int dst_id) {
  uint32_t b[8][8];
  xmd32<8>(b, digest, dst_id);
  return h2c_g2_map({fp_from_be512(b[0], b[1]), fp_from_be512(b[2], b[3])}, {fp_from_be512(b[4], b[5]), fp_from_be512(b[6], b[7])});
}

// psi (untwist-Frobenius-twist) on E2 and its square, Jacobian
DH_DEV jac<fp2> g2_psi(const jac<fp2>& p) {
  jac<fp2> r;
  r.x = fp2_mul(fp2_conj(p.x), fp2_c(cst::PSI_X));
  r.y = fp2_mul(fp2_conj(p.y), fp2_c(cst::PSI_Y));
  r.z = fp2_conj(p.z);
  return r;
}
DH_DEV jac<fp2> g2_psi2(const jac<fp2>& p) {
  return {fp2_mul(p.x, fp2_c(cst::PSI2_X)), fp2_mul(p.y, fp2_c(cst::PSI2_Y)), p.z};
}

// clear_cofactor(G2) = [h_eff] P, computed with the endomorphism method of RFC 9380 Appendix G.3
// (Budroni-Pintore): 2 x 64-bit scalar multiplications instead of one 636-bit one; same point.
DH_DEV jac<fp2> h2c_clear_g2(const jac<fp2>& p) {
  jac<fp2> t1 = jac_neg(jac_mul_uabs_j(p));      // [u] P  (u < 0)
  jac<fp2> t2 = g2_psi(p);
  jac<fp2> t3 = g2_psi2(jac_dbl(p));
  t3 = jac_add(t3, jac_neg(t2));
  t2 = jac_add(t1, t2);
  t2 = jac_neg(jac_mul_uabs_j(t2));             // [u] (t1 + t2)
  t3 = jac_add(t3, t2);
  t3 = jac_add(t3, jac_neg(t1));
  return jac_add(t3, jac_neg(p));
}

}  // namespace dh
