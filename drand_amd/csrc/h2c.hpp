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

// 11-isogeny E1' -> E1 on x = X/Z (RFC 9380 E.2), Jacobian output, Z' = 0 if a denominator vanishes.
DH_DEV jac<fp> iso11(const swu_out<fp>& s) {
  using namespace cst;
  // Horner with the powers of Z folded in: acc_d = acc_d * X + c_{d-j} * Z^j, j = 1..deg
  fp xn = fp_c(ISO11_XNUM[ISO11_XNUM_LEN - 1]);
  fp xd = fp_c(ISO11_XDEN[ISO11_XDEN_LEN - 1]);
  fp yn = fp_c(ISO11_YNUM[ISO11_YNUM_LEN - 1]);
  fp yd = fp_c(ISO11_YDEN[ISO11_YDEN_LEN - 1]);
  fp zp = s.xd;
#pragma unroll 1
  for (int j = 1; j < ISO11_YNUM_LEN; j++) {
    if (j > 1) zp = fp_mul(zp, s.xd);
    yn = fp_add(fp_mul(yn, s.xn), fp_mul(fp_c(ISO11_YNUM[ISO11_YNUM_LEN - 1 - j]), zp));
    yd = fp_add(fp_mul(yd, s.xn), fp_mul(fp_c(ISO11_YDEN[ISO11_YDEN_LEN - 1 - j]), zp));
    if (j < ISO11_XNUM_LEN) xn = fp_add(fp_mul(xn, s.xn), fp_mul(fp_c(ISO11_XNUM[ISO11_XNUM_LEN - 1 - j]), zp));
    if (j < ISO11_XDEN_LEN) xd = fp_add(fp_mul(xd, s.xn), fp_mul(fp_c(ISO11_XDEN[ISO11_XDEN_LEN - 1 - j]), zp));
  }
  // x' = xn / (xd Z), y' = y yn / yd  (deg xn = deg xd + 1, deg yn = deg yd)
  fp a = fp_mul(xd, s.xd);
  jac<fp> r;
  r.z = fp_mul(a, yd);
  r.x = fp_mul(fp_mul(xn, yd), r.z);
  r.y = fp_mul(fp_mul(fp_mul(s.y, yn), a), fp_sqr(r.z));
  return r;
}

// hash_to_curve(G1) without clear_cofactor: Q = iso(swu(u0)) + iso(swu(u1))
DH_DEV jac<fp> h2c_g1_noclear(const sha_h& digest, int dst_id) {
  uint32_t b[4][8];
  xmd32<4>(b, digest, dst_id);
  fp u0 = fp_from_be512(b[0], b[1]);
  fp u1 = fp_from_be512(b[2], b[3]);
  jac<fp> q0 = iso11(sswu_g1(u0));
  jac<fp> q1 = iso11(sswu_g1(u1));
  return jac_add(q0, q1);
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

// 3-isogeny E2' -> E2 (RFC 9380 E.3), same homogeneous evaluation as iso11
DH_DEV jac<fp2> iso3(const swu_out<fp2>& s) {
  using namespace cst;
  fp2 xn = fp2_c(ISO3_XNUM[ISO3_XNUM_LEN - 1]);
  fp2 xd = fp2_c(ISO3_XDEN[ISO3_XDEN_LEN - 1]);
  fp2 yn = fp2_c(ISO3_YNUM[ISO3_YNUM_LEN - 1]);
  fp2 yd = fp2_c(ISO3_YDEN[ISO3_YDEN_LEN - 1]);
  fp2 zp = s.xd;
#pragma unroll 1
  for (int j = 1; j < ISO3_YNUM_LEN; j++) {
    if (j > 1) zp = fp2_mul(zp, s.xd);
    yn = fp2_add(fp2_mul(yn, s.xn), fp2_mul(fp2_c(ISO3_YNUM[ISO3_YNUM_LEN - 1 - j]), zp));
    yd = fp2_add(fp2_mul(yd, s.xn), fp2_mul(fp2_c(ISO3_YDEN[ISO3_YDEN_LEN - 1 - j]), zp));
    if (j < ISO3_XNUM_LEN) xn = fp2_add(fp2_mul(xn, s.xn), fp2_mul(fp2_c(ISO3_XNUM[ISO3_XNUM_LEN - 1 - j]), zp));
    if (j < ISO3_XDEN_LEN) xd = fp2_add(fp2_mul(xd, s.xn), fp2_mul(fp2_c(ISO3_XDEN[ISO3_XDEN_LEN - 1 - j]), zp));
  }
  fp2 a = fp2_mul(xd, s.xd);
  jac<fp2> r;
  r.z = fp2_mul(a, yd);
  r.x = fp2_mul(fp2_mul(xn, yd), r.z);
  r.y = fp2_mul(fp2_mul(fp2_mul(s.y, yn), a), fp2_sqr(r.z));
  return r;
}

DH_DEV jac<fp2> h2c_g2_noclear(const sha_h& digest, int dst_id) {
  uint32_t b[8][8];
  xmd32<8>(b, digest, dst_id);
  fp2 u0 = {fp_from_be512(b[0], b[1]), fp_from_be512(b[2], b[3])};
  fp2 u1 = {fp_from_be512(b[4], b[5]), fp_from_be512(b[6], b[7])};
  jac<fp2> q0 = iso3(sswu_g2(u0));
  jac<fp2> q1 = iso3(sswu_g2(u1));
  return jac_add(q0, q1);
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
