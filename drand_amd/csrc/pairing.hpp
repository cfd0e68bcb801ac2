// Fp6 / Fp12 tower and the optimal-ate pairing check for BLS12-381, per lane.
// Tower: Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v), xi = 1 + i (same as kilic/bls12-381).
// Replaces kilic/bls12-381 v0.1.0 Engine (AddPair / AddPairInv / Check: multi-Miller loop + final
// exponentiation) that kyber-bls12381 v0.2.5 ValidatePairing runs inside bls.Verify for every
// /root/reference/crypto/schemes.go:70-72 VerifyBeacon call.
//
// The batch path runs ONE such check per group of rounds (random-linear-combination), so these are
// latency routines: one lane per check. Miller loop lines follow Costello-Lange-Naehrig (eprint 2010/354)
// on the M-twist with homogeneous coordinates; final exponentiation uses the (p^4-p^2+1)/r hard-part
// decomposition with exponent 3 (Hayashida-Hayasaka-Teruya), cyclotomic squarings (Granger-Scott).
#pragma once
#include "curve.hpp"

namespace dh {

// the tower routines are large: keep them out of line so the kernels stay compact
#define DH_NOINL __device__ __noinline__

struct fp6 {
  fp2 c0, c1, c2;
};
struct fp12 {
  fp6 c0, c1;
};

DH_DEV fp6 fp6_add(const fp6& a, const fp6& b) { return {fp2_add(a.c0, b.c0), fp2_add(a.c1, b.c1), fp2_add(a.c2, b.c2)}; }
DH_DEV fp6 fp6_sub(const fp6& a, const fp6& b) { return {fp2_sub(a.c0, b.c0), fp2_sub(a.c1, b.c1), fp2_sub(a.c2, b.c2)}; }
DH_DEV fp6 fp6_neg(const fp6& a) { return {fp2_neg(a.c0), fp2_neg(a.c1), fp2_neg(a.c2)}; }
DH_DEV fp6 fp6_zero() { return {fp2_zero(), fp2_zero(), fp2_zero()}; }

DH_NOINL fp6 fp6_mul(const fp6& a, const fp6& b) {
  fp2 t0 = fp2_mul(a.c0, b.c0), t1 = fp2_mul(a.c1, b.c1), t2 = fp2_mul(a.c2, b.c2);
  fp2 u0 = fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c1, a.c2), fp2_add(b.c1, b.c2)), t1), t2);
  u0 = fp2_add(fp2_mul_xi(u0), t0);
  fp2 u1 = fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b.c0, b.c1)), t0), t1);
  u1 = fp2_add(u1, fp2_mul_xi(t2));
  fp2 u2 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c2), fp2_add(b.c0, b.c2)), t0), t2), t1);
  return {u0, u1, u2};
}

// a * (b0 + b1 v): sparse (b2 = 0)
DH_NOINL fp6 fp6_mul_01(const fp6& a, const fp2& b0, const fp2& b1) {
  fp2 t0 = fp2_mul(a.c0, b0), t1 = fp2_mul(a.c1, b1);
  fp2 u0 = fp2_add(fp2_mul_xi(fp2_mul(a.c2, b1)), t0);                                   // (a2 b1) xi + a0 b0
  fp2 u1 = fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b0, b1)), t0), t1);      // a0 b1 + a1 b0
  fp2 u2 = fp2_add(fp2_mul(a.c2, b0), t1);                                              // a2 b0 + a1 b1
  return {u0, u1, u2};
}
// a * (b1 v)
DH_DEV fp6 fp6_mul_1(const fp6& a, const fp2& b1) {
  return {fp2_mul_xi(fp2_mul(a.c2, b1)), fp2_mul(a.c0, b1), fp2_mul(a.c1, b1)};
}

DH_DEV fp6 fp6_mul_v(const fp6& a) { return {fp2_mul_xi(a.c2), a.c0, a.c1}; }

DH_NOINL fp6 fp6_inv(const fp6& a) {
  fp2 c0 = fp2_sub(fp2_sqr(a.c0), fp2_mul_xi(fp2_mul(a.c1, a.c2)));
  fp2 c1 = fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1));
  fp2 c2 = fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2));
  fp2 t = fp2_add(fp2_mul_xi(fp2_add(fp2_mul(a.c2, c1), fp2_mul(a.c1, c2))), fp2_mul(a.c0, c0));
  t = fp2_inv(t);
  return {fp2_mul(c0, t), fp2_mul(c1, t), fp2_mul(c2, t)};
}

DH_NOINL fp6 fp6_frob(const fp6& a, int k) {  // k in 1..3
  fp2 c0 = a.c0, c1 = a.c1, c2 = a.c2;
  if (k & 1) {
    c0 = fp2_conj(c0);
    c1 = fp2_conj(c1);
    c2 = fp2_conj(c2);
  }
  c1 = fp2_mul(c1, fp2_c(cst::FROB6_C1[k - 1]));
  c2 = fp2_mul(c2, fp2_c(cst::FROB6_C2[k - 1]));
  return {c0, c1, c2};
}

DH_DEV fp12 fp12_one() {
  fp12 r;
  r.c0 = fp6_zero();
  r.c1 = fp6_zero();
  r.c0.c0 = fp2_one();
  return r;
}

DH_NOINL fp12 fp12_mul(const fp12& a, const fp12& b) {
  fp6 t0 = fp6_mul(a.c0, b.c0), t1 = fp6_mul(a.c1, b.c1);
  fp6 s = fp6_sub(fp6_sub(fp6_mul(fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1)), t0), t1);
  return {fp6_add(t0, fp6_mul_v(t1)), s};
}

// complex squaring in Fp12 over Fp6: 2 Fp6 multiplications
DH_NOINL fp12 fp12_sqr(const fp12& a) {
  fp6 ab = fp6_mul(a.c0, a.c1);
  fp6 t = fp6_mul(fp6_add(a.c0, a.c1), fp6_add(a.c0, fp6_mul_v(a.c1)));
  fp6 c0 = fp6_sub(fp6_sub(t, ab), fp6_mul_v(ab));
  return {c0, fp6_add(ab, ab)};
}

DH_DEV fp12 fp12_conj(const fp12& a) { return {a.c0, fp6_neg(a.c1)}; }

DH_NOINL fp12 fp12_inv(const fp12& a) {
  fp6 t = fp6_sub(fp6_mul(a.c0, a.c0), fp6_mul_v(fp6_mul(a.c1, a.c1)));
  t = fp6_inv(t);
  return {fp6_mul(a.c0, t), fp6_neg(fp6_mul(a.c1, t))};
}

DH_NOINL fp12 fp12_frob(const fp12& a, int k) {
  fp6 c0 = fp6_frob(a.c0, k), c1 = fp6_frob(a.c1, k);
  const fp2 w = fp2_c(cst::FROB12_C[k - 1]);
  c1.c0 = fp2_mul(c1.c0, w);
  c1.c1 = fp2_mul(c1.c1, w);
  c1.c2 = fp2_mul(c1.c2, w);
  return {c0, c1};
}

DH_DEV bool fp12_is_one(const fp12& a) {
  fp12 one = fp12_one();
  return fp2_eq(a.c0.c0, one.c0.c0) && fp2_is_zero(a.c0.c1) && fp2_is_zero(a.c0.c2) && fp2_is_zero(a.c1.c0) &&
         fp2_is_zero(a.c1.c1) && fp2_is_zero(a.c1.c2);
}

// f *= line with coefficients at positions (c0.c0 = a, c0.c1 = b, c1.c1 = c):  l = (a + b v) + (c v) w
DH_NOINL fp12 fp12_mul_line(const fp12& f, const fp2& a, const fp2& b, const fp2& c) {
  fp6 t0 = fp6_mul_01(f.c0, a, b);
  fp6 t1 = fp6_mul_1(f.c1, c);
  fp6 s = fp6_sub(fp6_sub(fp6_mul_01(fp6_add(f.c0, f.c1), a, fp2_add(b, c)), t0), t1);
  return {fp6_add(t0, fp6_mul_v(t1)), s};
}

// ---- Miller loop steps on a homogeneous twist point T (CLN 2010/354, M-twist)
DH_NOINL void ml_dbl(jac<fp2>& r, fp2& c0, fp2& c1, fp2& c2) {
  fp2 t0 = fp2_sqr(r.x), t1 = fp2_sqr(r.y), t2 = fp2_sqr(t1);
  fp2 t3 = fp2_dbl(fp2_sub(fp2_sub(fp2_sqr(fp2_add(t1, r.x)), t0), t2));
  fp2 t4 = fp2_add(fp2_dbl(t0), t0);
  fp2 t6 = fp2_add(r.x, t4);
  fp2 t5 = fp2_sqr(t4);
  fp2 zz = fp2_sqr(r.z);
  fp2 nx = fp2_sub(fp2_sub(t5, t3), t3);
  fp2 nz = fp2_sub(fp2_sub(fp2_sqr(fp2_add(r.z, r.y)), t1), zz);
  fp2 ny = fp2_sub(fp2_mul(fp2_sub(t3, nx), t4), fp2_dbl(fp2_dbl(fp2_dbl(t2))));
  t3 = fp2_neg(fp2_dbl(fp2_mul(t4, zz)));
  t6 = fp2_sub(fp2_sub(fp2_sqr(t6), t0), t5);
  t6 = fp2_sub(t6, fp2_dbl(fp2_dbl(t1)));
  t0 = fp2_dbl(fp2_mul(nz, zz));
  r.x = nx;
  r.y = ny;
  r.z = nz;
  c0 = t0;
  c1 = t3;
  c2 = t6;
}

DH_NOINL void ml_add(jac<fp2>& r, const aff<fp2>& q, fp2& c0, fp2& c1, fp2& c2) {
  fp2 zz = fp2_sqr(r.z), yy = fp2_sqr(q.y);
  fp2 t0 = fp2_mul(zz, q.x);
  fp2 t1 = fp2_mul(fp2_sub(fp2_sub(fp2_sqr(fp2_add(q.y, r.z)), yy), zz), zz);
  fp2 t2 = fp2_sub(t0, r.x);
  fp2 t3 = fp2_sqr(t2);
  fp2 t4 = fp2_dbl(fp2_dbl(t3));
  fp2 t5 = fp2_mul(t4, t2);
  fp2 t6 = fp2_sub(fp2_sub(t1, r.y), r.y);
  fp2 t9 = fp2_mul(t6, q.x);
  fp2 t7 = fp2_mul(t4, r.x);
  fp2 nx = fp2_sub(fp2_sub(fp2_sub(fp2_sqr(t6), t5), t7), t7);
  fp2 nz = fp2_sub(fp2_sub(fp2_sqr(fp2_add(r.z, t2)), zz), t3);
  fp2 t10 = fp2_add(q.y, nz);
  fp2 t8 = fp2_mul(fp2_sub(t7, nx), t6);
  fp2 ny = fp2_sub(t8, fp2_dbl(fp2_mul(r.y, t5)));
  t10 = fp2_sub(fp2_sub(fp2_sqr(t10), yy), fp2_sqr(nz));
  t9 = fp2_sub(fp2_dbl(t9), t10);
  t10 = fp2_dbl(nz);
  t1 = fp2_dbl(fp2_neg(t6));
  r.x = nx;
  r.y = ny;
  r.z = nz;
  c0 = t10;
  c1 = t1;
  c2 = t9;
}

// multi-Miller loop over NP pairs (P_k affine G1, Q_k affine G2); skip[k] drops a pair (infinity)
template <int NP>
DH_DEV fp12 miller_loop(const aff<fp> P[NP], const aff<fp2> Q[NP], const bool skip[NP]) {
  fp12 f = fp12_one();
  jac<fp2> T[NP];
#pragma unroll
  for (int k = 0; k < NP; k++) T[k] = jac_from_aff(Q[k]);
  bool started = false;
#pragma unroll 1
  for (int b = 62; b >= 0; b--) {
    if (started) f = fp12_sqr(f);
    started = true;
#pragma unroll
    for (int k = 0; k < NP; k++) {
      if (skip[k]) continue;
      fp2 c0, c1, c2;
      ml_dbl(T[k], c0, c1, c2);
      f = fp12_mul_line(f, c2, fp2_mul_fp(c1, P[k].x), fp2_mul_fp(c0, P[k].y));
    }
    if ((cst::U_ABS >> b) & 1) {
#pragma unroll
      for (int k = 0; k < NP; k++) {
        if (skip[k]) continue;
        fp2 c0, c1, c2;
        ml_add(T[k], Q[k], c0, c1, c2);
        f = fp12_mul_line(f, c2, fp2_mul_fp(c1, P[k].x), fp2_mul_fp(c0, P[k].y));
      }
    }
  }
  return fp12_conj(f);  // u < 0
}

// Granger-Scott cyclotomic squaring (valid after the easy part of the final exponentiation)
DH_DEV void fp4_sqr(fp2& r0, fp2& r1, const fp2& a, const fp2& b) {
  fp2 t0 = fp2_sqr(a), t1 = fp2_sqr(b);
  r0 = fp2_add(fp2_mul_xi(t1), t0);
  r1 = fp2_sub(fp2_sub(fp2_sqr(fp2_add(a, b)), t0), t1);
}
DH_NOINL fp12 fp12_cyc_sqr(const fp12& a) {
  // element = (g0 + g1 v + g2 v^2) + (h0 + h1 v + h2 v^2) w ; pairs (g0,h1), (h0,g2), (g1,h2)
  fp2 t0, t1, t2, t3, t4, t5;
  fp4_sqr(t0, t1, a.c0.c0, a.c1.c1);
  fp4_sqr(t2, t3, a.c1.c0, a.c0.c2);
  fp4_sqr(t4, t5, a.c0.c1, a.c1.c2);
  fp12 r;
  // g0' = 3 t0 - 2 g0 ; h1' = 3 t1 + 2 h1
  r.c0.c0 = fp2_add(fp2_dbl(fp2_sub(t0, a.c0.c0)), t0);
  r.c1.c1 = fp2_add(fp2_dbl(fp2_add(t1, a.c1.c1)), t1);
  // h0' = 3 xi t5 + 2 h0 ; g2' = 3 t4 - 2 g2
  fp2 t5x = fp2_mul_xi(t5);
  r.c1.c0 = fp2_add(fp2_dbl(fp2_add(t5x, a.c1.c0)), t5x);
  r.c0.c2 = fp2_add(fp2_dbl(fp2_sub(t4, a.c0.c2)), t4);
  // g1' = 3 t2 - 2 g1 ; h2' = 3 t3 + 2 h2
  r.c0.c1 = fp2_add(fp2_dbl(fp2_sub(t2, a.c0.c1)), t2);
  r.c1.c2 = fp2_add(fp2_dbl(fp2_add(t3, a.c1.c2)), t3);
  return r;
}

// a^u for u = -|u| on a cyclotomic element: conj(a^|u|)
DH_NOINL fp12 cyc_exp_u(const fp12& a) {
  fp12 acc = a;
#pragma unroll 1
  for (int b = 62; b >= 0; b--) {
    acc = fp12_cyc_sqr(acc);
    if ((cst::U_ABS >> b) & 1) acc = fp12_mul(acc, a);
  }
  return fp12_conj(acc);
}

DH_NOINL fp12 final_exp(const fp12& f) {
  // easy part: f^((p^6 - 1)(p^2 + 1))
  fp12 t0 = fp12_mul(fp12_conj(f), fp12_inv(f));
  t0 = fp12_mul(t0, fp12_frob(t0, 2));
  // hard part: 3 (p^4 - p^2 + 1) / r = l0 + l1 p + l2 p^2 + l3 p^3
  //   l3 = (u - 1)^2, l2 = l3 u, l1 = l2 u - l3, l0 = l1 u + 3
  fp12 a = fp12_mul(cyc_exp_u(t0), fp12_conj(t0));  // t0^(u-1)
  fp12 b = fp12_mul(cyc_exp_u(a), fp12_conj(a));    // t0^l3
  fp12 c = cyc_exp_u(b);                            // t0^l2
  fp12 d = fp12_mul(cyc_exp_u(c), fp12_conj(b));    // t0^l1
  fp12 e = fp12_mul(cyc_exp_u(d), fp12_mul(fp12_cyc_sqr(t0), t0));  // t0^l0
  e = fp12_mul(e, fp12_frob(d, 1));
  e = fp12_mul(e, fp12_frob(c, 2));
  return fp12_mul(e, fp12_frob(b, 3));
}

// prod_k e(P_k, Q_k) == 1 ; pairs with an infinity are skipped (as kilic's engine does)
template <int NP>
DH_DEV bool pairing_check(const jac<fp> P[NP], const jac<fp2> Q[NP]) {
  aff<fp> pa[NP];
  aff<fp2> qa[NP];
  bool skip[NP];
  bool all_skip = true;
#pragma unroll
  for (int k = 0; k < NP; k++) {
    skip[k] = jac_is_inf(P[k]) || jac_is_inf(Q[k]);
    all_skip = all_skip && skip[k];
    if (!skip[k]) {
      pa[k] = jac_to_aff(P[k]);
      qa[k] = jac_to_aff(Q[k]);
    } else {
      pa[k] = {fp_zero(), fp_zero()};
      qa[k] = {fp2_zero(), fp2_zero()};
    }
  }
  if (all_skip) return true;
  return fp12_is_one(final_exp(miller_loop<NP>(pa, qa, skip)));
}

}  // namespace dh
