// Fp2 = Fp[i]/(i^2 + 1) on gfx950 (per-lane, 24 VGPRs per element).
// Replaces kilic/bls12-381 v0.1.0 fp2.go as used for G2 signatures / keys
// (/root/reference/crypto/schemes.go:99-101,140-142,178-180).
#pragma once
#include "fp.hpp"

namespace dh {

struct fp2 {
  fp c0, c1;
};

DH_DEV fp2 fp2_zero() { return {fp_zero(), fp_zero()}; }
DH_DEV fp2 fp2_one() { return {fp_one(), fp_zero()}; }
DH_DEV fp2 fp2_c(const uint32_t (*c)[12]) { return {fp_c(c[0]), fp_c(c[1])}; }
DH_DEV fp2 fp2_add(const fp2& a, const fp2& b) { return {fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; }
DH_DEV fp2 fp2_sub(const fp2& a, const fp2& b) { return {fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; }
DH_DEV fp2 fp2_dbl(const fp2& a) { return {fp_dbl(a.c0), fp_dbl(a.c1)}; }
DH_DEV fp2 fp2_neg(const fp2& a) { return {fp_neg(a.c0), fp_neg(a.c1)}; }
DH_DEV fp2 fp2_conj(const fp2& a) { return {a.c0, fp_neg(a.c1)}; }

// Karatsuba: 3 Fp products
DH_DEV fp2 fp2_mul(const fp2& a, const fp2& b) {
  fp t0 = fp_mul(a.c0, b.c0);
  fp t1 = fp_mul(a.c1, b.c1);
  fp t2 = fp_mul(fp_add_nr(a.c0, a.c1), fp_add_nr(b.c0, b.c1));  // unreduced sums < 2p feed the product
  return {fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
}

// complex squaring: 2 Fp products (operand coordinates must be canonical, < p: they are added / subtracted here)
DH_DEV fp2 fp2_sqr(const fp2& a) {
  fp t0 = fp_mul(fp_add_nr(a.c0, a.c1), fp_sub(a.c0, a.c1));
  fp t1 = fp_mul(fp_add_nr(a.c0, a.c0), a.c1);  // 2 a0 a1 with the doubling folded into the operand
  return {t0, t1};
}


DH_DEV fp2 fp2_mul_fp(const fp2& a, const fp& b) { return {fp_mul(a.c0, b), fp_mul(a.c1, b)}; }

// multiply by the Fp6 non-residue xi = 1 + i
DH_DEV fp2 fp2_mul_xi(const fp2& a) { return {fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)}; }

DH_DEV bool fp2_is_zero(const fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
DH_DEV bool fp2_eq(const fp2& a, const fp2& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
DH_DEV fp2 fp2_select(bool c, const fp2& a, const fp2& b) { return {fp_select(c, a.c0, b.c0), fp_select(c, a.c1, b.c1)}; }

DH_DEV fp2 fp2_inv(const fp2& a) {
  fp n = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  fp ni = fp_inv(n);
  return {fp_mul(a.c0, ni), fp_neg(fp_mul(a.c1, ni))};
}

// variable time, public inputs only (fp_inv_vt)
DH_DEV fp2 fp2_inv_vt(const fp2& a) {
  fp n = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  fp ni = fp_inv_vt(n);
  return {fp_mul(a.c0, ni), fp_neg(fp_mul(a.c1, ni))};
}

DH_DEV fp2 fp2_pow_words(const fp2& x, const uint32_t* e, int nbits) {
  fp2 acc = x;
  for (int b = nbits - 2; b >= 0; b--) {
    acc = fp2_sqr(acc);
    if ((e[b >> 5] >> (b & 31)) & 1) acc = fp2_mul(acc, x);
  }
  return acc;
}

DH_DEV fp2 fp2_pow_small(const fp2& x, uint32_t e) {
  fp2 acc = fp2_one();
  for (int b = 31; b >= 0; b--) {
    acc = fp2_sqr(acc);
    if ((e >> b) & 1) acc = fp2_mul(acc, x);
  }
  return acc;
}

// x^e for a fixed exponent given as a sliding-window schedule (w = 3, see fp_pow_sched)
DH_DEV fp2 fp2_pow_sched(const fp2& x, const uint32_t* sched, int len) {
  const fp2 x2 = fp2_sqr(x);
  const fp2 t1 = fp2_mul(x, x2);
  const fp2 t2 = fp2_mul(t1, x2);
  const fp2 t3 = fp2_mul(t2, x2);
  auto pick = [&](uint32_t k) { return k == 0 ? x : (k == 1 ? t1 : (k == 2 ? t2 : t3)); };
  fp2 acc = pick(sched[0]);
  uint32_t next = sched[1];  // the tables end with a 0 entry: the read one step ahead stays in bounds
#pragma unroll 1
  for (int i = 1; i < len; i++) {
    const uint32_t op = next;
    next = sched[i + 1];  // scalar load issued a whole step before its use
    const uint32_t nsq = op >> 8, k = op & 0xff;
#pragma unroll 1
    for (uint32_t j = 0; j < nsq; j++) acc = fp2_sqr(acc);
    if (k != 0xff) acc = fp2_mul(acc, pick(k));
  }
  return acc;
}

// RFC 9380 sgn0 for Fp2
DH_DEV uint32_t fp2_sgn0(const fp2& a) {
  fp c0 = fp_from_mont(a.c0), c1 = fp_from_mont(a.c1);
  uint32_t s0 = c0.v[0] & 1, s1 = c1.v[0] & 1;
  uint32_t z0 = fp_is_zero(c0) ? 1u : 0u;
  return s0 | (z0 & s1);
}

// RFC 9380 Appendix F.2.1.1 sqrt_ratio (generic, here c1 = 3 for q = p^2).
// Returns isQR; y = sqrt(u/v) if QR else sqrt(Z*u/v).
DH_DEV bool fp2_sqrt_ratio(fp2& y, const fp2& u, const fp2& v) {
  fp2 tv1 = fp2_c(cst::SQRT_RATIO2_C6);
  fp2 tv2 = fp2_pow_small(v, cst::SR2_C4);
  fp2 tv3 = fp2_mul(fp2_sqr(tv2), v);
  fp2 tv5 = fp2_mul(u, tv3);
  tv5 = fp2_pow_sched(tv5, cst::SCHED_SR2_C3, cst::SCHED_SR2_C3_LEN);
  tv5 = fp2_mul(tv5, tv2);
  tv2 = fp2_mul(tv5, v);
  tv3 = fp2_mul(tv5, u);
  fp2 tv4 = fp2_mul(tv3, tv2);
  tv5 = fp2_pow_small(tv4, cst::SR2_C5);
  bool isQR = fp2_eq(tv5, fp2_one());
  tv2 = fp2_mul(tv3, fp2_c(cst::SQRT_RATIO2_C7));
  tv5 = fp2_mul(tv4, tv1);
  tv3 = fp2_select(isQR, tv3, tv2);
  tv4 = fp2_select(isQR, tv4, tv5);
#pragma unroll
  for (int i = cst::SR2_C1; i >= 2; i--) {
    tv5 = tv4;
    for (int k = 0; k < i - 2; k++) tv5 = fp2_sqr(tv5);
    bool e1 = fp2_eq(tv5, fp2_one());
    tv2 = fp2_mul(tv3, tv1);
    tv1 = fp2_sqr(tv1);
    tv5 = fp2_mul(tv4, tv1);
    tv3 = fp2_select(e1, tv3, tv2);
    tv4 = fp2_select(e1, tv4, tv5);
  }
  y = tv3;
  return isQR;
}

// The same sqrt_ratio contract with two Fp exponentiations instead of one Fp2 exponentiation (~4.3 Fp-exponent
// equivalents): with n = N(v), u/v = W / n^2 for W = u conj(v) n, so sqrt(u/v) = sqrt(W) / n. W is a square
// iff alpha = N(W) is a square in Fp (alpha^k, k = (p-3)/4, gives Legendre and sqrt(alpha)); otherwise Z W is
// (N(Z W) = N(Z) alpha: the same exponentiation times the constant N(Z)^k). The complex method then needs
// delta = (W0 + sqrt(alpha)) / 2 and delta^k; exponentiating delta n^4 instead yields delta^k n^-2 (Fermat),
// which folds the division by n in. If delta is not a square, sqrt(-delta) gives the root (p = 3 mod 4).
// Any square root is returned (SSWU fixes the sign with sgn0 afterwards), so the output point is identical.
DH_DEV bool fp2_sqrt_ratio_cm(fp2& y, const fp2& u, const fp2& v) {
  const fp one = fp_one();
  const fp n = fp_add(fp_sqr(v.c0), fp_sqr(v.c1));
  fp2 W = fp2_mul(u, fp2_conj(v));
  W = {fp_mul(W.c0, n), fp_mul(W.c1, n)};
  fp alpha = fp_add(fp_sqr(W.c0), fp_sqr(W.c1));
  fp e = fp_pow_sched(alpha, cst::SCHED_SR1_C1, cst::SCHED_SR1_C1_LEN);
  const bool sq = fp_is_zero(alpha) || fp_eq(fp_mul(fp_sqr(e), alpha), one);
  const fp2 ZW = fp2_mul(fp2_c(cst::SSWU2_Z), W);
  W = fp2_select(sq, W, ZW);
  alpha = fp_select(sq, alpha, fp_mul(alpha, fp_c(cst::SSWU2_NZ)));
  e = fp_select(sq, e, fp_mul(e, fp_c(cst::SSWU2_NZ_K)));
  const fp lam = fp_mul(e, alpha);  // sqrt(alpha)
  fp delta = fp_mul(fp_add(W.c0, lam), fp_c(cst::INV2));
  delta = fp_select(fp_is_zero(delta), W.c0, delta);  // only when W1 = 0: then W0 itself
  const fp n4 = fp_sqr(fp_sqr(n));
  const fp tp = fp_pow_sched(fp_mul(delta, n4), cst::SCHED_SR1_C1, cst::SCHED_SR1_C1_LEN);  // delta^k n^-2
  const bool dsq = fp_eq(fp_mul(fp_mul(fp_sqr(tp), n4), delta), one);
  const fp tn = fp_mul(tp, n);
  const fp a = fp_mul(tn, delta);                           // sqrt(delta) / n
  const fp b = fp_mul(fp_mul(W.c1, tn), fp_c(cst::INV2));  // W1 / (2 sqrt(delta)) / n
  // delta not a square: x1 = -sigma t delta, x0 = sigma W1 t / 2 (sigma = (-1)^k)
  const fp nb = cst::SIGMA_K_NEG ? fp_neg(b) : b;
  const fp na = cst::SIGMA_K_NEG ? a : fp_neg(a);
  y.c0 = fp_select(dsq, a, nb);
  y.c1 = fp_select(dsq, b, na);
  return sq;
}

// square root in Fp2 (any root); false if a is not a square. "Complex" method for p = 3 mod 4 with two
// Fp exponentiations (k = (p-3)/4) and no data-dependent branch:
//   g = sqrt(a0^2 + a1^2); d = (a0 + g) / 2; t = d^k; s = t d = d^((p+1)/4); s t = (d | p) (Legendre)
//   1 / s = +-t, so a1 / 2s = +-a1 t / 2 without an inversion;
//   if d is a residue: (x0, x1) = (s, a1 / 2s)   else (s^2 = -d): (x0, x1) = (a1 / 2s, s)
// a1 == 0 is handled directly (sqrt(a0) or i sqrt(-a0)). The result is checked by squaring.
DH_DEV bool fp2_sqrt(fp2& r, const fp2& a) {
  if (fp_is_zero(a.c1)) {
    fp s0, s1;
    bool q0 = fp_sqrt(s0, a.c0);
    bool q1 = fp_sqrt(s1, fp_neg(a.c0));
    r = q0 ? fp2{s0, fp_zero()} : fp2{fp_zero(), s1};
    return q0 || q1;
  }
  fp g;
  fp_sqrt(g, fp_add(fp_sqr(a.c0), fp_sqr(a.c1)));  // a non-square norm shows up in the final check
  fp d = fp_add(a.c0, g);
  d = fp_is_zero(d) ? fp_sub(a.c0, g) : d;
  d = fp_mul(d, fp_c(cst::INV2));
  const fp t = fp_pow_sched(d, cst::SCHED_SR1_C1, cst::SCHED_SR1_C1_LEN);
  const fp s = fp_mul(t, d);
  const bool qr = fp_eq(fp_mul(s, t), fp_one());
  fp h = fp_mul(fp_mul(a.c1, t), fp_c(cst::INV2));  // a1 t / 2 = +-a1 / 2s
  h = qr ? h : fp_neg(h);
  r = qr ? fp2{s, h} : fp2{h, s};
  return fp2_eq(fp2_sqr(r), a);
}

}  // namespace dh
