// Lazily reduced Fp2 and G2 point arithmetic on 28-bit limbs (the G2 counterpart of fp28.hpp), for the G2
// signature subgroup test (k_sub_sig_g2) and the G2 MSM (k_msm.hip MSM28).
//
// An Fp2 element is a pair of fp28.hpp values (each an integer < K p congruent to c R', 14 normalised limbs). The
// product is Karatsuba (3 out-of-line 28-bit products), the squaring the complex method (2 products); a product
// accepts operands whose component bounds Ka, Kb (units of p) keep (Ka0 + Ka1)(Kb0 + Kb1) < 2500 and returns
// components < (4, 6), a squaring (2, 4). Sums and differences are limb-wise with one signed carry pass (a - b =
// a + K p - b), and f28_red is a cheap partial reduction to < 2p (the top three limbs as a double give q with
// q p <= a, then a - q p: ~70 VALU instead of a ~450-instruction product). Point coordinates keep X, Y < 2 (X3, Y3
// reduced at the end of every formula) and Z < 12 per component, which closes every formula below; each step's
// bound is written next to it and asserted by the integer model tests/fp2_28_model.py (tests/test_fp2_28_model.py).
// Infinity is a flag; the MSM takes the additions without exceptional-case tests and one zero test of Z per run
// (the poison argument of fp28.hpp j28_madd_fast holds verbatim over Fp2).
#pragma once
#include "fp28.hpp"
#include "fp2.hpp"

namespace dh {

// q p <= a < 2^392 with q from the top three limbs: a - q p < 2p (tests/fp2_28_model.py red)
DH_DEV f28 f28_red(const f28& a) {
  const double hi = ((double)a.l[13] * 268435456.0 + (double)a.l[12]) * 268435456.0 + (double)a.l[11];
  const uint32_t q = (uint32_t)(hi * 1.3029181615380006e-22);  // 2^308 / p * (1 - 2^-40)
  f28 r;
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    const int64_t t = (int64_t)a.l[i] - (int64_t)((uint64_t)q * m28::P[i]) + c;
    r.l[i] = (uint32_t)t & m28::MASK;
    c = t >> 28;
  }
  return r;
}

struct f228 {
  f28 c0, c1;
};

DH_DEV f228 f2_add(const f228& a, const f228& b) { return {f28_add(a.c0, b.c0), f28_add(a.c1, b.c1)}; }
DH_DEV f228 f2_scale(const f228& a, int c) { return {f28_scale(a.c0, c), f28_scale(a.c1, c)}; }
template <int K0, int K1>
DH_DEV f228 f2_lin(const f228& a, int ca, const f228& b, int cb) {
  return {f28_lin<K0>(a.c0, ca, b.c0, cb), f28_lin<K1>(a.c1, ca, b.c1, cb)};
}
template <int K0, int K1>
DH_DEV f228 f2_lin3(const f228& a, int ca, const f228& b, int cb, const f228& c, int cc) {
  return {f28_lin3<K0>(a.c0, ca, b.c0, cb, c.c0, cc), f28_lin3<K1>(a.c1, ca, b.c1, cb, c.c1, cc)};
}
DH_DEV f228 f2_red(const f228& a) { return {f28_red(a.c0), f28_red(a.c1)}; }
// -a = 3p - a for a < 3 (points, affine coordinates)
DH_DEV f228 f2_neg3(const f228& a) { return {f28_lin<3>(a.c0, -1, a.c0, 0), f28_lin<3>(a.c1, -1, a.c1, 0)}; }
DH_DEV f228 f2_conj(const f228& a) { return {a.c0, f28_lin<2>(a.c1, -1, a.c1, 0)}; }  // a1 < 2

// Karatsuba: (a0 b0 - a1 b1 + 2p, (a0 + a1)(b0 + b1) - a0 b0 - a1 b1 + 4p) -> (4, 6). NC: the sums a0 + a1, b0 + b1
// feed only the third product and keep their limbs unnormalised (f28_add_nc): fewer instructions, but the
// independent limb sums lengthen live ranges, which the register-starved MSM reduction kernels pay for in scratch
// (G2 MSM 15.8 -> 17.8 ms with NC everywhere); the subgroup test's doubling chain gains (k_sub_sig_g2 -3%)
template <bool NC = false>
DH_DEV f228 f2_mul(const f228& a, const f228& b) {
  const f28 t0 = f28_mul(a.c0, b.c0);
  const f28 t1 = f28_mul(a.c1, b.c1);
  const f28 t2 = NC ? f28_mul(f28_add_nc(a.c0, a.c1), f28_add_nc(b.c0, b.c1)) : f28_mul(f28_add(a.c0, a.c1), f28_add(b.c0, b.c1));
  return {f28_lin<2>(t0, 1, t1, -1), f28_lin3<4>(t2, 1, t0, -1, t1, -1)};
}
// complex squaring ((a0 + a1)(a0 - a1 + K p), 2 a0 a1), K >= a1's bound -> (2, 4). NC (as f2_mul): both operands of
// the first product skip the carry pass, the difference with K' = kp_above(K) (it needs a1 below (K' - 1) p)
template <int K, bool NC = false>
DH_DEV f228 f2_sqr(const f228& a) {
  const f28 t0 = NC ? f28_mul(f28_add_nc(a.c0, a.c1), f28_sub_nc<kp_above(K)>(a.c0, a.c1))
                    : f28_mul(f28_add(a.c0, a.c1), f28_lin<K>(a.c0, 1, a.c1, -1));
  const f28 t1 = f28_mul(a.c0, a.c1);
  return {t0, f28_scale(t1, 2)};
}
DH_DEV bool f2_zero(const f228& a) { return f28_zero(a.c0) && f28_zero(a.c1); }
DH_DEV f228 f2_one() {
  f228 r;
  r.c0 = f28_one();
#pragma unroll
  for (int i = 0; i < 14; i++) r.c1.l[i] = 0;
  return r;
}
DH_DEV f228 f2_from_fp2(const fp2& x) { return {f28_from_fp(x.c0), f28_from_fp(x.c1)}; }
DH_DEV fp2 f2_to_fp2(const f228& a) { return {f28_to_fp(a.c0), f28_to_fp(a.c1)}; }

struct j228 {
  f228 x, y, z;
  bool inf;
};
DH_DEV j228 j228_inf() {
  j228 r;
  r.x = f2_one();
  r.y = f2_one();
#pragma unroll
  for (int i = 0; i < 14; i++) r.z.c0.l[i] = r.z.c1.l[i] = 0;
  r.inf = true;
  return r;
}

// The formulas are written in the order that keeps the fewest Fp2 values live (an Fp2 value is 28 VGPRs and every
// product call clobbers 46 fixed registers): each intermediate dies as early as the formula allows.
// dbl-2009-l (a = 0): X, Y < 2, Z < 12 -> (2, 2, 12)
template <bool NC = false>
DH_DEV j228 j228_dbl(const j228& p) {
  j228 r;
  r.inf = p.inf;
  r.z = f2_scale(f2_mul<NC>(p.y, p.z), 2);                     // (8, 12)
  const f228 b = f2_sqr<3, NC>(p.y);                           // (2, 4)
  const f228 c = f2_sqr<4, NC>(b);                             // (2, 4)
  const f228 t = f2_sqr<7, NC>(f2_add(p.x, b));                // X + B < (5, 7)
  const f228 a = f2_sqr<3, NC>(p.x);                           // (2, 4)
  const f228 d = f2_lin3<8, 16>(t, 2, a, -2, c, -2);           // (12, 24)
  const f228 e = f2_scale(a, 3);                               // (6, 12)
  r.x = f2_red(f2_lin<24, 48>(f2_sqr<12, NC>(e), 1, d, -2));   // (26, 52) -> < 2
  const f228 m = f2_mul<NC>(e, f2_lin<3, 3>(d, 1, r.x, -1));   // e < 12, D - X3 + 3p < 27
  r.y = f2_red(f2_lin<16, 32>(m, 1, c, -8));                   // (20, 38) -> < 2
  return r;
}

// madd-2007-bl, q affine (< 3): P (2, 2, 12) -> (2, 2, 12). EXACT: the exceptional-case tests of curve.hpp
// jac_add_aff. q's coordinates come from ldq(0) / ldq(1) at their single use, so they are never live across the
// formula (the MSM reads them from memory there).
template <bool EXACT, bool NC = false, class LDQ>
DH_DEV j228 j228_madd_ld(const j228& p, LDQ ldq) {
  if (p.inf) return j228{ldq(0), ldq(1), f2_one(), false};
  const f228 z1z1 = f2_sqr<12, NC>(p.z);                       // (2, 4)
  const f228 rr = f2_lin<3, 3>(f2_mul<NC>(f2_mul<NC>(ldq(1), p.z), z1z1), 1, p.y, -1);  // S2 - Y1 + 3p: (7, 9)
  const f228 h = f2_lin<3, 3>(f2_mul<NC>(ldq(0), z1z1), 1, p.x, -1);  // U2 - X1 + 3p: (7, 9)
  if (EXACT && f2_zero(h)) {
    if (f2_zero(rr)) return j228_dbl<NC>(p);
    return j228_inf();
  }
  const f228 hh = f2_sqr<9, NC>(h);                            // (2, 4)
  j228 r;
  r.inf = false;
  r.z = f2_lin3<4, 8>(f2_sqr<21, NC>(f2_add(p.z, h)), 1, z1z1, -1, hh, -1);  // Z + H < 21 -> (6, 12)
  const f228 i = f2_scale(hh, 4);                              // (8, 16)
  const f228 j = f2_mul<NC>(h, i);                             // (4, 6)
  const f228 v = f2_mul<NC>(p.x, i);                           // (4, 6)
  const f228 r2 = f2_scale(rr, 2);                             // (14, 18)
  r.x = f2_red(f2_lin3<12, 18>(f2_sqr<18, NC>(r2), 1, j, -1, v, -2));  // (14, 22) -> < 2
  const f228 yj = f2_mul<NC>(p.y, j);                          // (4, 6)
  const f228 m = f2_mul<NC>(r2, f2_lin<3, 3>(v, 1, r.x, -1));  // (4, 6)
  r.y = f2_red(f2_lin<8, 12>(m, 1, yj, -2));                   // (12, 18) -> < 2
  return r;
}
template <bool EXACT, bool NC = false>
DH_DEV j228 j228_madd(const j228& p, const f228& qx, const f228& qy) {
  return j228_madd_ld<EXACT, NC>(p, [&](int k) { return k ? qy : qx; });
}

// add-2007-bl: (2, 2, 12) x (2, 2, 12) -> (2, 2, 6). EXACT as curve.hpp jac_add. q's coordinates come from ldq(k)
// (k = 0, 1, 2 for x, y, z) where they are used, so a caller can leave q in memory.
template <bool EXACT, class LDQ>
DH_DEV j228 j228_add_ld(const j228& p, bool q_inf, LDQ ldq) {
  if (q_inf) return p;
  if (p.inf) return j228{ldq(0), ldq(1), ldq(2), false};
  const f228 z1z1 = f2_sqr<12>(p.z);                           // (2, 4)
  f228 z2z2, zz, t;
  {
    const f228 z2 = ldq(2);
    z2z2 = f2_sqr<12>(z2);                                     // (2, 4)
    zz = f2_lin3<4, 8>(f2_sqr<24>(f2_add(p.z, z2)), 1, z1z1, -1, z2z2, -1);  // 2 Z1 Z2: (6, 12)
    t = f2_mul(z2, z2z2);                                      // Z2^3: (4, 6)
  }
  const f228 s1 = f2_mul(p.y, t);                              // Y1 Z2^3: (4, 6)
  const f228 u1 = f2_mul(p.x, z2z2);                           // (4, 6)
  const f228 rr = f2_lin<4, 6>(f2_mul(ldq(1), f2_mul(p.z, z1z1)), 1, s1, -1);  // S2 - S1: (8, 12)
  const f228 h = f2_lin<4, 6>(f2_mul(ldq(0), z1z1), 1, u1, -1);  // U2 - U1: (8, 12)
  if (EXACT && f2_zero(h)) {
    if (f2_zero(rr)) return j228_dbl(p);
    return j228_inf();
  }
  j228 r;
  r.inf = false;
  r.z = f2_mul(zz, h);                                         // (4, 6)
  const f228 i = f2_sqr<24>(f2_scale(h, 2));                   // 2H < (16, 24) -> (2, 4)
  const f228 j = f2_mul(h, i);                                 // (4, 6)
  const f228 v = f2_mul(u1, i);                                // (4, 6)
  const f228 r2 = f2_scale(rr, 2);                             // (16, 24)
  r.x = f2_red(f2_lin3<12, 18>(f2_sqr<24>(r2), 1, j, -1, v, -2));  // (14, 22) -> < 2
  const f228 sj = f2_mul(s1, j);                               // (4, 6)
  const f228 m = f2_mul(r2, f2_lin<3, 3>(v, 1, r.x, -1));      // (4, 6)
  r.y = f2_red(f2_lin<8, 12>(m, 1, sj, -2));                   // (12, 18) -> < 2
  return r;
}
template <bool EXACT>
DH_DEV j228 j228_add(const j228& p, const j228& q) {
  return j228_add_ld<EXACT>(p, q.inf, [&](int k) { return k == 0 ? q.x : k == 1 ? q.y : q.z; });
}
DH_DEV bool j228_poisoned(const j228& p) { return !p.inf && f2_zero(p.z); }

// psi(x, y) = (conj(x) PSI_X, conj(y) PSI_Y) as 28-bit Montgomery constants (PSI_X's c0 is 0)
__device__ __constant__ uint32_t PSI_X28[2][14] = {
    {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {0x58a1811u, 0x96e4867u, 0x1d5c11cu, 0x543e856u, 0x13e6366u, 0x4b0fc91u, 0xae5efbbu, 0x8680210u, 0x9941307u,
     0xf700269u, 0xb02eef7u, 0x9086bfcu, 0x6855919u, 0x001291eu}};
__device__ __constant__ uint32_t PSI_Y28[2][14] = {
    {0xcc17b84u, 0xcc5da55u, 0x1835de7u, 0x3e1e677u, 0x9e4ae31u, 0x9b9a07au, 0xd662557u, 0xb7f1997u, 0x71cc4dau,
     0xa667f92u, 0x65115feu, 0x4a3370cu, 0xe5b746au, 0x000d16du},
    {0x33e2f27u, 0x32a25aau, 0x27ca1d2u, 0xc1e049eu, 0xc3f707au, 0x055ca94u, 0x2010b7bu, 0x3b93794u, 0xd5a86aau,
     0xa544de3u, 0x556a044u, 0x9c66da5u, 0x38ec515u, 0x000cea3u}};
DH_DEV f228 f2_c28(const uint32_t (*c)[14]) { return {f28_c(c[0]), f28_c(c[1])}; }

// psi^2 constants (Fp: the c1 parts are 0)
__device__ __constant__ uint32_t PSI2_X28[14] = {0x2421b59u, 0xbee4867u, 0x1d31002u, 0x4760184u, 0x4cc5086u, 0xc76dc00u, 0xaae891bu,
                                                 0xac70ad2u, 0xfe377c4u, 0xe4686b8u, 0x5ed1568u, 0x8f5a180u, 0x02b5c1fu, 0x000d1a4u};
__device__ __constant__ uint32_t PSI2_Y28[14] = {0xcb7adf3u, 0x26fffffu, 0x3fd4ea0u, 0xf320443u, 0x9b20bcbu, 0x1d54a7eu, 0xf2fca33u,
                                                 0x19759edu, 0xac6b042u, 0x39151c5u, 0x691dcb4u, 0xe56da35u, 0xb903c85u, 0x0014896u};
DH_DEV j228 j228_neg(const j228& p) { return {p.x, f2_neg3(p.y), p.z, p.inf}; }  // Y < 3 stays a valid coordinate
DH_DEV j228 j228_psi(const j228& p) {  // (conj(X) PSI_X, conj(Y) PSI_Y, conj(Z)), Z < 12
  return {f2_red(f2_mul(f2_conj(p.x), f2_c28(PSI_X28))), f2_red(f2_mul(f2_conj(p.y), f2_c28(PSI_Y28))),
          {p.z.c0, f28_lin<12>(p.z.c1, -1, p.z.c1, 0)}, p.inf};
}
DH_DEV j228 j228_psi2(const j228& p) {
  const f28 cx = f28_c(PSI2_X28), cy = f28_c(PSI2_Y28);
  return {{f28_mul(p.x.c0, cx), f28_mul(p.x.c1, cx)}, {f28_mul(p.y.c0, cy), f28_mul(p.y.c1, cy)}, p.z, p.inf};
}
// the doubling runs of [|u|] between |u|'s set bits below the top one (62, 60, 57, 48, 16: 1, 2, 3, 9, 32, 16)
DH_DEV int uabs_run(int r) { return r == 0 ? 1 : r == 1 ? 2 : r == 2 ? 3 : r == 3 ? 9 : r == 4 ? 32 : 16; }
DH_DEV j228 j228_mul_uabs(const j228& p) {  // [|u|] P, Jacobian base; doublings in runs (g2_mul_uabs_ld)
  j228 acc = p;
#pragma unroll 1
  for (int r = 0; r < 6; r++) {
    const int k = uabs_run(r);
#pragma unroll 1
    for (int i = 0; i < k; i++) acc = j228_dbl(acc);
    if (r < 5) acc = j228_add<true>(acc, p);
  }
  return acc;
}
// clear_cofactor(G2) = [h_eff] P by the endomorphism method of RFC 9380 Appendix G.3, the steps of h2c.hpp
// h2c_clear_g2 on the lazy form (tests/fp2_28_model.py clear): the G2 group check's and the leaves' hash side
DH_DEV jac<fp2> g2_clear28(const jac<fp2>& q) {
  j228 p{f2_from_fp2(q.x), f2_from_fp2(q.y), f2_from_fp2(q.z), fp2_is_zero(q.z)};
  const j228 t1 = j228_neg(j228_mul_uabs(p));
  j228 t3 = j228_add<true>(j228_psi2(j228_dbl(p)), j228_neg(j228_psi(p)));
  const j228 t2 = j228_neg(j228_mul_uabs(j228_add<true>(t1, j228_psi(p))));
  t3 = j228_add<true>(j228_add<true>(j228_add<true>(t3, t2), j228_neg(t1)), j228_neg(p));
  if (t3.inf) return jac_inf<fp2>();
  return {f2_to_fp2(t3.x), f2_to_fp2(t3.y), f2_to_fp2(t3.z)};
}

// G2 subgroup test of an affine point (codec.hpp g2_in_subgroup, same algorithm): psi(P) == [u] P = -[|u|] P,
// |u| = 0xd201000000010000, on the lazy form (tests/fp2_28_model.py in_subgroup). ld() returns P (12 x 32 form); it is
// called where P's coordinates are needed (the loop's five mixed additions, the final comparison), so a caller that
// keeps P in memory (k_sub_sig_g2) holds no copy of it in registers across the doublings.
// [|u|] P on the lazy form; EXACT = false takes the mixed additions without their exceptional-case tests (the MSM's
// fast formulas): an exceptional case (acc = +-P, or a 2-torsion doubling) leaves Z = 0 mod p, which every later step
// keeps, so a poisoned result (Z = 0 without the infinity flag) is recomputed with the exact formulas
// The 63 doublings run as the six runs between |u|'s set bits (uabs_run), each an inner loop with the mixed addition
// after it, so the doublings' loop carries none of the addition's live values.
template <bool EXACT, class Q>
DH_DEV j228 g2_mul_uabs_ld(Q q) {
  j228 acc{q(0), q(1), f2_one(), false};
#pragma unroll 1
  for (int r = 0; r < 6; r++) {
    const int k = uabs_run(r);
#pragma unroll 1
    for (int i = 0; i < k; i++) acc = j228_dbl<true>(acc);
    if (r < 5) acc = j228_madd_ld<EXACT, true>(acc, q);
  }
  return acc;
}
template <class LD>
DH_DEV bool g2_in_subgroup28(LD ld) {
  auto q = [&](int k) { const aff<fp2> a = ld(); return f2_from_fp2(k ? a.y : a.x); };
  j228 acc = g2_mul_uabs_ld<false>(q);
  if (j228_poisoned(acc)) acc = g2_mul_uabs_ld<true>(q);
  if (acc.inf) return false;  // psi(P) is finite
  const f228 z2 = f2_sqr<12>(acc.z);
  const f228 px = f2_mul(f2_conj(q(0)), f2_c28(PSI_X28));               // (4, 6)
  if (!f2_zero(f2_lin<3, 3>(f2_mul(px, z2), 1, acc.x, -1))) return false;  // psi(P).x Z^2 == X
  const f228 py = f2_mul(f2_conj(q(1)), f2_c28(PSI_Y28));               // (4, 6)
  return f2_zero(f2_add(f2_mul(py, f2_mul(z2, acc.z)), acc.y));         // psi(P).y Z^3 == -Y
}
DH_DEV bool g2_in_subgroup28(const aff<fp2>& p) {
  return g2_in_subgroup28([&] { return p; });
}

}  // namespace dh
