// Lazy-reduced Fp arithmetic on 14 x 28-bit limbs (Montgomery radix R' = 2^392) for the G1 signature subgroup test,
// the largest share of k_prep_sig (two 64-bit scalar multiplications per round, ~990 field products).
//
// A value is an integer v < K p (K tracked per formula below) congruent to a R' for the field element a, held in 14
// NORMALISED limbs (< 2^28). The products (fp_mul28.hpp mont_mul / mont_sqr, out of line: dh_fp28_mul_vec /
// dh_fp28_sqr_vec) accept any two such values with X Y < 2^392 p (about 2500 p^2) and return < 2p; sums and
// differences are limb-wise with one signed carry pass and no modular reduction (a - b is a + k p - b for a k p
// above b's bound). So no product slices 12 <-> 14 limbs or subtracts p, and no addition reduces: the point
// formulas keep their operands below ~50 p. Equality tests reduce first (f28_zero: one product by 1); infinity is a
// flag (j28).
// Bounds (units of p): dbl (X, Y, Z) <= (48, 50, 2500/Y) -> (26, 18, 4); madd with q < 2 -> (8, 6, 6); add -> (8, 6, 2).
#pragma once
#include "fp.hpp"

namespace dh {

struct f28 {
  uint32_t l[14];
};

#define DH_FP28_CALL_CLOBBERS                                                                                  \
  "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v48", "v49", "v50", "v51", "v52", "v53", "s0", "s1", \
      "s2", "s3", "s4", "s5", "s6", "s7", "s8", "s9", "s10", "s11", "s12", "s13", "s14", "s15", "s16", "s17", "s30", \
      "s31", "vcc", "scc"

DH_DEV fp28vec f28_vec(const f28& a) {
  fp28vec v;
#pragma unroll
  for (int i = 0; i < 14; i++) v[i] = a.l[i];
  v[14] = v[15] = 0;
  return v;
}
DH_DEV f28 f28_unvec(const fp28vec& v) {
  f28 a;
#pragma unroll
  for (int i = 0; i < 14; i++) a.l[i] = v[i];
  return a;
}

DH_DEV f28 f28_mul(const f28& a, const f28& b) {
  DH_COUNT_PROD();
  fp28vec x = f28_vec(a), y = f28_vec(b);
  asm(DH_FP_CALL("dh_fp28_mul_vec") : "+{v[0:15]}"(x), "+{v[16:31]}"(y) : : DH_FP28_CALL_CLOBBERS);
  return f28_unvec(x);
}
DH_DEV f28 f28_sqr(const f28& a) {
  DH_COUNT_PROD();
  fp28vec x = f28_vec(a);
  asm(DH_FP_CALL("dh_fp28_sqr_vec")
      : "+{v[0:15]}"(x)
      :
      : "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31",
        DH_FP28_CALL_CLOBBERS);
  return f28_unvec(x);
}

// multiples of p (normalised limbs) for differences: a - b = a + k p - b, k p >= b
template <int K>
DH_DEV uint32_t kp_limb(int i);
#define DH_KP(K, ...)                                                 \
  template <>                                                         \
  DH_DEV uint32_t kp_limb<K>(int i) {                                 \
    const uint32_t t[14] = {__VA_ARGS__};                             \
    return t[i];                                                      \
  }
DH_KP(2, 0xfff5556u, 0xfdfffffu, 0x7ffff73u, 0xfffd62au, 0xc483d57u, 0x41ed61eu, 0xece61a5u, 0xe70a257u, 0x8ee9709u,
      0x9759aecu, 0x74f6c86u, 0xcd34963u, 0x3d472ffu, 0x0034022u)
DH_KP(4, 0xffeaaacu, 0xfbfffffu, 0xffffee7u, 0xfffac54u, 0x8907aafu, 0x83dac3du, 0xd9cc34au, 0xce144afu, 0x1dd2e13u,
      0x2eb35d9u, 0xe9ed90du, 0x9a692c6u, 0x7a8e5ffu, 0x0068044u)
DH_KP(6, 0xffe0002u, 0xf9fffffu, 0x7fffe5bu, 0xfff827fu, 0x4d8b807u, 0xc5c825cu, 0xc6b24efu, 0xb51e707u, 0xacbc51du,
      0xc60d0c5u, 0x5ee4593u, 0x679dc2au, 0xb7d58ffu, 0x009c066u)
DH_KP(8, 0xffd5558u, 0xf7fffffu, 0xffffdcfu, 0xfff58a9u, 0x120f55fu, 0x07b587bu, 0xb398695u, 0x9c2895fu, 0x3ba5c27u,
      0x5d66bb2u, 0xd3db21au, 0x34d258du, 0xf51cbffu, 0x00d0088u)
DH_KP(16, 0xffaaab0u, 0xeffffffu, 0xffffb9fu, 0xffeb153u, 0x241eabfu, 0x0f6b0f6u, 0x6730d2au, 0x38512bfu, 0x774b84fu,
      0xbacd764u, 0xa7b6434u, 0x69a4b1bu, 0xea397feu, 0x01a0111u)
DH_KP(18, 0xffa0006u, 0xedfffffu, 0x7fffb13u, 0xffe877eu, 0xe8a2817u, 0x5158714u, 0x5416ecfu, 0x1f5b517u, 0x0634f59u,
      0x5227251u, 0x1cad0bbu, 0x36d947fu, 0x2780afeu, 0x01d4134u)
DH_KP(24, 0xff80008u, 0xe7fffffu, 0xffff96fu, 0xffe09fdu, 0x362e01fu, 0x1720971u, 0x1ac93bfu, 0xd479c1fu, 0xb2f1476u,
      0x1834316u, 0x7b9164fu, 0x9e770a9u, 0xdf563fdu, 0x027019au)
DH_KP(26, 0xff7555eu, 0xe5fffffu, 0x7fff8e3u, 0xffde028u, 0xfab1d77u, 0x590df8fu, 0x07af564u, 0xbb83e77u, 0x41dab80u,
      0xaf8de03u, 0xf0882d5u, 0x6baba0cu, 0x1c9d6fdu, 0x02a41bdu)
DH_KP(3, 0xfff0001u, 0xfcfffffu, 0xbffff2du, 0xfffc13fu, 0x26c5c03u, 0xe2e412eu, 0xe359277u, 0xda8f383u, 0xd65e28eu,
      0xe306862u, 0x2f722c9u, 0xb3cee15u, 0x5beac7fu, 0x004e033u)
DH_KP(7, 0xffdaaadu, 0xf8fffffu, 0xbfffe15u, 0xfff6d94u, 0xafcd6b3u, 0x66bed6bu, 0xbd255c2u, 0xa8a3833u, 0xf4310a2u,
      0x11b9e3bu, 0x195fbd7u, 0x4e380dcu, 0xd67927fu, 0x00b6077u)
DH_KP(9, 0xffd0003u, 0xf6fffffu, 0x3fffd89u, 0xfff43bfu, 0x745140bu, 0xa8ac38au, 0xaa0b767u, 0x8fada8bu, 0x831a7acu,
      0xa913928u, 0x8e5685du, 0x1b6ca3fu, 0x13c057fu, 0x00ea09au)
DH_KP(12, 0xffc0004u, 0xf3fffffu, 0xffffcb7u, 0xfff04feu, 0x9b1700fu, 0x8b904b8u, 0x8d649dfu, 0x6a3ce0fu, 0x5978a3bu,
      0x8c1a18bu, 0xbdc8b27u, 0xcf3b854u, 0x6fab1feu, 0x01380cdu)
DH_KP(21, 0xff90007u, 0xeafffffu, 0x3fffa41u, 0xffe48beu, 0x0f6841bu, 0x343c843u, 0x3770147u, 0xf9ea89bu, 0xdc931e7u,
      0x352dab3u, 0x4c1f385u, 0xeaa8294u, 0x836b77du, 0x0222167u)
DH_KP(32, 0xff55560u, 0xdffffffu, 0xffff73fu, 0xffd62a7u, 0x483d57fu, 0x1ed61ecu, 0xce61a54u, 0x70a257eu, 0xee9709eu,
      0x759aec8u, 0x4f6c869u, 0xd349637u, 0xd472ffcu, 0x0340223u)
DH_KP(48, 0xff00010u, 0xcffffffu, 0xffff2dfu, 0xffc13fbu, 0x6c5c03fu, 0x2e412e2u, 0x359277eu, 0xa8f383eu, 0x65e28edu,
      0x306862du, 0xf722c9eu, 0x3cee152u, 0xbeac7fbu, 0x04e0335u)
#undef DH_KP

// ca a + cb b + K p limb-wise with one signed carry pass. The negative coefficients add up to >= -8 and the positive
// ones to <= 6, so every limb sum stays inside int32 (limbs < 2^28: a sum is >= -8 (2^28 - 1) - 8 carry); the
// caller's bounds keep the value in [0, 2^392)
template <int K>
DH_DEV f28 f28_lin(const f28& a, int ca, const f28& b, int cb) {
  f28 r;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    int32_t t = ca * (int32_t)a.l[i] + cb * (int32_t)b.l[i] + c;
    if constexpr (K != 0) t += (int32_t)kp_limb<K>(i);
    r.l[i] = (uint32_t)t & m28::MASK;
    c = t >> 28;
  }
  return r;
}
// ca a + cb b + cc c + K p (same limits on the coefficients as f28_lin)
template <int K>
DH_DEV f28 f28_lin3(const f28& a, int ca, const f28& b, int cb, const f28& c3, int cc) {
  f28 r;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    int32_t t = ca * (int32_t)a.l[i] + cb * (int32_t)b.l[i] + cc * (int32_t)c3.l[i] + c;
    if constexpr (K != 0) t += (int32_t)kp_limb<K>(i);
    r.l[i] = (uint32_t)t & m28::MASK;
    c = t >> 28;
  }
  return r;
}
DH_DEV f28 f28_add(const f28& a, const f28& b) { return f28_lin<0>(a, 1, b, 1); }
template <int K>
DH_DEV f28 f28_sub(const f28& a, const f28& b) { return f28_lin<K>(a, 1, b, -1); }
DH_DEV f28 f28_scale(const f28& a, int c) { return f28_lin<0>(a, c, a, 0); }

// Operands that feed only a product skip the carry pass. fp_mul28.hpp accumulates a column of 14 limb products plus
// 14 quotient-digit products and the carry-in in 64 bits: with one operand's limbs < 2^29.6 and the other's < 2^29 a
// column stays below 14 * 2^58.6 + 14 * 2^56 + 2^36 < 2^63, so limbs need not be normalised there (the value, which
// the bounds are about, is the same integer). a + b limb by limb: limbs < 2^29.
DH_DEV f28 f28_add_nc(const f28& a, const f28& b) {
  f28 r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.l[i] = a.l[i] + b.l[i];
  return r;
}
// a + K p - b limb by limb, K p in a redundant form (limb 0 + 2^28, limbs 1..12 + 2^28 - 1, limb 13 - 1: the same
// value) so that every limb is >= 0 given normalised a, b and b's top limb below K p's (b < (K - 1) p suffices);
// limbs < 2^29.6
template <int K>
DH_DEV f28 f28_sub_nc(const f28& a, const f28& b) {
  f28 r;
  r.l[0] = a.l[0] + kp_limb<K>(0) + (1u << 28) - b.l[0];
#pragma unroll
  for (int i = 1; i < 13; i++) r.l[i] = a.l[i] + kp_limb<K>(i) + ((1u << 28) - 1) - b.l[i];
  r.l[13] = a.l[13] + kp_limb<K>(13) - 1 - b.l[13];
  return r;
}
// the smallest K' > K with a K' p constant (kp_limb): f28_sub_nc<kp_above(K)> takes any b < K p
constexpr int kp_above(int K) {
  return K < 3 ? 3 : K < 4 ? 4 : K < 6 ? 6 : K < 7 ? 7 : K < 8 ? 8 : K < 9 ? 9 : K < 12 ? 12 : K < 16 ? 16 : K < 18 ? 18
       : K < 21 ? 21 : K < 24 ? 24 : K < 26 ? 26 : K < 32 ? 32 : 48;
}
DH_DEV f28 f28_one() {  // R' mod p
  const uint32_t k[14] = {0x347fcb8u, 0xd800000u, 0x002b119u, 0x0cde6d2u, 0xc7212e0u, 0x83a2090u, 0x037669fu,
                          0xda0f73eu, 0x9b09b42u, 0x1297bb0u, 0x515d98fu, 0x012ca7cu, 0x659fcfau, 0x000577au};
  f28 r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.l[i] = k[i];
  return r;
}

// a == 0 mod p (a < 2^392): a / R' by one product lands in [0, 2p)
DH_DEV bool f28_zero(const f28& a) {
  f28 one;
#pragma unroll
  for (int i = 0; i < 14; i++) one.l[i] = i == 0;
  const f28 r = f28_mul(a, one);
  uint32_t z = 0, d = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    z |= r.l[i];
    d |= r.l[i] ^ m28::P[i];
  }
  return z == 0 || d == 0;
}

// 12 x 32-bit Montgomery (radix 2^384, < p) -> 28-bit form: one product with 2^400 mod p, < 1.002 p
DH_DEV f28 f28_from_fp(const fp& x) {
  f28 a, c;
  m28::split<0>(a.l, x.v);
  const uint32_t k[14] = {0x80e6299u, 0x3500034u, 0xeb12856u, 0xdeb2699u, 0xc988670u, 0x4ef6697u, 0x70983e8u,
                          0xa4e6fe9u, 0x3e8a053u, 0xecf271eu, 0xc20d323u, 0x6eb6385u, 0x47f1286u, 0x00156dau};
#pragma unroll
  for (int i = 0; i < 14; i++) c.l[i] = k[i];
  return f28_mul(a, c);
}

// Jacobian point with an explicit infinity flag: the subgroup test's points lie on E(Fp), whose order h r is odd
// (no 2-torsion), so the formulas below only reach infinity through their special cases, which set the flag; a
// finite point's Z never vanishes (Z3 = 2YZ, 2 Z H, 2 Z1 Z2 H with Y, Z, H != 0), and no product is spent testing it
// 28-bit form (< 2p) -> 12 x 32-bit Montgomery form, canonical: one product with 2^384 mod p
DH_DEV fp f28_to_fp(const f28& a) {
  f28 c;
  const uint32_t k[14] = {0x002fffdu, 0x0900000u, 0xc000276u, 0x000bc40u, 0x8baebf4u, 0x5753c75u, 0x55f4898u,
                          0x7052574u, 0x7ce5853u, 0x56ec6d7u, 0x71a97a2u, 0xe4935c0u, 0xec3fa80u, 0x0015f65u};
#pragma unroll
  for (int i = 0; i < 14; i++) c.l[i] = k[i];
  const f28 r = f28_mul(a, c);
  fp o;
  m28::join(o.v, r.l);
  m28::final_sub(o.v);
  return o;
}

DH_DEV f28 f28_c(const uint32_t* c) {
  f28 r;
#pragma unroll
  for (int i = 0; i < 14; i++) r.l[i] = c[i];
  return r;
}

struct j28 {
  f28 x, y, z;
  bool inf;
};

// the products inlined (fp_mul28.hpp), for the doubling that makes up the subgroup test's loops: the compiler
// allocates its operands freely instead of moving them into the call's fixed registers
DH_DEV f28 f28_mul_inl(const f28& a, const f28& b) {
  DH_COUNT_PROD();
  f28 r;
  m28::mont_mul(r.l, a.l, b.l);
  return r;
}
DH_DEV f28 f28_sqr_inl(const f28& a) {
  DH_COUNT_PROD();
  f28 r;
  m28::mont_sqr(r.l, a.l);
  return r;
}

// dbl-2009-l (a = 0), 2M + 5S. In X <= 48, Y <= 50, Y Z <= 2500 -> out (26, 18, 4); infinity propagates.
// INL: products inlined (the subgroup test's hot loops) or entered out of line (the rare special cases)
template <bool INL = false>
DH_DEV j28 j28_dbl(const j28& p) {
  auto sq = [](const f28& x) { return INL ? f28_sqr_inl(x) : f28_sqr(x); };
  auto mu = [](const f28& x, const f28& y) { return INL ? f28_mul_inl(x, y) : f28_mul(x, y); };
  const f28 a = sq(p.x);                                               // < 2
  const f28 b = sq(p.y);                                               // < 2
  const f28 c = sq(b);                                                 // < 2
  const f28 t = sq(INL ? f28_add_nc(p.x, b) : f28_add(p.x, b));       // (X + B)^2, X + B < 50
  const f28 d = f28_lin3<8>(t, 2, a, -2, c, -2);                       // D = 2 (T + 4p - A - C) < 12
  const f28 e = f28_scale(a, 3);                                       // E = 3A < 6
  const f28 f = sq(e);                                                 // < 2
  j28 r;
  r.x = f28_lin<24>(f, 1, d, -2);                                      // F + 24p - 2D < 26
  // E (D + 26p - X3): 6 x 38 -> < 2 (the carry-free form: D + 32p - X3, 6 x 44)
  const f28 m = mu(e, INL ? f28_sub_nc<kp_above(26)>(d, r.x) : f28_sub<26>(d, r.x));
  r.y = f28_lin<16>(m, 1, c, -8);                                      // M + 16p - 8C < 18
  r.z = f28_scale(mu(p.y, p.z), 2);                                    // < 4
  r.inf = p.inf;
  return r;
}

DH_DEV j28 j28_inf() {
  j28 r;
  r.x = f28_one();
  r.y = f28_one();
#pragma unroll
  for (int i = 0; i < 14; i++) r.z.l[i] = 0;
  r.inf = true;
  return r;
}

// madd-2007-bl, q affine (x, y < 2), full special cases as curve.hpp jac_add_aff. In (26, 18, 6) -> out (8, 6, 6)
DH_DEV j28 j28_madd(const j28& p, const f28& qx, const f28& qy) {
  if (p.inf) return j28{qx, qy, f28_one(), false};
  const f28 z1z1 = f28_sqr(p.z);                                       // < 2
  const f28 u2 = f28_mul(qx, z1z1);                                    // < 2
  const f28 s2 = f28_mul(f28_mul(qy, p.z), z1z1);                      // < 2
  const f28 h = f28_sub<26>(u2, p.x);                                  // < 28
  const f28 rr = f28_sub<18>(s2, p.y);                                 // < 20
  if (f28_zero(h)) {
    if (f28_zero(rr)) return j28_dbl(p);
    return j28_inf();
  }
  const f28 hh = f28_sqr(h);                                           // 28^2 -> < 2
  const f28 i = f28_scale(hh, 4);                                      // < 8
  const f28 j = f28_mul(h, i);                                         // 28 x 8 -> < 2
  const f28 r2 = f28_scale(rr, 2);                                     // < 40
  const f28 v = f28_mul(p.x, i);                                       // 26 x 8 -> < 2
  j28 r;
  r.inf = false;
  r.x = f28_lin3<6>(f28_sqr(r2), 1, j, -1, v, -2);                    // R^2 + 6p - J - 2V < 8
  const f28 m = f28_mul(r2, f28_sub<8>(v, r.x));                       // 40 x 10 -> < 2
  r.y = f28_lin<4>(m, 1, f28_mul(p.y, j), -2);                         // < 6
  r.z = f28_lin3<4>(f28_sqr(f28_add(p.z, h)), 1, z1z1, -1, hh, -1);    // (Z + H)^2, Z + H < 34 -> < 6
  return r;
}

// add-2007-bl, full special cases as curve.hpp jac_add. In (26, 18, 6) x (26, 18, 6) -> out (8, 6, 2)
DH_DEV j28 j28_add(const j28& p, const j28& q) {
  if (p.inf) return q;
  if (q.inf) return p;
  const f28 z1z1 = f28_sqr(p.z), z2z2 = f28_sqr(q.z);                 // < 2
  const f28 u1 = f28_mul(p.x, z2z2), u2 = f28_mul(q.x, z1z1);         // < 2
  const f28 s1 = f28_mul(f28_mul(p.y, q.z), z2z2);                    // < 2
  const f28 s2 = f28_mul(f28_mul(q.y, p.z), z1z1);                    // < 2
  const f28 h = f28_sub<2>(u2, u1);                                    // < 4
  const f28 rr = f28_sub<2>(s2, s1);                                   // < 4
  if (f28_zero(h)) {
    if (f28_zero(rr)) return j28_dbl(p);
    return j28_inf();
  }
  const f28 i = f28_sqr(f28_scale(h, 2));                              // < 2
  const f28 j = f28_mul(h, i);                                         // < 2
  const f28 r2 = f28_scale(rr, 2);                                     // < 8
  const f28 v = f28_mul(u1, i);                                        // < 2
  j28 r;
  r.inf = false;
  r.x = f28_lin3<6>(f28_sqr(r2), 1, j, -1, v, -2);                    // < 8
  const f28 m = f28_mul(r2, f28_sub<8>(v, r.x));                       // 8 x 10 -> < 2
  r.y = f28_lin<4>(m, 1, f28_mul(s1, j), -2);                          // < 6
  const f28 zz = f28_lin3<4>(f28_sqr(f28_add(p.z, q.z)), 1, z1z1, -1, z2z2, -1);  // < 6
  r.z = f28_mul(zz, h);                                                // 6 x 4 -> < 2
  return r;
}

// The MSM's bucket additions (k_msm.hip) use the two formulas above WITHOUT their exceptional-case tests (one
// product each): when h = 0 mod p (the added point equals the accumulator or its negative) Z3 = 2 Z1 H (madd) or
// 2 Z1 Z2 H (add) vanishes mod p, and every later step keeps Z = 0 mod p (madd: Z3 = 2 Z1 H, add: 2 Z1 Z2 H, dbl:
// 2 Y Z, whatever the other operand). So ONE zero test of Z at the end of a run of additions (j28_poisoned) finds
// every run that met such a case, and that run is recomputed with the exact formulas. Same bounds as the exact ones.
DH_DEV j28 j28_madd_fast(const j28& p, const f28& qx, const f28& qy) {
  if (p.inf) return j28{qx, qy, f28_one(), false};
  const f28 z1z1 = f28_sqr(p.z);
  const f28 u2 = f28_mul(qx, z1z1);
  const f28 s2 = f28_mul(f28_mul(qy, p.z), z1z1);
  const f28 h = f28_sub<26>(u2, p.x);
  const f28 rr = f28_sub<18>(s2, p.y);
  const f28 hh = f28_sqr(h);
  const f28 i = f28_scale(hh, 4);
  const f28 j = f28_mul(h, i);
  const f28 r2 = f28_scale(rr, 2);
  const f28 v = f28_mul(p.x, i);
  j28 r;
  r.inf = false;
  r.x = f28_lin3<6>(f28_sqr(r2), 1, j, -1, v, -2);
  const f28 m = f28_mul(r2, f28_sub<8>(v, r.x));
  r.y = f28_lin<4>(m, 1, f28_mul(p.y, j), -2);
  r.z = f28_lin3<4>(f28_sqr(f28_add(p.z, h)), 1, z1z1, -1, hh, -1);
  return r;
}
DH_DEV j28 j28_add_fast(const j28& p, const j28& q) {
  if (p.inf) return q;
  if (q.inf) return p;
  const f28 z1z1 = f28_sqr(p.z), z2z2 = f28_sqr(q.z);
  const f28 u1 = f28_mul(p.x, z2z2), u2 = f28_mul(q.x, z1z1);
  const f28 s1 = f28_mul(f28_mul(p.y, q.z), z2z2);
  const f28 s2 = f28_mul(f28_mul(q.y, p.z), z1z1);
  const f28 h = f28_sub<2>(u2, u1);
  const f28 rr = f28_sub<2>(s2, s1);
  const f28 i = f28_sqr(f28_scale(h, 2));
  const f28 j = f28_mul(h, i);
  const f28 r2 = f28_scale(rr, 2);
  const f28 v = f28_mul(u1, i);
  j28 r;
  r.inf = false;
  r.x = f28_lin3<6>(f28_sqr(r2), 1, j, -1, v, -2);
  const f28 m = f28_mul(r2, f28_sub<8>(v, r.x));
  r.y = f28_lin<4>(m, 1, f28_mul(s1, j), -2);
  const f28 zz = f28_lin3<4>(f28_sqr(f28_add(p.z, q.z)), 1, z1z1, -1, z2z2, -1);
  r.z = f28_mul(zz, h);
  return r;
}
DH_DEV bool j28_poisoned(const j28& p) { return !p.inf && f28_zero(p.z); }
// -y for a y < 2p (loaded points): 2p - y
DH_DEV f28 f28_neg2(const f28& y) { return f28_lin<2>(y, -1, y, 0); }

// G1 subgroup test of an affine point (curve.hpp / codec.hpp g1_in_subgroup, same algorithm): phi(P) == -[u^2] P
// with [u^2] P = [|u|]([|u|] P), |u| = 0xd201000000010000. ld() returns P; it is called at the start and again
// for the final comparison, so a caller that keeps P in memory (k_prep_sig) leaves no copy of it live across the
// second multiplication, whose add steps need ~200 VGPRs besides the call's clobbers.
template <class LD>
DH_DEV bool g1_in_subgroup28(LD ld) {
  j28 t;
  {
    const aff<fp> p = ld();
    const f28 x = f28_from_fp(p.x), y = f28_from_fp(p.y);
    j28 acc{x, y, f28_one(), false};
#pragma unroll 1
    for (int b = 62; b >= 0; b--) {
      acc = j28_dbl<true>(acc);
      if ((cst::U_ABS >> b) & 1) acc = j28_madd(acc, x, y);
    }
    t = acc;  // (26, 18, 4): the last step is a doubling
  }
  j28 acc = t;
#pragma unroll 1
  for (int b = 62; b >= 0; b--) {
    acc = j28_dbl<true>(acc);
    if ((cst::U_ABS >> b) & 1) acc = j28_add(acc, t);
  }
  if (acc.inf) return false;  // phi(P) is finite
  asm volatile("" ::: "memory");      // reload P rather than keep it live through the loop
  const aff<fp> p = ld();
  const f28 bx = f28_from_fp(fp_mul(p.x, fp_c(cst::BETA)));           // phi(P).x < 2
  const f28 y = f28_from_fp(p.y);
  const f28 z2 = f28_sqr(acc.z), z3 = f28_mul(z2, acc.z);              // < 2
  if (!f28_zero(f28_sub<26>(f28_mul(bx, z2), acc.x))) return false;   // x: phi(P).x Z^2 == X
  return f28_zero(f28_add(f28_mul(y, z3), acc.y));                     // y: P.y Z^3 == -Y
}

}  // namespace dh
