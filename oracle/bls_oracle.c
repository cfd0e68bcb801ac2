/*
 * bls_oracle.c — CPU restatement of drand's beacon-verification path. TEST INFRASTRUCTURE.
 *
 * This file is the checker, never the product: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load it (as oracle/liboracle.so). It restates, in plain C with
 * 6 x 64-bit Montgomery limbs, the per-round algorithm that drand runs through kyber:
 *
 *   crypto.Scheme.VerifyBeacon        /root/reference/crypto/schemes.go:70-72
 *     DigestBeacon (chained)          /root/reference/crypto/schemes.go:106-114
 *     DigestBeacon (unchained, g1)    /root/reference/crypto/schemes.go:147-151, 187-191
 *     tbls.VerifyRecovered -> bls.Verify      [kyber v1.1.18 sign/bls, un-vendored]
 *       decode sig (ZCash compressed + subgroup check)  [kilic/bls12-381 v0.1.0 FromCompressed]
 *       hash-to-curve (RFC 9380 XMD:SHA-256 SSWU RO)    [kilic HashToCurve, kyber-bls12381 DSTs]
 *       2-pairing check                                 [kilic Engine AddPair/AddPairInv/Check]
 *   crypto.RandomnessFromSignature    /root/reference/crypto/schemes.go:249-252
 *   tbls.Recover / share.RecoverCommit [kyber v1.1.18], called at
 *                                     /root/reference/chain/beacon/chainstore.go:202,207
 *   mock chain generator pattern      /root/reference/client/test/result/mock/result.go:84-127
 *
 * Pinned by the reference KATs /root/reference/crypto/schemes_test.go:81-130 and
 * /root/reference/crypto/curve_test.go:10-31 (tests/test_oracle.py, KATs in tests/kat.py), and cross-checked
 * against the independent pure-Python model oracle/bls_py.py.
 *
 * Build: see oracle/Makefile (gcc -O3 -shared -fPIC -pthread).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t l[6]; } fp_t;
typedef struct { fp_t c0, c1; } fp2_t;
typedef struct { fp2_t c0, c1, c2; } fp6_t;
typedef struct { fp6_t c0, c1; } fp12_t;
typedef struct { fp_t x, y, z; } g1_t;    /* Jacobian; z == 0 <=> infinity */
typedef struct { fp2_t x, y, z; } g2_t;

static const uint64_t P[6] = {0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL,
                              0x64774b84f38512bfULL, 0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL};
static const uint64_t NP0 = 0x89f3fffcfffcfffdULL; /* -p^-1 mod 2^64 */
static const uint64_t RSC[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL,
                                0x73eda753299d7d48ULL}; /* group order r */

static fp_t FP_ONE, FP_R2;

/* ------------------------------------------------------------------ Fp */
static int geq_p(const uint64_t *a) {
  for (int i = 5; i >= 0; i--) {
    if (a[i] > P[i]) return 1;
    if (a[i] < P[i]) return 0;
  }
  return 1;
}
static void sub_p(uint64_t *a) {
  u128 b = 0;
  for (int i = 0; i < 6; i++) {
    u128 t = (u128)a[i] - P[i] - b;
    a[i] = (uint64_t)t;
    b = (t >> 64) & 1;
  }
}
static void fp_add(fp_t *r, const fp_t *a, const fp_t *b) {
  u128 c = 0;
  for (int i = 0; i < 6; i++) {
    c += (u128)a->l[i] + b->l[i];
    r->l[i] = (uint64_t)c;
    c >>= 64;
  }
  if (geq_p(r->l)) sub_p(r->l);
}
static void fp_sub(fp_t *r, const fp_t *a, const fp_t *b) {
  u128 br = 0;
  uint64_t t[6];
  for (int i = 0; i < 6; i++) {
    u128 d = (u128)a->l[i] - b->l[i] - br;
    t[i] = (uint64_t)d;
    br = (d >> 64) & 1;
  }
  if (br) {
    u128 c = 0;
    for (int i = 0; i < 6; i++) {
      c += (u128)t[i] + P[i];
      t[i] = (uint64_t)c;
      c >>= 64;
    }
  }
  memcpy(r->l, t, sizeof t);
}
static int fp_is_zero(const fp_t *a) {
  uint64_t z = 0;
  for (int i = 0; i < 6; i++) z |= a->l[i];
  return z == 0;
}
static int fp_eq(const fp_t *a, const fp_t *b) { return memcmp(a, b, sizeof *a) == 0; }
static void fp_neg(fp_t *r, const fp_t *a) {
  fp_t z;
  memset(&z, 0, sizeof z);
  fp_sub(r, &z, a);
}
static void fp_mul(fp_t *r, const fp_t *a, const fp_t *b) {
  uint64_t t[8] = {0};
  for (int i = 0; i < 6; i++) {
    u128 c = 0;
    for (int j = 0; j < 6; j++) {
      c += (u128)a->l[j] * b->l[i] + t[j];
      t[j] = (uint64_t)c;
      c >>= 64;
    }
    c += t[6];
    t[6] = (uint64_t)c;
    t[7] = (uint64_t)(c >> 64);
    uint64_t m = t[0] * NP0;
    c = (u128)m * P[0] + t[0];
    c >>= 64;
    for (int j = 1; j < 6; j++) {
      c += (u128)m * P[j] + t[j];
      t[j - 1] = (uint64_t)c;
      c >>= 64;
    }
    c += t[6];
    t[5] = (uint64_t)c;
    t[6] = t[7] + (uint64_t)(c >> 64);
  }
  if (t[6] || geq_p(t)) sub_p(t);
  memcpy(r->l, t, 48);
}
static void fp_sqr(fp_t *r, const fp_t *a) { fp_mul(r, a, a); }
static void fp_pow(fp_t *r, const fp_t *a, const uint64_t *e, int nwords) {
  fp_t acc = FP_ONE, base = *a;
  for (int i = nwords * 64 - 1; i >= 0; i--) {
    fp_sqr(&acc, &acc);
    if ((e[i >> 6] >> (i & 63)) & 1) fp_mul(&acc, &acc, &base);
  }
  *r = acc;
}
static uint64_t E_PM2[6], E_SQRT[6], E_LEG[6];
static void fp_inv(fp_t *r, const fp_t *a) { fp_pow(r, a, E_PM2, 6); }
static int fp_sqrt(fp_t *r, const fp_t *a) {
  fp_t s, c;
  fp_pow(&s, a, E_SQRT, 6);
  fp_sqr(&c, &s);
  *r = s;
  return fp_eq(&c, a);
}
static int fp_is_square(const fp_t *a) {
  fp_t t;
  if (fp_is_zero(a)) return 1;
  fp_pow(&t, a, E_LEG, 6);
  return fp_eq(&t, &FP_ONE);
}
static void fp_from_u64s(fp_t *r, const uint64_t *x) { /* canonical < p -> Montgomery */
  fp_t t;
  memcpy(t.l, x, 48);
  fp_mul(r, &t, &FP_R2);
}
static void fp_canon(uint64_t *out, const fp_t *a) {
  fp_t one, t;
  memset(&one, 0, sizeof one);
  one.l[0] = 1;
  fp_mul(&t, a, &one);
  memcpy(out, t.l, 48);
}
static void fp_set_u64(fp_t *r, uint64_t v) {
  uint64_t x[6] = {v, 0, 0, 0, 0, 0};
  fp_from_u64s(r, x);
}
static int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  return c - 'A' + 10;
}
static void u64s_from_hex(uint64_t *x, int nwords, const char *h) {
  memset(x, 0, 8 * nwords);
  int n = (int)strlen(h);
  for (int i = 0; i < n; i++) {
    int v = hexval(h[n - 1 - i]);
    x[i / 16] |= (uint64_t)v << (4 * (i % 16));
  }
}
static void fp_from_hex(fp_t *r, const char *h) {
  uint64_t x[6];
  u64s_from_hex(x, 6, h);
  fp_from_u64s(r, x);
}
static void be48_to_u64s(uint64_t *x, const uint8_t *b) {
  for (int i = 0; i < 6; i++) {
    uint64_t v = 0;
    for (int k = 0; k < 8; k++) v = (v << 8) | b[40 - 8 * i + k];
    x[i] = v;
  }
}
static void u64s_to_be48(uint8_t *b, const uint64_t *x) {
  for (int i = 0; i < 6; i++)
    for (int k = 0; k < 8; k++) b[40 - 8 * i + k] = (uint8_t)(x[i] >> (56 - 8 * k));
}
static int lt_p(const uint64_t *x) { return !geq_p(x); }
static int canon_gt_half(const uint64_t *x) { /* x > (p-1)/2 */
  uint64_t h[6];
  for (int i = 0; i < 6; i++) h[i] = (P[i] >> 1) | (i < 5 ? (P[i + 1] << 63) : 0);
  for (int i = 5; i >= 0; i--) {
    if (x[i] > h[i]) return 1;
    if (x[i] < h[i]) return 0;
  }
  return 0;
}
static int fp_sgn0(const fp_t *a) {
  uint64_t c[6];
  fp_canon(c, a);
  return (int)(c[0] & 1);
}

/* ------------------------------------------------------------------ Fp2 */
static void fp2_add(fp2_t *r, const fp2_t *a, const fp2_t *b) { fp_add(&r->c0, &a->c0, &b->c0); fp_add(&r->c1, &a->c1, &b->c1); }
static void fp2_sub(fp2_t *r, const fp2_t *a, const fp2_t *b) { fp_sub(&r->c0, &a->c0, &b->c0); fp_sub(&r->c1, &a->c1, &b->c1); }
static void fp2_neg(fp2_t *r, const fp2_t *a) { fp_neg(&r->c0, &a->c0); fp_neg(&r->c1, &a->c1); }
static void fp2_conj(fp2_t *r, const fp2_t *a) { r->c0 = a->c0; fp_neg(&r->c1, &a->c1); }
static void fp2_mul(fp2_t *r, const fp2_t *a, const fp2_t *b) {
  fp_t t0, t1, t2, t3;
  fp_mul(&t0, &a->c0, &b->c0);
  fp_mul(&t1, &a->c1, &b->c1);
  fp_add(&t2, &a->c0, &a->c1);
  fp_add(&t3, &b->c0, &b->c1);
  fp_mul(&t2, &t2, &t3);
  fp_sub(&r->c0, &t0, &t1);
  fp_sub(&t2, &t2, &t0);
  fp_sub(&r->c1, &t2, &t1);
}
static void fp2_sqr(fp2_t *r, const fp2_t *a) { fp2_mul(r, a, a); }
static void fp2_mul_fp(fp2_t *r, const fp2_t *a, const fp_t *b) { fp_mul(&r->c0, &a->c0, b); fp_mul(&r->c1, &a->c1, b); }
static void fp2_mul_xi(fp2_t *r, const fp2_t *a) { /* (1+i) */
  fp_t t0, t1;
  fp_sub(&t0, &a->c0, &a->c1);
  fp_add(&t1, &a->c0, &a->c1);
  r->c0 = t0;
  r->c1 = t1;
}
static int fp2_is_zero(const fp2_t *a) { return fp_is_zero(&a->c0) && fp_is_zero(&a->c1); }
static int fp2_eq(const fp2_t *a, const fp2_t *b) { return fp_eq(&a->c0, &b->c0) && fp_eq(&a->c1, &b->c1); }
static void fp2_inv(fp2_t *r, const fp2_t *a) {
  fp_t n, t;
  fp_sqr(&n, &a->c0);
  fp_sqr(&t, &a->c1);
  fp_add(&n, &n, &t);
  fp_inv(&n, &n);
  fp_mul(&r->c0, &a->c0, &n);
  fp_mul(&t, &a->c1, &n);
  fp_neg(&r->c1, &t);
}
static void fp2_zero(fp2_t *r) { memset(r, 0, sizeof *r); }
static void fp2_one(fp2_t *r) { r->c0 = FP_ONE; memset(&r->c1, 0, sizeof r->c1); }
static int fp2_is_square(const fp2_t *a) {
  fp_t n, t;
  fp_sqr(&n, &a->c0);
  fp_sqr(&t, &a->c1);
  fp_add(&n, &n, &t);
  return fp_is_square(&n);
}
/* complex-method square root (mirrors oracle/bls_py.py f2sqrt) */
static int fp2_sqrt(fp2_t *r, const fp2_t *a) {
  fp_t inv2, two;
  fp_set_u64(&two, 2);
  fp_inv(&inv2, &two);
  if (fp_is_zero(&a->c1)) {
    fp_t s;
    if (fp_sqrt(&s, &a->c0)) { r->c0 = s; memset(&r->c1, 0, sizeof r->c1); return 1; }
    fp_t na;
    fp_neg(&na, &a->c0);
    if (!fp_sqrt(&s, &na)) return 0;
    memset(&r->c0, 0, sizeof r->c0);
    r->c1 = s;
    return 1;
  }
  fp_t n, t, s, d;
  fp_sqr(&n, &a->c0);
  fp_sqr(&t, &a->c1);
  fp_add(&n, &n, &t);
  if (!fp_sqrt(&d, &n)) return 0;
  fp_add(&t, &a->c0, &d);
  fp_mul(&t, &t, &inv2);
  if (!fp_sqrt(&s, &t)) {
    fp_sub(&t, &a->c0, &d);
    fp_mul(&t, &t, &inv2);
    if (!fp_sqrt(&s, &t)) return 0;
  }
  fp_t s2, is2;
  fp_add(&s2, &s, &s);
  fp_inv(&is2, &s2);
  r->c0 = s;
  fp_mul(&r->c1, &a->c1, &is2);
  fp2_t chk;
  fp2_sqr(&chk, r);
  return fp2_eq(&chk, a);
}
static int fp2_sgn0(const fp2_t *a) {
  uint64_t c0[6], c1[6];
  fp_canon(c0, &a->c0);
  fp_canon(c1, &a->c1);
  int z0 = 1;
  for (int i = 0; i < 6; i++) z0 &= c0[i] == 0;
  return (int)((c0[0] & 1) | (z0 & (c1[0] & 1)));
}
static void fp2_pow(fp2_t *r, const fp2_t *a, const uint64_t *e, int nwords) {
  fp2_t acc, base = *a;
  fp2_one(&acc);
  for (int i = nwords * 64 - 1; i >= 0; i--) {
    fp2_sqr(&acc, &acc);
    if ((e[i >> 6] >> (i & 63)) & 1) fp2_mul(&acc, &acc, &base);
  }
  *r = acc;
}

/* ------------------------------------------------------------------ Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v) */
static fp2_t FROB6_C1[4], FROB6_C2[4], FROB12_C[4];
static void fp6_add(fp6_t *r, const fp6_t *a, const fp6_t *b) { fp2_add(&r->c0, &a->c0, &b->c0); fp2_add(&r->c1, &a->c1, &b->c1); fp2_add(&r->c2, &a->c2, &b->c2); }
static void fp6_sub(fp6_t *r, const fp6_t *a, const fp6_t *b) { fp2_sub(&r->c0, &a->c0, &b->c0); fp2_sub(&r->c1, &a->c1, &b->c1); fp2_sub(&r->c2, &a->c2, &b->c2); }
static void fp6_neg(fp6_t *r, const fp6_t *a) { fp2_neg(&r->c0, &a->c0); fp2_neg(&r->c1, &a->c1); fp2_neg(&r->c2, &a->c2); }
static void fp6_mul(fp6_t *r, const fp6_t *a, const fp6_t *b) {
  fp2_t t0, t1, t2, s0, s1, u0, u1, u2;
  fp2_mul(&t0, &a->c0, &b->c0);
  fp2_mul(&t1, &a->c1, &b->c1);
  fp2_mul(&t2, &a->c2, &b->c2);
  /* c0 = ((a1+a2)(b1+b2) - t1 - t2) xi + t0 */
  fp2_add(&s0, &a->c1, &a->c2);
  fp2_add(&s1, &b->c1, &b->c2);
  fp2_mul(&u0, &s0, &s1);
  fp2_sub(&u0, &u0, &t1);
  fp2_sub(&u0, &u0, &t2);
  fp2_mul_xi(&u0, &u0);
  fp2_add(&u0, &u0, &t0);
  /* c1 = (a0+a1)(b0+b1) - t0 - t1 + t2 xi */
  fp2_add(&s0, &a->c0, &a->c1);
  fp2_add(&s1, &b->c0, &b->c1);
  fp2_mul(&u1, &s0, &s1);
  fp2_sub(&u1, &u1, &t0);
  fp2_sub(&u1, &u1, &t1);
  fp2_mul_xi(&s0, &t2);
  fp2_add(&u1, &u1, &s0);
  /* c2 = (a0+a2)(b0+b2) - t0 - t2 + t1 */
  fp2_add(&s0, &a->c0, &a->c2);
  fp2_add(&s1, &b->c0, &b->c2);
  fp2_mul(&u2, &s0, &s1);
  fp2_sub(&u2, &u2, &t0);
  fp2_sub(&u2, &u2, &t2);
  fp2_add(&u2, &u2, &t1);
  r->c0 = u0; r->c1 = u1; r->c2 = u2;
}
static void fp6_mul_v(fp6_t *r, const fp6_t *a) { /* * v */
  fp2_t t;
  fp2_mul_xi(&t, &a->c2);
  r->c2 = a->c1;
  r->c1 = a->c0;
  r->c0 = t;
}
static void fp6_inv(fp6_t *r, const fp6_t *a) {
  fp2_t c0, c1, c2, t, t2;
  /* c0 = a0^2 - xi a1 a2 */
  fp2_sqr(&c0, &a->c0);
  fp2_mul(&t, &a->c1, &a->c2);
  fp2_mul_xi(&t, &t);
  fp2_sub(&c0, &c0, &t);
  /* c1 = xi a2^2 - a0 a1 */
  fp2_sqr(&c1, &a->c2);
  fp2_mul_xi(&c1, &c1);
  fp2_mul(&t, &a->c0, &a->c1);
  fp2_sub(&c1, &c1, &t);
  /* c2 = a1^2 - a0 a2 */
  fp2_sqr(&c2, &a->c1);
  fp2_mul(&t, &a->c0, &a->c2);
  fp2_sub(&c2, &c2, &t);
  /* t = a0 c0 + xi (a2 c1 + a1 c2) */
  fp2_mul(&t, &a->c2, &c1);
  fp2_mul(&t2, &a->c1, &c2);
  fp2_add(&t, &t, &t2);
  fp2_mul_xi(&t, &t);
  fp2_mul(&t2, &a->c0, &c0);
  fp2_add(&t, &t, &t2);
  fp2_inv(&t, &t);
  fp2_mul(&r->c0, &c0, &t);
  fp2_mul(&r->c1, &c1, &t);
  fp2_mul(&r->c2, &c2, &t);
}
static void fp6_frob(fp6_t *r, const fp6_t *a, int k) {
  fp2_t c0 = a->c0, c1 = a->c1, c2 = a->c2;
  if (k & 1) { fp2_conj(&c0, &c0); fp2_conj(&c1, &c1); fp2_conj(&c2, &c2); }
  fp2_mul(&c1, &c1, &FROB6_C1[k]);
  fp2_mul(&c2, &c2, &FROB6_C2[k]);
  r->c0 = c0; r->c1 = c1; r->c2 = c2;
}
static void fp12_one(fp12_t *r) { memset(r, 0, sizeof *r); r->c0.c0.c0 = FP_ONE; }
static int fp12_eq(const fp12_t *a, const fp12_t *b) { return memcmp(a, b, sizeof *a) == 0; }
static void fp12_mul(fp12_t *r, const fp12_t *a, const fp12_t *b) {
  fp6_t t0, t1, s0, s1;
  fp6_mul(&t0, &a->c0, &b->c0);
  fp6_mul(&t1, &a->c1, &b->c1);
  fp6_add(&s0, &a->c0, &a->c1);
  fp6_add(&s1, &b->c0, &b->c1);
  fp6_mul(&s0, &s0, &s1);
  fp6_sub(&s0, &s0, &t0);
  fp6_sub(&r->c1, &s0, &t1);
  fp6_mul_v(&t1, &t1);
  fp6_add(&r->c0, &t0, &t1);
}
static void fp12_sqr(fp12_t *r, const fp12_t *a) { fp12_mul(r, a, a); }
static void fp12_conj(fp12_t *r, const fp12_t *a) { r->c0 = a->c0; fp6_neg(&r->c1, &a->c1); }
static void fp12_inv(fp12_t *r, const fp12_t *a) {
  fp6_t t0, t1;
  fp6_mul(&t0, &a->c0, &a->c0);
  fp6_mul(&t1, &a->c1, &a->c1);
  fp6_mul_v(&t1, &t1);
  fp6_sub(&t0, &t0, &t1);
  fp6_inv(&t0, &t0);
  fp6_mul(&r->c0, &a->c0, &t0);
  fp6_mul(&t1, &a->c1, &t0);
  fp6_neg(&r->c1, &t1);
}
static void fp12_frob(fp12_t *r, const fp12_t *a, int k) {
  fp6_t c0, c1;
  fp6_frob(&c0, &a->c0, k);
  fp6_frob(&c1, &a->c1, k);
  fp2_mul(&c1.c0, &c1.c0, &FROB12_C[k]);
  fp2_mul(&c1.c1, &c1.c1, &FROB12_C[k]);
  fp2_mul(&c1.c2, &c1.c2, &FROB12_C[k]);
  r->c0 = c0;
  r->c1 = c1;
}
/* sparse multiply by a line l = (a at c0.c0, b at c0.c1, c at c1.c1) */
static void fp12_mul_line(fp12_t *f, const fp2_t *a, const fp2_t *b, const fp2_t *c) {
  fp12_t l;
  memset(&l, 0, sizeof l);
  l.c0.c0 = *a;
  l.c0.c1 = *b;
  l.c1.c1 = *c;
  fp12_mul(f, f, &l);
}

/* ------------------------------------------------------------------ curve constants */
static fp_t B1, G1X, G1Y, BETA;
static fp2_t B2, G2X, G2Y, PSI_X, PSI_Y;
static fp_t SSWU1_A, SSWU1_B, SSWU1_Z;
static fp2_t SSWU2_A, SSWU2_B, SSWU2_Z;
static fp_t ISO11[4][16];
static int ISO11_N[4] = {12, 11, 16, 16};
static fp2_t ISO3[4][4];
static int ISO3_N[4] = {4, 3, 4, 4};
static uint64_t H_EFF2[10];
static const uint64_t U_ABS = 0xd201000000010000ULL;

/* ------------------------------------------------------------------ G1 (Jacobian, a = 0) */
static int g1_is_inf(const g1_t *p) { return fp_is_zero(&p->z); }
static void g1_set_inf(g1_t *p) { memset(p, 0, sizeof *p); p->x = FP_ONE; p->y = FP_ONE; }
static void g1_dbl(g1_t *r, const g1_t *p) {
  if (g1_is_inf(p)) { *r = *p; return; }
  fp_t a, b, c, d, e, f, t;
  fp_sqr(&a, &p->x);
  fp_sqr(&b, &p->y);
  fp_sqr(&c, &b);
  fp_add(&t, &p->x, &b);
  fp_sqr(&t, &t);
  fp_sub(&t, &t, &a);
  fp_sub(&t, &t, &c);
  fp_add(&d, &t, &t);
  fp_add(&e, &a, &a);
  fp_add(&e, &e, &a);
  fp_sqr(&f, &e);
  fp_t x3, y3, z3;
  fp_add(&t, &d, &d);
  fp_sub(&x3, &f, &t);
  fp_sub(&t, &d, &x3);
  fp_mul(&y3, &e, &t);
  fp_add(&c, &c, &c);
  fp_add(&c, &c, &c);
  fp_add(&c, &c, &c);
  fp_sub(&y3, &y3, &c);
  fp_mul(&z3, &p->y, &p->z);
  fp_add(&z3, &z3, &z3);
  r->x = x3; r->y = y3; r->z = z3;
}
static void g1_add(g1_t *r, const g1_t *p, const g1_t *q) {
  if (g1_is_inf(p)) { *r = *q; return; }
  if (g1_is_inf(q)) { *r = *p; return; }
  fp_t z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t;
  fp_sqr(&z1z1, &p->z);
  fp_sqr(&z2z2, &q->z);
  fp_mul(&u1, &p->x, &z2z2);
  fp_mul(&u2, &q->x, &z1z1);
  fp_mul(&s1, &p->y, &q->z);
  fp_mul(&s1, &s1, &z2z2);
  fp_mul(&s2, &q->y, &p->z);
  fp_mul(&s2, &s2, &z1z1);
  if (fp_eq(&u1, &u2)) {
    if (fp_eq(&s1, &s2)) { g1_dbl(r, p); return; }
    g1_set_inf(r);
    r->z = (fp_t){{0}};
    return;
  }
  fp_sub(&h, &u2, &u1);
  fp_add(&i, &h, &h);
  fp_sqr(&i, &i);
  fp_mul(&j, &h, &i);
  fp_sub(&rr, &s2, &s1);
  fp_add(&rr, &rr, &rr);
  fp_mul(&v, &u1, &i);
  fp_t x3, y3, z3;
  fp_sqr(&x3, &rr);
  fp_sub(&x3, &x3, &j);
  fp_sub(&x3, &x3, &v);
  fp_sub(&x3, &x3, &v);
  fp_sub(&t, &v, &x3);
  fp_mul(&y3, &rr, &t);
  fp_mul(&t, &s1, &j);
  fp_add(&t, &t, &t);
  fp_sub(&y3, &y3, &t);
  fp_add(&z3, &p->z, &q->z);
  fp_sqr(&z3, &z3);
  fp_sub(&z3, &z3, &z1z1);
  fp_sub(&z3, &z3, &z2z2);
  fp_mul(&z3, &z3, &h);
  r->x = x3; r->y = y3; r->z = z3;
}
static void g1_neg(g1_t *r, const g1_t *p) { *r = *p; fp_neg(&r->y, &p->y); }
static void g1_mul(g1_t *r, const g1_t *p, const uint64_t *k, int nwords) {
  g1_t acc, base = *p;
  g1_set_inf(&acc);
  acc.z = (fp_t){{0}};
  for (int i = nwords * 64 - 1; i >= 0; i--) {
    g1_dbl(&acc, &acc);
    if ((k[i >> 6] >> (i & 63)) & 1) g1_add(&acc, &acc, &base);
  }
  *r = acc;
}
static void g1_affine(fp_t *x, fp_t *y, const g1_t *p) {
  fp_t zi, zi2;
  fp_inv(&zi, &p->z);
  fp_sqr(&zi2, &zi);
  fp_mul(x, &p->x, &zi2);
  fp_mul(&zi2, &zi2, &zi);
  fp_mul(y, &p->y, &zi2);
}
static int g1_eq(const g1_t *a, const g1_t *b) {
  if (g1_is_inf(a) || g1_is_inf(b)) return g1_is_inf(a) && g1_is_inf(b);
  fp_t z1, z2, t1, t2;
  fp_sqr(&z1, &a->z);
  fp_sqr(&z2, &b->z);
  fp_mul(&t1, &a->x, &z2);
  fp_mul(&t2, &b->x, &z1);
  if (!fp_eq(&t1, &t2)) return 0;
  fp_mul(&z1, &z1, &a->z);
  fp_mul(&z2, &z2, &b->z);
  fp_mul(&t1, &a->y, &z2);
  fp_mul(&t2, &b->y, &z1);
  return fp_eq(&t1, &t2);
}
/* subgroup check: faithful = r * P == O (kilic InCorrectSubgroup); fast = phi(P) == [-u^2] P */
static int g_fast_subgroup = 0;
static int g1_in_subgroup(const g1_t *p) {
  if (!g_fast_subgroup) {
    g1_t t;
    g1_mul(&t, p, RSC, 4);
    return g1_is_inf(&t);
  }
  g1_t t, phi = *p;
  uint64_t uu = U_ABS;
  g1_mul(&t, p, &uu, 1);
  g1_mul(&t, &t, &uu, 1); /* [u^2] P */
  g1_neg(&t, &t);
  fp_mul(&phi.x, &phi.x, &BETA);
  return g1_eq(&phi, &t);
}

/* ------------------------------------------------------------------ G2 (Jacobian over Fp2) */
static int g2_is_inf(const g2_t *p) { return fp2_is_zero(&p->z); }
static void g2_set_inf(g2_t *p) { memset(p, 0, sizeof *p); fp2_one(&p->x); fp2_one(&p->y); }
static void g2_dbl(g2_t *r, const g2_t *p) {
  if (g2_is_inf(p)) { *r = *p; return; }
  fp2_t a, b, c, d, e, f, t;
  fp2_sqr(&a, &p->x);
  fp2_sqr(&b, &p->y);
  fp2_sqr(&c, &b);
  fp2_add(&t, &p->x, &b);
  fp2_sqr(&t, &t);
  fp2_sub(&t, &t, &a);
  fp2_sub(&t, &t, &c);
  fp2_add(&d, &t, &t);
  fp2_add(&e, &a, &a);
  fp2_add(&e, &e, &a);
  fp2_sqr(&f, &e);
  fp2_t x3, y3, z3;
  fp2_add(&t, &d, &d);
  fp2_sub(&x3, &f, &t);
  fp2_sub(&t, &d, &x3);
  fp2_mul(&y3, &e, &t);
  fp2_add(&c, &c, &c);
  fp2_add(&c, &c, &c);
  fp2_add(&c, &c, &c);
  fp2_sub(&y3, &y3, &c);
  fp2_mul(&z3, &p->y, &p->z);
  fp2_add(&z3, &z3, &z3);
  r->x = x3; r->y = y3; r->z = z3;
}
static void g2_add(g2_t *r, const g2_t *p, const g2_t *q) {
  if (g2_is_inf(p)) { *r = *q; return; }
  if (g2_is_inf(q)) { *r = *p; return; }
  fp2_t z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t;
  fp2_sqr(&z1z1, &p->z);
  fp2_sqr(&z2z2, &q->z);
  fp2_mul(&u1, &p->x, &z2z2);
  fp2_mul(&u2, &q->x, &z1z1);
  fp2_mul(&s1, &p->y, &q->z);
  fp2_mul(&s1, &s1, &z2z2);
  fp2_mul(&s2, &q->y, &p->z);
  fp2_mul(&s2, &s2, &z1z1);
  if (fp2_eq(&u1, &u2)) {
    if (fp2_eq(&s1, &s2)) { g2_dbl(r, p); return; }
    g2_set_inf(r);
    fp2_zero(&r->z);
    return;
  }
  fp2_sub(&h, &u2, &u1);
  fp2_add(&i, &h, &h);
  fp2_sqr(&i, &i);
  fp2_mul(&j, &h, &i);
  fp2_sub(&rr, &s2, &s1);
  fp2_add(&rr, &rr, &rr);
  fp2_mul(&v, &u1, &i);
  fp2_t x3, y3, z3;
  fp2_sqr(&x3, &rr);
  fp2_sub(&x3, &x3, &j);
  fp2_sub(&x3, &x3, &v);
  fp2_sub(&x3, &x3, &v);
  fp2_sub(&t, &v, &x3);
  fp2_mul(&y3, &rr, &t);
  fp2_mul(&t, &s1, &j);
  fp2_add(&t, &t, &t);
  fp2_sub(&y3, &y3, &t);
  fp2_add(&z3, &p->z, &q->z);
  fp2_sqr(&z3, &z3);
  fp2_sub(&z3, &z3, &z1z1);
  fp2_sub(&z3, &z3, &z2z2);
  fp2_mul(&z3, &z3, &h);
  r->x = x3; r->y = y3; r->z = z3;
}
static void g2_neg(g2_t *r, const g2_t *p) { *r = *p; fp2_neg(&r->y, &p->y); }
static void g2_mul(g2_t *r, const g2_t *p, const uint64_t *k, int nwords) {
  g2_t acc, base = *p;
  g2_set_inf(&acc);
  fp2_zero(&acc.z);
  for (int i = nwords * 64 - 1; i >= 0; i--) {
    g2_dbl(&acc, &acc);
    if ((k[i >> 6] >> (i & 63)) & 1) g2_add(&acc, &acc, &base);
  }
  *r = acc;
}
static void g2_affine(fp2_t *x, fp2_t *y, const g2_t *p) {
  fp2_t zi, zi2;
  fp2_inv(&zi, &p->z);
  fp2_sqr(&zi2, &zi);
  fp2_mul(x, &p->x, &zi2);
  fp2_mul(&zi2, &zi2, &zi);
  fp2_mul(y, &p->y, &zi2);
}
static int g2_eq(const g2_t *a, const g2_t *b) {
  if (g2_is_inf(a) || g2_is_inf(b)) return g2_is_inf(a) && g2_is_inf(b);
  fp2_t z1, z2, t1, t2;
  fp2_sqr(&z1, &a->z);
  fp2_sqr(&z2, &b->z);
  fp2_mul(&t1, &a->x, &z2);
  fp2_mul(&t2, &b->x, &z1);
  if (!fp2_eq(&t1, &t2)) return 0;
  fp2_mul(&z1, &z1, &a->z);
  fp2_mul(&z2, &z2, &b->z);
  fp2_mul(&t1, &a->y, &z2);
  fp2_mul(&t2, &b->y, &z1);
  return fp2_eq(&t1, &t2);
}
static void g2_psi(g2_t *r, const g2_t *p) { /* Jacobian: psi acts coordinate-wise, z conj */
  g2_t t;
  fp2_conj(&t.x, &p->x);
  fp2_conj(&t.y, &p->y);
  fp2_conj(&t.z, &p->z);
  fp2_mul(&t.x, &t.x, &PSI_X);
  fp2_mul(&t.y, &t.y, &PSI_Y);
  *r = t;
}
static int g2_in_subgroup(const g2_t *p) {
  if (!g_fast_subgroup) {
    g2_t t;
    g2_mul(&t, p, RSC, 4);
    return g2_is_inf(&t);
  }
  g2_t t, s;
  uint64_t uu = U_ABS;
  g2_mul(&t, p, &uu, 1);
  g2_neg(&t, &t); /* [u] P */
  g2_psi(&s, p);
  return g2_eq(&s, &t);
}

/* ------------------------------------------------------------------ ZCash codec */
static int g1_decompress(g1_t *out, const uint8_t *b) {
  uint8_t flags = b[0];
  if (!(flags & 0x80)) return 0;
  if (flags & 0x40) {
    if (flags & 0x3f) return 0;
    for (int i = 1; i < 48; i++) if (b[i]) return 0;
    g1_set_inf(out);
    fp_t z; memset(&z, 0, sizeof z); out->z = z;
    return 2; /* infinity */
  }
  uint8_t tmp[48];
  memcpy(tmp, b, 48);
  tmp[0] &= 0x1f;
  uint64_t x[6];
  be48_to_u64s(x, tmp);
  if (!lt_p(x)) return 0;
  fp_t X, Y, rhs;
  fp_from_u64s(&X, x);
  fp_sqr(&rhs, &X);
  fp_mul(&rhs, &rhs, &X);
  fp_add(&rhs, &rhs, &B1);
  if (!fp_sqrt(&Y, &rhs)) return 0;
  uint64_t yc[6];
  fp_canon(yc, &Y);
  if (canon_gt_half(yc) != !!(flags & 0x20)) fp_neg(&Y, &Y);
  out->x = X; out->y = Y; out->z = FP_ONE;
  if (!g1_in_subgroup(out)) return 0;
  return 1;
}
static void g1_compress(uint8_t *b, const g1_t *p) {
  if (g1_is_inf(p)) { memset(b, 0, 48); b[0] = 0xc0; return; }
  fp_t x, y;
  g1_affine(&x, &y, p);
  uint64_t xc[6], yc[6];
  fp_canon(xc, &x);
  fp_canon(yc, &y);
  u64s_to_be48(b, xc);
  b[0] |= 0x80;
  if (canon_gt_half(yc)) b[0] |= 0x20;
}
static int fp2_lex_largest(const fp2_t *y) {
  uint64_t c0[6], c1[6];
  fp_canon(c0, &y->c0);
  fp_canon(c1, &y->c1);
  int z1 = 1;
  for (int i = 0; i < 6; i++) z1 &= c1[i] == 0;
  if (!z1) return canon_gt_half(c1);
  return canon_gt_half(c0);
}
static int g2_decompress(g2_t *out, const uint8_t *b) {
  uint8_t flags = b[0];
  if (!(flags & 0x80)) return 0;
  if (flags & 0x40) {
    if (flags & 0x3f) return 0;
    for (int i = 1; i < 96; i++) if (b[i]) return 0;
    g2_set_inf(out);
    fp2_zero(&out->z);
    return 2;
  }
  uint8_t tmp[48];
  memcpy(tmp, b, 48);
  tmp[0] &= 0x1f;
  uint64_t x1[6], x0[6];
  be48_to_u64s(x1, tmp);
  be48_to_u64s(x0, b + 48);
  if (!lt_p(x0) || !lt_p(x1)) return 0;
  fp2_t X, Y, rhs;
  fp_from_u64s(&X.c0, x0);
  fp_from_u64s(&X.c1, x1);
  fp2_sqr(&rhs, &X);
  fp2_mul(&rhs, &rhs, &X);
  fp2_add(&rhs, &rhs, &B2);
  if (!fp2_sqrt(&Y, &rhs)) return 0;
  if (fp2_lex_largest(&Y) != !!(flags & 0x20)) fp2_neg(&Y, &Y);
  out->x = X; out->y = Y; fp2_one(&out->z);
  if (!g2_in_subgroup(out)) return 0;
  return 1;
}
static void g2_compress(uint8_t *b, const g2_t *p) {
  if (g2_is_inf(p)) { memset(b, 0, 96); b[0] = 0xc0; return; }
  fp2_t x, y;
  g2_affine(&x, &y, p);
  uint64_t c0[6], c1[6];
  fp_canon(c0, &x.c0);
  fp_canon(c1, &x.c1);
  u64s_to_be48(b, c1);
  u64s_to_be48(b + 48, c0);
  b[0] |= 0x80;
  if (fp2_lex_largest(&y)) b[0] |= 0x20;
}

/* ------------------------------------------------------------------ SHA-256 (FIPS 180-4) */
typedef struct { uint32_t h[8]; uint8_t buf[64]; uint64_t len; int n; } sha_t;
static const uint32_t KSHA[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98,
    0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
    0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8,
    0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
    0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819,
    0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
    0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};
#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void sha_block(uint32_t *h, const uint8_t *p) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++) w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; i++) {
    uint32_t t1 = hh + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + KSHA[i] + w[i];
    uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}
static void sha_init(sha_t *s) {
  static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memcpy(s->h, iv, 32);
  s->len = 0;
  s->n = 0;
}
static void sha_update(sha_t *s, const uint8_t *d, size_t n) {
  s->len += n;
  while (n) {
    size_t k = 64 - s->n;
    if (k > n) k = n;
    memcpy(s->buf + s->n, d, k);
    s->n += (int)k;
    d += k;
    n -= k;
    if (s->n == 64) { sha_block(s->h, s->buf); s->n = 0; }
  }
}
static void sha_final(sha_t *s, uint8_t *out) {
  uint64_t bits = s->len * 8;
  uint8_t pad = 0x80;
  sha_update(s, &pad, 1);
  uint8_t z = 0;
  while (s->n != 56) sha_update(s, &z, 1);
  uint8_t l[8];
  for (int i = 0; i < 8; i++) l[i] = (uint8_t)(bits >> (56 - 8 * i));
  sha_update(s, l, 8);
  for (int i = 0; i < 8; i++) {
    out[4 * i] = s->h[i] >> 24; out[4 * i + 1] = s->h[i] >> 16; out[4 * i + 2] = s->h[i] >> 8; out[4 * i + 3] = s->h[i];
  }
}
void or_sha256(uint8_t *out, const uint8_t *d, size_t n) {
  sha_t s;
  sha_init(&s);
  sha_update(&s, d, n);
  sha_final(&s, out);
}

/* ------------------------------------------------------------------ hash to curve (RFC 9380) */
void or_expand_message_xmd(uint8_t *out, size_t len, const uint8_t *msg, size_t mlen, const uint8_t *dst, size_t dlen) {
  size_t ell = (len + 31) / 32;
  uint8_t zpad[64] = {0}, b0[32], bi[32], lib[2] = {(uint8_t)(len >> 8), (uint8_t)len}, zero = 0, dl = (uint8_t)dlen;
  sha_t s;
  sha_init(&s);
  sha_update(&s, zpad, 64);
  sha_update(&s, msg, mlen);
  sha_update(&s, lib, 2);
  sha_update(&s, &zero, 1);
  sha_update(&s, dst, dlen);
  sha_update(&s, &dl, 1);
  sha_final(&s, b0);
  uint8_t prev[32];
  memset(prev, 0, 32);
  for (size_t i = 1; i <= ell; i++) {
    uint8_t x[32], ic = (uint8_t)i;
    for (int k = 0; k < 32; k++) x[k] = (i == 1) ? b0[k] : (uint8_t)(b0[k] ^ prev[k]);
    sha_init(&s);
    sha_update(&s, x, 32);
    sha_update(&s, &ic, 1);
    sha_update(&s, dst, dlen);
    sha_update(&s, &dl, 1);
    sha_final(&s, bi);
    size_t off = (i - 1) * 32, k = len - off < 32 ? len - off : 32;
    memcpy(out + off, bi, k);
    memcpy(prev, bi, 32);
  }
}
static fp_t K2_256; /* 2^256 mod p in Montgomery form */
static void fp_from_be64(fp_t *r, const uint8_t *b) { /* 64 big-endian bytes -> Fp (mod p) */
  uint64_t hi[6] = {0}, lo[6] = {0};
  for (int i = 0; i < 4; i++) {
    uint64_t v = 0, w = 0;
    for (int k = 0; k < 8; k++) {
      v = (v << 8) | b[24 - 8 * i + k];
      w = (w << 8) | b[56 - 8 * i + k];
    }
    hi[i] = v;
    lo[i] = w;
  }
  fp_t H, L;
  fp_from_u64s(&H, hi);
  fp_from_u64s(&L, lo);
  fp_mul(&H, &H, &K2_256);
  fp_add(r, &H, &L);
}
static void sswu1(fp_t *xo, fp_t *yo, const fp_t *u) {
  fp_t tv1, x1, gx1, x, y, t, u2;
  fp_sqr(&u2, u);
  fp_t zu2; fp_mul(&zu2, &SSWU1_Z, &u2);
  fp_sqr(&tv1, &zu2);
  fp_add(&tv1, &tv1, &zu2); /* Z^2 u^4 + Z u^2 */
  if (fp_is_zero(&tv1)) {
    fp_mul(&t, &SSWU1_Z, &SSWU1_A);
    fp_inv(&t, &t);
    fp_mul(&x1, &SSWU1_B, &t);
  } else {
    fp_inv(&t, &tv1);
    fp_add(&t, &t, &FP_ONE);
    fp_t nba; fp_inv(&nba, &SSWU1_A); fp_mul(&nba, &nba, &SSWU1_B); fp_neg(&nba, &nba);
    fp_mul(&x1, &nba, &t);
  }
  fp_sqr(&gx1, &x1); fp_add(&gx1, &gx1, &SSWU1_A); fp_mul(&gx1, &gx1, &x1); fp_add(&gx1, &gx1, &SSWU1_B);
  if (fp_is_square(&gx1)) { x = x1; fp_sqrt(&y, &gx1); }
  else {
    fp_t x2, gx2;
    fp_mul(&x2, &zu2, &x1);
    fp_sqr(&gx2, &x2); fp_add(&gx2, &gx2, &SSWU1_A); fp_mul(&gx2, &gx2, &x2); fp_add(&gx2, &gx2, &SSWU1_B);
    x = x2; fp_sqrt(&y, &gx2);
  }
  if (fp_sgn0(u) != fp_sgn0(&y)) fp_neg(&y, &y);
  *xo = x; *yo = y;
}
static void sswu2(fp2_t *xo, fp2_t *yo, const fp2_t *u) {
  fp2_t tv1, x1, gx1, x, y, t, u2, zu2;
  fp2_sqr(&u2, u);
  fp2_mul(&zu2, &SSWU2_Z, &u2);
  fp2_sqr(&tv1, &zu2);
  fp2_add(&tv1, &tv1, &zu2);
  if (fp2_is_zero(&tv1)) {
    fp2_mul(&t, &SSWU2_Z, &SSWU2_A);
    fp2_inv(&t, &t);
    fp2_mul(&x1, &SSWU2_B, &t);
  } else {
    fp2_inv(&t, &tv1);
    fp2_t one; fp2_one(&one);
    fp2_add(&t, &t, &one);
    fp2_t nba; fp2_inv(&nba, &SSWU2_A); fp2_mul(&nba, &nba, &SSWU2_B); fp2_neg(&nba, &nba);
    fp2_mul(&x1, &nba, &t);
  }
  fp2_sqr(&gx1, &x1); fp2_add(&gx1, &gx1, &SSWU2_A); fp2_mul(&gx1, &gx1, &x1); fp2_add(&gx1, &gx1, &SSWU2_B);
  if (fp2_is_square(&gx1)) { x = x1; fp2_sqrt(&y, &gx1); }
  else {
    fp2_t x2, gx2;
    fp2_mul(&x2, &zu2, &x1);
    fp2_sqr(&gx2, &x2); fp2_add(&gx2, &gx2, &SSWU2_A); fp2_mul(&gx2, &gx2, &x2); fp2_add(&gx2, &gx2, &SSWU2_B);
    x = x2; fp2_sqrt(&y, &gx2);
  }
  if (fp2_sgn0(u) != fp2_sgn0(&y)) fp2_neg(&y, &y);
  *xo = x; *yo = y;
}
static void iso11(g1_t *out, const fp_t *x, const fp_t *y) {
  fp_t v[4];
  for (int k = 0; k < 4; k++) {
    fp_t acc; memset(&acc, 0, sizeof acc);
    for (int i = ISO11_N[k] - 1; i >= 0; i--) { fp_mul(&acc, &acc, x); fp_add(&acc, &acc, &ISO11[k][i]); }
    v[k] = acc;
  }
  /* affine: X = xn/xd, Y = y yn/yd ; Jacobian with Z = xd*yd */
  fp_t Z, Z2, t;
  fp_mul(&Z, &v[1], &v[3]);
  fp_sqr(&Z2, &Z);
  fp_mul(&out->x, &v[0], &v[3]);
  fp_mul(&out->x, &out->x, &Z); /* xn/xd * Z^2 = xn * xd * yd^2 -> xn * yd * Z */
  fp_mul(&t, y, &v[2]);
  fp_mul(&t, &t, &Z2);
  fp_mul(&out->y, &t, &v[1]); /* y yn/yd * Z^3 = y yn xd^3 yd^2 = y yn Z^2 xd */
  out->z = Z;
}
static void iso3(g2_t *out, const fp2_t *x, const fp2_t *y) {
  fp2_t v[4];
  for (int k = 0; k < 4; k++) {
    fp2_t acc; fp2_zero(&acc);
    for (int i = ISO3_N[k] - 1; i >= 0; i--) { fp2_mul(&acc, &acc, x); fp2_add(&acc, &acc, &ISO3[k][i]); }
    v[k] = acc;
  }
  fp2_t Z, Z2, t;
  fp2_mul(&Z, &v[1], &v[3]);
  fp2_sqr(&Z2, &Z);
  fp2_mul(&out->x, &v[0], &v[3]);
  fp2_mul(&out->x, &out->x, &Z);
  fp2_mul(&t, y, &v[2]);
  fp2_mul(&t, &t, &Z2);
  fp2_mul(&out->y, &t, &v[1]);
  out->z = Z;
}
static void hash_to_g1(g1_t *out, const uint8_t *msg, size_t mlen, const uint8_t *dst, size_t dlen) {
  uint8_t u[128];
  or_expand_message_xmd(u, 128, msg, mlen, dst, dlen);
  fp_t u0, u1, x, y;
  fp_from_be64(&u0, u);
  fp_from_be64(&u1, u + 64);
  g1_t q0, q1;
  sswu1(&x, &y, &u0);
  iso11(&q0, &x, &y);
  sswu1(&x, &y, &u1);
  iso11(&q1, &x, &y);
  g1_add(&q0, &q0, &q1);
  uint64_t h = 0xd201000000010001ULL;
  g1_mul(out, &q0, &h, 1);
}
static void hash_to_g2(g2_t *out, const uint8_t *msg, size_t mlen, const uint8_t *dst, size_t dlen) {
  uint8_t u[256];
  or_expand_message_xmd(u, 256, msg, mlen, dst, dlen);
  fp2_t u0, u1, x, y;
  fp_from_be64(&u0.c0, u);
  fp_from_be64(&u0.c1, u + 64);
  fp_from_be64(&u1.c0, u + 128);
  fp_from_be64(&u1.c1, u + 192);
  g2_t q0, q1;
  sswu2(&x, &y, &u0);
  iso3(&q0, &x, &y);
  sswu2(&x, &y, &u1);
  iso3(&q1, &x, &y);
  g2_add(&q0, &q0, &q1);
  g2_mul(out, &q0, H_EFF2, 10);
}

/* ------------------------------------------------------------------ pairing (optimal ate, M-twist) */
/* Line formulas after Costello-Lange-Naehrig (eprint 2010/354, Alg. 26/27) on a homogeneous-Jacobian G2 point. */
static void dbl_step(g2_t *r, fp2_t *c0, fp2_t *c1, fp2_t *c2) {
  fp2_t t0, t1, t2, t3, t4, t5, t6, zz;
  fp2_sqr(&t0, &r->x);
  fp2_sqr(&t1, &r->y);
  fp2_sqr(&t2, &t1);
  fp2_add(&t3, &t1, &r->x); fp2_sqr(&t3, &t3); fp2_sub(&t3, &t3, &t0); fp2_sub(&t3, &t3, &t2); fp2_add(&t3, &t3, &t3);
  fp2_add(&t4, &t0, &t0); fp2_add(&t4, &t4, &t0);
  fp2_add(&t6, &r->x, &t4);
  fp2_sqr(&t5, &t4);
  fp2_sqr(&zz, &r->z);
  fp2_t nx, ny, nz;
  fp2_sub(&nx, &t5, &t3); fp2_sub(&nx, &nx, &t3);
  fp2_add(&nz, &r->z, &r->y); fp2_sqr(&nz, &nz); fp2_sub(&nz, &nz, &t1); fp2_sub(&nz, &nz, &zz);
  fp2_sub(&ny, &t3, &nx); fp2_mul(&ny, &ny, &t4);
  fp2_add(&t2, &t2, &t2); fp2_add(&t2, &t2, &t2); fp2_add(&t2, &t2, &t2);
  fp2_sub(&ny, &ny, &t2);
  fp2_mul(&t3, &t4, &zz); fp2_add(&t3, &t3, &t3); fp2_neg(&t3, &t3);
  fp2_sqr(&t6, &t6); fp2_sub(&t6, &t6, &t0); fp2_sub(&t6, &t6, &t5);
  fp2_add(&t1, &t1, &t1); fp2_add(&t1, &t1, &t1);
  fp2_sub(&t6, &t6, &t1);
  fp2_mul(&t0, &nz, &zz); fp2_add(&t0, &t0, &t0);
  r->x = nx; r->y = ny; r->z = nz;
  *c0 = t0; *c1 = t3; *c2 = t6;
}
static void add_step(g2_t *r, const fp2_t *qx, const fp2_t *qy, fp2_t *c0, fp2_t *c1, fp2_t *c2) {
  fp2_t zz, yy, t0, t1, t2, t3, t4, t5, t6, t7, t8, t9, t10;
  fp2_sqr(&zz, &r->z);
  fp2_sqr(&yy, qy);
  fp2_mul(&t0, &zz, qx);
  fp2_add(&t1, qy, &r->z); fp2_sqr(&t1, &t1); fp2_sub(&t1, &t1, &yy); fp2_sub(&t1, &t1, &zz); fp2_mul(&t1, &t1, &zz);
  fp2_sub(&t2, &t0, &r->x);
  fp2_sqr(&t3, &t2);
  fp2_add(&t4, &t3, &t3); fp2_add(&t4, &t4, &t4);
  fp2_mul(&t5, &t4, &t2);
  fp2_sub(&t6, &t1, &r->y); fp2_sub(&t6, &t6, &r->y);
  fp2_mul(&t9, &t6, qx);
  fp2_mul(&t7, &t4, &r->x);
  fp2_t nx, ny, nz;
  fp2_sqr(&nx, &t6); fp2_sub(&nx, &nx, &t5); fp2_sub(&nx, &nx, &t7); fp2_sub(&nx, &nx, &t7);
  fp2_add(&nz, &r->z, &t2); fp2_sqr(&nz, &nz); fp2_sub(&nz, &nz, &zz); fp2_sub(&nz, &nz, &t3);
  fp2_add(&t10, qy, &nz);
  fp2_sub(&t8, &t7, &nx); fp2_mul(&t8, &t8, &t6);
  fp2_mul(&t0, &r->y, &t5); fp2_add(&t0, &t0, &t0);
  fp2_sub(&ny, &t8, &t0);
  fp2_sqr(&t10, &t10); fp2_sub(&t10, &t10, &yy);
  fp2_t zt; fp2_sqr(&zt, &nz);
  fp2_sub(&t10, &t10, &zt);
  fp2_add(&t9, &t9, &t9); fp2_sub(&t9, &t9, &t10);
  fp2_add(&t10, &nz, &nz);
  fp2_neg(&t6, &t6);
  fp2_add(&t1, &t6, &t6);
  r->x = nx; r->y = ny; r->z = nz;
  *c0 = t10; *c1 = t1; *c2 = t9;
}
/* f *= line(c0,c1,c2) evaluated at affine P = (px, py):  (c2) + (c1*px) v + (c0*py) v w  in positions 0,1,4 */
static void ell(fp12_t *f, const fp2_t *c0, const fp2_t *c1, const fp2_t *c2, const fp_t *px, const fp_t *py) {
  fp2_t a = *c2, b, c;
  fp2_mul_fp(&b, c1, px);
  fp2_mul_fp(&c, c0, py);
  fp12_mul_line(f, &a, &b, &c);
}
/* multi Miller loop over n pairs (P_i affine G1, Q_i affine G2); skips pairs with an infinity */
static void miller_loop(fp12_t *f, int n, const fp_t *px, const fp_t *py, const fp2_t *qx, const fp2_t *qy, const int *skip) {
  g2_t T[8];
  fp12_one(f);
  for (int k = 0; k < n; k++) { T[k].x = qx[k]; T[k].y = qy[k]; fp2_one(&T[k].z); }
  int started = 0;
  for (int b = 62; b >= 0; b--) {
    if (started) fp12_sqr(f, f);
    started = 1;
    for (int k = 0; k < n; k++) {
      if (skip[k]) continue;
      fp2_t c0, c1, c2;
      dbl_step(&T[k], &c0, &c1, &c2);
      ell(f, &c0, &c1, &c2, &px[k], &py[k]);
    }
    if ((U_ABS >> b) & 1) {
      for (int k = 0; k < n; k++) {
        if (skip[k]) continue;
        fp2_t c0, c1, c2;
        add_step(&T[k], &qx[k], &qy[k], &c0, &c1, &c2);
        ell(f, &c0, &c1, &c2, &px[k], &py[k]);
      }
    }
  }
  fp12_conj(f, f); /* u < 0 */
}
static void cyc_exp_u(fp12_t *r, const fp12_t *a) { /* a^u, u negative: conj(a^|u|) */
  fp12_t acc = *a;
  for (int b = 62; b >= 0; b--) {
    fp12_sqr(&acc, &acc);
    if ((U_ABS >> b) & 1) fp12_mul(&acc, &acc, a);
  }
  fp12_conj(r, &acc);
}
static void final_exp(fp12_t *r, const fp12_t *f) {
  fp12_t t0, t1, a, b, c, d, e, t;
  /* easy part: f^(p^6-1)(p^2+1) */
  fp12_conj(&t0, f);
  fp12_inv(&t1, f);
  fp12_mul(&t0, &t0, &t1);
  fp12_frob(&t1, &t0, 2);
  fp12_mul(&t0, &t0, &t1);
  /* hard part, 3(p^4-p^2+1)/r = l0 + l1 p + l2 p^2 + l3 p^3 with l3=(u-1)^2, l2=l3 u, l1=l2 u - l3, l0=l1 u + 3 */
  cyc_exp_u(&a, &t0);
  fp12_conj(&t, &t0);
  fp12_mul(&a, &a, &t); /* f^(u-1) */
  cyc_exp_u(&b, &a);
  fp12_conj(&t, &a);
  fp12_mul(&b, &b, &t); /* f^(u-1)^2 = f^l3 */
  cyc_exp_u(&c, &b);    /* f^l2 */
  cyc_exp_u(&d, &c);
  fp12_conj(&t, &b);
  fp12_mul(&d, &d, &t); /* f^l1 */
  cyc_exp_u(&e, &d);
  fp12_sqr(&t, &t0);
  fp12_mul(&t, &t, &t0);
  fp12_mul(&e, &e, &t); /* f^l0 */
  fp12_frob(&t, &d, 1);
  fp12_mul(&e, &e, &t);
  fp12_frob(&t, &c, 2);
  fp12_mul(&e, &e, &t);
  fp12_frob(&t, &b, 3);
  fp12_mul(r, &e, &t);
}
/* prod e(P_i, Q_i) == 1 ? */
static int pairing_check(int n, const g1_t *P, const g2_t *Q) {
  fp_t px[8], py[8];
  fp2_t qx[8], qy[8];
  int skip[8];
  for (int k = 0; k < n; k++) {
    skip[k] = g1_is_inf(&P[k]) || g2_is_inf(&Q[k]);
    if (skip[k]) continue;
    g1_affine(&px[k], &py[k], &P[k]);
    g2_affine(&qx[k], &qy[k], &Q[k]);
  }
  fp12_t f, g, one;
  miller_loop(&f, n, px, py, qx, qy, skip);
  final_exp(&g, &f);
  fp12_one(&one);
  return fp12_eq(&g, &one);
}

/* ------------------------------------------------------------------ init */
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static void init_consts(void) {
  uint64_t one_raw[6] = {1, 0, 0, 0, 0, 0};
  /* R2 = 2^768 mod p by doubling, R mod p by doubling 2^0 384 times */
  fp_t t;
  memcpy(t.l, one_raw, 48);
  for (int i = 0; i < 768; i++) {
    u128 c = 0;
    uint64_t x[6];
    for (int k = 0; k < 6; k++) { c += (u128)t.l[k] * 2; x[k] = (uint64_t)c; c >>= 64; }
    memcpy(t.l, x, 48);
    if (geq_p(t.l)) sub_p(t.l);
    if (i == 383) FP_ONE = t;
  }
  FP_R2 = t;
  /* exponents */
  u128 br = 0;
  for (int i = 0; i < 6; i++) { u128 d = (u128)P[i] - (i == 0 ? 2 : 0) - br; E_PM2[i] = (uint64_t)d; br = (d >> 64) & 1; }
  /* (p+1)/4 and (p-1)/2 */
  uint64_t pp1[6];
  u128 c = 1;
  for (int i = 0; i < 6; i++) { c += P[i]; pp1[i] = (uint64_t)c; c >>= 64; }
  for (int i = 0; i < 6; i++) E_SQRT[i] = (pp1[i] >> 2) | (i < 5 ? pp1[i + 1] << 62 : 0);
  for (int i = 0; i < 6; i++) E_LEG[i] = (P[i] >> 1) | (i < 5 ? P[i + 1] << 63 : 0);
  fp_set_u64(&B1, 4);
  B2.c0 = B1; B2.c1 = B1;
  fp_from_hex(&G1X, "17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb");
  fp_from_hex(&G1Y, "08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1");
  fp_from_hex(&G2X.c0, "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8");
  fp_from_hex(&G2X.c1, "13e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e");
  fp_from_hex(&G2Y.c0, "0ce5d527727d6e118cc9cdc6da2e351aadfd9baa8cbdd3a76d429a695160d12c923ac9cc3baca289e193548608b82801");
  fp_from_hex(&G2Y.c1, "0606c4a02ea734cc32acd2b02bc28b99cb3e287e85a763af267492ab572e99ab3f370d275cec1da1aaa9075ff05f79be");
  fp_from_hex(&BETA, "5f19672fdf76ce51ba69c6076a0f77eaddb3a93be6f89688de17d813620a00022e01fffffffefffe");
  fp_from_hex(&SSWU1_A, "144698a3b8e9433d693a02c96d4982b0ea985383ee66a8d8e8981aefd881ac98936f8da0e0f97f5cf428082d584c1d");
  fp_from_hex(&SSWU1_B, "12e2908d11688030018b12e8753eee3b2016c1f0f24f4070a0b9c14fcef35ef55a23215a316ceaa5d1cc48e98e172be0");
  fp_set_u64(&SSWU1_Z, 11);
  memset(&SSWU2_A, 0, sizeof SSWU2_A);
  fp_set_u64(&SSWU2_A.c1, 240);
  fp_set_u64(&SSWU2_B.c0, 1012);
  SSWU2_B.c1 = SSWU2_B.c0;
  fp_t two, one;
  fp_set_u64(&two, 2);
  fp_set_u64(&one, 1);
  fp_neg(&SSWU2_Z.c0, &two);
  fp_neg(&SSWU2_Z.c1, &one);
  static const char *iso11[4][16] = {
      {"11a05f2b1e833340b809101dd99815856b303e88a2d7005ff2627b56cdb4e2c85610c2d5f2e62d6eaeac1662734649b7",
       "17294ed3e943ab2f0588bab22147a81c7c17e75b2f6a8417f565e33c70d1e86b4838f2a6f318c356e834eef1b3cb83bb",
       "d54005db97678ec1d1048c5d10a9a1bce032473295983e56878e501ec68e25c958c3e3d2a09729fe0179f9dac9edcb0",
       "1778e7166fcc6db74e0609d307e55412d7f5e4656a8dbf25f1b33289f1b330835336e25ce3107193c5b388641d9b6861",
       "e99726a3199f4436642b4b3e4118e5499db995a1257fb3f086eeb65982fac18985a286f301e77c451154ce9ac8895d9",
       "1630c3250d7313ff01d1201bf7a74ab5db3cb17dd952799b9ed3ab9097e68f90a0870d2dcae73d19cd13c1c66f652983",
       "d6ed6553fe44d296a3726c38ae652bfb11586264f0f8ce19008e218f9c86b2a8da25128c1052ecaddd7f225a139ed84",
       "17b81e7701abdbe2e8743884d1117e53356de5ab275b4db1a682c62ef0f2753339b7c8f8c8f475af9ccb5618e3f0c88e",
       "80d3cf1f9a78fc47b90b33563be990dc43b756ce79f5574a2c596c928c5d1de4fa295f296b74e956d71986a8497e317",
       "169b1f8e1bcfa7c42e0c37515d138f22dd2ecb803a0c5c99676314baf4bb1b7fa3190b2edc0327797f241067be390c9e",
       "10321da079ce07e272d8ec09d2565b0dfa7dccdde6787f96d50af36003b14866f69b771f8c285decca67df3f1605fb7b",
       "6e08c248e260e70bd1e962381edee3d31d79d7e22c837bc23c0bf1bc24c6b68c24b1b80b64d391fa9c8ba2e8ba2d229"},
      {"8ca8d548cff19ae18b2e62f4bd3fa6f01d5ef4ba35b48ba9c9588617fc8ac62b558d681be343df8993cf9fa40d21b1c",
       "12561a5deb559c4348b4711298e536367041e8ca0cf0800c0126c2588c48bf5713daa8846cb026e9e5c8276ec82b3bff",
       "b2962fe57a3225e8137e629bff2991f6f89416f5a718cd1fca64e00b11aceacd6a3d0967c94fedcfcc239ba5cb83e19",
       "3425581a58ae2fec83aafef7c40eb545b08243f16b1655154cca8abc28d6fd04976d5243eecf5c4130de8938dc62cd8",
       "13a8e162022914a80a6f1d5f43e7a07dffdfc759a12062bb8d6b44e833b306da9bd29ba81f35781d539d395b3532a21e",
       "e7355f8e4e667b955390f7f0506c6e9395735e9ce9cad4d0a43bcef24b8982f7400d24bc4228f11c02df9a29f6304a5",
       "772caacf16936190f3e0c63e0596721570f5799af53a1894e2e073062aede9cea73b3538f0de06cec2574496ee84a3a",
       "14a7ac2a9d64a8b230b3f5b074cf01996e7f63c21bca68a81996e1cdf9822c580fa5b9489d11e2d311f7d99bbdcc5a5e",
       "a10ecf6ada54f825e920b3dafc7a3cce07f8d1d7161366b74100da67f39883503826692abba43704776ec3a79a1d641",
       "95fc13ab9e92ad4476d6e3eb3a56680f682b4ee96f7d03776df533978f31c1593174e4b4b7865002d6384d168ecdd0a",
       "1"},
      {"90d97c81ba24ee0259d1f094980dcfa11ad138e48a869522b52af6c956543d3cd0c7aee9b3ba3c2be9845719707bb33",
       "134996a104ee5811d51036d776fb46831223e96c254f383d0f906343eb67ad34d6c56711962fa8bfe097e75a2e41c696",
       "cc786baa966e66f4a384c86a3b49942552e2d658a31ce2c344be4b91400da7d26d521628b00523b8dfe240c72de1f6",
       "1f86376e8981c217898751ad8746757d42aa7b90eeb791c09e4a3ec03251cf9de405aba9ec61deca6355c77b0e5f4cb",
       "8cc03fdefe0ff135caf4fe2a21529c4195536fbe3ce50b879833fd221351adc2ee7f8dc099040a841b6daecf2e8fedb",
       "16603fca40634b6a2211e11db8f0a6a074a7d0d4afadb7bd76505c3d3ad5544e203f6326c95a807299b23ab13633a5f0",
       "4ab0b9bcfac1bbcb2c977d027796b3ce75bb8ca2be184cb5231413c4d634f3747a87ac2460f415ec961f8855fe9d6f2",
       "987c8d5333ab86fde9926bd2ca6c674170a05bfe3bdd81ffd038da6c26c842642f64550fedfe935a15e4ca31870fb29",
       "9fc4018bd96684be88c9e221e4da1bb8f3abd16679dc26c1e8b6e6a1f20cabe69d65201c78607a360370e577bdba587",
       "e1bba7a1186bdb5223abde7ada14a23c42a0ca7915af6fe06985e7ed1e4d43b9b3f7055dd4eba6f2bafaaebca731c30",
       "19713e47937cd1be0dfd0b8f1d43fb93cd2fcbcb6caf493fd1183e416389e61031bf3a5cce3fbafce813711ad011c132",
       "18b46a908f36f6deb918c143fed2edcc523559b8aaf0c2462e6bfe7f911f643249d9cdf41b44d606ce07c8a4d0074d8e",
       "b182cac101b9399d155096004f53f447aa7b12a3426b08ec02710e807b4633f06c851c1919211f20d4c04f00b971ef8",
       "245a394ad1eca9b72fc00ae7be315dc757b3b080d4c158013e6632d3c40659cc6cf90ad1c232a6442d9d3f5db980133",
       "5c129645e44cf1102a159f748c4a3fc5e673d81d7e86568d9ab0f5d396a7ce46ba1049b6579afb7866b1e715475224b",
       "15e6be4e990f03ce4ea50b3b42df2eb5cb181d8f84965a3957add4fa95af01b2b665027efec01c7704b456be69c8b604"},
      {"16112c4c3a9c98b252181140fad0eae9601a6de578980be6eec3232b5be72e7a07f3688ef60c206d01479253b03663c1",
       "1962d75c2381201e1a0cbd6c43c348b885c84ff731c4d59ca4a10356f453e01f78a4260763529e3532f6102c2e49a03d",
       "58df3306640da276faaae7d6e8eb15778c4855551ae7f310c35a5dd279cd2eca6757cd636f96f891e2538b53dbf67f2",
       "16b7d288798e5395f20d23bf89edb4d1d115c5dbddbcd30e123da489e726af41727364f2c28297ada8d26d98445f5416",
       "be0e079545f43e4b00cc912f8228ddcc6d19c9f0f69bbb0542eda0fc9dec916a20b15dc0fd2ededda39142311a5001d",
       "8d9e5297186db2d9fb266eaac783182b70152c65550d881c5ecd87b6f0f5a6449f38db9dfa9cce202c6477faaf9b7ac",
       "166007c08a99db2fc3ba8734ace9824b5eecfdfa8d0cf8ef5dd365bc400a0051d5fa9c01a58b1fb93d1a1399126a775c",
       "16a3ef08be3ea7ea03bcddfabba6ff6ee5a4375efa1f4fd7feb34fd206357132b920f5b00801dee460ee415a15812ed9",
       "1866c8ed336c61231a1be54fd1d74cc4f9fb0ce4c6af5920abc5750c4bf39b4852cfe2f7bb9248836b233d9d55535d4a",
       "167a55cda70a6e1cea820597d94a84903216f763e13d87bb5308592e7ea7d4fbc7385ea3d529b35e346ef48bb8913f55",
       "4d2f259eea405bd48f010a01ad2911d9c6dd039bb61a6290e591b36e636a5c871a5c29f4f83060400f8b49cba8f6aa8",
       "accbb67481d033ff5852c1e48c50c477f94ff8aefce42d28c0f9a88cea7913516f968986f7ebbea9684b529e2561092",
       "ad6b9514c767fe3c3613144b45f1496543346d98adf02267d5ceef9a00d9b8693000763e3b90ac11e99b138573345cc",
       "2660400eb2e4f3b628bdd0d53cd76f2bf565b94e72927c1cb748df27942480e420517bd8714cc80d1fadc1326ed06f7",
       "e0fa1d816ddc03e6b24255e0d7819c171c40f65e273b853324efcd6356caa205ca2f570f13497804415473a1d634b8f",
       "1"}};
  for (int k = 0; k < 4; k++)
    for (int i = 0; i < ISO11_N[k]; i++) fp_from_hex(&ISO11[k][i], iso11[k][i]);
  static const char *iso3[4][4][2] = {
      {{"5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6",
        "5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6"},
       {"0", "11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71a"},
       {"11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71e",
        "8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38d"},
       {"171d6541fa38ccfaed6dea691f5fb614cb14b4e7f4e810aa22d6108f142b85757098e38d0f671c7188e2aaaaaaaa5ed1", "0"}},
      {{"0", "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa63"},
       {"c", "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa9f"},
       {"1", "0"},
       {"0", "0"}},
      {{"1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706",
        "1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706"},
       {"0", "5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97be"},
       {"11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71c",
        "8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38f"},
       {"124c9ad43b6cf79bfbf7043de3811ad0761b0f37a1e26286b0e977c69aa274524e79097a56dc4bd9e1b371c71c718b10", "0"}},
      {{"1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa8fb",
        "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa8fb"},
       {"0", "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffa9d3"},
       {"12", "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaa99"},
       {"1", "0"}}};
  for (int k = 0; k < 4; k++)
    for (int i = 0; i < ISO3_N[k]; i++) { fp_from_hex(&ISO3[k][i].c0, iso3[k][i][0]); fp_from_hex(&ISO3[k][i].c1, iso3[k][i][1]); }
  u64s_from_hex(H_EFF2, 10, "bc69f08f2ee75b3584c6a0ea91b352888e2a8e9145ad7689986ff031508ffe1329c2f178731db956d82bf015d1212b02ec0ec69d7477c1ae954cbc06689f6a359894c0adebbf6b4e8020005aaa95551");
  /* 2^256 mod p: Montgomery(2^256) */
  uint64_t k256[6] = {0, 0, 0, 0, 1, 0};
  fp_from_u64s(&K2_256, k256);
  /* Frobenius / psi coefficients: computed from xi = 1 + i */
  fp2_t xi;
  xi.c0 = one; xi.c1 = one;
  /* e = (p^k - 1)/6 computed with 10-word big integers */
  for (int k = 1; k <= 3; k++) {
    enum { NW = 20 };
    uint64_t pk[NW] = {0}, tmpw[NW];
    pk[0] = 1;
    for (int j = 0; j < k; j++) { /* pk *= p */
      memset(tmpw, 0, sizeof tmpw);
      for (int a = 0; a < NW; a++) {
        u128 cc = 0;
        for (int bb = 0; bb < 6 && a + bb < NW; bb++) {
          cc += (u128)pk[a] * P[bb] + tmpw[a + bb];
          tmpw[a + bb] = (uint64_t)cc;
          cc >>= 64;
        }
        if (a + 6 < NW) tmpw[a + 6] += (uint64_t)cc;
      }
      memcpy(pk, tmpw, sizeof pk);
    }
    pk[0] -= 1; /* p^k - 1 (no borrow: p^k odd) */
    uint64_t e6[NW], e3[NW], e23[NW];
    u128 rem = 0;
    for (int a = NW - 1; a >= 0; a--) { u128 cur = (rem << 64) | pk[a]; e6[a] = (uint64_t)(cur / 6); rem = cur % 6; }
    rem = 0;
    for (int a = NW - 1; a >= 0; a--) { u128 cur = (rem << 64) | pk[a]; e3[a] = (uint64_t)(cur / 3); rem = cur % 3; }
    u128 cc = 0;
    for (int a = 0; a < NW; a++) { cc += (u128)e3[a] * 2; e23[a] = (uint64_t)cc; cc >>= 64; }
    fp2_pow(&FROB12_C[k], &xi, e6, NW);
    fp2_pow(&FROB6_C1[k], &xi, e3, NW);
    fp2_pow(&FROB6_C2[k], &xi, e23, NW);
  }
  /* psi: x * conj / xi^((p-1)/3), y * conj / xi^((p-1)/2) */
  fp2_inv(&PSI_X, &FROB6_C1[1]);
  {
    uint64_t e2[6];
    for (int i = 0; i < 6; i++) e2[i] = (P[i] >> 1) | (i < 5 ? P[i + 1] << 63 : 0); /* (p-1)/2 */
    fp2_t t2;
    fp2_pow(&t2, &xi, e2, 6);
    fp2_inv(&PSI_Y, &t2);
  }
}
static void ensure_init(void) { pthread_once(&g_once, init_consts); }

/* ------------------------------------------------------------------ drand scheme layer */
enum { SCH_CHAINED = 0, SCH_UNCHAINED = 1, SCH_G1_LEGACY = 2, SCH_G1_RFC9380 = 3 };
static const char DST_G2[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_";
static const char DST_G1[] = "BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_";
static int sig_on_g1(int sch) { return sch == SCH_G1_LEGACY || sch == SCH_G1_RFC9380; }
static const char *sch_dst(int sch) { return sch == SCH_G1_RFC9380 ? DST_G1 : DST_G2; }

void or_init(int fast_subgroup) { ensure_init(); g_fast_subgroup = fast_subgroup; }

void or_digest_beacon(uint8_t *out, int sch, uint64_t round, const uint8_t *prev, size_t prevlen) {
  sha_t s;
  sha_init(&s);
  if (sch == SCH_CHAINED && prevlen > 0) sha_update(&s, prev, prevlen);
  uint8_t r[8];
  for (int i = 0; i < 8; i++) r[i] = (uint8_t)(round >> (56 - 8 * i));
  sha_update(&s, r, 8);
  sha_final(&s, out);
}

/* bls.Verify: 1 valid, 0 invalid */
int or_verify(int sch, const uint8_t *pk, size_t pklen, const uint8_t *msg, size_t mlen, const uint8_t *sig, size_t siglen) {
  ensure_init();
  const char *dst = sch_dst(sch);
  if (sig_on_g1(sch)) {
    if (pklen != 96 || siglen != 48) return 0;
    g2_t PK; g1_t S, H;
    if (g2_decompress(&PK, pk) != 1) return 0;
    if (g1_decompress(&S, sig) != 1) return 0;
    hash_to_g1(&H, msg, mlen, (const uint8_t *)dst, strlen(dst));
    /* e(H, pk) == e(S, g2)  <=>  e(H, pk) e(-S, g2) == 1 */
    g1_t Ps[2]; g2_t Qs[2];
    Ps[0] = H; Qs[0] = PK;
    g1_neg(&Ps[1], &S);
    Qs[1].x = G2X; Qs[1].y = G2Y; fp2_one(&Qs[1].z);
    return pairing_check(2, Ps, Qs);
  } else {
    if (pklen != 48 || siglen != 96) return 0;
    g1_t PK; g2_t S, H;
    if (g1_decompress(&PK, pk) != 1) return 0;
    if (g2_decompress(&S, sig) != 1) return 0;
    hash_to_g2(&H, msg, mlen, (const uint8_t *)dst, strlen(dst));
    /* e(pk, H) == e(g1, S) */
    g1_t Ps[2]; g2_t Qs[2];
    Ps[0] = PK; Qs[0] = H;
    Ps[1].x = G1X; fp_neg(&Ps[1].y, &G1Y); Ps[1].z = FP_ONE;
    Qs[1] = S;
    return pairing_check(2, Ps, Qs);
  }
}

int or_verify_beacon(int sch, const uint8_t *pk, size_t pklen, uint64_t round, const uint8_t *sig, size_t siglen,
                     const uint8_t *prev, size_t prevlen) {
  uint8_t d[32];
  or_digest_beacon(d, sch, round, prev, prevlen);
  return or_verify(sch, pk, pklen, d, 32, sig, siglen);
}

void or_randomness(uint8_t *out, const uint8_t *sig, size_t siglen) { or_sha256(out, sig, siglen); }

/* scalar from 32-byte big-endian (reduced mod r is the caller's job) */
static void sc_from_be32(uint64_t *k, const uint8_t *b) {
  for (int i = 0; i < 4; i++) {
    uint64_t v = 0;
    for (int j = 0; j < 8; j++) v = (v << 8) | b[24 - 8 * i + j];
    k[i] = v;
  }
}

int or_sign(int sch, const uint8_t *sk32, const uint8_t *msg, size_t mlen, uint8_t *sig_out) {
  ensure_init();
  uint64_t k[4];
  sc_from_be32(k, sk32);
  const char *dst = sch_dst(sch);
  if (sig_on_g1(sch)) {
    g1_t H;
    hash_to_g1(&H, msg, mlen, (const uint8_t *)dst, strlen(dst));
    g1_mul(&H, &H, k, 4);
    g1_compress(sig_out, &H);
    return 48;
  }
  g2_t H;
  hash_to_g2(&H, msg, mlen, (const uint8_t *)dst, strlen(dst));
  g2_mul(&H, &H, k, 4);
  g2_compress(sig_out, &H);
  return 96;
}

int or_public_key(int sch, const uint8_t *sk32, uint8_t *pk_out) {
  ensure_init();
  uint64_t k[4];
  sc_from_be32(k, sk32);
  if (sig_on_g1(sch)) {
    g2_t G; G.x = G2X; G.y = G2Y; fp2_one(&G.z);
    g2_mul(&G, &G, k, 4);
    g2_compress(pk_out, &G);
    return 96;
  }
  g1_t G; G.x = G1X; G.y = G1Y; G.z = FP_ONE;
  g1_mul(&G, &G, k, 4);
  g1_compress(pk_out, &G);
  return 48;
}

/* hash_to_curve output as compressed bytes (cross-check helper) */
int or_hash_to_curve(int g2, const uint8_t *msg, size_t mlen, const uint8_t *dst, size_t dlen, uint8_t *out) {
  ensure_init();
  if (g2) { g2_t H; hash_to_g2(&H, msg, mlen, dst, dlen); g2_compress(out, &H); return 96; }
  g1_t H; hash_to_g1(&H, msg, mlen, dst, dlen); g1_compress(out, &H); return 48;
}

/* decode check: 1 ok, 2 infinity, 0 invalid */
int or_decode(int g2, const uint8_t *b) {
  ensure_init();
  if (g2) { g2_t t; return g2_decompress(&t, b); }
  g1_t t; return g1_decompress(&t, b);
}

/* ------------------------------------------------------------------ batch (threaded) */
typedef struct {
  int sch; const uint8_t *pk; size_t pklen; const uint64_t *rounds; const uint8_t *sigs; size_t sig_stride;
  const uint8_t *prevs; size_t prev_stride; const uint32_t *prev_lens; uint8_t *verdict; uint8_t *rand_out;
  size_t lo, hi;
} job_t;
static void *batch_worker(void *arg) {
  job_t *j = (job_t *)arg;
  size_t siglen = sig_on_g1(j->sch) ? 48 : 96;
  for (size_t i = j->lo; i < j->hi; i++) {
    const uint8_t *prev = j->prevs ? j->prevs + i * j->prev_stride : NULL;
    size_t plen = j->prevs ? (j->prev_lens ? j->prev_lens[i] : j->prev_stride) : 0;
    j->verdict[i] = (uint8_t)or_verify_beacon(j->sch, j->pk, j->pklen, j->rounds[i], j->sigs + i * j->sig_stride, siglen, prev, plen);
    if (j->rand_out) or_randomness(j->rand_out + 32 * i, j->sigs + i * j->sig_stride, siglen);
  }
  return NULL;
}
/* Per-round VerifyBeacon over n rounds with nthreads OS threads (the CPU baseline). */
void or_verify_batch(int sch, const uint8_t *pk, size_t pklen, const uint64_t *rounds, const uint8_t *sigs, size_t sig_stride,
                     const uint8_t *prevs, size_t prev_stride, const uint32_t *prev_lens, size_t n, int nthreads,
                     uint8_t *verdict, uint8_t *rand_out) {
  ensure_init();
  if (nthreads < 1) nthreads = 1;
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  job_t *jobs = (job_t *)calloc((size_t)nthreads, sizeof(job_t));
  for (int t = 0; t < nthreads; t++) {
    job_t *j = &jobs[t];
    j->sch = sch; j->pk = pk; j->pklen = pklen; j->rounds = rounds; j->sigs = sigs; j->sig_stride = sig_stride;
    j->prevs = prevs; j->prev_stride = prev_stride; j->prev_lens = prev_lens; j->verdict = verdict; j->rand_out = rand_out;
    j->lo = n * (size_t)t / (size_t)nthreads;
    j->hi = n * (size_t)(t + 1) / (size_t)nthreads;
    pthread_create(&th[t], NULL, batch_worker, j);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
}

/* ------------------------------------------------------------------ scalar field (mod r) for tbls */
static void sc_mod_r_sub(uint64_t *a) { /* if a >= r: a -= r */
  int ge = 1;
  for (int i = 3; i >= 0; i--) { if (a[i] > RSC[i]) { ge = 1; break; } if (a[i] < RSC[i]) { ge = 0; break; } }
  if (!ge) return;
  u128 br = 0;
  for (int i = 0; i < 4; i++) { u128 d = (u128)a[i] - RSC[i] - br; a[i] = (uint64_t)d; br = (d >> 64) & 1; }
}
static void sc_mul(uint64_t *r, const uint64_t *a, const uint64_t *b) { /* schoolbook + bitwise reduction (slow, simple) */
  uint64_t t[8] = {0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) { c += (u128)a[i] * b[j] + t[i + j]; t[i + j] = (uint64_t)c; c >>= 64; }
    t[i + 4] = (uint64_t)c;
  }
  uint64_t acc[4] = {0};
  for (int bit = 511; bit >= 0; bit--) {
    /* acc = 2 acc + bit */
    uint64_t carry = acc[3] >> 63;
    for (int i = 3; i > 0; i--) acc[i] = (acc[i] << 1) | (acc[i - 1] >> 63);
    acc[0] = (acc[0] << 1) | ((t[bit >> 6] >> (bit & 63)) & 1);
    if (carry) { /* acc + 2^256 - r ... handle by subtracting r until < r (acc < 2r guaranteed before shift) */
      u128 br = 0;
      for (int i = 0; i < 4; i++) { u128 d = (u128)acc[i] - RSC[i] - br; acc[i] = (uint64_t)d; br = (d >> 64) & 1; }
    }
    sc_mod_r_sub(acc);
  }
  memcpy(r, acc, 32);
}
static void sc_sub(uint64_t *r, const uint64_t *a, const uint64_t *b) {
  u128 br = 0;
  uint64_t t[4];
  for (int i = 0; i < 4; i++) { u128 d = (u128)a[i] - b[i] - br; t[i] = (uint64_t)d; br = (d >> 64) & 1; }
  if (br) { u128 c = 0; for (int i = 0; i < 4; i++) { c += (u128)t[i] + RSC[i]; t[i] = (uint64_t)c; c >>= 64; } }
  memcpy(r, t, 32);
}
static void sc_inv(uint64_t *r, const uint64_t *a) {
  uint64_t e[4], acc[4] = {1, 0, 0, 0};
  memcpy(e, RSC, 32);
  e[0] -= 2;
  for (int i = 255; i >= 0; i--) {
    sc_mul(acc, acc, acc);
    if ((e[i >> 6] >> (i & 63)) & 1) sc_mul(acc, acc, a);
  }
  memcpy(r, acc, 32);
}

/*
 * tbls.Recover semantics [kyber v1.1.18 sign/tbls + share.RecoverCommit], called at
 * /root/reference/chain/beacon/chainstore.go:202:
 *   for each partial in the given order: parse 2-byte BE index; VerifyPartial against
 *   PubPoly.Eval(index) (x = index+1, Horner over the t commits); decode; keep; stop at t kept.
 *   < t kept -> error. Then sort kept by index, drop duplicate indices, take the first t and
 *   Lagrange-interpolate at 0 in the signature group.
 * commits: t compressed key-group points (48 B for G2-sig schemes, 96 B for G1-sig).
 * partials: npart entries of (2 + siglen) bytes. Returns siglen on success, -1 on failure.
 */
int or_recover(int sch, const uint8_t *commits, int t, int n, const uint8_t *msg, size_t mlen, const uint8_t *partials,
               int npart, uint8_t *sig_out) {
  ensure_init();
  (void)n;
  int g1sig = sig_on_g1(sch);
  size_t siglen = g1sig ? 48 : 96, keylen = g1sig ? 96 : 48, plen = 2 + siglen;
  int *idx = (int *)malloc(sizeof(int) * (size_t)npart);
  int kept = 0;
  for (int k = 0; k < npart && kept < t; k++) {
    const uint8_t *pp = partials + (size_t)k * plen;
    int index = (pp[0] << 8) | pp[1];
    /* PubPoly.Eval(index): Horner at x = index + 1 over commits (key group) */
    uint64_t x = (uint64_t)index + 1;
    uint8_t keyb[96];
    if (g1sig) {
      g2_t acc, c;
      g2_set_inf(&acc); fp2_zero(&acc.z);
      int bad = 0;
      for (int j = t - 1; j >= 0; j--) {
        g2_mul(&acc, &acc, &x, 1);
        if (g2_decompress(&c, commits + (size_t)j * keylen) == 0) bad = 1;
        g2_add(&acc, &acc, &c);
      }
      if (bad) continue;
      g2_compress(keyb, &acc);
    } else {
      g1_t acc, c;
      g1_set_inf(&acc); acc.z = (fp_t){{0}};
      int bad = 0;
      for (int j = t - 1; j >= 0; j--) {
        g1_mul(&acc, &acc, &x, 1);
        if (g1_decompress(&c, commits + (size_t)j * keylen) == 0) bad = 1;
        g1_add(&acc, &acc, &c);
      }
      if (bad) continue;
      g1_compress(keyb, &acc);
    }
    if (!or_verify(sch, keyb, keylen, msg, mlen, pp + 2, siglen)) continue;
    idx[kept++] = k;
  }
  if (kept < t) { free(idx); return -1; }
  /* sort kept by share index (stable insertion), dedup, take first t */
  int *sel = (int *)malloc(sizeof(int) * (size_t)kept);
  int ns = 0;
  for (int a = 0; a < kept; a++) {
    const uint8_t *pp = partials + (size_t)idx[a] * plen;
    int ia = (pp[0] << 8) | pp[1];
    int pos = ns;
    while (pos > 0) {
      const uint8_t *q = partials + (size_t)sel[pos - 1] * plen;
      int ib = (q[0] << 8) | q[1];
      if (ib <= ia) break;
      pos--;
    }
    memmove(sel + pos + 1, sel + pos, sizeof(int) * (size_t)(ns - pos));
    sel[pos] = idx[a];
    ns++;
  }
  int nd = 0;
  for (int a = 0; a < ns; a++) {
    const uint8_t *pp = partials + (size_t)sel[a] * plen;
    int ia = (pp[0] << 8) | pp[1];
    if (nd > 0) {
      const uint8_t *q = partials + (size_t)sel[nd - 1] * plen;
      if (((q[0] << 8) | q[1]) == ia) continue;
    }
    sel[nd++] = sel[a];
    if (nd == t) break;
  }
  free(idx);
  if (nd < t) { free(sel); return -1; }
  /* Lagrange at 0: lambda_i = prod_{j != i} x_j / (x_j - x_i) */
  g1_t acc1; g2_t acc2;
  g1_set_inf(&acc1); acc1.z = (fp_t){{0}};
  g2_set_inf(&acc2); fp2_zero(&acc2.z);
  for (int a = 0; a < t; a++) {
    const uint8_t *pa = partials + (size_t)sel[a] * plen;
    uint64_t xa[4] = {(uint64_t)((pa[0] << 8) | pa[1]) + 1, 0, 0, 0};
    uint64_t num[4] = {1, 0, 0, 0}, den[4] = {1, 0, 0, 0};
    for (int b = 0; b < t; b++) {
      if (b == a) continue;
      const uint8_t *pb = partials + (size_t)sel[b] * plen;
      uint64_t xb[4] = {(uint64_t)((pb[0] << 8) | pb[1]) + 1, 0, 0, 0}, d[4];
      sc_mul(num, num, xb);
      sc_sub(d, xb, xa);
      sc_mul(den, den, d);
    }
    sc_inv(den, den);
    uint64_t lam[4];
    sc_mul(lam, num, den);
    if (g1sig) {
      g1_t s; g1_decompress(&s, pa + 2); g1_mul(&s, &s, lam, 4); g1_add(&acc1, &acc1, &s);
    } else {
      g2_t s; g2_decompress(&s, pa + 2); g2_mul(&s, &s, lam, 4); g2_add(&acc2, &acc2, &s);
    }
  }
  free(sel);
  if (g1sig) g1_compress(sig_out, &acc1); else g2_compress(sig_out, &acc2);
  return (int)siglen;
}

/* PubPoly.Eval(i) as compressed key-group bytes (fixture helper) */
int or_pubpoly_eval(int sch, const uint8_t *commits, int t, int index, uint8_t *out) {
  ensure_init();
  int g1sig = sig_on_g1(sch);
  size_t keylen = g1sig ? 96 : 48;
  uint64_t x = (uint64_t)index + 1;
  if (g1sig) {
    g2_t acc, c; g2_set_inf(&acc); fp2_zero(&acc.z);
    for (int j = t - 1; j >= 0; j--) { g2_mul(&acc, &acc, &x, 1); if (g2_decompress(&c, commits + (size_t)j * keylen) == 0) return -1; g2_add(&acc, &acc, &c); }
    g2_compress(out, &acc); return 96;
  }
  g1_t acc, c; g1_set_inf(&acc); acc.z = (fp_t){{0}};
  for (int j = t - 1; j >= 0; j--) { g1_mul(&acc, &acc, &x, 1); if (g1_decompress(&c, commits + (size_t)j * keylen) == 0) return -1; g1_add(&acc, &acc, &c); }
  g1_compress(out, &acc); return 48;
}
