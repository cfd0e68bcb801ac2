// BLS12-381 base field Fp on gfx950: 12 x 32-bit limbs, Montgomery form (R = 2^384).
//
// One field element lives in 12 VGPRs of one lane; every lane of a wave works on its own
// beacon, so all arithmetic here is per-lane SIMT code with no cross-lane traffic.
// Multiplication is CIOS with the "no final carry word" shortcut (p's top limb < 2^31),
// written so that each partial product lowers to one v_mad_u64_u32.
//
// Replaces the Fp arithmetic of kilic/bls12-381 v0.1.0 (arithmetic_x86.s / fp.go) that
// kyber-bls12381 v0.2.5 uses behind /root/reference/crypto/schemes.go:98,139,177.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "consts.hpp"
#include "fp_mul28.hpp"
#include "inv_bingcd.hpp"

namespace dh {

#define DH_DEV __device__ __forceinline__
// out-of-line helper (a real call); the field products themselves are the out-of-line fp_mul_vec /
// fp_sqr_vec (measured: point formulas must stay inline — by-reference arguments go through scratch)
#define DH_OOL __device__ __noinline__

struct fp {
  uint32_t v[12];
};

// p, little-endian 32-bit limbs
#define DH_P0 0xffffaaabu
#define DH_P1 0xb9feffffu
#define DH_P2 0xb153ffffu
#define DH_P3 0x1eabfffeu
#define DH_P4 0xf6b0f624u
#define DH_P5 0x6730d2a0u
#define DH_P6 0xf38512bfu
#define DH_P7 0x64774b84u
#define DH_P8 0x434bacd7u
#define DH_P9 0x4b1ba7b6u
#define DH_P10 0x397fe69au
#define DH_P11 0x1a0111eau
#define DH_NP0 0xfffcfffdu  // -p^-1 mod 2^32

DH_DEV uint32_t p_limb(int i) {
  switch (i) {
    case 0: return DH_P0; case 1: return DH_P1; case 2: return DH_P2; case 3: return DH_P3;
    case 4: return DH_P4; case 5: return DH_P5; case 6: return DH_P6; case 7: return DH_P7;
    case 8: return DH_P8; case 9: return DH_P9; case 10: return DH_P10; default: return DH_P11;
  }
}

DH_DEV fp fp_zero() {
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = 0;
  return r;
}

// R mod p (Montgomery one)
DH_DEV fp fp_one() {
  fp r;
  r.v[0] = 0x0002fffdu; r.v[1] = 0x76090000u; r.v[2] = 0xc40c0002u; r.v[3] = 0xebf4000bu;
  r.v[4] = 0x53c758bau; r.v[5] = 0x5f489857u; r.v[6] = 0x70525745u; r.v[7] = 0x77ce5853u;
  r.v[8] = 0xa256ec6du; r.v[9] = 0x5c071a97u; r.v[10] = 0xfa80e493u; r.v[11] = 0x15f65ec3u;
  return r;
}

// R^2 mod p (to enter Montgomery form)
DH_DEV fp fp_r2() {
  fp r;
  r.v[0] = 0x1c341746u; r.v[1] = 0xf4df1f34u; r.v[2] = 0x09d104f1u; r.v[3] = 0x0a76e6a6u;
  r.v[4] = 0x4c95b6d5u; r.v[5] = 0x8de5476cu; r.v[6] = 0x939d83c0u; r.v[7] = 0x67eb88a9u;
  r.v[8] = 0xb519952du; r.v[9] = 0x9a793e85u; r.v[10] = 0x92cae3aau; r.v[11] = 0x11988fe5u;
  return r;
}

// Multi-limb carry chains use clang's __builtin_addc / __builtin_subc: they lower to one v_add_co / v_addc_co
// (v_sub_co / v_subb_co) per limb with the carry in VCC or an SGPR pair. The uint64_t "t >> 32" / "t >> 63"
// formulation compiled to 64-bit v_lshl_add_u64 + v_ashrrev + v_mov per limb (~140 VALU per fp_add, 48 now).

// r = a - p if a >= p else a   (a < 2p)
DH_DEV void fp_reduce_once(fp& a) {
  uint32_t d[12];
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d[i] = __builtin_subc(a.v[i], p_limb(i), br, &br);
  // br == 0  <=>  a >= p
#pragma unroll
  for (int i = 0; i < 12; i++) a.v[i] = br ? a.v[i] : d[i];
}

DH_DEV fp fp_add(const fp& a, const fp& b) {
  fp r;
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
  fp_reduce_once(r);  // a+b < 2p < 2^382, no limb overflow
  return r;
}

// a + b WITHOUT the reduction, for operands that only feed a Montgomery product: a, b < p gives a sum < 2p, and
// the product (fp_mul28.hpp mul) is exact and fully reduced for inputs < 2p: before its one conditional
// subtraction it is < x y / 2^384 + p < 2p
// (t = (xy + mp) / R < 4p^2/R + p < 2p before its one conditional subtraction).
DH_DEV fp fp_add_nr(const fp& a, const fp& b) {
  fp r;
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
  return r;
}

DH_DEV fp fp_sub(const fp& a, const fp& b) {
  fp r;
  unsigned br = 0, c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
  // if negative add p back
  const uint32_t mask = 0u - br;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = __builtin_addc(r.v[i], p_limb(i) & mask, c, &c);
  return r;
}

DH_DEV fp fp_neg(const fp& a) {
  // p - a, and 0 -> 0
  uint32_t nz = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) nz |= a.v[i];
  const uint32_t mask = nz ? 0xffffffffu : 0u;
  fp r;
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = __builtin_subc(p_limb(i) & mask, a.v[i], br, &br);
  return r;
}

DH_DEV fp fp_dbl(const fp& a) { return fp_add(a, a); }

DH_DEV uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
  return (uint64_t)a * (uint64_t)b + c;
}

// Textbook CIOS Montgomery product (kept as the microbenchmark baseline, bench/microbench_fp.hip).
DH_DEV fp fp_mul_cios(const fp& a, const fp& b) {
  uint32_t t[12];
#pragma unroll
  for (int j = 0; j < 12; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint32_t bi = b.v[i];
    uint64_t A = mad64(a.v[0], bi, t[0]);
    t[0] = (uint32_t)A;
    const uint32_t m = t[0] * DH_NP0;
    uint64_t C = mad64(m, DH_P0, t[0]);
#pragma unroll
    for (int j = 1; j < 12; j++) {
      A = mad64(a.v[j], bi, (uint64_t)t[j] + (A >> 32));
      t[j] = (uint32_t)A;
      C = mad64(m, p_limb(j), (uint64_t)t[j] + (C >> 32));
      t[j - 1] = (uint32_t)C;
    }
    t[11] = (uint32_t)(C >> 32) + (uint32_t)(A >> 32);
  }
  fp r;
#pragma unroll
  for (int j = 0; j < 12; j++) r.v[j] = t[j];
  fp_reduce_once(r);
  return r;
}

// The field product used everywhere: product-scanning Montgomery on 14 x 28-bit limbs behind the 12 x 32-bit
// interface (fp_mul28.hpp: one v_mad_u64_u32 per partial product, no carry adds; the 32-bit form of
// bench/fp32/fp_mul_fips.hpp needs a v_addc per product and measured slower), one out-of-line copy
// per code object so that the large kernels (pairing, hash-to-curve) stay compact; define DH_MUL_INLINE to
// inline it instead.
//
// Call convention. A plain call makes the caller assume the standard AMDGPU C convention: every
// caller-saved VGPR (v0-v39 and the v48-55, v64-71, ... stripes, ~148 registers) dies at the call, so
// only ~108 VGPRs can carry values across a product — 4 Fp2 elements. The G2 point formulas keep more
// than that live and spilled to scratch around EVERY product (k_prep_msg<fp2>: 19.3 KB of scratch per
// lane). The products are therefore entered through an inline-asm `s_swappc_b64` whose clobber list is
// exactly what the two bodies touch: v0-v39, v48-v53, s0-s17, s30-s31, vcc and scc. The bodies are ordinary compiled functions: they may set SCC and mask EXEC around a
// branch (restoring it), so SCC must be in the list — without it a loop condition held in SCC across a
// product was lost. Everything else stays live in registers across the call. drand_amd/tools/check_fp_abi.py
// disassembles every built code object and fails the build if a body touches a register outside that list,
// leaves EXEC modified, uses the stack or calls out, so a compiler change cannot silently break the contract.
typedef uint32_t fpvec __attribute__((ext_vector_type(12)));

extern "C" __device__ __noinline__ __attribute__((used)) fpvec dh_fp_mul_vec(fpvec a, fpvec b) {
  uint32_t x[12], y[12], r[12];
#pragma unroll
  for (int i = 0; i < 12; i++) { x[i] = a[i]; y[i] = b[i]; }
  m28::mul(r, x, y);
  fpvec o;
#pragma unroll
  for (int i = 0; i < 12; i++) o[i] = r[i];
  return o;
}
extern "C" __device__ __noinline__ __attribute__((used)) fpvec dh_fp_sqr_vec(fpvec a) {
  uint32_t x[12], r[12];
#pragma unroll
  for (int i = 0; i < 12; i++) x[i] = a[i];
  m28::sqr(r, x);
  fpvec o;
#pragma unroll
  for (int i = 0; i < 12; i++) o[i] = r[i];
  return o;
}

// The same products on values already in the 28-bit representation (fp_mul28.hpp mont_mul / mont_sqr: 14 limbs,
// radix 2^392, no slicing or final subtraction), for the chains that stay in it (fp28.hpp). Operands travel in 16
// VGPRs (limbs 0-13; the backend has no 14-register class), a in v0-v15, b in v16-v31.
typedef uint32_t fp28vec __attribute__((ext_vector_type(16)));
extern "C" __device__ __noinline__ __attribute__((used)) fp28vec dh_fp28_mul_vec(fp28vec a, fp28vec b) {
  uint32_t x[14], y[14], r[14];
#pragma unroll
  for (int i = 0; i < 14; i++) { x[i] = a[i]; y[i] = b[i]; }
  m28::mont_mul(r, x, y);
  fp28vec o;
#pragma unroll
  for (int i = 0; i < 14; i++) o[i] = r[i];
  o[14] = o[15] = 0;
  return o;
}
extern "C" __device__ __noinline__ __attribute__((used)) fp28vec dh_fp28_sqr_vec(fp28vec a) {
  uint32_t x[14], r[14];
#pragma unroll
  for (int i = 0; i < 14; i++) x[i] = a[i];
  m28::mont_sqr(r, x);
  fp28vec o;
#pragma unroll
  for (int i = 0; i < 14; i++) o[i] = r[i];
  o[14] = o[15] = 0;
  return o;
}

#define DH_FP_CALL_CLOBBERS                                                                                    \
  "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", \
      "v48", "v49", "v50", "v51", "v52", "v53", "s0", "s1", "s2", "s3", "s4", "s5", "s6", "s7", "s8", "s9", "s10",  \
      "s11", "s12", "s13", "s14", "s15", "s16", "s17", "s30", "s31", "vcc", "scc"
// a = a * b (a in v0-v11, b in v12-v23 and clobbered); the callee address is formed exactly as the compiler
// forms it for a direct call
#define DH_FP_CALL(fn) \
  "s_getpc_b64 s[14:15]\n\ts_add_u32 s14, s14, " fn "@rel32@lo+4\n\ts_addc_u32 s15, s15, " fn "@rel32@hi+12\n\ts_swappc_b64 s[30:31], s[14:15]"

DH_DEV fpvec to_vec(const fp& a) {
  fpvec v;
#pragma unroll
  for (int i = 0; i < 12; i++) v[i] = a.v[i];
  return v;
}
DH_DEV fp from_vec(const fpvec& v) {
  fp a;
#pragma unroll
  for (int i = 0; i < 12; i++) a.v[i] = v[i];
  return a;
}

DH_DEV fp fp_mul(const fp& a, const fp& b) {
  DH_COUNT_PROD();
#ifdef DH_MUL_INLINE
  fp r;
  m28::mul(r.v, a.v, b.v);
  return r;
#else
  fpvec x = to_vec(a), y = to_vec(b);
  asm(DH_FP_CALL("dh_fp_mul_vec") : "+{v[0:11]}"(x), "+{v[12:23]}"(y) : : DH_FP_CALL_CLOBBERS);
  return from_vec(x);
#endif
}

DH_DEV fp fp_sqr(const fp& a) {
  DH_COUNT_PROD();
#ifdef DH_MUL_INLINE
  fp r;
  m28::sqr(r.v, a.v);
  return r;
#else
  fpvec x = to_vec(a);
  asm(DH_FP_CALL("dh_fp_sqr_vec")
      : "+{v[0:11]}"(x)
      :
      : "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", DH_FP_CALL_CLOBBERS);
  return from_vec(x);
#endif
}


DH_DEV bool fp_is_zero(const fp& a) {
  uint32_t nz = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) nz |= a.v[i];
  return nz == 0;
}

DH_DEV bool fp_eq(const fp& a, const fp& b) {
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d |= a.v[i] ^ b.v[i];
  return d == 0;
}

DH_DEV fp fp_select(bool c, const fp& a, const fp& b) {
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}

DH_DEV fp fp_to_mont(const fp& a) { return fp_mul(a, fp_r2()); }

DH_DEV fp fp_from_mont(const fp& a) {
  fp one = fp_zero();
  one.v[0] = 1;
  return fp_mul(a, one);
}

// load a constant-memory Montgomery element
DH_DEV fp fp_c(const uint32_t* c) {
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.v[i] = c[i];
  return r;
}

DH_DEV fp fp_mul_c(const fp& a, const uint32_t* c) { return fp_mul(a, fp_c(c)); }

// x^e for a fixed exponent given as a sliding-window schedule (consts.hpp SCHED_*, w = 3):
// table x, x^3, x^5, x^7; sched[0] = first table index, then (squarings << 8 | index), index 0xff =
// squarings only. 378 squarings + ~105 multiplications for the 381-bit exponents (binary: ~228).
// The chain runs on 14 x 28-bit limbs in Montgomery radix R' = 2^392 (fp_mul28.hpp mont_mul / mont_sqr, inlined):
// x R enters as x R' by one product with 2^400 mod p and leaves by one product with 2^384 mod p, so the ~480
// products in between skip the 12 <-> 14 limb slicing and the final subtraction of the out-of-line bodies
// (~110 of their ~610 instructions). Every intermediate value stays < 1.002 p with normalised limbs.
struct fp28 {
  uint32_t l[14];
};
DH_DEV fp28 fp28_mul(const fp28& a, const fp28& b) {
  DH_COUNT_PROD();
  fp28 r;
  m28::mont_mul(r.l, a.l, b.l);
  return r;
}
DH_DEV fp28 fp28_sqr(const fp28& a) {
  DH_COUNT_PROD();
  fp28 r;
  m28::mont_sqr(r.l, a.l);
  return r;
}
DH_DEV fp28 fp28_from(const fp& x) {  // x R -> x R'
  fp28 a, c;
  m28::split<0>(a.l, x.v);
  const uint32_t k[14] = {0x80e6299u, 0x3500034u, 0xeb12856u, 0xdeb2699u, 0xc988670u, 0x4ef6697u, 0x70983e8u,
                          0xa4e6fe9u, 0x3e8a053u, 0xecf271eu, 0xc20d323u, 0x6eb6385u, 0x47f1286u, 0x00156dau};  // 2^400 mod p
#pragma unroll
  for (int i = 0; i < 14; i++) c.l[i] = k[i];
  return fp28_mul(a, c);
}
DH_DEV fp fp28_to(const fp28& a) {  // x R' -> x R, canonical
  fp28 c;
  const uint32_t k[14] = {0x002fffdu, 0x0900000u, 0xc000276u, 0x000bc40u, 0x8baebf4u, 0x5753c75u, 0x55f4898u,
                          0x7052574u, 0x7ce5853u, 0x56ec6d7u, 0x71a97a2u, 0xe4935c0u, 0xec3fa80u, 0x0015f65u};  // 2^384 mod p
#pragma unroll
  for (int i = 0; i < 14; i++) c.l[i] = k[i];
  const fp28 r = fp28_mul(a, c);
  fp o;
  m28::join(o.v, r.l);
  m28::final_sub(o.v);
  return o;
}

DH_DEV fp fp_pow_sched(const fp& x0, const uint32_t* sched, int len) {
  const fp28 x = fp28_from(x0);
  const fp28 x2 = fp28_sqr(x);
  const fp28 t1 = fp28_mul(x, x2);
  const fp28 t2 = fp28_mul(t1, x2);
  const fp28 t3 = fp28_mul(t2, x2);
  auto pick = [&](uint32_t k) { return k == 0 ? x : (k == 1 ? t1 : (k == 2 ? t2 : t3)); };
  fp28 acc = pick(sched[0]);
  uint32_t next = sched[1];  // the tables end with a 0 entry: the read one step ahead stays in bounds
#pragma unroll 1
  for (int i = 1; i < len; i++) {
    const uint32_t op = next;
    next = sched[i + 1];  // scalar load issued a whole step before its use
    const uint32_t nsq = op >> 8, k = op & 0xff;
#pragma unroll 1
    for (uint32_t j = 0; j < nsq; j++) acc = fp28_sqr(acc);
    if (k != 0xff) acc = fp28_mul(acc, pick(k));
  }
  return fp28_to(acc);
}

DH_DEV fp fp_inv(const fp& x) { return fp_pow_sched(x, cst::SCHED_INV, cst::SCHED_INV_LEN); }

// Inversion of a PUBLIC element in variable time (verification data only — signatures, hash points, RLC sums; the
// signing helpers keep the fixed exponentiation above): inv_bingcd.hpp, Pornin's optimized binary GCD (25 rounds of
// 31 divsteps on 64-bit approximations, the 12-word linear combinations once per round). It replaced (r06) a binary
// extended Euclid with multi-bit halving, ~450 iterations of ~100 dependent VALU ops each (0.19 ms on one lane: the
// pairing VM's inversion phase was 7% of a check, and every one-lane affine conversion and the MSM point prep's
// per-workgroup inversion waited on it). a = yR gives a^-1 = y^-1 R^-1, and one product by R^3 mod p returns the
// Montgomery form y^-1 R.
// in place: a (integer in [1, p)) -> a^-1 mod p
DH_DEV void inv_vt_int(uint32_t a[12]) { bgcd::inverse(a); }

DH_DEV fp fp_inv_vt(const fp& a) {
  if (fp_is_zero(a)) return a;
  fp r = a;
  inv_vt_int(r.v);
  const fp r3 = {{0xd94ca1e0u, 0xed48ac6bu, 0x03a7adf8u, 0x315f831eu, 0x615e29ddu, 0x9a53352au, 0x921e1761u, 0x34c04e5eu,
                  0x65724728u, 0x2512d435u, 0x91755d4du, 0x0aa63460u}};  // R^3 mod p
  return fp_mul(r, r3);
}

// returns true and r = sqrt(a) if a is a square
DH_DEV bool fp_sqrt(fp& r, const fp& a) {
  r = fp_pow_sched(a, cst::SCHED_SQRT, cst::SCHED_SQRT_LEN);
  return fp_eq(fp_sqr(r), a);
}

// canonical (non-Montgomery) integer comparison helpers
DH_DEV bool int_gt_half_p(const fp& canon) {
  // (p-1)/2 limbs
  const uint32_t h[12] = {0xffffd555u, 0xdcff7fffu, 0x58a9ffffu, 0x0f55ffffu, 0x7b587b12u, 0xb3986950u,
                          0x79c2895fu, 0xb23ba5c2u, 0x21a5d66bu, 0x258dd3dbu, 0x1cbff34du, 0x0d0088f5u};
  // canon > h ?
  bool gt = false, decided = false;
#pragma unroll
  for (int i = 11; i >= 0; i--) {
    bool g = canon.v[i] > h[i], l = canon.v[i] < h[i];
    gt = decided ? gt : g;
    decided = decided || g || l;
  }
  return gt;
}

DH_DEV bool int_lt_p(const uint32_t* x) {
  bool lt = false, decided = false;
#pragma unroll
  for (int i = 11; i >= 0; i--) {
    uint32_t pl = p_limb(i);
    bool l = x[i] < pl, g = x[i] > pl;
    lt = decided ? lt : l;
    decided = decided || g || l;
  }
  return lt;
}

// RFC 9380 sgn0 for Fp: parity of the canonical value
DH_DEV uint32_t fp_sgn0(const fp& a) { return fp_from_mont(a).v[0] & 1; }

// 48 big-endian bytes (top 3 bits masked by the caller) -> limbs (no reduction)
DH_DEV void be48_to_limbs(uint32_t* out, const uint8_t* in) {
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint8_t* q = in + 44 - 4 * i;
    out[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
}

DH_DEV void limbs_to_be48(uint8_t* out, const fp& canon) {
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint8_t* q = out + 44 - 4 * i;
    uint32_t v = canon.v[i];
    q[0] = v >> 24; q[1] = v >> 16; q[2] = v >> 8; q[3] = v;
  }
}

}  // namespace dh
