// ZCash compressed point codec and subgroup checks, per lane.
// Replaces kilic/bls12-381 v0.1.0 G1.FromCompressed / G2.FromCompressed / ToCompressed and
// InCorrectSubgroup, reached via kyber-bls12381 v0.2.5 Point.UnmarshalBinary (e.g.
// /root/reference/key/encoding.go:22-29, /root/reference/chain/convert.go:21-24) and inside bls.Verify.
//
// Accept/reject rules (mirrored by oracle/bls_oracle.c g1_decompress / g2_decompress):
//   byte0 bit7 (compression) must be set; bit6 (infinity) => all other bits/bytes zero, decoded as the
//   point at infinity (status DEC_INF, which every verify path rejects); x (and for G2 both x.c1, x.c0)
//   must be < p; x^3 + b must be a square; bit5 selects the lexicographically largest y (G2: compare
//   c1, then c0 when c1 == 0); the point must be in the r-torsion subgroup.
// Subgroup tests (exact for BLS12-381): G1  phi(P) == [-u^2] P  with phi(x, y) = (beta x, y);
//                                      G2  psi(P) == [u] P.
#pragma once
#include "h2c.hpp"
#include "fp28.hpp"
#include "fp2_28.hpp"

namespace dh {

enum : uint8_t { DEC_OK = 1, DEC_INF = 2, DEC_BAD = 0 };

DH_DEV bool fp_lex_gt_half(const fp& mont_y) { return int_gt_half_p(fp_from_mont(mont_y)); }

DH_DEV bool fp2_lex_largest(const fp2& y) {
  fp c0 = fp_from_mont(y.c0), c1 = fp_from_mont(y.c1);
  return fp_is_zero(c1) ? int_gt_half_p(c0) : int_gt_half_p(c1);
}

// raw 48 big-endian bytes (flags masked) -> limbs; 4-byte aligned source
DH_DEV void be48_words(uint32_t out[12], const uint8_t* in, bool mask_flags) {
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint32_t w = __builtin_bswap32(*(const uint32_t*)(in + 44 - 4 * i));
    out[i] = w;
  }
  if (mask_flags) out[11] &= 0x1fffffffu;
}

DH_DEV bool g1_in_subgroup(const aff<fp>& p) {
  // t = [u^2] P = [|u|]([|u|] P); need phi(P) == -t. Run on lazily reduced 28-bit limbs (fp28.hpp)
  return g1_in_subgroup28([&] { return p; });
}

DH_DEV bool g2_in_subgroup(const aff<fp2>& p) {
  // psi(P) == [u] P = -[|u|] P, on lazily reduced 28-bit limbs (fp2_28.hpp)
  return g2_in_subgroup28(p);
}

// decode a 48-byte compressed G1 point (4-byte aligned); optional subgroup check
DH_DEV uint8_t g1_decompress(aff<fp>& out, const uint8_t* b, bool subgroup) {
  uint32_t w[12];
  be48_words(w, b, false);
  const uint32_t flags = w[11] >> 29;
  if (!(flags & 4)) return DEC_BAD;
  w[11] &= 0x1fffffffu;
  if (flags & 2) {
    uint32_t nz = flags & 1;
#pragma unroll
    for (int i = 0; i < 12; i++) nz |= w[i];
    return nz ? DEC_BAD : DEC_INF;
  }
  if (!int_lt_p(w)) return DEC_BAD;
  fp x;
#pragma unroll
  for (int i = 0; i < 12; i++) x.v[i] = w[i];
  x = fp_to_mont(x);
  fp rhs = fp_add(fp_mul(fp_sqr(x), x), fp_c(cst::B1));
  fp y;
  if (!fp_sqrt(y, rhs)) return DEC_BAD;
  if (fp_lex_gt_half(y) != (bool)(flags & 1)) y = fp_neg(y);
  out.x = x;
  out.y = y;
  if (subgroup && !g1_in_subgroup(out)) return DEC_BAD;
  return DEC_OK;
}

// decode a 96-byte compressed G2 point (x.c1 || x.c0)
DH_DEV uint8_t g2_decompress(aff<fp2>& out, const uint8_t* b, bool subgroup) {
  uint32_t w1[12], w0[12];
  be48_words(w1, b, false);
  be48_words(w0, b + 48, false);
  const uint32_t flags = w1[11] >> 29;
  if (!(flags & 4)) return DEC_BAD;
  w1[11] &= 0x1fffffffu;
  if (flags & 2) {
    uint32_t nz = flags & 1;
#pragma unroll
    for (int i = 0; i < 12; i++) nz |= w1[i] | w0[i];
    return nz ? DEC_BAD : DEC_INF;
  }
  if (!int_lt_p(w0) || !int_lt_p(w1)) return DEC_BAD;
  fp2 x;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    x.c0.v[i] = w0[i];
    x.c1.v[i] = w1[i];
  }
  x.c0 = fp_to_mont(x.c0);
  x.c1 = fp_to_mont(x.c1);
  fp2 rhs = fp2_add(fp2_mul(fp2_sqr(x), x), fp2_c(cst::B2));
  fp2 y;
  if (!fp2_sqrt(y, rhs)) return DEC_BAD;
  if (fp2_lex_largest(y) != (bool)(flags & 1)) y = fp2_neg(y);
  out.x = x;
  out.y = y;
  if (subgroup && !g2_in_subgroup(out)) return DEC_BAD;
  return DEC_OK;
}

DH_DEV void st_be48(uint8_t* out, const fp& canon) {
#pragma unroll
  for (int i = 0; i < 12; i++) *(uint32_t*)(out + 44 - 4 * i) = __builtin_bswap32(canon.v[i]);
}

// compressed encodings of a finite affine point / of a Jacobian point (infinity: the 0xc0 encoding)
DH_DEV void g1_compress_aff(uint8_t* out, const aff<fp>& a) {
  st_be48(out, fp_from_mont(a.x));
  out[0] |= 0x80 | (fp_lex_gt_half(a.y) ? 0x20 : 0);
}
DH_DEV void g2_compress_aff(uint8_t* out, const aff<fp2>& a) {
  st_be48(out, fp_from_mont(a.x.c1));
  st_be48(out + 48, fp_from_mont(a.x.c0));
  out[0] |= 0x80 | (fp2_lex_largest(a.y) ? 0x20 : 0);
}
DH_DEV void g1_compress(uint8_t* out, const jac<fp>& p) {
  if (jac_is_inf(p)) {
    for (int i = 0; i < 48; i++) out[i] = 0;
    out[0] = 0xc0;
    return;
  }
  g1_compress_aff(out, jac_to_aff(p));
}

DH_DEV void g2_compress(uint8_t* out, const jac<fp2>& p) {
  if (jac_is_inf(p)) {
    for (int i = 0; i < 96; i++) out[i] = 0;
    out[0] = 0xc0;
    return;
  }
  g2_compress_aff(out, jac_to_aff(p));
}

}  // namespace dh
