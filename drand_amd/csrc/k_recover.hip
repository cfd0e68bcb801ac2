// Threshold-BLS Recover on gfx950: kyber v1.1.18 sign/tbls Recover + share.RecoverCommit as called at
// /root/reference/chain/beacon/chainstore.go:202 (then VerifyRecovered at :207), batched over rounds.
//
//   k_repack_partials   (2-byte BE index || sig) records -> aligned signatures + share indices
//   k_pubpoly_eval      PubPoly.Eval(i) = sum_j C_j (i+1)^j for every signer index (Horner, small scalars)
//   [partial signatures decoded by k_prep_sig, hash points by k_prep_msg32, RLC scalars by k_scalars]
//   batch VerifyPartial: sum_{j,i} r_ji sigma_ji  vs  per signer i: [h] sum_j r_ji Q_j  (grouped MSM), then
//   k_pair_miller       one lane per pair of the multi-pairing prod_i e(pk_i, B_i) e(-g, A) -> Miller value
//   k_pair_product      one lane: product of the Miller values, final exponentiation, == 1
//   k_partial_leaf      per-partial VerifyPartial (only when the batch check fails)
//   k_partial_meta      per round: the round of each partial; indices outside the group are rejected
//   k_select_lagrange   per round: first t valid partials, index order, duplicates dropped, Lagrange at 0 (F_r)
//   k_lagrange          per round: sum_k lambda_k sigma_k (Straus, shared doublings)
//   k_compress          recovered signatures -> compressed bytes
#include "kcommon.hpp"
#include "fr.hpp"

namespace dh {

// per Lagrange term: NAF pos mask (8 words), neg mask (8), width-4 NAF nibbles (32), regular 4-bit window digits (32)
constexpr int LAM_WORDS = 80;

__global__ void k_repack_partials(const uint8_t* __restrict__ raw, size_t n, int sig_len, uint8_t* __restrict__ sigs,
                                  uint32_t* __restrict__ idx) {
  size_t i = gtid();
  if (i >= n) return;
  const uint8_t* r = raw + i * (size_t)(2 + sig_len);
  idx[i] = ((uint32_t)r[0] << 8) | r[1];
  uint32_t* o = (uint32_t*)(sigs + i * (size_t)sig_len);
  for (int w = 0; w < sig_len / 4; w++) {
    const uint8_t* q = r + 2 + 4 * w;
    o[w] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
  }
}

// commits: t affine key-group points (AoS); out[i] = Eval(i) Jacobian, x = i + 1
template <class K>
__global__ void k_pubpoly_eval(const uint32_t* __restrict__ commits, int t, int n_nodes, uint32_t* __restrict__ out) {
  size_t i = gtid();
  if (i >= (size_t)n_nodes) return;
  const uint32_t x = (uint32_t)i + 1;
  jac<K> acc = jac_from_aff(ld_aff_aos<K>(commits, t - 1));
  for (int j = t - 2; j >= 0; j--) {
    // acc = [x] acc + C_j
    jac<K> base = acc, r = jac_inf<K>();
    for (int b = 31 - __builtin_clz(x); b >= 0; b--) {
      r = jac_dbl(r);
      if ((x >> b) & 1) r = jac_add(r, base);
    }
    acc = jac_add_aff(r, ld_aff_aos<K>(commits, j));
  }
  st_jac_aos<K>(out, i, acc);
}

// Miller loop of one pair per lane. P side G1, Q side G2 (Jacobian AoS arrays); cofactor clearing of the
// hash side is applied here (clear_p / clear_q); neg_p negates P. Output: fp12 Miller value, skip flag.
__global__ __launch_bounds__(64) void k_pair_miller(const uint32_t* __restrict__ P, const uint32_t* __restrict__ Q,
                                                    size_t npairs, int clear_p, int clear_q, const uint8_t* __restrict__ live,
                                                    uint32_t* __restrict__ f_out, uint8_t* __restrict__ skip_out) {
  size_t i = gtid();
  if (i >= npairs) return;
  jac<fp> p = ld_jac_aos<fp>(P, i);
  jac<fp2> q = ld_jac_aos<fp2>(Q, i);
  if (clear_p) p = h2c_clear_g1(p);
  if (clear_q) q = h2c_clear_g2(q);
  bool skip = jac_is_inf(p) || jac_is_inf(q) || (live && !live[i]);
  fp12 f = fp12_one();
  if (!skip) {
    aff<fp> pa[1] = {jac_to_aff(p)};
    aff<fp2> qa[1] = {jac_to_aff(q)};
    bool sk[1] = {false};
    f = miller_loop<1>(pa, qa, sk);
  }
  uint32_t* o = f_out + i * 144;
  const fp2* c = &f.c0.c0;
  for (int k = 0; k < 6; k++) {
    st_f<fp2>(o + 24 * k, c[k]);
  }
  skip_out[i] = skip ? 1 : 0;
}

__global__ void k_pair_product(const uint32_t* __restrict__ f_in, const uint8_t* __restrict__ skip, size_t npairs,
                               uint8_t* __restrict__ pass) {
  if (gtid() != 0) return;
  fp12 acc = fp12_one();
  for (size_t i = 0; i < npairs; i++) {
    if (skip[i]) continue;
    fp12 f;
    fp2* c = &f.c0.c0;
    for (int k = 0; k < 6; k++) ld_f<fp2>(c[k], f_in + i * 144 + 24 * k);
    acc = fp12_mul(acc, f);
  }
  *pass = fp12_is_one(final_exp(acc)) ? 1 : 0;
}

// one lane per round j: round_of[e] = j for its partials e in [off[j], off[j+1]) (offsets relative to the first
// partial); a share index outside the group has no public share (include/drandhip.h): status -> DEC_BAD, so its RLC
// scalar is 0 and the batch check ignores it
__global__ __launch_bounds__(256) void k_partial_meta(const uint32_t* __restrict__ off, size_t n_rounds,
                                                      const uint32_t* __restrict__ share_idx, int n_nodes,
                                                      uint32_t* __restrict__ round_of, uint8_t* __restrict__ status) {
  size_t j = gtid();
  if (j >= n_rounds) return;
  for (uint32_t e = off[j]; e < off[j + 1]; e++) {
    round_of[e] = (uint32_t)j;
    if (share_idx[e] >= (uint32_t)n_nodes) status[e] = DEC_BAD;
  }
}

// MSM group of partial e for the per-signer sums: its share index (those outside the group carry a zero scalar)
__global__ __launch_bounds__(256) void k_clamp_group(const uint32_t* __restrict__ share_idx, size_t np, uint32_t hi,
                                                     uint32_t* __restrict__ grp) {
  size_t e = gtid();
  if (e < np) grp[e] = min(share_idx[e], hi);
}

// after the batch check: ok[e] = 1 iff partial e decoded (subgroup point, index inside the group)
__global__ __launch_bounds__(256) void k_ok_from_status(const uint8_t* __restrict__ status, size_t np, uint8_t* __restrict__ ok) {
  size_t e = gtid();
  if (e < np) ok[e] = status[e] == DEC_OK ? 1 : 0;
}

// Recover's selection and Lagrange basis per round, one lane per round (kyber v1.1.18 tbls.Recover +
// share.RecoverCommit / xyCommit, restated in oracle/bls_oracle.c or_recover): the first t valid partials in arrival
// order (Recover stops at t), sorted by share index (stable), duplicate indices dropped; fewer than t distinct ->
// not recovered. Then (k_lambda) lambda_k = prod_{m != k} x_m / (x_m - x_k) over x = index + 1 in F_r (one batch
// inversion), written for k_lagrange as NAF digit masks (G1) and width-4 NAF nibbles (G2). sel/key: t words per round;
// den: 8 t words per round (scratch); lam: LAM_WORDS (48) t words per round: per term pos mask (8), neg mask (8),
// nibbles (32).
__global__ __launch_bounds__(64) void k_select_lagrange(const uint32_t* __restrict__ off, const uint8_t* __restrict__ ok,
                                                        const uint32_t* __restrict__ share_idx, int t, size_t n_rounds,
                                                        uint32_t* __restrict__ sel, uint32_t* __restrict__ key,
                                                        uint8_t* __restrict__ rok) {
  const size_t j = gtid();
  if (j >= n_rounds) return;
  uint32_t* S = sel + j * (size_t)t;
  uint32_t* K = key + j * (size_t)t;
  int kept = 0;
  for (uint32_t e = off[j]; e < off[j + 1] && kept < t; e++) {
    if (!ok[e]) continue;
    const uint32_t ki = share_idx[e];
    int pos = kept;
    while (pos > 0 && K[pos - 1] > ki) {
      K[pos] = K[pos - 1];
      S[pos] = S[pos - 1];
      pos--;
    }
    K[pos] = ki;
    S[pos] = e;
    kept++;
  }
  int nd = 0;
  for (int a = 0; a < kept; a++) {
    if (nd && K[nd - 1] == K[a]) continue;
    K[nd] = K[a];
    S[nd] = S[a];
    nd++;
  }
  rok[j] = nd < t ? 0 : 1;
}

// lambda rows per recovered round; a round whose selected indices equal round 0's (the usual case: the same nodes
// answer every round) points at round 0's rows (lam_set[j] = 0) instead of recomputing the same basis, otherwise
// lam_set[j] = j. lam_set is what k_lagrange reads.
__global__ __launch_bounds__(64) void k_lambda(const uint32_t* __restrict__ key, const uint8_t* __restrict__ rok, int t,
                                               size_t n_rounds, uint32_t* __restrict__ den, uint32_t* __restrict__ lam,
                                               uint32_t* __restrict__ lam_set, uint32_t* __restrict__ own, int masks) {
  const size_t j = gtid();
  if (j >= n_rounds || !rok[j]) return;
  const uint32_t* K = key + j * (size_t)t;
  if (j > 0 && rok[0]) {
    bool same = true;
    for (int k = 0; k < t && same; k++) same = K[k] == key[k];
    if (same) {
      lam_set[j] = 0;
      return;
    }
  }
  lam_set[j] = (uint32_t)j;
  if (j > 0) atomicAdd(own, 1u);
  uint32_t* D = den + j * (size_t)t * 8;
  uint32_t* L = lam + j * (size_t)t * LAM_WORDS;
  // x_m in Montgomery form once per round, parked in each term's nibble words (written in pass 2, after the last use)
  for (int m = 0; m < t; m++) {
    const fr xm = fr_from_u32(K[m] + 1);
    for (int w = 0; w < 8; w++) L[LAM_WORDS * m + 16 + w] = xm.v[w];
  }
  auto ldx = [&](int m) {
    fr x;
    for (int w = 0; w < 8; w++) x.v[w] = L[LAM_WORDS * m + 16 + w];
    return x;
  };
  // pass 1: lambda_k = N / (x_k prod_{m != k} (x_m - x_k)) with N = prod_m x_m: the denominators (scratch) and their
  // prefix products (into lam's first words); one product per (k, m) (r04 formed each numerator too and converted x_m
  // to Montgomery form in the inner loop: three products per pair)
  fr pre = fr_one(), N = fr_one();
  for (int k = 0; k < t; k++) {
    const fr xk = ldx(k);
    N = fr_mul(N, xk);
    fr dk = xk;
    for (int m = 0; m < t; m++)
      if (m != k) dk = fr_mul(dk, fr_sub(ldx(m), xk));
    for (int w = 0; w < 8; w++) {
      L[LAM_WORDS * k + w] = pre.v[w];
      D[8 * k + w] = dk.v[w];
    }
    pre = fr_mul(pre, dk);
  }
  // pass 2: one inversion of the product, then lambda_k from the back
  fr inv = fr_inv(pre);
  for (int k = t - 1; k >= 0; k--) {
    fr pk, dk;
    for (int w = 0; w < 8; w++) {
      pk.v[w] = L[LAM_WORDS * k + w];
      dk.v[w] = D[8 * k + w];
    }
    const fr dinv = fr_mul(inv, pk);
    inv = fr_mul(inv, dk);
    uint32_t words[8], sw[8], pos[8], neg[8];
    fr_to_words(fr_mul(N, dinv), words);
    // the NAFs recode the shorter of lambda and r - lambda (digits negated for the latter): the chains skip the
    // doublings above the highest digit, so a small +-lambda costs a short chain (fr_short)
    const bool flip = fr_short(words, sw);
    if (masks) {  // the G1 chain's NAF digit masks (G2 reads the nibbles)
      fr_naf_masks(sw, pos, neg);
      for (int w = 0; w < 8; w++) {
        L[LAM_WORDS * k + w] = flip ? neg[w] : pos[w];
        L[LAM_WORDS * k + 8 + w] = flip ? pos[w] : neg[w];
      }
    }
    if (masks) continue;  // G1 chains read the NAF masks only
    // G2: the width-4 NAF for round 0's basis, which coherent waves share (k_lagrange runs every other basis on the
    // regular windows); the regular digits for every basis
    if (j == 0) {
      uint32_t* nib = L + LAM_WORDS * k + 16;
      fr_wnaf4(sw, nib);
      if (flip)
        for (int w = 0; w < 32; w++) {
          // a nonzero nibble v (1..4 or 9..12) changes sign: v ^ 8
          const uint32_t x = nib[w], nz = (x | (x >> 1) | (x >> 2) | (x >> 3)) & 0x11111111u;
          nib[w] = x ^ (nz << 3);
        }
    }
    fr_reg4(words, L + LAM_WORDS * k + 48);
  }
}

// VerifyPartial for each listed partial e: pubshare = shares[idx[e]], hash point q[round_of[e]]
template <class F>
__global__ __launch_bounds__(64) void k_partial_leaf(const uint32_t* __restrict__ list, size_t m,
                                                     const uint32_t* __restrict__ sig_aff, const uint8_t* __restrict__ status,
                                                     const uint32_t* __restrict__ share_idx,
                                                     const uint32_t* __restrict__ round_of, const uint32_t* __restrict__ q_pts,
                                                     const uint32_t* __restrict__ shares, int n_nodes,
                                                     uint8_t* __restrict__ ok_out) {
  size_t t = gtid();
  if (t >= m) return;
  const uint32_t e = list[t];
  const uint32_t si = share_idx[e];
  if (status[e] != DEC_OK || si >= (uint32_t)n_nodes) {
    ok_out[e] = 0;
    return;
  }
  jac<F> S = jac_from_aff(ld_aff_aos<F>(sig_aff, e));
  bool ok;
  if constexpr (sizeof(F) == sizeof(fp2)) {
    jac<fp2> H = h2c_clear_g2(ld_jac_aos<fp2>(q_pts, round_of[e]));
    jac<fp> pk = ld_jac_aos<fp>(shares, si);
    jac<fp> Pp[2] = {pk, jac_neg(g1_gen())};
    jac<fp2> Qq[2] = {H, S};
    ok = pairing_check<2>(Pp, Qq);
  } else {
    jac<fp> H = h2c_clear_g1(ld_jac_aos<fp>(q_pts, round_of[e]));
    jac<fp2> pk = ld_jac_aos<fp2>(shares, si);
    jac<fp> Pp[2] = {H, jac_neg(S)};
    jac<fp2> Qq[2] = {pk, g2_gen()};
    ok = pairing_check<2>(Pp, Qq);
  }
  ok_out[e] = ok ? 1 : 0;
}

// sigma_j = sum_k lambda_{j,k} sigma_{sel[j,k]}: Straus over t points with shared doublings.
// lam: per term the NAF masks of lambda (16 words); row set lam_set[j], or the round's own rows when lam_set is null.
// LG_LANES lanes per round, each running Straus (shared doublings) over every LG_LANES-th term of the
// interpolation sum sum_k lambda_k sigma_k; the partial sums meet in LDS and one lane of the round adds them. One
// lane per round left most of the chip idle at 10^4-10^5 rounds and ran 33 terms x 127 additions serially. With the
// width-4 NAF the 256 doublings per lane are a quarter of the chain's products, so r04 measured 2 lanes against 4 on
// one box: k_lagrange 119.7 -> 103.2 ms per 100k rounds (the last partial wave of workgroups sliced either way;
// profiles/r04/config_recover_lanes*). A workgroup is LG_LANES waves over the same 64 rounds, wave q
// running term lane q of each: rounds that selected the same signers (the usual case: the same nodes answer every
// round) have the same lambdas, so all 64 lanes of a wave take the same digits and branches. r03 put the LG_LANES
// lanes of a round side by side in ONE wave, whose lanes then followed LG_LANES different digit patterns and ran
// every addition step up to LG_LANES times, diverged.
constexpr int LG_LANES = 2, LG_MAXK = 17;  // terms per lane and pass (t <= 34: one pass)
// G2: the chain on the lazily reduced 28-bit form (fp2_28.hpp) over width-4 NAF digits and each partial's table of
// P, 3P, 5P, 7P (1/5 of the positions take an addition instead of 1/3), with the MSM's fast mixed additions (no
// exceptional-case tests); a chain that met an exceptional case ends with Z = 0 mod p and runs again with the exact
// formulas. G1 keeps the 32-bit Straus chain over the NAF masks.
// a point coordinate pair in the 28-bit form as the tables hold it, converted once per partial (k_wnaf_table_g2)
// instead of at each of the additions that read it: x.c0, x.c1, y.c0, y.c1, 16 words each (14 limbs + 2 pad)
constexpr int A28_WORDS = 64;
DH_DEV f28 ld_f28w(const uint32_t* p) {
  f28 a;
  const uint4* q = (const uint4*)p;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint4 t = q[i];
    a.l[4 * i] = t.x;
    a.l[4 * i + 1] = t.y;
    if (4 * i + 2 < 14) a.l[4 * i + 2] = t.z;
    if (4 * i + 3 < 14) a.l[4 * i + 3] = t.w;
  }
  return a;
}
DH_DEV void st_f28w(uint32_t* p, const f28& a) {
  uint4* q = (uint4*)p;
#pragma unroll
  for (int i = 0; i < 4; i++)
    q[i] = make_uint4(a.l[4 * i], a.l[4 * i + 1], 4 * i + 2 < 14 ? a.l[4 * i + 2] : 0u, 4 * i + 3 < 14 ? a.l[4 * i + 3] : 0u);
}
// G2 table per valid partial: the odd multiples P, 3P, ..., (2 NE - 1) P affine in the 28-bit form (NE x 64 words):
// NE = 4 for the width-4 NAF chains (digits up to 7), NE = 8 when some wave's rounds do not share one Lagrange basis and
// run the regular 4-bit windows (digits up to 15). The multiples come from co-Z additions (Meloni's ZADDU, the
// odd-multiples chain of Longa and Gebotys): 2P and P share a Z after the doubling (DBLU from affine P, 2M + 4S), and
// each (2j + 1) P = 2P + (2j - 1) P is one ZADDU (5M + 2S) that also returns 2P on the new Z, so the entries' Z's
// differ only by the factors d_j = X(2P) - X((2j - 1) P): Z_j = Z_{j-1} d_j. r04 took a doubling, a mixed and NE - 2
// full Jacobian additions (16M + ... each) and normalised every entry's own Z. Now each partial contributes ONE Z (its
// last entry's) to the lane's Montgomery chain over its TB_K partials (one variable-time Fp2 inversion per lane), and
// the walk back turns 1/Z_last into every 1/Z_j by the parked d_j's. The partials reaching k_lagrange decoded to
// subgroup points (order r), so 2P is never +-(2j - 1) P and no co-Z step meets an exceptional case.
constexpr int TB_K = 8;
DH_DEV void st_f228w(uint32_t* p, const f228& a) {
  st_f28w(p, a.c0);
  st_f28w(p + 16, a.c1);
}
DH_DEV f228 ld_f228w(const uint32_t* p) { return f228{ld_f28w(p), ld_f28w(p + 16)}; }
template <int NE>
__global__ __launch_bounds__(256) void k_wnaf_table_g2(const uint32_t* __restrict__ paff, const uint8_t* __restrict__ ok,
                                                       size_t n, uint32_t* __restrict__ tbl, uint32_t* __restrict__ zs) {
  // words per partial: table; scratch d_1 .. d_{NE-1}, Z_last, the product of the lane's earlier Z_last's (32 each)
  constexpr size_t TW = (size_t)NE * A28_WORDS, ZW = (size_t)(NE - 1) * 64;
  static_assert((NE + 1) * 32 <= ZW, "co-Z scratch");
  const size_t nth = (n + TB_K - 1) / TB_K;
  const size_t t = gtid();
  if (t >= nth) return;
  f228 pre = f2_one();
  bool any = false;
  uint32_t valid = 0;  // bit k: the lane's k-th partial is valid
#pragma unroll 1
  for (int k = 0; k < TB_K; k++) {
    const size_t e = t + (size_t)k * nth;  // lanes of a wave take consecutive partials
    if (e >= n || !ok[e]) continue;
    valid |= 1u << k;
    const aff<fp2> a = ld_aff_aos<fp2>(paff, e);
    const f228 px{f28_from_fp(a.x.c0), f28_from_fp(a.x.c1)}, py{f28_from_fp(a.y.c0), f28_from_fp(a.y.c1)};
    uint32_t* o = tbl + TW * e;
    uint32_t* z = zs + ZW * e;
    st_f228w(o, px);
    st_f228w(o + 32, py);
    // DBLU: 2P = (M^2 - 2S, M (S - X2) - 8B^2, 2y) and P on the same Z = (S, 8B^2), B = y^2, S = 4xB, M = 3x^2
    // (bounds in units of p per component; every stored value reduced below 2)
    const f228 B = f2_red(f2_sqr<2, true>(py));
    const f228 S = f2_red(f2_scale(f2_red(f2_mul<true>(px, B)), 4));
    const f228 M = f2_scale(f2_red(f2_sqr<2, true>(px)), 3);                                    // < 6
    f228 tx = f2_red(f2_lin<4, 4>(f2_sqr<6, true>(M), 1, S, -2));                               // (2, 4) + 4p - 2S
    // 8B^2: the scale's limb sums 8 (2^28 - 1) + a carry <= 7 stay inside int32 (f28_lin)
    const f228 e8 = f2_red(f2_scale(f2_red(f2_sqr<2, true>(B)), 8));
    f228 ty = f2_red(f2_lin<2, 2>(f2_mul<true>(M, f2_lin<2, 2>(S, 1, tx, -1)), 1, e8, -1));     // 6 x 4 -> (4, 6) + 2p - 8B^2
    f228 zl = f2_red(f2_scale(py, 2));                                                      // Z of 2P and P
    f228 rx = S, ry = e8;
#pragma unroll 1
    for (int j = 1; j < NE; j++) {
      // ZADDU(T = 2P, R = (2j - 1) P): R' = T + R, T' = T, both on Z d
      const f228 d = f2_lin<2, 2>(tx, 1, rx, -1);                                         // < 4
      const f228 C = f2_red(f2_sqr<4, true>(d));
      const f228 w1 = f2_red(f2_mul<true>(tx, C)), w2 = f2_red(f2_mul<true>(rx, C));
      const f228 ee = f2_lin<2, 2>(ty, 1, ry, -1);                                        // < 4
      const f228 a1 = f2_red(f2_mul<true>(ty, f2_lin<2, 2>(w1, 1, w2, -1)));
      rx = f2_red(f2_lin3<4, 4>(f2_sqr<4, true>(ee), 1, w1, -1, w2, -1));                       // (2, 4) + 4p - W1 - W2
      ry = f2_red(f2_lin<2, 2>(f2_mul<true>(ee, f2_lin<2, 2>(w1, 1, rx, -1)), 1, a1, -1));      // 4 x 4 -> (4, 6) + 2p - A1
      tx = w1;
      ty = a1;
      zl = f2_red(f2_mul<true>(zl, d));
      st_f228w(z + 32 * (j - 1), f2_red(d));
      uint32_t* sl = o + A28_WORDS * j;
      st_f228w(sl, rx);
      st_f228w(sl + 32, ry);
    }
    st_f228w(z + 32 * (NE - 1), zl);
    if (any) st_f228w(z + 32 * NE, pre);  // the product of the lane's Z_last's before this one
    pre = any ? f2_red(f2_mul<true>(pre, zl)) : zl;
    any = true;
  }
  if (!any) return;
  f228 inv = f2_from_fp2(fp2_inv_vt(f2_to_fp2(pre)));  // 1 / (product of the lane's Z_last's)
#pragma unroll 1
  for (int k = TB_K - 1; k >= 0; k--) {
    if (!(valid >> k & 1)) continue;
    const size_t e = t + (size_t)k * nth;
    const uint32_t* z = zs + ZW * e;
    uint32_t* o = tbl + TW * e;
    const bool earlier = (valid & ((1u << k) - 1)) != 0;  // a valid partial before this one in the lane
    // 1 / Z_last: inv for the lane's first partial, else inv * (product before it); inv moves past Z_last
    f228 zi = inv;
    if (earlier) {
      zi = f2_red(f2_mul<true>(inv, ld_f228w(z + 32 * NE)));
      inv = f2_red(f2_mul<true>(inv, ld_f228w(z + 32 * (NE - 1))));
    }
#pragma unroll 1
    for (int j = NE - 1; j >= 1; j--) {
      uint32_t* sl = o + A28_WORDS * j;
      const f228 z2 = f2_red(f2_sqr<2, true>(zi));
      st_f228w(sl, f2_red(f2_mul<true>(ld_f228w(sl), z2)));
      st_f228w(sl + 32, f2_red(f2_mul<true>(ld_f228w(sl + 32), f2_red(f2_mul<true>(z2, zi)))));
      if (j > 1) zi = f2_red(f2_mul<true>(zi, ld_f228w(z + 32 * (j - 1))));  // 1 / Z_{j-1} = d_j / Z_j
    }
  }
}
// need[e] = 1 for the partials some recovered round selected (sel, t per round): the tables are built for those only
// (with more than t partials per round, every valid partial got a table that no round reads)
__global__ void k_mark_selected(const uint32_t* __restrict__ sel, const uint8_t* __restrict__ rok, int t, size_t n_rounds,
                                uint8_t* __restrict__ need) {
  const size_t i = gtid();
  if (i >= n_rounds * (size_t)t) return;
  if (rok[i / t]) need[sel[i]] = 1;
}
hipError_t launch_mark_selected(const uint32_t* sel, const uint8_t* rok, int t, size_t n_rounds, size_t np, uint8_t* need,
                                hipStream_t st) {
  hipError_t e = hipMemsetAsync(need, 0, np, st);
  if (e != hipSuccess || !n_rounds) return e;
  hipLaunchKernelGGL(k_mark_selected, dim3(nblk(n_rounds * (size_t)t, 256)), dim3(256), 0, st, sel, rok, t, n_rounds, need);
  return hipGetLastError();
}

hipError_t launch_wnaf_table_g2(const uint32_t* paff, const uint8_t* ok, size_t n, int entries, uint32_t* tbl, uint32_t* zs,
                                hipStream_t st) {
  if (!n) return hipSuccess;
  if (entries == 8)
    hipLaunchKernelGGL(k_wnaf_table_g2<8>, dim3(nblk((n + TB_K - 1) / TB_K, 256)), dim3(256), 0, st, paff, ok, n, tbl, zs);
  else
    hipLaunchKernelGGL(k_wnaf_table_g2<4>, dim3(nblk((n + TB_K - 1) / TB_K, 256)), dim3(256), 0, st, paff, ok, n, tbl, zs);
  return hipGetLastError();
}
size_t wnaf_table_scratch_bytes(size_t n, int entries) { return n * (size_t)(entries - 1) * 64 * 4; }
size_t lam_words() { return LAM_WORDS; }

// the width-4 NAF Straus chain of one lane's terms over their tables (nibble words of the current 8 positions in nw)
// a table entry's coordinates for j228_madd_ld, loaded where the formula uses them (k = 0: x, 1: y, negated for a
// negative digit): the chain's mixed addition then holds neither coordinate across the products before its use
DH_DEV auto entry_ld(const uint32_t* pt, bool neg) {
  return [pt, neg](int k) {
    const f228 c{ld_f28w(pt + 32 * k), ld_f28w(pt + 32 * k + 16)};
    return k && neg ? f2_neg3(c) : c;
  };
}
template <bool EXACT>
DH_DEV j228 lagrange_wnaf28(const uint32_t* __restrict__ L, int q, int nl, int c0, int nc, const uint32_t* __restrict__ tbl,
                            uint32_t tw, const uint32_t* idx, uint32_t* nw) {
  j228 acc = j228_inf();
#pragma unroll 1
  for (int b = 255; b >= 0; b--) {
    if ((b & 7) == 7)
      for (int i = 0; i < nc; i++) nw[i] = L[(size_t)(q + nl * (c0 + i)) * LAM_WORDS + 16 + (b >> 3)];
    if (!acc.inf) acc = j228_dbl<true>(acc);
#pragma unroll 1
    for (int i = 0; i < nc; i++) {
      const uint32_t v = (nw[i] >> (4 * (b & 7))) & 15;
      if (v) {
        const uint32_t* pt = tbl + (size_t)tw * idx[i] + A28_WORDS * ((v & 7) - 1);
        acc = j228_madd_ld<EXACT, true>(acc, entry_ld(pt, v & 8));
      }
    }
  }
  return acc;
}

// the regular 4-bit window chain (fr_reg4 digits, every one odd and nonzero) of one lane's terms over their 8-entry
// tables: four doublings and one mixed addition per term at each of the 64 windows, with no digit-dependent branch —
// the path of a wave whose rounds use different Lagrange bases (random signer subsets), where the width-4 NAF's
// per-lane digits left the wave running nearly every position's addition for some lane (k_lagrange 540-590 ms per
// 100k random-subset rounds against 103-120 ms coherent, profiles/r04/config_recover_random_*)
template <bool EXACT>
DH_DEV j228 lagrange_reg28(const uint32_t* __restrict__ L, int q, int nl, int c0, int nc, const uint32_t* __restrict__ tbl,
                           uint32_t tw, const uint32_t* idx, uint32_t* nw) {
  j228 acc = j228_inf();
#pragma unroll 1
  for (int wi = 63; wi >= 0; wi--) {
    if ((wi & 7) == 7)
      for (int i = 0; i < nc; i++) nw[i] = L[(size_t)(q + nl * (c0 + i)) * LAM_WORDS + 48 + (wi >> 3)];
    if (!acc.inf) {
#pragma unroll 1
      for (int d = 0; d < 4; d++) acc = j228_dbl<true>(acc);
    }
#pragma unroll 1
    for (int i = 0; i < nc; i++) {
      const uint32_t v = (nw[i] >> (4 * (wi & 7))) & 15;
      const uint32_t* pt = tbl + (size_t)tw * idx[i] + A28_WORDS * (v & 7);
      acc = j228_madd_ld<EXACT, true>(acc, entry_ld(pt, v & 8));
    }
  }
  return acc;
}

// Blocks [0, full) take every term of their 64 rounds (term lanes q = 0 .. LG_LANES - 1, written to out); the
// remainder blocks, the last partial wave of workgroups over the chip, are split into S slices each (grid entries
// full + r * S + s): slice s runs term lanes s * LG_LANES + q of NL = S * LG_LANES and writes its partial sum to
// part_out[(j - 64 full) * S + s], summed into out by k_lagrange_sum. At 100k rounds the 1,563 blocks are 6 waves of
// 256 CUs and 27 blocks whose full-length chains left the other CUs idle for the 7th (~12% of the kernel); sliced,
// that wave's chains are ~1/3 as long.
template <class F>
__global__ __launch_bounds__(64 * LG_LANES) void k_lagrange(const uint32_t* __restrict__ sel, const uint32_t* __restrict__ lam,
                                                            const uint32_t* __restrict__ lam_set, const uint8_t* __restrict__ ok,
                                                            int t, size_t n_rounds, const uint32_t* __restrict__ sig_aff,
                                                            const uint32_t* __restrict__ tbl, uint32_t tw, int reg,
                                                            uint32_t* __restrict__ out, uint32_t full, uint32_t S,
                                                            uint32_t* __restrict__ part_out) {
  constexpr int JW = sizeof(F) / 4 * 3;
  __shared__ uint32_t part[(LG_LANES - 1) * 64 * JW];  // the partial sums of waves 1 .. LG_LANES - 1
  __shared__ uint32_t idxS[64 * LG_LANES][LG_MAXK], lpS[64 * LG_LANES][LG_MAXK], lnS[64 * LG_LANES][LG_MAXK];
  __shared__ uint32_t accS[sizeof(F) == sizeof(fp2) ? 64 * LG_LANES * JW : 1];  // G2: the lanes' sums over passes
  const bool sliced = blockIdx.x >= full;
  const uint32_t r = blockIdx.x - full;
  const size_t blk = sliced ? full + r / S : blockIdx.x;
  const int sl = sliced ? (int)(r % S) : 0, nl = sliced ? (int)S * LG_LANES : LG_LANES;
  const int q = sl * LG_LANES + (int)(threadIdx.x / 64);  // term lane: wave-uniform
  const size_t j = blk * 64 + threadIdx.x % 64;
  jac<F> acc = jac_inf<F>();
  // wave-uniform: do the wave's recovered rounds share one Lagrange basis (lam_set)? If not and the tables hold 8
  // entries (reg), the regular windows instead of the width-4 NAF
  const bool live = j < n_rounds && ok[j];
  const uint32_t myset = live ? (lam_set ? lam_set[j] : (uint32_t)j) : 0xffffffffu;
  const unsigned long long act = __ballot(live);
  const uint32_t ref = __shfl(myset, act ? __ffsll((long long)act) - 1 : 0);
  // (a wave coherent on a basis other than round 0's runs the regular windows too: k_lambda writes the width-4 NAF
  // nibbles for round 0's basis only)
  const bool regular = reg && (!__all(!live || myset == ref) || ref != 0);
  // G2: the width-4 NAF nibbles exist for round 0's basis only (k_lambda parks x_m in the other bases' nibble words),
  // so a wave on another basis needs the regular windows, i.e. tables of 8 entries (reg). The host sets reg whenever
  // any round has a basis of its own (drandhip.cpp recover_core, `own`), so this never fires; if it did, the wave's
  // rounds are left at infinity, which VerifyRecovered rejects (not recovered) instead of reading x_m values as digits.
  // (G1 chains read NAF digit masks, which k_lambda writes for every basis.)
  const bool lost_basis = sizeof(F) == sizeof(fp2) && !reg && ref != 0;
  if (live && !lost_basis) {
    const uint32_t* L = lam + (lam_set ? (size_t)lam_set[j] : j) * t * LAM_WORDS;  // per term: NAF masks, wNAF nibbles
    const uint32_t* Sel = sel + j * (size_t)t;
    const int nt = q < t ? (t - q + nl - 1) / nl : 0;  // terms of this lane: k = q + nl i
    // digit masks of the current 32-bit chunk and the point indices live in LDS (dynamic indices, no scratch)
    uint32_t* idx = idxS[threadIdx.x];
    uint32_t* lp = lpS[threadIdx.x];
    uint32_t* ln = lnS[threadIdx.x];
    for (int c0 = 0; c0 < nt; c0 += LG_MAXK) {  // more than LG_MAXK terms: several passes
      const int nc = nt - c0 < LG_MAXK ? nt - c0 : LG_MAXK;
      for (int i = 0; i < nc; i++) idx[i] = Sel[q + nl * (c0 + i)];
      if constexpr (sizeof(F) == sizeof(fp2)) {
        // width-4 NAF over the partials' tables; a chain that met an exceptional case (poisoned) runs again with
        // the exact formulas. The running sum of the passes waits in the lane's LDS slot (accS), not in 72 registers
        // live across the chain, which holds 512
        j228 a28 = regular ? lagrange_reg28<false>(L, q, nl, c0, nc, tbl, tw, idx, lp)
                           : lagrange_wnaf28<false>(L, q, nl, c0, nc, tbl, tw, idx, lp);
        if (j228_poisoned(a28))
          a28 = regular ? lagrange_reg28<true>(L, q, nl, c0, nc, tbl, tw, idx, lp)
                        : lagrange_wnaf28<true>(L, q, nl, c0, nc, tbl, tw, idx, lp);
        if (!a28.inf) {
          const jac<F> s{f2_to_fp2(a28.x), f2_to_fp2(a28.y), f2_to_fp2(a28.z)};
          st_jac_aos<F>(accS, threadIdx.x, c0 ? jac_add(ld_jac_aos<F>(accS, threadIdx.x), s) : s);
        } else if (!c0) {
          st_jac_aos<F>(accS, threadIdx.x, jac_inf<F>());
        }
        asm volatile("" ::: "memory");  // the sum is reloaded from LDS, not kept in registers across the next chain
        if (c0 + LG_MAXK >= nt) acc = ld_jac_aos<F>(accS, threadIdx.x);
        continue;
      }
      jac<F> part_acc = jac_inf<F>();
      for (int b = 255; b >= 0; b--) {
        if ((b & 31) == 31)
          for (int i = 0; i < nc; i++) {
            const uint32_t* Lk = L + (size_t)(q + nl * (c0 + i)) * LAM_WORDS;
            lp[i] = Lk[b >> 5];
            ln[i] = Lk[8 + (b >> 5)];
          }
        part_acc = jac_dbl(part_acc);
        for (int i = 0; i < nc; i++) {
          const uint32_t pb = (lp[i] >> (b & 31)) & 1, nb = (ln[i] >> (b & 31)) & 1;
          if (pb | nb) {
            aff<F> pt = ld_aff_aos<F>(sig_aff, idx[i]);
            if (nb) pt.y = f_neg(pt.y);
            part_acc = jac_add_aff(part_acc, pt);
          }
        }
      }
      acc = jac_add(acc, part_acc);
    }
  }
  const int w = (int)(threadIdx.x / 64);
  if (w) st_jac_aos<F>(part, threadIdx.x - 64, acc);
  __syncthreads();
  if (w == 0 && j < n_rounds) {
    for (int r2 = 1; r2 < LG_LANES; r2++) acc = jac_add(acc, ld_jac_aos<F>(part, (size_t)(r2 - 1) * 64 + threadIdx.x));
    if (sliced) st_jac_aos<F>(part_out, (j - (size_t)full * 64) * S + sl, acc);
    else st_jac_aos<F>(out, j, acc);
  }
}
template <class F>
__global__ __launch_bounds__(64) void k_lagrange_sum(const uint32_t* __restrict__ part, uint32_t S, size_t j0, size_t n_rounds,
                                                     uint32_t* __restrict__ out) {
  const size_t j = j0 + gtid();
  if (j >= n_rounds) return;
  jac<F> acc = ld_jac_aos<F>(part, (j - j0) * S);
  for (uint32_t s = 1; s < S; s++) acc = jac_add(acc, ld_jac_aos<F>(part, (j - j0) * S + s));
  st_jac_aos<F>(out, j, acc);
}

template <class F>
__global__ __launch_bounds__(64) void k_compress(const uint32_t* __restrict__ pts, size_t n, uint8_t* __restrict__ out,
                                                 uint32_t* __restrict__ aff_out, uint8_t* __restrict__ status_out) {
  size_t j = gtid();
  if (j >= n) return;
  jac<F> p = ld_jac_aos<F>(pts, j);
  const bool inf = jac_is_inf(p);
  if (inf) {
    if constexpr (sizeof(F) == sizeof(fp)) g1_compress(out + 48 * j, p);
    else g2_compress(out + 96 * j, p);
  }
  const aff<F> a = inf ? aff<F>{F{}, F{}} : jac_to_aff(p);
  if (!inf) {
    if constexpr (sizeof(F) == sizeof(fp)) g1_compress_aff(out + 48 * j, a);
    else g2_compress_aff(out + 96 * j, a);
  }
  // the affine point and decode status VerifyRecovered's batch needs (what decoding these bytes gives: the point is a
  // combination of subgroup-checked partials, so it is in the subgroup; infinity is rejected like a decoded one)
  if (aff_out) {
    st_aff_aos<F>(aff_out, j, a);
    status_out[j] = inf ? DEC_BAD : DEC_OK;
  }
}

// assemble the pairs of the batched VerifyPartial check:
//   G2 signatures: (share_i, [h] B_i) for i < n_nodes, then (-g1, A)
//   G1 signatures: ([h] B_i, share_i) for i < n_nodes, then (-A, g2)
template <class F>
__global__ __launch_bounds__(64) void k_recover_pairs(const uint32_t* __restrict__ shares, const uint32_t* __restrict__ B,
                                                      const uint32_t* __restrict__ A, int n_nodes,
                                                      uint32_t* __restrict__ P, uint32_t* __restrict__ Q) {
  size_t i = gtid();
  if (i > (size_t)n_nodes) return;
  if constexpr (sizeof(F) == sizeof(fp2)) {
    if (i < (size_t)n_nodes) {
      st_jac_aos<fp>(P, i, ld_jac_aos<fp>(shares, i));
      st_jac_aos<fp2>(Q, i, h2c_clear_g2(ld_jac_aos<fp2>(B, i)));
    } else {
      st_jac_aos<fp>(P, i, jac_neg(g1_gen()));
      st_jac_aos<fp2>(Q, i, ld_jac_aos<fp2>(A, 0));
    }
  } else {
    if (i < (size_t)n_nodes) {
      st_jac_aos<fp>(P, i, h2c_clear_g1(ld_jac_aos<fp>(B, i)));
      st_jac_aos<fp2>(Q, i, ld_jac_aos<fp2>(shares, i));
    } else {
      st_jac_aos<fp>(P, i, jac_neg(ld_jac_aos<fp>(A, 0)));
      st_jac_aos<fp2>(Q, i, g2_gen());
    }
  }
}

// ---------------------------------------------------------------- launchers
hipError_t launch_repack_partials(const uint8_t* raw, size_t n, int sig_len, uint8_t* sigs, uint32_t* idx, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_repack_partials, dim3(nblk(n, 256)), dim3(256), 0, st, raw, n, sig_len, sigs, idx);
  return hipGetLastError();
}

hipError_t launch_pubpoly_eval(int key_g2, const uint32_t* commits, int t, int n_nodes, uint32_t* out, hipStream_t st) {
  if (key_g2) hipLaunchKernelGGL(k_pubpoly_eval<fp2>, dim3(nblk(n_nodes, 64)), dim3(64), 0, st, commits, t, n_nodes, out);
  else hipLaunchKernelGGL(k_pubpoly_eval<fp>, dim3(nblk(n_nodes, 64)), dim3(64), 0, st, commits, t, n_nodes, out);
  return hipGetLastError();
}

hipError_t launch_pair_check(const uint32_t* P, const uint32_t* Q, size_t npairs, int clear_p, int clear_q,
                             const uint8_t* live, uint32_t* f_tmp, uint8_t* skip_tmp, uint8_t* pass, hipStream_t st) {
  hipLaunchKernelGGL(k_pair_miller, dim3(nblk(npairs, 64)), dim3(64), 0, st, P, Q, npairs, clear_p, clear_q, live, f_tmp,
                     skip_tmp);
  hipLaunchKernelGGL(k_pair_product, dim3(1), dim3(64), 0, st, f_tmp, skip_tmp, npairs, pass);
  return hipGetLastError();
}

hipError_t launch_partial_leaf(int sig_g2, const uint32_t* list, size_t m, const uint32_t* sig_aff, const uint8_t* status,
                               const uint32_t* share_idx, const uint32_t* round_of, const uint32_t* q_pts,
                               const uint32_t* shares, int n_nodes, uint8_t* ok_out, hipStream_t st) {
  if (!m) return hipSuccess;
  if (sig_g2)
    hipLaunchKernelGGL(k_partial_leaf<fp2>, dim3(nblk(m, 64)), dim3(64), 0, st, list, m, sig_aff, status, share_idx, round_of,
                       q_pts, shares, n_nodes, ok_out);
  else
    hipLaunchKernelGGL(k_partial_leaf<fp>, dim3(nblk(m, 64)), dim3(64), 0, st, list, m, sig_aff, status, share_idx, round_of,
                       q_pts, shares, n_nodes, ok_out);
  return hipGetLastError();
}

hipError_t launch_partial_meta(const uint32_t* off, size_t n_rounds, const uint32_t* share_idx, int n_nodes, uint32_t* round_of,
                               uint8_t* status, hipStream_t st) {
  if (!n_rounds) return hipSuccess;
  hipLaunchKernelGGL(k_partial_meta, dim3(nblk(n_rounds, 256)), dim3(256), 0, st, off, n_rounds, share_idx, n_nodes, round_of,
                     status);
  return hipGetLastError();
}

hipError_t launch_clamp_group(const uint32_t* share_idx, size_t np, uint32_t hi, uint32_t* grp, hipStream_t st) {
  if (!np) return hipSuccess;
  hipLaunchKernelGGL(k_clamp_group, dim3(nblk(np, 256)), dim3(256), 0, st, share_idx, np, hi, grp);
  return hipGetLastError();
}

hipError_t launch_ok_from_status(const uint8_t* status, size_t np, uint8_t* ok, hipStream_t st) {
  if (!np) return hipSuccess;
  hipLaunchKernelGGL(k_ok_from_status, dim3(nblk(np, 256)), dim3(256), 0, st, status, np, ok);
  return hipGetLastError();
}

hipError_t launch_select_lagrange(const uint32_t* off, const uint8_t* ok, const uint32_t* share_idx, int t, size_t n_rounds,
                                  uint32_t* sel, uint32_t* key, uint32_t* den, uint32_t* lam, uint32_t* lam_set, uint8_t* rok,
                                  uint32_t* own, int g1, hipStream_t st) {
  if (!n_rounds) return hipSuccess;
  hipError_t e = hipMemsetAsync(own, 0, 4, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_select_lagrange, dim3(nblk(n_rounds, 64)), dim3(64), 0, st, off, ok, share_idx, t, n_rounds, sel, key,
                     rok);
  hipLaunchKernelGGL(k_lambda, dim3(nblk(n_rounds, 64)), dim3(64), 0, st, key, rok, t, n_rounds, den, lam, lam_set, own, g1);
  return hipGetLastError();
}

static int cu_count() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return v > 0 ? v : 256;
  }();
  return n;
}
// workgroups resident at once: LG_LANES waves each at one wave per SIMD (the kernel holds 512 registers), 4 SIMDs per CU
static size_t lagrange_slots() { return (size_t)cu_count() * (4 / LG_LANES); }
size_t lagrange_tmp_bytes(int sig_g2) { return lagrange_slots() * 64 * (sig_g2 ? 72 : 36) * 4; }

template <class F>
static void lagrange_grid(const uint32_t* sel, const uint32_t* lam, const uint32_t* lam_set, const uint8_t* ok, int t,
                          size_t n_rounds, const uint32_t* sig_aff, const uint32_t* tbl, int entries, uint32_t* out,
                          uint32_t* tmp, hipStream_t st) {
  // blocks beyond the last full wave of resident workgroups are sliced (k_lagrange)
  const size_t nb = nblk(n_rounds, 64), ncu = lagrange_slots();
  size_t full = nb, rem = 0, S = 1;
  const size_t max_s = (size_t)(t + LG_LANES - 1) / LG_LANES;
  if (tmp && nb > ncu && nb % ncu && nb % ncu <= ncu / 2 && max_s > 1) {
    rem = nb % ncu;
    full = nb - rem;
    S = std::min(max_s, ncu / rem);
  }
  hipLaunchKernelGGL(k_lagrange<F>, dim3(full + rem * S), dim3(64 * LG_LANES), 0, st, sel, lam, lam_set, ok, t, n_rounds,
                     sig_aff, tbl, (uint32_t)(entries * A28_WORDS), entries == 8 ? 1 : 0, out, (uint32_t)full, (uint32_t)S,
                     tmp);
  if (rem)
    hipLaunchKernelGGL(k_lagrange_sum<F>, dim3(nblk(n_rounds - full * 64, 64)), dim3(64), 0, st, tmp, (uint32_t)S, full * 64,
                       n_rounds, out);
}

hipError_t launch_lagrange(int sig_g2, const uint32_t* sel, const uint32_t* lam, const uint32_t* lam_set, const uint8_t* ok,
                           int t, size_t n_rounds, const uint32_t* sig_aff, const uint32_t* tbl, int entries, uint32_t* out,
                           uint32_t* tmp, hipStream_t st) {
  if (!n_rounds) return hipSuccess;
  if (sig_g2) lagrange_grid<fp2>(sel, lam, lam_set, ok, t, n_rounds, sig_aff, tbl, entries, out, tmp, st);
  else lagrange_grid<fp>(sel, lam, lam_set, ok, t, n_rounds, sig_aff, tbl, entries, out, tmp, st);
  return hipGetLastError();
}

hipError_t launch_compress(int sig_g2, const uint32_t* pts, size_t n, uint8_t* out, uint32_t* aff_out, uint8_t* status_out,
                           hipStream_t st) {
  if (!n) return hipSuccess;
  if (sig_g2) hipLaunchKernelGGL(k_compress<fp2>, dim3(nblk(n, 64)), dim3(64), 0, st, pts, n, out, aff_out, status_out);
  else hipLaunchKernelGGL(k_compress<fp>, dim3(nblk(n, 64)), dim3(64), 0, st, pts, n, out, aff_out, status_out);
  return hipGetLastError();
}

hipError_t launch_recover_pairs(int sig_g2, const uint32_t* shares, const uint32_t* B, const uint32_t* A, int n_nodes,
                                uint32_t* P, uint32_t* Q, hipStream_t st) {
  if (sig_g2)
    hipLaunchKernelGGL(k_recover_pairs<fp2>, dim3(nblk(n_nodes + 1, 64)), dim3(64), 0, st, shares, B, A, n_nodes, P, Q);
  else
    hipLaunchKernelGGL(k_recover_pairs<fp>, dim3(nblk(n_nodes + 1, 64)), dim3(64), 0, st, shares, B, A, n_nodes, P, Q);
  return hipGetLastError();
}

DH_COUNTER_ACCESSOR(recover)

}  // namespace dh
