// Host-side declarations of the kernel launchers in kernels.hip (internal to libdrandhip).
#pragma once
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace dh {

// Pippenger geometry for one MSM level: entries are cut into groups of `gsize` consecutive entries;
// each group has nwin windows of c bits (signed digits) with nbuck = 2^(c-1) + 1 buckets (index = |digit|,
// 0 unused); bucket reduction splits the digits of a window into nseg segments of seglen digits.
// Scalars: 127-bit integers (halves = 1), or with the endomorphism split (halves = 2) a pair (a, b) of 63-bit
// integers in one uint4 (x, y = a; z, w = b): entry e then stands for two points, P_e with scalar a and
// endo(P_e) (stored half_stride points further on) with scalar b, i.e. P_e with the scalar a + b*mu mod r.
// G2 (halves = 4): four 31-bit parts (x, y, z, w) for P_e, psi(P_e), psi^2(P_e), psi^3(P_e) (part h at h * half_stride
// points on), i.e. the scalar a + b z + c z^2 + d z^3 (psi = [z] on G2).
struct msm_geom {
  uint32_t gsize;
  int c;
  int nwin;
  uint32_t nbuck;
  uint32_t nseg;
  uint32_t seglen;
  uint32_t halves;       // 1; 2 for the endomorphism split; 4 for the G2 psi split
  uint32_t half_stride;  // point index offset of endo(P) (halves = 2) / of each psi power (halves = 4)
};
inline size_t msm_entries(const msm_geom& g, size_t m) { return m * (size_t)g.nwin * g.halves; }

// device workspace of one MSM level (sized by the caller from msm_geom)
struct msm_ws {
  uint32_t* cnt;       // nkeys
  uint32_t* off;       // nkeys + 1
  uint32_t* scan_tmp;  // ceil(nkeys / 4096)
  uint32_t* list;      // msm_entries(g, m)
  uint32_t* buckets;   // nkeys Jacobian points (x2 for launch_msm28: both point sets)
  uint32_t* segs;      // ngroups * nwin * nseg Jacobian points (x2 for launch_msm28)
  uint32_t* out2;      // launch_msm28: 2 * ngroups Jacobian points (sigma sums, then hash sums)
  uint32_t* part;      // balanced bucket pass: 2 Jacobian partial sums per chunk (x2 for launch_msm28)
  uint32_t* meta;      // balanced bucket pass: 2 words per chunk (head kind, tail key)
  size_t max_entries;  // set by launch_msm_sort: upper bound of sorted-list entries (msm_entries)
  uint32_t* runs = nullptr;  // MSM28: the segments' running sums (as many points as segs)
};

// balanced bucket accumulation: entries per chunk, and workspace sizes for `max_entries` list entries
inline uint32_t msm_chunk_len(size_t max_entries, size_t cap = 32, size_t target_chunks = 262144) {
  // the shortest chunk: 8 entries (a 131k-round shard at c = 16 holds ~8 entries per bucket, so shorter chunks cut
  // most buckets and leave their sums to k_msm_bucket_fix: 4 -> 8 took the shard's MSM from 2.75 to 2.42 ms,
  // profiles/r03k); DRANDHIP_MSM_LMIN overrides it for experiments
  static const size_t lmin = [] {
    const char* e = getenv("DRANDHIP_MSM_LMIN");
    const long v = e ? atol(e) : 0;
    return (size_t)(v >= 1 && v <= 64 ? v : 8);
  }();
  size_t L = max_entries / target_chunks;
  if (L < lmin) L = lmin;
  return (uint32_t)(L > cap ? cap : L);
}
inline size_t msm_nchunks(size_t max_entries) { return max_entries / msm_chunk_len(max_entries) + 2; }
inline size_t msm_part_bytes(size_t max_entries, size_t jac_words, int nsets) {
  return msm_nchunks(max_entries) * 2 * jac_words * 4 * (size_t)nsets;
}
inline size_t msm_meta_bytes(size_t max_entries) { return msm_nchunks(max_entries) * 2 * 4; }

hipError_t launch_prep(int sig_g2, const uint8_t* sigs, size_t stride, size_t n, uint8_t* status, uint32_t* sig_aff,
                       uint8_t* rand_out, hipStream_t st);
// small-batch path: the signature pass split at the decoded point (decode + randomness; subgroup test -> sub_bad[i]
// = 1 when a decoded point is not in the subgroup; verdict[i] = 0 where sub_bad[i])
hipError_t launch_dec_sig(int sig_g2, const uint8_t* sigs, size_t stride, size_t n, uint8_t* status, uint32_t* sig_aff,
                          uint8_t* rand_out, hipStream_t st);
hipError_t launch_sub_flag(int sig_g2, size_t n, const uint8_t* status, const uint32_t* sig_aff, uint8_t* sub_bad, hipStream_t st);
hipError_t launch_and_subgroup(size_t n, const uint8_t* sub_bad, uint8_t* verdict, hipStream_t st);
// small-batch path: launch_hash with the G1 hash's two SSWU maps in workgroups of their own (G2: launch_hash);
// tmp: hash_small_tmp_bytes
size_t hash_small_tmp_bytes(int sig_g2, size_t n);
hipError_t launch_hash_small(int sig_g2, const uint64_t* rounds, const uint8_t* prevs, size_t prev_stride, const uint32_t* prev_lens,
                             const uint8_t* msgs32, size_t n, int chained, int dst_id, uint8_t* status, uint32_t* q_out,
                             uint32_t* tmp, hipStream_t st);
// hash points Q_i (before cofactor clearing) of the beacon digests of (rounds, prevs) or of the given 32-byte
// msgs32; a chained record longer than its slot marks status[i] = DEC_BAD. tmp: hash_tmp_bytes(sig_g2, n).
size_t hash_tmp_bytes(int sig_g2, size_t n);
hipError_t launch_hash(int sig_g2, const uint64_t* rounds, const uint8_t* prevs, size_t prev_stride, const uint32_t* prev_lens,
                       const uint8_t* msgs32, size_t n, int chained, int dst_id, uint8_t* status, uint32_t* q_out, uint32_t* tmp,
                       hipStream_t st);
// RLC scalars from SHA-256(seed || i): 127-bit (glv = 0) or a pair of 63-bit halves (glv = 1, msm_geom.halves = 2);
// 0 for rounds whose status is not DEC_OK (status null: every round gets its scalar)
// parts: 1 = one 127-bit scalar, 2 = two 63-bit halves, 4 = four 31-bit parts (msm_geom halves)
hipError_t launch_scalars(const uint32_t* seed_words, size_t n, const uint8_t* status, uint4* scal, int parts, hipStream_t st);
hipError_t launch_decode_key(int key_g2, const uint8_t* pk, uint32_t* key_aff, uint8_t* ok, hipStream_t st);
hipError_t launch_iota(uint32_t* v, size_t n, hipStream_t st);
hipError_t launch_scan(const uint32_t* cnt, size_t nk, uint32_t* off, uint32_t* tmp, hipStream_t st);
// The RLC MSM on lazily reduced 28-bit points (k_msm.hip MSM28): launch_msm_prep28 converts the batch's sigma
// (affine) and hash points (Jacobian, made affine) with their endomorphism images into S and Q (G1 32 / G2 64 words
// per point, parts x n points each: the images of point i at i + h n; a hash point at infinity marks its round
// DEC_BAD); the workspace's bucket / partial / segment arrays hold 48 / 96-word Jacobian points
hipError_t launch_msm_prep28(int sig_g2, size_t n, uint8_t* status, const uint32_t* sig_aff, const uint32_t* q_pts,
                             uint32_t* S, uint32_t* Q, hipStream_t st, uint32_t sets = 3);
// one point set (S of launch_msm_prep28) with point / scalar / group indices: ngroups 12 x 32-bit Jacobian sums into out
hipError_t launch_msm28_set(int sig_g2, const msm_geom& g, const uint32_t* pidx, const uint32_t* sidx, const uint32_t* grp,
                            size_t m, size_t ngroups, const uint4* scal, const uint32_t* P, msm_ws& ws, uint32_t* out,
                            hipStream_t st);
hipError_t launch_msm28(int sig_g2, const msm_geom& g, const uint32_t* entries, size_t m, size_t ngroups, const uint4* scal,
                        const uint32_t* S, const uint32_t* Q, msm_ws& ws, uint32_t* outA, uint32_t* outB, hipStream_t st,
                        const uint8_t* skip, bool presorted);
hipError_t launch_msm_sort(const msm_geom& g, const uint32_t* pidx, const uint32_t* sidx, const uint32_t* grp, size_t m,
                           size_t ngroups, const uint4* scal, msm_ws& ws, hipStream_t st);
hipError_t launch_group_check(int sig_g2, const uint32_t* A, const uint32_t* B, size_t ngroups, const uint32_t* key_aff,
                              uint8_t* pass, hipStream_t st);
// node-wide check: sum the k (A, B) level-0 partial-sum pairs, record i = [A_i | B_i | status word | pad] at
// parts + i * rec_words (Jacobian AoS); flag[0] (nullable) = 1 when any record's status word is nonzero
hipError_t launch_sum_partials(int sig_g2, const uint32_t* parts, size_t k, size_t rec_words, uint32_t* outA, uint32_t* outB,
                               uint8_t* flag, hipStream_t st);
// res[0] = abandon flag, res[1] = pairing check -> res[2] = 2 abandoned / 1 passed / 0 failed; passed: verdict[i] =
// (status[i] == DEC_OK) for i < n
hipError_t launch_node_mark(size_t n, uint8_t* res, const uint8_t* status, uint8_t* verdict, hipStream_t st);
hipError_t launch_mark_groups(const uint32_t* entries, size_t m, size_t gsize, const uint8_t* pass, const uint8_t* status,
                              uint8_t* verdict, hipStream_t st);
// bisection: out = the entries of the groups with pass == 0, in order; rank[ngroups] = the number of failing groups
// (flags: ngroups words, rank: ngroups + 1, scan_tmp: launch_scan's)
hipError_t launch_compact_failing(const uint32_t* entries, size_t m, size_t gsize, size_t ngroups, const uint8_t* pass,
                                  uint32_t* flags, uint32_t* rank, uint32_t* scan_tmp, uint32_t* out, hipStream_t st);
hipError_t launch_leaf_check(int sig_g2, const uint32_t* entries, size_t m, const uint32_t* sig_aff, const uint32_t* q_pts,
                             const uint32_t* key_aff, const uint8_t* status, uint8_t* verdict, hipStream_t st);

// lane-parallel pairing checks (k_vm.hip): pairs = 2 x 72 words per check, live = 2 bytes, done = 1 byte
// key_h: [h_eff] pk for G1-signature schemes (k_decode_key writes it after the key), or null for [h_eff] B
hipError_t launch_group_check_vm(int sig_g2, const uint32_t* A, const uint32_t* B, size_t ngroups, const uint32_t* key_aff,
                                 const uint32_t* key_h,
                                 uint32_t* pairs, uint8_t* live, uint8_t* pass, hipStream_t st);
// G2-signature group checks with the cofactor clearing inside the pairing program (k_vm.hip k_vm_pairing_c)
size_t group_check_c_pair_words();
hipError_t launch_group_check_vm_c(const uint32_t* A, const uint32_t* B, size_t ngroups, const uint32_t* key_aff, uint32_t* pairs,
                                   uint8_t* live, uint8_t* done, uint8_t* pass, hipStream_t st);
hipError_t launch_leaf_check_vm(int sig_g2, const uint32_t* entries, size_t m, const uint32_t* sig_aff, const uint32_t* q_pts,
                                const uint32_t* key_aff, const uint32_t* key_h, const uint8_t* status, uint32_t* pairs,
                                uint8_t* live, uint8_t* done, uint8_t* verdict, hipStream_t st);

// G2-signature leaves with the hash point's clearing inside the program (NP2C); same buffers as launch_group_check_vm_c
hipError_t launch_leaf_check_vm_c(const uint32_t* entries, size_t m, const uint32_t* sig_aff, const uint32_t* q_pts,
                                  const uint32_t* key_aff, const uint8_t* status, uint32_t* pairs, uint8_t* live, uint8_t* done,
                                  uint8_t* verdict, hipStream_t st);

// G1-signature checks on Jacobian G1 sides (NP2J, no prep kernel): groups (A, B Jacobian AoS) and leaves;
// key_h = [h_eff] pk (affine)
hipError_t launch_group_check_g1j(const uint32_t* A, const uint32_t* B, size_t ngroups, const uint32_t* key_h, uint8_t* pass,
                                  hipStream_t st);
hipError_t launch_leaf_check_g1j(const uint32_t* entries, size_t m, const uint32_t* sig_aff, const uint32_t* q_pts,
                                 const uint32_t* key_h, const uint8_t* status, uint8_t* verdict, hipStream_t st);

hipError_t launch_multi_pairing_vm(const uint32_t* P, const uint32_t* Q, size_t n, uint32_t* pairs, uint8_t* live,
                                   uint32_t* f_tmp, uint8_t* pass, hipStream_t st);

// synthetic signer: q_tmp n x 72 words and h_tmp hash_tmp_bytes(1, n) for G2 signatures (unused for G1)
hipError_t launch_sign(int sig_g2, const uint32_t* sk, const uint64_t* rounds, const uint8_t* prevs, size_t prev_stride,
                       const uint32_t* prev_lens, const uint8_t* msgs32, size_t n, int chained, int dst_id, uint8_t* out,
                       uint32_t* q_tmp, uint32_t* h_tmp, hipStream_t st);
// RFC 9380 hash_to_curve of arbitrary messages / DST, compressed (k_sign.hip)
hipError_t launch_h2c_generic(int g2, const uint8_t* msgs, const uint32_t* off, size_t n, const uint8_t* dst, uint32_t dlen,
                              uint8_t* scratch, size_t sstride, uint8_t* out, hipStream_t st);
hipError_t launch_pubkey(int key_g2, const uint32_t* sk, uint8_t* out, hipStream_t st);

// tbls Recover (k_recover.hip)
hipError_t launch_repack_partials(const uint8_t* raw, size_t n, int sig_len, uint8_t* sigs, uint32_t* idx, hipStream_t st);
hipError_t launch_pubpoly_eval(int key_g2, const uint32_t* commits, int t, int n_nodes, uint32_t* out, hipStream_t st);
hipError_t launch_pair_check(const uint32_t* P, const uint32_t* Q, size_t npairs, int clear_p, int clear_q,
                             const uint8_t* live, uint32_t* f_tmp, uint8_t* skip_tmp, uint8_t* pass, hipStream_t st);
hipError_t launch_partial_leaf(int sig_g2, const uint32_t* list, size_t m, const uint32_t* sig_aff, const uint8_t* status,
                               const uint32_t* share_idx, const uint32_t* round_of, const uint32_t* q_pts,
                               const uint32_t* shares, int n_nodes, uint8_t* ok_out, hipStream_t st);
// per round: round_of for its partials, indices >= n_nodes rejected (status); ok from status after a passed batch
hipError_t launch_partial_meta(const uint32_t* off, size_t n_rounds, const uint32_t* share_idx, int n_nodes, uint32_t* round_of,
                               uint8_t* status, hipStream_t st);
hipError_t launch_clamp_group(const uint32_t* share_idx, size_t np, uint32_t hi, uint32_t* grp, hipStream_t st);
hipError_t launch_ok_from_status(const uint8_t* status, size_t np, uint8_t* ok, hipStream_t st);
// per round: Recover's selection + Lagrange coefficients (sel/key: t words, den: 8t words, lam: lam_words() t words
// per round); lam_set[j] = the round whose lambda rows round j uses (0 when its selected indices equal round 0's, else
// j); *own = the number of rounds j > 0 with their own rows (device word)
size_t lam_words();
hipError_t launch_select_lagrange(const uint32_t* off, const uint8_t* ok, const uint32_t* share_idx, int t, size_t n_rounds,
                                  uint32_t* sel, uint32_t* key, uint32_t* den, uint32_t* lam, uint32_t* lam_set, uint8_t* rok,
                                  uint32_t* own, int g1, hipStream_t st);
// tbl (G2): per valid partial (ok) the odd multiples P, 3P, ..., (2 entries - 1) P affine 28-bit (entries = 4 or 8,
// 64 words each) from the partials' affine points (12 x 32-bit AOS); zs: wnaf_table_scratch_bytes(n, entries) of
// scratch (the batched inversion's Z's); unused for G1
hipError_t launch_mark_selected(const uint32_t* sel, const uint8_t* rok, int t, size_t n_rounds, size_t np, uint8_t* need,
                                hipStream_t st);
hipError_t launch_wnaf_table_g2(const uint32_t* paff, const uint8_t* ok, size_t n, int entries, uint32_t* tbl, uint32_t* zs,
                                hipStream_t st);
size_t wnaf_table_scratch_bytes(size_t n, int entries);
// tmp: lagrange_tmp_bytes(sig_g2) of scratch for the sliced last wave of workgroups (null: no slicing)
// entries: the G2 tables' width (8: waves whose rounds use different bases run the regular windows)
hipError_t launch_lagrange(int sig_g2, const uint32_t* sel, const uint32_t* lam, const uint32_t* lam_set, const uint8_t* ok,
                           int t, size_t n_rounds, const uint32_t* sig_aff, const uint32_t* tbl, int entries, uint32_t* out,
                           uint32_t* tmp, hipStream_t st);
size_t lagrange_tmp_bytes(int sig_g2);
// compressed bytes of n Jacobian points; aff_out / status_out (nullable): their affine form and a decode status
// (DEC_OK, DEC_BAD for infinity) — what decoding the bytes of a subgroup point gives
hipError_t launch_compress(int sig_g2, const uint32_t* pts, size_t n, uint8_t* out, uint32_t* aff_out, uint8_t* status_out,
                           hipStream_t st);
hipError_t launch_recover_pairs(int sig_g2, const uint32_t* shares, const uint32_t* B, const uint32_t* A, int n_nodes,
                                uint32_t* P, uint32_t* Q, hipStream_t st);

#ifdef DH_COUNT_PRODUCTS
// counting build: field products executed since the last take, per translation unit (fp_mul28.hpp)
hipError_t count_take_prep(unsigned long long* v);
hipError_t count_take_msm(unsigned long long* v);
hipError_t count_take_check(unsigned long long* v);
hipError_t count_take_sign(unsigned long long* v);
hipError_t count_take_recover(unsigned long long* v);
hipError_t count_take_vm(unsigned long long* v);
#endif

}  // namespace dh
