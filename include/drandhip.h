/*
 * drandhip.h — C ABI of libdrandhip, the MI355X (gfx950) beacon-verification engine for drand.
 *
 * Plain pointers and sizes only (cgo / ctypes / JNI friendly). Every entry point is thread-safe and
 * reentrant: concurrent callers each get their own HIP stream and device workspace from an internal
 * pool. Inputs are borrowed for the duration of the call and never retained; outputs are written into
 * caller-owned buffers. Batch calls block until their results are on the host.
 *
 * Replaces, for the verification hot path, the kyber / kyber-bls12381 / kilic arithmetic that drand
 * reaches through (reference at /root/reference, drand snapshot 2025-01-17):
 *   crypto.Scheme.VerifyBeacon            crypto/schemes.go:70-72
 *   crypto.Scheme.DigestBeacon            crypto/schemes.go:106-114 (chained), 147-151, 187-191
 *   crypto.RandomnessFromSignature        crypto/schemes.go:249-252
 *   crypto.SchemeFromName                 crypto/schemes.go:206-217
 *   sign.ThresholdScheme.VerifyRecovered  [kyber v1.1.18 sign/tbls], called at crypto/schemes.go:71,
 *                                         chain/beacon/chainstore.go:207
 *   sign.ThresholdScheme.Recover          [kyber v1.1.18 sign/tbls], called at chain/beacon/chainstore.go:202
 * and adds the batch entry point the serial per-round loops need:
 *   chain/beacon/sync_manager.go:191-225 (CheckPastBeacons), client/verify.go:139-160, lp2p relays.
 * INTEGRATION.md shows the cgo binding a drand maintainer would add.
 */
#ifndef DRANDHIP_H
#define DRANDHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* return codes (>= 0 success) */
#define DH_OK 0
#define DH_EINVAL (-1)   /* bad argument: unknown scheme, wrong key/sig length, unsupported message shape */
#define DH_EDEVICE (-2)  /* HIP runtime / kernel failure; the caller should fall back to its CPU path */
#define DH_ENOMEM (-3)   /* device allocation failed */
#define DH_EKEY (-4)     /* the group public key does not decode to a subgroup point */
#define DH_ERECOVER (-5) /* Recover: fewer than t valid partial signatures */
#define DH_EBUSY (-6)    /* every library worker is held (DRANDHIP_MAX_WORKERS, default 24): dh_batch_begin at once,
                            a blocking call after DRANDHIP_LEASE_TIMEOUT_MS when node batches hold them all */
#define DH_EABANDONED (-7) /* node-wide batch: some rank's dh_batch_begin failed, every rank abandons the batch */

/* scheme ids, in the order of crypto/schemes.go:206-219 plus the RFC 9380 quicknet scheme */
#define DH_SCHEME_CHAINED 0      /* "pedersen-bls-chained":   sig G2 (96 B), key G1 (48 B), msg SHA256(prev||round) */
#define DH_SCHEME_UNCHAINED 1    /* "pedersen-bls-unchained": sig G2, key G1, msg SHA256(round) */
#define DH_SCHEME_G1_LEGACY 2    /* "bls-unchained-on-g1":    sig G1 (48 B), key G2 (96 B), G2 hash DST (legacy) */
#define DH_SCHEME_G1_RFC9380 3   /* "bls-unchained-g1-rfc9380" (quicknet): sig G1, key G2, G1 hash DST */

/*
 * Select the device: bit i of device_mask = HIP device i, at most one bit (one process per GPU);
 * 0 = device 0 or the device already selected. Idempotent; asking for another device after initialisation is
 * DH_EINVAL until dh_shutdown.
 */
int dh_init(uint32_t device_mask);
/*
 * Release all device resources. Safe while other threads are inside calls: their workers are retired and freed
 * when those calls return. Calls after this re-initialise lazily.
 */
void dh_shutdown(void);

/* crypto.SchemeFromName: scheme id or DH_EINVAL */
int dh_scheme_from_name(const char* name);
/* byte lengths for a scheme: compressed signature / group public key; DH_EINVAL for unknown ids */
int dh_sig_len(int scheme);
int dh_key_len(int scheme);

/*
 * Batch VerifyBeacon over n rounds sharing one group public key.
 *   pk           compressed key-group point (dh_key_len bytes)
 *   rounds[i]    round numbers
 *   sigs         n signatures, record i at sigs + i*sig_stride (sig_stride >= dh_sig_len, multiple of 4)
 *   prevs        chained scheme only (NULL otherwise): previous signature of round i at prevs + i*prev_stride;
 *                length prev_lens[i] (or prev_stride when prev_lens is NULL), any length <= prev_stride: the
 *                record is hashed as stored, like crypto/schemes.go:106-114 (0 = none, 32 = genesis seed,
 *                96 = stored G2 signature; a corrupted 31- or 100-byte record simply fails its round).
 *                prev_lens[i] > prev_stride is DH_EINVAL here and rejects round i on the device entry point.
 *   verdict_out  n bytes: 1 = VerifyBeacon returns nil, 0 = it returns an error
 *   rand_out     n*32 bytes SHA-256(sig) (RandomnessFromSignature) or NULL
 *   seed         0 = draw the random-linear-combination seed from the OS CSPRNG; otherwise deterministic
 * One call runs on one internal stream by default (its per-round kernels, then its MSM and pairing checks on a
 * high-priority stream): a 4M-round call runs at ~94% of the rate of 8 concurrent 1M calls, a 1M-round call at
 * ~85% (its ~8 ms latency tail, MSM + pairing check, is exposed). DRANDHIP_SPLIT="chunk,workers" / dh_set_split cut a call into
 * chunks verified on several streams instead.
 * Returns DH_OK or a negative error code (no verdicts are valid on error).
 */
int dh_verify_batch(int scheme, const uint8_t* pk, size_t pk_len, const uint64_t* rounds, const uint8_t* sigs,
                    size_t sig_stride, const uint8_t* prevs, size_t prev_stride, const uint32_t* prev_lens, size_t n,
                    uint8_t* verdict_out, uint8_t* rand_out, uint64_t seed);

/* Set the one-call split of dh_verify_batch / dh_verify_batch_device (chunk_rounds 0 = one stream per call, the
 * default). */
int dh_set_split(uint64_t chunk_rounds, int workers);

/*
 * Same as dh_verify_batch with every array already resident in device memory (HIP device pointers). The inputs
 * may still be in production on `hip_stream` (a hipStream_t): the library's streams wait for that stream's work
 * first; NULL = the inputs are ready. Blocks until done. `stats_out` (nullable, host) receives
 * {levels, groups_failed, leaf_rounds, rounds_rejected} (levels: the deepest chunk's).
 */
int dh_verify_batch_device(int scheme, const uint8_t* pk, size_t pk_len, const uint64_t* d_rounds, const uint8_t* d_sigs,
                           size_t sig_stride, const uint8_t* d_prevs, size_t prev_stride, const uint32_t* d_prev_lens,
                           size_t n, uint8_t* d_verdict_out, uint8_t* d_rand_out, uint64_t seed, void* hip_stream,
                           uint64_t stats_out[4]);

/* Single VerifyBeacon (crypto/schemes.go:70-72): 1 valid, 0 invalid, < 0 error */
int dh_verify_beacon(int scheme, const uint8_t* pk, size_t pk_len, uint64_t round, const uint8_t* sig, size_t sig_len,
                     const uint8_t* prev, size_t prev_len);

/*
 * ThresholdScheme.VerifyRecovered(pk, msg, sig) (kyber sign/tbls = bls.Verify; called at
 * chain/beacon/chainstore.go:207 on every recovered signature) for a 32-byte msg (a beacon digest):
 * 1 valid / 0 invalid / < 0 error.
 */
int dh_verify_recovered(int scheme, const uint8_t* pk, size_t pk_len, const uint8_t* msg32, const uint8_t* sig,
                        size_t sig_len);

/*
 * Batch VerifyRecovered: n (32-byte digest, signature) pairs under one key, host buffers, same batching and
 * bit-exact per-item verdicts as dh_verify_batch (verdict_out[i] = 1 valid, 0 invalid).
 */
int dh_verify_recovered_batch(int scheme, const uint8_t* pk, size_t pk_len, const uint8_t* msgs32, const uint8_t* sigs,
                              size_t sig_stride, size_t n, uint8_t* verdict_out, uint64_t seed);

/* crypto.Scheme.DigestBeacon for n rounds (host-side SHA-256, no device): out n*32 bytes */
int dh_digest_batch(int scheme, const uint64_t* rounds, const uint8_t* prevs, size_t prev_stride,
                    const uint32_t* prev_lens, size_t n, uint8_t* out);

/* RandomnessFromSignature for n signatures on the device: out n*32 bytes */
int dh_randomness_batch(int scheme, const uint8_t* sigs, size_t sig_stride, size_t n, uint8_t* out);

/*
 * Batch tbls Recover (kyber sign/tbls Recover + share.RecoverCommit, called at chain/beacon/chainstore.go:202):
 * for each of n_rounds rounds, partials[part_off[j] .. part_off[j+1]) are (2-byte BE index || sig) records
 * of (2 + sig_len) bytes for message msgs32[j] (32-byte digests). Each partial is verified against
 * PubPoly.Eval(index) (commits = t compressed key-group points); the first t valid ones (in the given
 * order) are kept, sorted by index, and Lagrange-interpolated at 0 in the signature group.
 * sig_out: n_rounds * sig_len bytes; status_out[j] = 1 recovered, 0 not enough valid partials. n_nodes <= 65536
 * (every 2-byte index); a caller that wants kyber's any-index semantics passes max(n, largest index + 1).
 */
int dh_recover_batch(int scheme, const uint8_t* commits, int t, int n_nodes, const uint8_t* msgs32,
                     const uint8_t* partials, const uint32_t* part_off, size_t n_rounds, uint8_t* sig_out,
                     uint8_t* status_out);

/*
 * Batch ThresholdScheme.VerifyPartial(pubPoly, msg, partial) (kyber sign/tbls; called per incoming partial at
 * chain/beacon/node.go:150): same input layout as dh_recover_batch; ok_out[k] (one byte per partial, in
 * input order) = 1 when the k-th partial's signature verifies under PubPoly.Eval(index) for its round's
 * message, 0 otherwise.
 * Deviation from kyber, documented: kyber's VerifyPartial evaluates PubPoly.Eval(i) for ANY index i, so a partial
 * validly signed with f(i+1) for i >= n_nodes would pass there; here indices >= n_nodes have no share in the group
 * and are reported invalid (and skipped by dh_recover_batch). drand never hands such a partial to the scheme:
 * chain/beacon/node.go:138-141 rejects indices outside the group before VerifyPartial and the partial cache.
 */
int dh_verify_partials_batch(int scheme, const uint8_t* commits, int t, int n_nodes, const uint8_t* msgs32,
                             const uint8_t* partials, const uint32_t* part_off, size_t n_rounds, uint8_t* ok_out);

/*
 * Node-wide batch check over the GPUs of one node (one process per GPU; the sharded form of
 * chain/beacon/sync_manager.go:191-225). Every rank prepares its shard of rounds and its level-0
 * random-linear-combination sums with dh_batch_begin, which writes one record of dh_partial_bytes(scheme) bytes into
 * d_partials_out (device memory): A = sum r_i sigma_i, B = sum r_i H(m_i) (Jacobian), a status word (0) and padding.
 * The ranks all-gather the records (RCCL over xGMI); a rank whose dh_batch_begin failed contributes a record with a
 * nonzero status word, so every rank learns it from the gathered data. dh_batch_check queues, on the batch's own
 * worker, the sum of the k gathered records and ONE pairing check e(g, sum A) = e(pk, [h] sum B) for the whole node;
 * when it passes, every decoded round of the batch is marked valid on the device. dh_batch_finish(b,
 * DH_NODE_CHECKED, ...) then waits for that result: it returns 1 (the node check passed), or 0 (it failed: the
 * shard's own level-0 check and bisection ran, so the verdicts are per-round exact either way), or DH_EABANDONED
 * (some rank's record carried a nonzero status: nothing is valid), or another error.
 *
 * Streams: the batch's record is written, and its check and bisection run, on ONE stream of the library,
 * dh_batch_stream(b) (a hipStream_t): the caller queues the collective there (e.g. torch.cuda.ExternalStream), so the
 * record, the all-gather and the check follow each other in stream order, with no host wait and, for one rank, no
 * cross-stream wait. dh_batch_begin returns as soon as the batch is queued; with hip_stream (a hipStream_t) non-NULL
 * it orders the batch after hip_stream's work (inputs still in production there), with NULL the inputs must be
 * complete (NULL means "no stream": work on the legacy NULL / default stream must be synchronised by the caller).
 * A host caller that wants the record itself waits for dh_batch_stream(b).
 * dh_batch_check orders the check after hip_stream's work when hip_stream is another stream (the gathered records
 * produced there); NULL or dh_batch_stream(b) adds no wait. The only host wait of a batch is in dh_batch_finish.
 *
 * A batch holds one library worker from begin to finish (DH_EBUSY if none is idle: begin never waits, since the
 * other ranks may be waiting in the collective); the arguments of dh_batch_begin must stay valid until
 * dh_batch_finish returns. A blocking call (any other entry point) made while EVERY worker is held by unfinished
 * batches waits at most DRANDHIP_LEASE_TIMEOUT_MS (default 30 s) for one and then fails with DH_EBUSY: finish the
 * batches first. A batch of one round contributes the identity to the node-wide sums, so its round always gets its
 * own check in dh_batch_finish, whatever the node-wide result. dh_batch_finish with node_pass 1 / 0 (a result the caller obtained itself, e.g. from
 * dh_check_partials) accepts every decoded round / runs the shard's own check and returns DH_OK; node_pass < 0
 * (other than DH_NODE_CHECKED) abandons the batch. dh_check_partials is the standalone check of k records (it
 * leases its own worker and blocks): pass_out = 1 / 0, DH_EABANDONED when a status word is nonzero.
 */
typedef struct dh_batch dh_batch;
#define DH_NODE_CHECKED 2 /* dh_batch_finish: take the result of dh_batch_check */
int dh_partial_bytes(int scheme);
int dh_batch_begin(int scheme, const uint8_t* pk, size_t pk_len, const uint64_t* d_rounds, const uint8_t* d_sigs,
                   size_t sig_stride, const uint8_t* d_prevs, size_t prev_stride, const uint32_t* d_prev_lens, size_t n,
                   uint8_t* d_verdict_out, uint8_t* d_rand_out, uint64_t seed, void* hip_stream, dh_batch** batch_out,
                   uint8_t* d_partials_out);
void* dh_batch_stream(dh_batch* batch);
int dh_batch_check(dh_batch* batch, const uint8_t* d_partials, size_t k, void* hip_stream);
int dh_check_partials(int scheme, const uint8_t* pk, size_t pk_len, const uint8_t* d_partials, size_t k, int* pass_out);
int dh_batch_finish(dh_batch* batch, int node_pass, uint64_t stats_out[4]);

/*
 * Synthetic-chain utilities (test fixtures and benchmark inputs; not part of the verification path):
 * sign n beacons with a 32-byte big-endian secret scalar, sig_i = [sk] H(DigestBeacon(round_i, prev_i)),
 * the mock chain pattern of client/test/result/mock/result.go:84-127; and the matching group key [sk] g.
 * sigs_out: n * dh_sig_len bytes; key_out: dh_key_len bytes.
 */
int dh_sign_batch(int scheme, const uint8_t* sk32, const uint64_t* rounds, const uint8_t* prevs, size_t n,
                  const uint32_t* prev_lens, size_t prev_stride, uint8_t* sigs_out);
int dh_public_key(int scheme, const uint8_t* sk32, uint8_t* key_out);

/*
 * RFC 9380 hash_to_curve (random-oracle encoding, expand_message_xmd with SHA-256) on the device for n arbitrary
 * messages (message i = msgs[msg_off[i] .. msg_off[i+1])) under one DST of 1..255 bytes: group 1 = G1 (SSWU on the
 * 11-isogenous curve), group 2 = G2 (3-isogenous). out: n compressed points (48 / 96 bytes). The general form of the
 * fixed-shape hashing inside the batch kernels (kilic HashToCurve as used by kyber-bls12381's Hash, [ext]); pinned
 * by the RFC 9380 J.9.1 / J.10.1 vectors in tests/kat.py.
 */
int dh_hash_to_curve(int group, const uint8_t* msgs, const uint32_t* msg_off, size_t n, const uint8_t* dst, size_t dst_len,
                     uint8_t* out);

/*
 * Live kernel timing: when enabled, every device stage of the verification path is bracketed by HIP
 * events on the stream it is launched on; dh_profile_read writes a JSON object
 * {"stage": {"count": c, "total_ms": t}, ...} into buf (returns the full length). dh_profile resets.
 */
int dh_profile(int enable);
int dh_profile_read(char* buf, size_t cap);

/* Human-readable description of the last error on the calling thread ("" if none). */
const char* dh_last_error_string(void);

/* Build / device description, e.g. "libdrandhip gfx950 ..." */
const char* dh_version(void);

#ifdef __cplusplus
}
#endif
#endif /* DRANDHIP_H */
