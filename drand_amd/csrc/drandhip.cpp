// libdrandhip host side: the C ABI of include/drandhip.h over the gfx950 kernels in kernels.hip.
//
// Threading model (SURVEY.md §8b "Threading"): one global device context (dh_init, idempotent), and a
// pool of workers, each = {hipStream_t, growable device workspace}. A call takes a free worker for its
// duration, so concurrent goroutines / threads never share a stream or a buffer; results are copied
// into caller memory before the call returns. No global mutable state is visible to callers.
//
// Verification flow of one batch (dh_verify_batch_device):
//   decode pk -> prep signatures (status, affine sigma, randomness) -> prep messages (Q_i, pre-cofactor)
//   -> RLC scalars -> level 0: one group = every round: MSM + pairing check
//   -> on failure, bisection levels with smaller groups (sizes from an expected-cost model: 1024, then 256/64/16/4
//      as the observed fault density says, or straight to leaves) over the failing groups only
//   -> leaves: per-round 2-pairing checks. Verdict = decode ok AND (group passed OR leaf passed),
//   which is the per-round VerifyBeacon verdict of /root/reference/crypto/schemes.go:70-72.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <sys/random.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cmath>
#include <functional>
#include <map>
#include <memory>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/drandhip.h"
#include "kernels.hpp"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(x)                                                                     \
  do {                                                                                 \
    hipError_t e__ = (x);                                                              \
    if (e__ != hipSuccess)                                                             \
      return fail(e__ == hipErrorOutOfMemory ? DH_ENOMEM : DH_EDEVICE, "%s: %s (%s:%d)", #x, \
                  hipGetErrorString(e__), __FILE__, __LINE__);                         \
  } while (0)

bool sig_on_g2(int scheme) { return scheme == DH_SCHEME_CHAINED || scheme == DH_SCHEME_UNCHAINED; }
int dst_id(int scheme) { return scheme == DH_SCHEME_G1_RFC9380 ? 1 : 0; }

// growable device buffer
struct dbuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max(bytes, (size_t)4096);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  template <class T>
  T* as() const {
    return (T*)p;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct worker {
  hipStream_t stream = nullptr;
  // high-priority stream for a batch's latency-bound tail (MSM, pairing checks, bisection): its small kernels
  // get wave slots ahead of other batches' saturating per-round kernels (verify_core)
  hipStream_t tail = nullptr;
  hipEvent_t handoff = nullptr;
  // node-wide batch (dh_batch_begin / dh_batch_check): the partial sums are complete (ordered onto the caller's
  // stream), and the gathered records are complete on the caller's stream (the tail waits for it)
  hipEvent_t part_ready = nullptr, gath_ready = nullptr;
  // small-batch path (verify_small): the hash kernels fork onto the tail stream beside the signature kernels and
  // join back (join); host inputs and outputs cross PCIe through one pinned staging buffer each way
  hipEvent_t join = nullptr, ev_dec = nullptr, ev_sub = nullptr;
  void* h_stage = nullptr;
  size_t h_stage_cap = 0;
  dbuf d_stage, sub_bad;
  bool busy = false;
  // leased by a node batch (dh_batch_begin until dh_batch_finish): held across calls, released only by the caller
  bool node_held = false;
  // per-round state
  dbuf status, sig_aff, q_pts, scal, entries, verdict_tmp, rand_tmp, h2c_tmp;
  // the MSM's 28-bit points (launch_msm_prep28, G1): sigma and its phi image (32 words each), hash points (48 words)
  dbuf s28, q28;
  // bisection on the device: the next level's entries, fail flags, their ranks and the scan's block sums
  dbuf entries_alt, cflags, crank, cscan;
  // host-API staging
  dbuf in_rounds, in_sigs, in_prevs, in_prev_lens, out_verdict, out_rand;
  // key
  dbuf key_raw, key_aff, key_ok;
  // node-wide check: the summed (A, B) of the gathered records, and {abandon flag, pairing check, result}
  dbuf node_sum, node_res;
  // MSM
  dbuf cnt, off, scan_tmp, list, buckets, segs, outA, outB, out2, pass, part, meta;
  // lane-parallel pairing checks
  dbuf vm_pairs, vm_live, vm_done;
  // tbls Recover
  dbuf r_commits, r_cstatus, r_caff, r_shares, r_raw, r_psigs, r_pidx, r_pstatus, r_paff, r_msgs, r_q, r_scal,
      r_round_of, r_e_pidx, r_e_sidx, r_e_grp, r_P, r_Q, r_f, r_skip, r_ok, r_sel, r_lam, r_lamset, r_rok, r_sig,
      r_sigbytes, r_status2, r_aff2, r_entries2, r_off, r_key, r_den, r_zs, r_tbl, r_rstat, r_ltmp, r_own, r_need;
  std::vector<uint8_t> h_verdict;
  // Recover: the (scheme, t, n_nodes, commits) whose decoded commits and public shares r_caff / r_shares hold
  std::vector<uint8_t> r_pub_key;
  // decoded group keys, KEY_SLOTS per worker (least recently used replaced): a chain's batches all use one key, and a
  // node or relay serving several chains alternates between a few; key_cur = the slot ensure_key selected (96 words:
  // the affine point, then [h_eff] pk for G1-signature schemes)
  static constexpr int KEY_SLOTS = 4;
  struct key_slot {
    uint8_t bytes[96];
    size_t len = 0;  // 0: empty
    int g2 = -1;
    uint8_t ok = 0;
    uint64_t used = 0;
  } keys[KEY_SLOTS];
  uint64_t key_clock = 0;
  dbuf key_tab;
  uint32_t* key_cur = nullptr;
  // fault density (faults per round) the last bisection of this worker observed at its first level: a replay's
  // consecutive windows fail alike, so a dense one starts its next bisection with smaller groups (next_group_size)
  double fault_density = 0;
  // set by dh_batch_begin while it queues a node batch on one stream (node_one_stream): no tail-stream handoff
  bool begin_one_stream = false;
  void release_all() {
    key_tab.release();
    dbuf* all[] = {&s28, &q28, &entries_alt, &cflags, &crank, &cscan, &status, &sig_aff, &q_pts, &scal, &entries, &verdict_tmp, &rand_tmp, &h2c_tmp, &in_rounds, &in_sigs,
                   &in_prevs, &in_prev_lens, &out_verdict, &out_rand, &key_raw, &key_aff, &key_ok, &cnt, &off,
                   &scan_tmp, &list, &buckets, &segs, &outA, &outB, &out2, &pass, &part, &meta, &vm_pairs, &vm_live, &vm_done, &r_commits, &r_cstatus, &r_caff, &r_shares,
                   &r_raw, &r_psigs, &r_pidx, &r_pstatus, &r_paff, &r_msgs, &r_q, &r_scal, &r_round_of, &r_e_pidx,
                   &r_e_sidx, &r_e_grp, &r_P, &r_Q, &r_f, &r_skip, &r_ok, &r_sel, &r_lam, &r_lamset, &r_rok, &r_sig,
                   &r_sigbytes, &r_status2, &r_aff2, &r_entries2, &r_off, &r_key, &r_den, &r_zs, &r_tbl, &r_rstat, &r_ltmp, &r_own, &r_need, &node_sum, &node_res};
    for (dbuf* b : all) b->release();
    d_stage.release();
    sub_bad.release();
    if (h_stage) (void)hipHostFree(h_stage);
    h_stage = nullptr;
    h_stage_cap = 0;
    for (hipEvent_t* e : {&join, &ev_dec, &ev_sub}) {
      if (*e) (void)hipEventDestroy(*e);
      *e = nullptr;
    }
    if (stream) (void)hipStreamDestroy(stream);
    if (tail) (void)hipStreamDestroy(tail);
    if (handoff) (void)hipEventDestroy(handoff);
    if (part_ready) (void)hipEventDestroy(part_ready);
    if (gath_ready) (void)hipEventDestroy(gath_ready);
    stream = tail = nullptr;
    handoff = part_ready = gath_ready = nullptr;
  }
};

struct context {
  std::mutex mu;
  std::condition_variable freed;  // a worker became idle
  bool inited = false;
  int device = 0;
  // at most this many workers (2 HIP streams each): a burst of callers waits for an idle worker instead of creating
  // streams until the runtime runs out of hardware-queue resources (r03: 16 node batches in flight, each holding two
  // workers, aborted HSA queues with HSA_STATUS_ERROR_OUT_OF_RESOURCES); DRANDHIP_MAX_WORKERS overrides
  size_t max_workers = [] {
    const char* e = getenv("DRANDHIP_MAX_WORKERS");
    const long v = e ? atol(e) : 0;
    return (size_t)(v >= 1 && v <= 256 ? v : 24);
  }();
  std::vector<worker*> pool;     // idle or leased workers
  std::vector<worker*> retired;  // leased when dh_shutdown ran: freed by their lease's end
};
context g_ctx;

// One device per process (the multi-GPU layout is one process per GPU): the mask must name at
// most one device; 0 means "device 0, or the device already selected".
int ensure_init_locked(uint32_t mask) {
  if (mask & (mask - 1)) return fail(DH_EINVAL, "device mask 0x%x names more than one device (one process per GPU)", mask);
  const int want = mask ? __builtin_ctz(mask) : -1;
  if (g_ctx.inited) {
    if (want >= 0 && want != g_ctx.device)
      return fail(DH_EINVAL, "already initialised on device %d (dh_shutdown first)", g_ctx.device);
    return DH_OK;
  }
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev <= 0) return fail(DH_EDEVICE, "no HIP device available (%s)", hipGetErrorString(e));
  const int dev = want >= 0 ? want : 0;
  if (dev >= ndev) return fail(DH_EINVAL, "device %d not present (%d devices)", dev, ndev);
  g_ctx.device = dev;
  g_ctx.inited = true;
  return DH_OK;
}

// How long a blocking call waits for a worker while EVERY worker is held by an unfinished node batch (those are
// released only by their callers' dh_batch_finish, possibly on the waiting thread itself): then DH_EBUSY, not a
// deadlock. DRANDHIP_LEASE_TIMEOUT_MS overrides (default 30 s).
static std::chrono::milliseconds node_held_timeout() {
  static const long v = [] {
    const char* e = getenv("DRANDHIP_LEASE_TIMEOUT_MS");
    const long x = e ? atol(e) : 0;
    return x > 0 ? x : 30000L;
  }();
  return std::chrono::milliseconds(v);
}

// A worker for the duration of a call. The pool holds at most g_ctx.max_workers: a blocking call waits for an idle
// one; wait = false (dh_batch_begin, whose lease spans a collective with the other ranks, so waiting could deadlock
// the node) fails with DH_EBUSY instead, and its worker is marked node_held until dh_batch_finish. A blocking call
// that finds every worker node_held waits at most node_held_timeout() and then fails with DH_EBUSY.
struct lease {
  worker* w = nullptr;
  int rc = DH_OK;
  explicit lease(bool wait = true) {
    std::unique_lock<std::mutex> lk(g_ctx.mu);
    rc = ensure_init_locked(0);
    if (rc != DH_OK) return;
    for (;;) {
      for (worker* x : g_ctx.pool)
        if (!x->busy) {
          w = x;
          break;
        }
      if (w) break;
      if (g_ctx.pool.size() < g_ctx.max_workers) {
        w = new worker();
        g_ctx.pool.push_back(w);
        break;
      }
      if (!wait) {
        rc = fail(DH_EBUSY, "all %zu library workers are busy (DRANDHIP_MAX_WORKERS)", g_ctx.max_workers);
        return;
      }
      const bool all_node_held =
          std::all_of(g_ctx.pool.begin(), g_ctx.pool.end(), [](const worker* x) { return x->node_held; });
      if (!all_node_held) {
        g_ctx.freed.wait(lk);
      } else if (g_ctx.freed.wait_for(lk, node_held_timeout()) == std::cv_status::timeout) {
        rc = fail(DH_EBUSY, "all %zu library workers are held by unfinished node batches (dh_batch_finish them first)",
                  g_ctx.max_workers);
        return;
      }
    }
    w->busy = true;
    w->node_held = !wait;
  }
  ~lease() {
    if (!w) return;
    std::lock_guard<std::mutex> lk(g_ctx.mu);
    w->busy = false;
    w->node_held = false;
    g_ctx.freed.notify_all();
    auto it = std::find(g_ctx.retired.begin(), g_ctx.retired.end(), w);
    if (it != g_ctx.retired.end()) {  // dh_shutdown ran during this call
      g_ctx.retired.erase(it);
      if (w->stream) (void)hipStreamSynchronize(w->stream);
      w->release_all();
      delete w;
    }
  }
};

// The tail stream is created on a worker's first local call: a worker that only ever runs node batches (one stream
// per batch) holds one stream. HIP hands a process's streams its hardware queues in creation order, round robin; with
// two streams per worker, the node batches' streams landed on every other queue (8 of 16), so more than 8 batches in
// flight doubled some queues up and not others, and the one host thread retiring batches in order waited on the
// doubled ones: 131k-round node batches 21.5 M/s at 8-11 in flight, 16.3 at 12, 19.5 at 16 (19.8 at 12 over 8
// queues, 16.7 at 8 over 4: profiles/r05/node_131072_sweep_r05k).
int set_device_and_stream(worker* w, bool need_tail = true) {
  HIP_TRY(hipSetDevice(g_ctx.device));
  if (!w->stream) HIP_TRY(hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking));
  if (!w->tail && need_tail) {
    int least = 0, greatest = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIP_TRY(hipStreamCreateWithPriority(&w->tail, hipStreamNonBlocking, greatest));
  }
  if (!w->handoff) HIP_TRY(hipEventCreateWithFlags(&w->handoff, hipEventDisableTiming));
  if (!w->part_ready) HIP_TRY(hipEventCreateWithFlags(&w->part_ready, hipEventDisableTiming));
  if (!w->gath_ready) HIP_TRY(hipEventCreateWithFlags(&w->gath_ready, hipEventDisableTiming));
  for (hipEvent_t* e : {&w->join, &w->ev_dec, &w->ev_sub})
    if (!*e) HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
  return DH_OK;
}

// The group key decoded on the device (a key_tab slot: the affine point, then [h_eff] pk for G1-signature schemes),
// cached per worker in KEY_SLOTS slots: a chain's batches all use one key, and decoding a G2 key is a one-lane kernel
// of a few ms. On a miss the stream is synchronised once to read the key's status; DH_EKEY when it is not a
// compressed subgroup point. Sets w->key_cur.
int ensure_key(worker* w, bool g2, const uint8_t* pk, size_t pk_len, hipStream_t st) {
  HIP_TRY(w->key_raw.ensure(96));
  HIP_TRY(w->key_ok.ensure(64));  // [0] key status, [32..63] RLC seed
  HIP_TRY(w->key_tab.ensure(worker::KEY_SLOTS * 96 * 4));  // fixed size keeps the slots valid
  const int kg = g2 ? 0 : 1;
  int slot = -1, victim = 0;
  for (int i = 0; i < worker::KEY_SLOTS; i++) {
    const worker::key_slot& k = w->keys[i];
    if (k.len == pk_len && k.g2 == kg && !memcmp(k.bytes, pk, pk_len)) slot = i;
    if (k.used < w->keys[victim].used) victim = i;
  }
  if (slot < 0) {
    slot = victim;
    worker::key_slot& k = w->keys[slot];
    k.len = 0;
    uint8_t ok = 0;
    uint32_t* dst = w->key_tab.as<uint32_t>() + (size_t)slot * 96;
    HIP_TRY(hipMemcpyAsync(w->key_raw.p, pk, pk_len, hipMemcpyHostToDevice, st));
    HIP_TRY(dh::launch_decode_key(g2 ? 0 : 1, w->key_raw.as<uint8_t>(), dst, w->key_ok.as<uint8_t>(), st));
    HIP_TRY(hipMemcpyAsync(&ok, w->key_ok.p, 1, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    memcpy(k.bytes, pk, pk_len);
    k.len = pk_len;
    k.g2 = kg;
    k.ok = ok;
  }
  w->keys[slot].used = ++w->key_clock;
  w->key_cur = w->key_tab.as<uint32_t>() + (size_t)slot * 96;
  if (w->keys[slot].ok != 1) return fail(DH_EKEY, "group public key is not a valid compressed subgroup point");
  return DH_OK;
}

// ---- host SHA-256 (DigestBeacon for dh_digest_batch; not used by the device path)
struct sha256_host {
  uint32_t h[8];
  uint8_t buf[64];
  uint64_t len;
  size_t n;
  static uint32_t ror(uint32_t x, int k) { return (x >> k) | (x << (32 - k)); }
  void init() {
    static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    memcpy(h, iv, sizeof h);
    len = 0;
    n = 0;
  }
  void block(const uint8_t* p) {
    static const uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
        0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
        0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
        0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
        0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
        0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
        0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
    uint32_t w[64];
    for (int i = 0; i < 16; i++) w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; i++)
      w[i] = w[i - 16] + (ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3)) + w[i - 7] +
             (ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10));
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
      uint32_t t1 = hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
      uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  void update(const uint8_t* d, size_t k) {
    len += k;
    while (k) {
      size_t t = std::min(k, 64 - n);
      memcpy(buf + n, d, t);
      n += t;
      d += t;
      k -= t;
      if (n == 64) {
        block(buf);
        n = 0;
      }
    }
  }
  void final(uint8_t out[32]) {
    uint64_t bits = len * 8;
    uint8_t pad = 0x80, z = 0;
    update(&pad, 1);
    while (n != 56) update(&z, 1);
    uint8_t l[8];
    for (int i = 0; i < 8; i++) l[i] = (uint8_t)(bits >> (56 - 8 * i));
    update(l, 8);
    for (int i = 0; i < 8; i++) {
      out[4 * i] = h[i] >> 24; out[4 * i + 1] = h[i] >> 16; out[4 * i + 2] = h[i] >> 8; out[4 * i + 3] = h[i];
    }
  }
};

uint64_t splitmix64(uint64_t& x) {
  uint64_t z = (x += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

int make_seed(uint64_t seed, uint32_t words[8]) {
  if (seed == 0) {
    uint8_t b[32];
    size_t got = 0;
    while (got < sizeof b) {
      ssize_t r = getrandom(b + got, sizeof b - got, 0);
      if (r <= 0) return fail(DH_EDEVICE, "getrandom failed");
      got += (size_t)r;
    }
    memcpy(words, b, 32);
  } else {
    uint64_t x = seed;
    for (int i = 0; i < 4; i++) {
      uint64_t v = splitmix64(x);
      words[2 * i] = (uint32_t)(v >> 32);
      words[2 * i + 1] = (uint32_t)v;
    }
  }
  return DH_OK;
}

// MSM geometry for groups of gsize rounds; parts: 1 = 127-bit scalars, 2 = the endomorphism split (2 x gsize points,
// 63-bit scalar halves), 4 = the G2 psi split (4 x gsize points, 31-bit scalar parts)
static bool window_ok(int sbits, int c) {
  // keep the top window's t bits at >= c - 4, since each of its 2^(t-1) buckets collects ~m / 2^(t-1) entries
  // and a bucket that spans many chunks is summed serially by k_msm_bucket_fix (127-bit scalars at c = 14 would
  // leave t = 1: two buckets holding the whole set)
  const int nw = (sbits + 1 + c - 1) / c, t = sbits - c * (nw - 1);
  return t >= c - 4;
}
dh::msm_geom geom_for(size_t gsize, int parts = 1) {
  const size_t npts = (size_t)parts * gsize;
  const int sbits = parts == 4 ? 31 : parts == 2 ? 63 : 127;  // scalar bits (k_scalars)
  int lg = 0;
  while (((size_t)1 << (lg + 1)) <= npts) lg++;
  int c = std::max(3, std::min(16, lg - 2));
  // DRANDHIP_MSM_C (experiments): the window width of batch-sized groups (>= 65,536 rounds)
  static const int c_env = [] {
    const char* e = getenv("DRANDHIP_MSM_C");
    const int v = e ? atoi(e) : 0;
    return v >= 4 && v <= 16 ? v : 0;
  }();
  if (c_env && gsize >= 65536) c = c_env;
  // c = lg(npts) - 2 (a 131k-round shard keeps c = 16: a cost model trading bucket-pass additions against the
  // reduction picked c = 13 there and measured 8.5 ms against 6.7, gpurun_out r03g)
  while (c > 3 && !window_ok(sbits, c)) c--;
  dh::msm_geom g;
  g.gsize = (uint32_t)gsize;
  g.c = c;
  g.nwin = (sbits + 1 + c - 1) / c;
  g.nbuck = (1u << (c - 1)) + 1;  // signed digits: |d| in [1, 2^(c-1)] (k_msm.hip: signed_digit)
  // bucket reduction: segments of ~8 digits, one thread each (k_msm_segsum): 16 additions + the segment's offset
  // multiple per thread, then a log-depth tree
  uint32_t nseg = std::max(1u, std::min(8192u, g.nbuck / 8));  // a power of two (nbuck = 2^(c-1) + 1)
  g.nseg = nseg;
  g.seglen = (g.nbuck - 1 + nseg - 1) / nseg;
  g.halves = (uint32_t)parts;
  g.half_stride = 0;  // set by the caller: the point-array offset of the endomorphism images
  return g;
}

// Bucket-reduction segments for a level of ngroups groups (nsets point sets): as many segments per (set, group, window)
// row as keep ~256k segment threads busy, at most nbuck / 8. Each extra segment costs its offset multiple (segoff:
// ~log2 k doublings) and a tree level; with thousands of groups (the bisection's 256- and 32-round levels) the rows
// alone fill the chip, and geom_for's fixed 8-bucket segments had doubled the reduction's additions there (a
// 129-bucket row: 16 segments = 256 + ~150 segoff additions against 256 + 7 for 2).
static void fit_segments(dh::msm_geom& g, size_t ngroups, size_t nsets) {
  const size_t rows = std::max<size_t>(1, nsets * ngroups * (size_t)g.nwin);
  const size_t want = ((size_t)1 << 18) / rows + 1;
  size_t nseg = std::max<size_t>(1, std::min<size_t>({want, (size_t)g.nseg}));
  if (nseg > 512) nseg &= ~(size_t)511;  // rows of more than 64 lanes of 8 segments fill whole waves (k_msm_rowtree28)
  g.nseg = (uint32_t)nseg;
  g.seglen = (g.nbuck - 1 + g.nseg - 1) / g.nseg;
}

constexpr size_t JAC_WORDS_G1 = 36, JAC_WORDS_G2 = 72;

// ---- live per-kernel timing with HIP events on the launching stream (dh_profile / dh_profile_read)
struct prof_entry {
  uint64_t count = 0;
  double ms = 0;
  unsigned long long prods = 0;  // field products executed (counting build only)
};
struct prof_pending {
  const char* name;
  hipEvent_t a, b;
  unsigned long long prods;
};
struct profiler {
  std::mutex mu;
  std::atomic<bool> on{false};  // read on every launch without the lock
  std::vector<std::pair<std::string, prof_entry>> table;
  std::vector<prof_pending> pending;  // launches whose end event had not completed when their call returned
  void add(const char* name, float ms, unsigned long long prods = 0) {
    std::lock_guard<std::mutex> lk(mu);
    add_locked(name, ms, prods);
  }
  void add_locked(const char* name, float ms, unsigned long long prods) {
    for (auto& e : table)
      if (e.first == name) {
        e.second.count++;
        e.second.ms += ms;
        e.second.prods += prods;
        return;
      }
    prof_entry pe;
    pe.count = 1;
    pe.ms = ms;
    pe.prods = prods;
    table.emplace_back(name, pe);
  }
};
profiler g_prof;

static void prof_settle(const char* name, hipEvent_t a, hipEvent_t b, unsigned long long prods) {
  float ms = 0;
  if (hipEventSynchronize(b) == hipSuccess && hipEventElapsedTime(&ms, a, b) == hipSuccess) g_prof.add(name, ms, prods);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
}
// resolve the deferred launches (waits for them); called with g_prof.mu held
static void prof_drain_locked() {
  for (auto& r : g_prof.pending) {
    float ms = 0;
    if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess)
      g_prof.add_locked(r.name, ms, r.prods);
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  g_prof.pending.clear();
}

#ifdef DH_COUNT_PRODUCTS
// counting build: products executed by every translation unit's kernels since the last take
static unsigned long long count_take_all() {
  unsigned long long t = 0, v = 0;
  hipError_t (*take[])(unsigned long long*) = {dh::count_take_prep, dh::count_take_msm, dh::count_take_check,
                                               dh::count_take_sign, dh::count_take_recover, dh::count_take_vm};
  for (auto f : take)
    if (f(&v) == hipSuccess) t += v;
  return t;
}
#endif

// records a launch bracketed by events when profiling is on; resolved after the stream syncs. The counting build
// also synchronises after each launch and attributes the products executed to it (one batch at a time).
struct timed_launches {
  struct rec {
    const char* name;
    hipEvent_t a, b;
    unsigned long long prods;
  };
  std::vector<rec> recs;
  hipStream_t st;
  explicit timed_launches(hipStream_t s) : st(s) {}
  template <class F>
  hipError_t run(const char* name, F&& f) {
    if (!g_prof.on.load(std::memory_order_relaxed)) return f();
    rec r{name, nullptr, nullptr, 0};
    (void)hipEventCreate(&r.a);
    (void)hipEventCreate(&r.b);
#ifdef DH_COUNT_PRODUCTS
    (void)hipDeviceSynchronize();
    (void)count_take_all();
#endif
    (void)hipEventRecord(r.a, st);
    hipError_t e = f();
    (void)hipEventRecord(r.b, st);
#ifdef DH_COUNT_PRODUCTS
    (void)hipDeviceSynchronize();
    r.prods = count_take_all();
#endif
    recs.push_back(r);
    return e;
  }
  // launches still running (a node batch's begin returns with its kernels queued) are resolved later, when the
  // profile is read, so timing never adds a host wait
  void resolve() {
    for (auto& r : recs) {
      if (hipEventQuery(r.b) == hipErrorNotReady) {
        std::lock_guard<std::mutex> lk(g_prof.mu);
        g_prof.pending.push_back({r.name, r.a, r.b, r.prods});
        continue;
      }
      prof_settle(r.name, r.a, r.b, r.prods);
    }
    recs.clear();
  }
  ~timed_launches() { resolve(); }
};

// Pairing checks: the lane-parallel program (k_vm.hip) unless DRANDHIP_LANE_PAIRING=1 selects the one-lane
// tower code (k_check.hip), kept as the independent second implementation the parity tests compare against.
static bool lane_pairing() {
  static const bool v = [] {
    const char* e = getenv("DRANDHIP_LANE_PAIRING");
    return e && e[0] == '1';
  }();
  return v;
}

// key_h: [h_eff] pk next to a decoded G2 key (k_decode_key), or null (the check clears B's cofactor itself)
// G2-signature group checks of up to this many groups clear B's cofactor inside the pairing program (NP2C: the
// clearing's doublings spread over the lanes) instead of on one lane before it; DRANDHIP_NP2C=0 turns it off. Above
// it the one-lane clearing wins: every group's lane runs in parallel, the NP2C workgroups queue for the CUs.
static size_t np2c_max_groups() {
  static const size_t v = [] {
    const char* e = getenv("DRANDHIP_NP2C");
    return e && e[0] == '0' ? (size_t)0 : (size_t)4096;
  }();
  return v;
}

// G2-signature leaves (per-round checks: bisection leaves and the small-batch path) likewise, up to this many per
// launch; DRANDHIP_NP2C_LEAVES overrides (0: every leaf clears its hash point on one lane first)
static size_t np2c_max_leaves() {
  static const size_t v = [] {
    const char* e = getenv("DRANDHIP_NP2C_LEAVES");
    return e ? (size_t)atol(e) : (size_t)4096;
  }();
  return v;
}

// G1-signature checks with [h_eff] pk at hand take their G1 sides in Jacobian form (NP2J: no prep kernel, no
// inversion before the program); DRANDHIP_G1_JAC=0 keeps the affine prep (k_vm_prep_groups / _leaves) for A/B runs
static bool g1_jac() {
  static const bool v = [] {
    const char* e = getenv("DRANDHIP_G1_JAC");
    return !(e && e[0] == '0');
  }();
  return v;
}

static hipError_t group_check(worker* w, bool g2, const uint32_t* A, const uint32_t* B, size_t ngroups, const uint32_t* key,
                              uint8_t* pass, hipStream_t st, const uint32_t* key_h = nullptr) {
  if (lane_pairing()) return dh::launch_group_check(g2, A, B, ngroups, key, pass, st);
  if (!g2 && key_h && g1_jac()) return dh::launch_group_check_g1j(A, B, ngroups, key_h, pass, st);
  hipError_t e;
  if (g2 && ngroups <= np2c_max_groups()) {
    if ((e = w->vm_pairs.ensure(ngroups * dh::group_check_c_pair_words() * 4)) != hipSuccess) return e;
    if ((e = w->vm_live.ensure(ngroups * 3)) != hipSuccess) return e;
    if ((e = w->vm_done.ensure(ngroups)) != hipSuccess) return e;
    return dh::launch_group_check_vm_c(A, B, ngroups, key, w->vm_pairs.as<uint32_t>(), w->vm_live.as<uint8_t>(),
                                       w->vm_done.as<uint8_t>(), pass, st);
  }
  if ((e = w->vm_pairs.ensure(ngroups * 2 * 72 * 4)) != hipSuccess) return e;
  if ((e = w->vm_live.ensure(ngroups * 2)) != hipSuccess) return e;
  return dh::launch_group_check_vm(g2, A, B, ngroups, key, g2 ? nullptr : key_h, w->vm_pairs.as<uint32_t>(),
                                   w->vm_live.as<uint8_t>(), pass, st);
}

// key_h as for group_check: the leaves of G1-signature schemes pair the uncleared hash point with [h_eff] pk
static hipError_t leaf_check(worker* w, bool g2, const uint32_t* entries, size_t m, const uint32_t* sig_aff,
                             const uint32_t* q_pts, const uint32_t* key, const uint8_t* status, uint8_t* verdict,
                             hipStream_t st, const uint32_t* key_h = nullptr) {
  if (lane_pairing()) return dh::launch_leaf_check(g2, entries, m, sig_aff, q_pts, key, status, verdict, st);
  if (!g2 && key_h && g1_jac()) return dh::launch_leaf_check_g1j(entries, m, sig_aff, q_pts, key_h, status, verdict, st);
  hipError_t e;
  if (g2 && m <= np2c_max_leaves()) {
    if ((e = w->vm_pairs.ensure(m * dh::group_check_c_pair_words() * 4)) != hipSuccess) return e;
    if ((e = w->vm_live.ensure(m * 3)) != hipSuccess) return e;
    if ((e = w->vm_done.ensure(m)) != hipSuccess) return e;
    return dh::launch_leaf_check_vm_c(entries, m, sig_aff, q_pts, key, status, w->vm_pairs.as<uint32_t>(),
                                      w->vm_live.as<uint8_t>(), w->vm_done.as<uint8_t>(), verdict, st);
  }
  if ((e = w->vm_pairs.ensure(m * 2 * 72 * 4)) != hipSuccess) return e;
  if ((e = w->vm_live.ensure(m * 2)) != hipSuccess) return e;
  if ((e = w->vm_done.ensure(m)) != hipSuccess) return e;
  return dh::launch_leaf_check_vm(g2, entries, m, sig_aff, q_pts, key, g2 ? nullptr : key_h, status,
                                  w->vm_pairs.as<uint32_t>(), w->vm_live.as<uint8_t>(), w->vm_done.as<uint8_t>(), verdict,
                                  st);
}

// Bisection ladder. DRANDHIP_BISECT="4096,256,16,2" fixes the group sizes after level 0 (tests, experiments);
// otherwise next_group_size picks each level from the failure rate the previous level observed.
static const std::vector<size_t>& fixed_ladder() {
  static const std::vector<size_t> v = [] {
    std::vector<size_t> r;
    const char* e = getenv("DRANDHIP_BISECT");
    while (e && *e) {
      char* end = nullptr;
      unsigned long x = strtoul(e, &end, 10);
      if (end == e) break;
      if (x >= 2) r.push_back(x);
      e = *end ? end + 1 : end;
    }
    return r;
  }();
  return v;
}

// Expected-cost choice of the next bisection level (group size; 1 = per-round leaf checks). Level costs
// fitted to the chained-replay sweep on one MI355X (bench/bisect_sweep.sh, ms at 1M G2 rounds): an MSM over m
// rounds costs ~9 + 1.8e-6 m nwin(g), a group-check launch ~12 + 0.0025 groups (the pairing program's
// latency floor), per-round leaf checks ~12 + 0.005 m. Faults are modelled as Poisson at the density the last
// level observed (faulty groups -> -ln(1 - f) faults per group, at least one per failing group; when every
// group failed, 5 per group). The next size minimises the expected cost of the rest of the descent.
static double msm_cost_ms(double m, size_t g) {
  const dh::msm_geom gg = geom_for(g, 2);
  return 9.0 + 1.8e-6 * m * (double)(gg.nwin * gg.halves) / 2.0;  // fitted on 127-bit entries (8 per round at c = 16)
}
static double check_cost_ms(double groups) { return 12.0 + 0.0025 * groups; }
static double leaf_cost_ms(double m) { return 12.0 + 0.005 * m; }

static double descent_cost(double m, double d, size_t gprev, size_t* best) {
  double c_best = leaf_cost_ms(m);
  if (best) *best = 1;
  for (size_t g = 4; g < gprev && (double)g < m; g *= 4) {
    const double q = -std::expm1(-d * (double)g);  // P(group of g holds a fault)
    const double m_next = m * q;
    const double c = msm_cost_ms(m, g) + check_cost_ms(m / (double)g) +
                     (m_next < 1.0 ? 0.0 : descent_cost(m_next, d / std::max(q, 1e-12), g, nullptr));
    if (c < c_best) {
      c_best = c;
      if (best) *best = g;
    }
  }
  return c_best;
}

static size_t next_group_size(size_t gsize, size_t ngroups, size_t nfail, size_t m_prev, size_t m_next, double hint) {
  // level 0 (one group) says only that some round is bad: 1024 costs about what 4096 does over 1M rounds and
  // its groups still pass at a 0.1% fault density (4096-round groups then all fail). When the worker's previous
  // bisection saw dense faults (> 1 per 2000 rounds: most 1024-groups fail), 256-round groups first: the ladder
  // sweep on a 0.2%-faulty chained window put 256-first ladders 5-9% ahead of 1024-first ones
  // (profiles/bisect_sweep_r03s.txt)
  const bool dense = hint > 1.0 / 2000;
  if (gsize == m_prev && m_prev > 4096) return dense ? 256 : 1024;
  // ... and continues 256 -> 32 -> 4 -> per-round leaves, the best ladder of that sweep (231.7 ms per 1M window
  // against 240-259 for the others); the cost model below was fitted on sparser failures
  if (dense && (gsize == 256 || gsize == 32)) return gsize == 256 ? 32 : 4;
  if (dense && gsize == 4) return 1;
  const double f = (double)nfail / (double)ngroups;
  const double per_group = nfail == ngroups ? 5.0 : -std::log1p(-f);
  const double faults = std::max((double)nfail, per_group * (double)ngroups);
  const double density = std::min(1.0, faults / (double)std::max<size_t>(m_next, 1));
  size_t g = 1;
  descent_cost((double)m_next, density, gsize, &g);
  return g;
}

static bool prep_sync() {
  static const bool v = [] {
    const char* e = getenv("DRANDHIP_PREP_SYNC");
    return !(e && e[0] == '0');
  }();
  return v;
}

// DRANDHIP_SKIP_LEVEL0=0 keeps level 0 on dense-fault workers (comparison runs)
static bool skip_level0() {
  static const bool v = [] {
    const char* e = getenv("DRANDHIP_SKIP_LEVEL0");
    return !(e && e[0] == '0');
  }();
  return v;
}


// core pipeline on device-resident inputs
// Phases of one batch (the node-wide check of dh_batch_begin / dh_batch_finish runs them separately):
enum verify_mode {
  VM_FULL = 0,        // prepare, then every level (local level-0 check)
  VM_BEGIN = 1,       // prepare and the level-0 MSM only: the partial sums are left in outA / outB
  VM_FINISH = 2,      // after VM_BEGIN: local level-0 check and bisection
  VM_FINISH_PASS = 3  // after VM_BEGIN, the node-wide check passed: every decoded round is valid
};

// One-call pipelining (run_split): the per-round kernels of consecutive chunks run one after another, each chunk's
// alone on the chip, while the latency-bound tails of earlier chunks (MSM reduction, pairing checks) run beside
// them on their own streams. A chunk's per-round kernels wait for the previous chunk's (an event), and it records
// its own event once they are queued.
struct prep_gate {
  hipEvent_t wait = nullptr;  // the previous chunk's per-round kernels (null: first chunk)
  hipEvent_t done = nullptr;  // this chunk's
  std::function<void()> recorded;  // host side: `done` is recorded, the next chunk may queue behind it
};

// MSM workspace of one bisection level (m entries in ngroups groups of geometry g, Jacobian width jw words)
static int msm_workspace(worker* w, const dh::msm_geom& g, size_t m, size_t ngroups, size_t jw, dh::msm_ws& ws) {
  const size_t nk = ngroups * g.nwin * (size_t)g.nbuck;
  HIP_TRY(w->cnt.ensure(nk * 4));
  HIP_TRY(w->off.ensure((nk + 1) * 4));
  HIP_TRY(w->scan_tmp.ensure(((nk + 4095) / 4096 + 1) * 4));
  HIP_TRY(w->list.ensure(dh::msm_entries(g, m) * 4));
  HIP_TRY(w->buckets.ensure(2 * nk * jw * 4));
  const size_t segs_bytes = 2 * ngroups * g.nwin * g.nseg * jw * 4;
  HIP_TRY(w->segs.ensure(2 * segs_bytes));  // segment sums, then (MSM28) the segments' running sums
  HIP_TRY(w->outA.ensure(ngroups * jw * 4));
  HIP_TRY(w->outB.ensure(ngroups * jw * 4));
  HIP_TRY(w->out2.ensure(2 * ngroups * jw * 4));
  HIP_TRY(w->pass.ensure(ngroups));
  HIP_TRY(w->part.ensure(dh::msm_part_bytes(dh::msm_entries(g, m), jw, 2)));
  HIP_TRY(w->meta.ensure(dh::msm_meta_bytes(dh::msm_entries(g, m))));
  ws = dh::msm_ws{w->cnt.as<uint32_t>(), w->off.as<uint32_t>(), w->scan_tmp.as<uint32_t>(), w->list.as<uint32_t>(),
                  w->buckets.as<uint32_t>(), w->segs.as<uint32_t>(), w->out2.as<uint32_t>(), w->part.as<uint32_t>(),
                  w->meta.as<uint32_t>(), 0, (uint32_t*)((uint8_t*)w->segs.p + segs_bytes)};
  return DH_OK;
}

int verify_core(worker* w, int scheme, const uint8_t* pk, size_t pk_len, const uint64_t* d_rounds, const uint8_t* d_sigs,
                size_t sig_stride, const uint8_t* d_prevs, size_t prev_stride, const uint32_t* d_prev_lens, size_t n,
                uint8_t* d_verdict, uint8_t* d_rand, uint64_t seed, hipStream_t st, uint64_t* stats,
                const uint8_t* d_msgs32 = nullptr, int mode = VM_FULL, prep_gate* gate = nullptr) {
  const bool g2 = sig_on_g2(scheme);
  const int sig_len = g2 ? 96 : 48, key_len = g2 ? 48 : 96;
  if ((int)pk_len != key_len) return fail(DH_EINVAL, "public key must be %d bytes for scheme %d", key_len, scheme);
  if (sig_stride < (size_t)sig_len || sig_stride % 4) return fail(DH_EINVAL, "bad signature stride %zu", sig_stride);
  if (stats) memset(stats, 0, 4 * sizeof(uint64_t));
  if (n == 0) return DH_OK;
  // the MSM runs on lazily reduced 28-bit points (k_msm.hip MSM28), whose workspace points take 48 (G1) / 96 (G2)
  // words; G2 splits each scalar in four psi parts, G1 in two endomorphism halves. (r01-r03 also kept a 12 x 32-bit
  // Pippenger behind DRANDHIP_MSM32 as a second implementation; removed in r04, git history has it.)
  const int parts = g2 ? 4 : 2;
  // sorted-list entries keep a sign bit and address parts * n points (the endomorphism images follow the n points)
  if (n >= ((size_t)1 << 31) / parts) return fail(DH_EINVAL, "batch too large");
  const size_t jw = g2 ? JAC_WORDS_G2 : JAC_WORDS_G1;
  const size_t aw = jw * 2 / 3;
  const size_t wsw = g2 ? 96 : 48;

  timed_launches T(st);
  // the whole batch on st (no tail-stream handoff, no level-0 presort there): a node batch's begin (begin_one_stream).
  // A local batch keeps the handoff after its host wait: measured on one stream too (gpurun_out r04aa), 1M rounds
  // 26.58 -> 26.41 M/s and one 1M call 46.2 -> 47.5 ms (the presort no longer overlaps the per-round kernels), 131k
  // rounds 20.76 -> 21.46 M/s.
  const bool one_stream = mode == VM_BEGIN && w->begin_one_stream;
  bool presorted = false;  // level-0 sorted lists already built on the tail stream
  // A local batch on a worker whose last bisection saw dense faults skips level 0: its one group is expected to fail,
  // so the batch starts at the dense ladder's 256-round groups (their check also answers "is the batch clean": a
  // batch whose groups all pass clears the hint). Saves the level-0 MSM and pairing check per dense window.
  // (with a fixed ladder, DRANDHIP_BISECT, its first size)
  const bool skip0 = mode == VM_FULL && w->fault_density > 1.0 / 2000 && n > 4096 && skip_level0();
  dh::msm_geom g0{};
  dh::msm_ws ws0{};
  if (mode <= VM_BEGIN) {
    // key (cached per worker; a miss synchronises once, before any per-round kernel is queued)
    int rc = ensure_key(w, g2, pk, pk_len, st);
    if (rc) return rc;

    // per-round prep
    HIP_TRY(w->status.ensure(n));
    HIP_TRY(w->sig_aff.ensure(n * aw * 4));
    HIP_TRY(w->q_pts.ensure(n * jw * 4));
    HIP_TRY(w->scal.ensure(n * 16));
    HIP_TRY(w->entries.ensure(n * 4));
    uint32_t seedw[8];
    rc = make_seed(seed, seedw);
    if (rc) return rc;
    uint32_t* d_seed = (uint32_t*)((uint8_t*)w->key_ok.p + 32);
    // The level-0 sort needs only the scalars, and the scalars only the seed: with a tail stream it runs there
    // while the per-round kernels decode and hash (its ~1 ms of small kernels left the one-call latency path).
    // Every round then carries a scalar; the bucket passes skip rounds whose status is not DEC_OK. A batch that skips
    // level 0 (skip0) has no level-0 sort.
    presorted = w->tail && st == w->stream && !skip0 && !one_stream;
    if (presorted) {
      hipStream_t ts = w->tail;
      HIP_TRY(hipMemcpyAsync(d_seed, seedw, 32, hipMemcpyHostToDevice, ts));
      HIP_TRY(dh::launch_scalars(d_seed, n, nullptr, w->scal.as<uint4>(), parts, ts));
      HIP_TRY(dh::launch_iota(w->entries.as<uint32_t>(), n, ts));
      g0 = geom_for(n, parts);
      g0.half_stride = (uint32_t)n;
      rc = msm_workspace(w, g0, n, 1, wsw, ws0);
      if (rc) return rc;
      HIP_TRY(dh::launch_msm_sort(g0, w->entries.as<uint32_t>(), nullptr, nullptr, n, 1, w->scal.as<uint4>(), ws0, ts));
    }
    if (gate && gate->wait) HIP_TRY(hipStreamWaitEvent(st, gate->wait, 0));
    HIP_TRY(T.run(g2 ? "k_prep_sig<fp2>" : "k_prep_sig<fp>", [&] {
      return dh::launch_prep(g2, d_sigs, sig_stride, n, w->status.as<uint8_t>(), w->sig_aff.as<uint32_t>(), d_rand, st);
    }));
    // hash points: of the beacon digests, or of the given 32-byte messages (VerifyRecovered); a chained record
    // longer than its slot rejects its round (status)
    HIP_TRY(w->h2c_tmp.ensure(dh::hash_tmp_bytes(g2, n)));
    HIP_TRY(T.run(d_msgs32 ? (g2 ? "k_prep_msg32<fp2>" : "k_prep_msg32<fp>") : (g2 ? "k_prep_msg<fp2>" : "k_prep_msg<fp>"), [&] {
      return dh::launch_hash(g2, d_rounds, d_prevs, prev_stride, d_prev_lens, d_msgs32, n,
                             scheme == DH_SCHEME_CHAINED && d_prevs && !d_msgs32 ? 1 : 0, dst_id(scheme), w->status.as<uint8_t>(),
                             w->q_pts.as<uint32_t>(), w->h2c_tmp.as<uint32_t>(), st);
    }));
    if (!presorted) {
      HIP_TRY(hipMemcpyAsync(d_seed, seedw, 32, hipMemcpyHostToDevice, st));
      HIP_TRY(dh::launch_scalars(d_seed, n, w->status.as<uint8_t>(), w->scal.as<uint4>(), parts, st));
    }
    HIP_TRY(w->s28.ensure(parts * n * (g2 ? 64 : 32) * 4));
    HIP_TRY(w->q28.ensure(parts * n * (g2 ? 64 : 32) * 4));
    HIP_TRY(T.run(g2 ? "k_msm_prep28<fp2>" : "k_msm_prep28<fp>", [&] {
      return dh::launch_msm_prep28(g2, n, w->status.as<uint8_t>(), w->sig_aff.as<uint32_t>(), w->q_pts.as<uint32_t>(),
                                   w->s28.as<uint32_t>(), w->q28.as<uint32_t>(), st);
    }));
    HIP_TRY(hipMemsetAsync(d_verdict, 0, n, st));
    if (gate) {
      HIP_TRY(hipEventRecord(gate->done, st));
      gate->recorded();
    }
    // The node batch (VM_BEGIN) queues its tail behind the per-round kernels with no host wait. A local batch
    // (VM_FULL) waits here first, as r03 did: its tail stream then carries no event wait while the per-round kernels
    // run, and with 8 batches in flight (16+ streams on 16 hardware queues) a queue blocked on such a wait holds up
    // the streams that share it (quicknet 1M: 25.5-25.9 M/s without this wait, 26.4-26.5 with it; DRANDHIP_PREP_SYNC=0
    // drops it for comparison).
    if (mode == VM_FULL && w->tail && st == w->stream && !one_stream && prep_sync()) HIP_TRY(hipStreamSynchronize(st));
    if (!presorted) HIP_TRY(dh::launch_iota(w->entries.as<uint32_t>(), n, st));
  }
  // the tail (MSM, checks, bisection) runs on the worker's high-priority stream, after the per-round kernels
  if (w->tail && st == w->stream && !one_stream) {
    if (mode <= VM_BEGIN) {
      HIP_TRY(hipEventRecord(w->handoff, st));
      HIP_TRY(hipStreamWaitEvent(w->tail, w->handoff, 0));
    }
    st = w->tail;
    T.st = st;
  }

  // bisection levels: group sizes n, then next_group_size() per level, then per-round leaves (a failing group is re-checked
  // as smaller groups with the same scalars; only rounds of failing pairs reach a per-round pairing check)
  size_t m = n;
  static const char* const msm_names[8] = {"msm_level0", "msm_bisect1", "msm_bisect2", "msm_bisect3",
                                           "msm_bisect4", "msm_bisect5", "msm_bisect6", "msm_bisect7+"};
  static const char* const chk_names[8] = {"k_group_check_level0", "k_group_check_bisect1", "k_group_check_bisect2",
                                           "k_group_check_bisect3", "k_group_check_bisect4", "k_group_check_bisect5",
                                           "k_group_check_bisect6", "k_group_check_bisect7+"};
  const std::vector<size_t>& fixed = fixed_ladder();
  size_t gsize = skip0 ? (fixed.empty() ? 256 : fixed[0]) : n;
  int level = skip0 ? 1 : 0;
  if (mode == VM_BEGIN && n < 2) {
    // a one-round batch has no level-0 group: it contributes the identity (Z = 0) to the node-wide sums, and
    // dh_batch_finish gives the round its own leaf check whatever the node check says
    HIP_TRY(w->outA.ensure(jw * 4));
    HIP_TRY(w->outB.ensure(jw * 4));
    HIP_TRY(hipMemsetAsync(w->outA.p, 0, jw * 4, st));
    HIP_TRY(hipMemsetAsync(w->outB.p, 0, jw * 4, st));
    return DH_OK;  // queued: dh_batch_begin orders the caller after it (or waits)
  }
  while (m > 0 && gsize > 1) {
    gsize = std::min(gsize, m);
    dh::msm_geom g = geom_for(gsize, parts);
    g.half_stride = (uint32_t)n;
    const size_t ngroups = (m + gsize - 1) / gsize;
    fit_segments(g, ngroups, 2);
    const bool pre = level == 0 && presorted;
    dh::msm_ws ws{};
    if (pre) {
      ws = ws0;
    } else {
      const int rc = msm_workspace(w, g, m, ngroups, wsw, ws);
      if (rc) return rc;
    }
    if (!(level == 0 && mode >= VM_FINISH)) {  // a resumed batch has its level-0 sums from dh_batch_begin
      // every level skips the rounds whose status is not DEC_OK (their scalars are nonzero after a presort)
      HIP_TRY(T.run(msm_names[std::min(level, 7)], [&] {
        return dh::launch_msm28(g2, pre ? g0 : g, w->entries.as<uint32_t>(), m, ngroups, w->scal.as<uint4>(),
                                w->s28.as<uint32_t>(), w->q28.as<uint32_t>(), ws, w->outA.as<uint32_t>(),
                                w->outB.as<uint32_t>(), st, w->status.as<uint8_t>(), pre);
      }));
    }
    if (level == 0 && mode == VM_BEGIN) return DH_OK;  // queued; dh_batch_begin orders the caller after it
    if (level == 0 && mode == VM_FINISH_PASS) {  // the node-wide check covers this batch's single level-0 group
      HIP_TRY(hipMemsetAsync(w->pass.p, 1, 1, st));
    } else {
      HIP_TRY(T.run(chk_names[std::min(level, 7)], [&] {
        return group_check(w, g2, w->outA.as<uint32_t>(), w->outB.as<uint32_t>(), ngroups, w->key_cur, w->pass.as<uint8_t>(),
                           st, w->key_cur + 48);
      }));
    }
    HIP_TRY(dh::launch_mark_groups(w->entries.as<uint32_t>(), m, gsize, w->pass.as<uint8_t>(), w->status.as<uint8_t>(),
                                   d_verdict, st));
    // failing groups' entries compacted on the device; only the failing-group count and the last group's flag
    // come back to the host (they size the next level)
    HIP_TRY(w->cflags.ensure(ngroups * 4));
    HIP_TRY(w->crank.ensure((ngroups + 1) * 4));
    HIP_TRY(w->cscan.ensure(((ngroups + 4095) / 4096 + 1) * 4));
    HIP_TRY(w->entries_alt.ensure(m * 4));
    HIP_TRY(dh::launch_compact_failing(w->entries.as<uint32_t>(), m, gsize, ngroups, w->pass.as<uint8_t>(),
                                       w->cflags.as<uint32_t>(), w->crank.as<uint32_t>(), w->cscan.as<uint32_t>(),
                                       w->entries_alt.as<uint32_t>(), st));
    uint32_t nfail32 = 0;
    uint8_t last_pass = 1;
    HIP_TRY(hipMemcpyAsync(&nfail32, w->crank.as<uint32_t>() + ngroups, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(&last_pass, w->pass.as<uint8_t>() + ngroups - 1, 1, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    level++;
    const size_t nfail = nfail32;
    if (stats) stats[1] += nfail;
    if (level == 1 && nfail == 0) w->fault_density = 0;  // a clean batch clears the density hint
    if (level == 2) {  // the first bisection level's failure rate: the density hint of the worker's next batch
      const double f = (double)nfail / (double)ngroups;
      w->fault_density = (f >= 1.0 ? 5.0 : -std::log1p(-f)) / (double)gsize;
    }
    if (nfail == 0) {
      m = 0;
      break;
    }
    std::swap(w->entries, w->entries_alt);
    const size_t m_prev = m;
    m = nfail * gsize - (last_pass ? 0 : ngroups * gsize - m_prev);  // only the last group may be short
    gsize = fixed.empty() ? next_group_size(gsize, ngroups, nfail, m_prev, m, w->fault_density)
                          : (size_t)(level - 1 < (int)fixed.size() ? fixed[level - 1] : 1);
  }
  if (m > 0) {
    HIP_TRY(T.run("k_leaf_check", [&] {
      return leaf_check(w, g2, w->entries.as<uint32_t>(), m, w->sig_aff.as<uint32_t>(), w->q_pts.as<uint32_t>(),
                        w->key_cur, w->status.as<uint8_t>(), d_verdict, st, w->key_cur + 48);
    }));
    if (stats) stats[2] = m;
  }
  if (stats) {  // rejected = decode/subgroup failures + failed leaves (1 MB D2H per 1M rounds, only when asked)
    w->h_verdict.resize(n);
    HIP_TRY(hipMemcpyAsync(w->h_verdict.data(), d_verdict, n, hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(hipStreamSynchronize(st));
  if (stats) {
    stats[0] = (uint64_t)level;
    size_t ok = 0;
    for (uint8_t v : w->h_verdict) ok += v ? 1 : 0;
    stats[3] = n - ok;
  }
  return DH_OK;
}

// ---- small batches: the one-beacon calls of the drop-in (VerifyBeacon from the gossip validator and the client,
// VerifyRecovered from the aggregator) and any batch of at most small_batch_max() rounds. No scalars, sort or MSM: the
// signature kernels (decode, subgroup test, randomness) on the worker's stream and the hash kernels on its tail stream
// run side by side, then every round gets its own 2-pairing check (the leaves of the batch path: bit-exact per-round
// verdicts by construction). A round's check is one wave per round, so up to a few hundred rounds cost what one does;
// larger batches amortise one group check over an MSM instead (verify_core). DRANDHIP_SMALL_N overrides (0: off).
static size_t small_batch_max() {
  static const size_t v = [] {
    const char* e = getenv("DRANDHIP_SMALL_N");
    return e ? (size_t)atol(e) : (size_t)64;
  }();
  return v;
}

// Queues the whole check on st (and the worker's tail stream); the caller reads the outputs after a stream sync.
// Lengths d_prev_lens the host has not checked (lens_checked): the hash kernels stay on st, behind the signature
// kernels, because a chained record longer than its slot marks its round in status (launch_hash).
int verify_small(worker* w, int scheme, const uint8_t* pk, size_t pk_len, const uint64_t* d_rounds, const uint8_t* d_sigs,
                 size_t sig_stride, const uint8_t* d_prevs, size_t prev_stride, const uint32_t* d_prev_lens, size_t n,
                 uint8_t* d_verdict, uint8_t* d_rand, const uint8_t* d_msgs32, hipStream_t st, bool lens_checked) {
  const bool g2 = sig_on_g2(scheme);
  const int sig_len = g2 ? 96 : 48, key_len = g2 ? 48 : 96;
  if ((int)pk_len != key_len) return fail(DH_EINVAL, "public key must be %d bytes for scheme %d", key_len, scheme);
  if (sig_stride < (size_t)sig_len || sig_stride % 4) return fail(DH_EINVAL, "bad signature stride %zu", sig_stride);
  if (n == 0) return DH_OK;
  int rc = ensure_key(w, g2, pk, pk_len, st);
  if (rc) return rc;
  const size_t jw = g2 ? JAC_WORDS_G2 : JAC_WORDS_G1;
  const size_t aw = jw * 2 / 3;
  HIP_TRY(w->status.ensure(n));
  HIP_TRY(w->sig_aff.ensure(n * aw * 4));
  HIP_TRY(w->q_pts.ensure(n * jw * 4));
  HIP_TRY(w->entries.ensure(n * 4));
  HIP_TRY(w->h2c_tmp.ensure(dh::hash_small_tmp_bytes(g2, n)));
  const bool chained = scheme == DH_SCHEME_CHAINED && d_prevs && !d_msgs32;
  const bool fork = w->tail && !(chained && d_prev_lens && !lens_checked);
  HIP_TRY(w->sub_bad.ensure(n));
  // Two streams: A = st decodes the signatures, then runs their subgroup tests; B = the tail stream hashes the
  // messages, waits for the decode, runs the per-round pairing checks beside the subgroup tests, then ANDs their
  // result into the verdicts; st joins B. Unforked (unchecked lengths): all of it on st, the hash after the decode.
  hipStream_t hs = fork ? w->tail : st;
  if (fork) {
    HIP_TRY(hipEventRecord(w->handoff, st));
    HIP_TRY(hipStreamWaitEvent(hs, w->handoff, 0));
  }
  timed_launches T(st), TH(hs);
  HIP_TRY(T.run(g2 ? "k_dec_sig_small<fp2>" : "k_dec_sig_small<fp>", [&] {
    return dh::launch_dec_sig(g2, d_sigs, sig_stride, n, w->status.as<uint8_t>(), w->sig_aff.as<uint32_t>(), d_rand, st);
  }));
  if (fork) HIP_TRY(hipEventRecord(w->ev_dec, st));
  HIP_TRY(TH.run(d_msgs32 ? (g2 ? "k_prep_msg32<fp2>" : "k_prep_msg32<fp>") : (g2 ? "k_prep_msg<fp2>" : "k_prep_msg<fp>"), [&] {
    return dh::launch_hash_small(g2, d_rounds, d_prevs, prev_stride, d_prev_lens, d_msgs32, n, chained ? 1 : 0, dst_id(scheme),
                                 fork ? nullptr : w->status.as<uint8_t>(), w->q_pts.as<uint32_t>(), w->h2c_tmp.as<uint32_t>(), hs);
  }));
  HIP_TRY(T.run(g2 ? "k_sub_sig_small<fp2>" : "k_sub_sig_small<fp>", [&] {
    return dh::launch_sub_flag(g2, n, w->status.as<uint8_t>(), w->sig_aff.as<uint32_t>(), w->sub_bad.as<uint8_t>(), st);
  }));
  if (fork) {
    HIP_TRY(hipEventRecord(w->ev_sub, st));
    HIP_TRY(hipStreamWaitEvent(hs, w->ev_dec, 0));
  }
  HIP_TRY(dh::launch_iota(w->entries.as<uint32_t>(), n, hs));
  HIP_TRY(TH.run("k_leaf_check", [&] {
    return leaf_check(w, g2, w->entries.as<uint32_t>(), n, w->sig_aff.as<uint32_t>(), w->q_pts.as<uint32_t>(),
                      w->key_cur, w->status.as<uint8_t>(), d_verdict, hs, w->key_cur + 48);
  }));
  if (fork) HIP_TRY(hipStreamWaitEvent(hs, w->ev_sub, 0));
  HIP_TRY(dh::launch_and_subgroup(n, w->sub_bad.as<uint8_t>(), d_verdict, hs));
  if (fork) {
    HIP_TRY(hipEventRecord(w->join, hs));
    HIP_TRY(hipStreamWaitEvent(st, w->join, 0));
  }
  return DH_OK;
}

// host-side staging of a small batch: the arrays packed into the worker's pinned buffer, one copy each way
struct stage_part {
  const void* src;
  size_t bytes;
  size_t slack = 0;  // zeroed bytes after the part (the digest kernel's word loads past the last chained record)
  size_t off = 0;
};
static int stage_in(worker* w, stage_part* parts, int k, size_t out_bytes, hipStream_t st, uint8_t** d_base, size_t* out_off) {
  size_t tot = 0;
  for (int i = 0; i < k; i++) {
    parts[i].off = tot;
    tot += (parts[i].bytes + parts[i].slack + 15) & ~(size_t)15;
  }
  *out_off = tot;
  const size_t need = tot + out_bytes;
  if (need > w->h_stage_cap) {
    if (w->h_stage) (void)hipHostFree(w->h_stage);
    w->h_stage = nullptr;
    w->h_stage_cap = 0;
    const size_t cap = std::max(need, (size_t)65536);
    HIP_TRY(hipHostMalloc(&w->h_stage, cap, hipHostMallocDefault));
    w->h_stage_cap = cap;
  }
  HIP_TRY(w->d_stage.ensure(need));
  uint8_t* h = (uint8_t*)w->h_stage;
  for (int i = 0; i < k; i++)
    if (parts[i].src && parts[i].bytes) {
      memcpy(h + parts[i].off, parts[i].src, parts[i].bytes);
      memset(h + parts[i].off + parts[i].bytes, 0, parts[i].slack);
    }
  if (tot) HIP_TRY(hipMemcpyAsync(w->d_stage.p, h, tot, hipMemcpyHostToDevice, st));
  *d_base = w->d_stage.as<uint8_t>();
  return DH_OK;
}

// the small-batch path behind the host-memory entry points (dh_verify_batch, dh_verify_recovered_batch): chained
// lengths were checked by the caller (dh_verify_batch)
static int verify_small_host(int scheme, const uint8_t* pk, size_t pk_len, const uint64_t* rounds, const uint8_t* sigs,
                             size_t sig_stride, const uint8_t* prevs, size_t prev_stride, const uint32_t* prev_lens,
                             const uint8_t* msgs32, size_t n, uint8_t* verdict_out, uint8_t* rand_out) {
  lease L;
  if (L.rc) return L.rc;
  worker* w = L.w;
  int rc = set_device_and_stream(w);
  if (rc) return rc;
  hipStream_t st = w->stream;
  stage_part parts[5] = {{rounds, rounds ? n * 8 : 0},
                         {sigs, n * sig_stride},
                         {prevs, prevs ? n * prev_stride : 0, 4},
                         {prev_lens, prevs && prev_lens ? n * 4 : 0},
                         {msgs32, msgs32 ? n * 32 : 0}};
  const size_t vbytes = (n + 15) & ~(size_t)15;
  uint8_t* d = nullptr;
  size_t out_off = 0;
  rc = stage_in(w, parts, 5, vbytes + (rand_out ? n * 32 : 0), st, &d, &out_off);
  if (rc) return rc;
  uint8_t* d_verdict = d + out_off;
  uint8_t* d_rand = rand_out ? d + out_off + vbytes : nullptr;
  rc = verify_small(w, scheme, pk, pk_len, rounds ? (const uint64_t*)(d + parts[0].off) : nullptr, d + parts[1].off, sig_stride,
                    prevs ? d + parts[2].off : nullptr, prev_stride, prevs && prev_lens ? (const uint32_t*)(d + parts[3].off) : nullptr,
                    n, d_verdict, d_rand, msgs32 ? d + parts[4].off : nullptr, st, true);
  if (rc) {
    (void)hipStreamSynchronize(st);
    if (w->tail) (void)hipStreamSynchronize(w->tail);
    return rc;
  }
  uint8_t* h_out = (uint8_t*)w->h_stage + out_off;
  HIP_TRY(hipMemcpyAsync(h_out, d_verdict, vbytes + (rand_out ? n * 32 : 0), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  memcpy(verdict_out, h_out, n);
  if (rand_out) memcpy(rand_out, h_out + vbytes, n * 32);
  return DH_OK;
}

int recover_core(worker* w, int scheme, const uint8_t* commits, int t, int n_nodes, const uint8_t* msgs32,
                 const uint8_t* partials, const uint32_t* part_off, size_t n_rounds, uint8_t* sig_out, uint8_t* status_out,
                 hipStream_t st, uint8_t* partial_ok_out = nullptr) {
  const bool g2 = sig_on_g2(scheme);
  const int sl = g2 ? 96 : 48, kl = g2 ? 48 : 96;
  const size_t jw = g2 ? JAC_WORDS_G2 : JAC_WORDS_G1, aw = jw * 2 / 3;
  const size_t kjw = g2 ? JAC_WORDS_G1 : JAC_WORDS_G2, kaw = kjw * 2 / 3;
  const size_t np = part_off[n_rounds] - part_off[0];
  const uint32_t base = part_off[0];
  memset(status_out, 0, n_rounds);
  if (n_rounds == 0) return DH_OK;
  timed_launches T(st);
  // 1./2. commits -> affine key-group points (all must decode) -> the public shares PubPoly.Eval(i), i < n_nodes.
  // Cached per worker under (scheme, t, n_nodes, commits): a node recovers every round against one group's
  // polynomial, and the evaluation is a ~6 ms latency-bound kernel (one lane per signer, 33-term Horner).
  std::vector<uint8_t> pub_key(9 + (size_t)t * kl);
  pub_key[0] = (uint8_t)scheme;
  memcpy(&pub_key[1], &t, 4);
  memcpy(&pub_key[5], &n_nodes, 4);
  memcpy(&pub_key[9], commits, (size_t)t * kl);
  const bool pub_hit = w->r_pub_key == pub_key;
  std::vector<uint8_t> cst(t, 1);
  if (!pub_hit) {
    w->r_pub_key.clear();
    HIP_TRY(w->r_commits.ensure((size_t)t * kl));
    HIP_TRY(w->r_cstatus.ensure(t));
    HIP_TRY(w->r_caff.ensure((size_t)t * kaw * 4));
    HIP_TRY(hipMemcpyAsync(w->r_commits.p, commits, (size_t)t * kl, hipMemcpyHostToDevice, st));
    HIP_TRY(dh::launch_prep(g2 ? 0 : 1, w->r_commits.as<uint8_t>(), kl, t, w->r_cstatus.as<uint8_t>(),
                            w->r_caff.as<uint32_t>(), nullptr, st));
    HIP_TRY(hipMemcpyAsync(cst.data(), w->r_cstatus.p, t, hipMemcpyDeviceToHost, st));
    HIP_TRY(w->r_shares.ensure((size_t)n_nodes * kjw * 4));
    HIP_TRY(T.run("k_pubpoly_eval", [&] {
      return dh::launch_pubpoly_eval(g2 ? 0 : 1, w->r_caff.as<uint32_t>(), t, n_nodes, w->r_shares.as<uint32_t>(), st);
    }));
  }
  // 3./4. partials: repack, decode + subgroup check
  HIP_TRY(w->r_raw.ensure(np * (2 + sl) + 4));
  HIP_TRY(w->r_psigs.ensure(np * sl + 4));
  HIP_TRY(w->r_pidx.ensure(np * 4 + 4));
  HIP_TRY(w->r_pstatus.ensure(np + 4));
  HIP_TRY(w->r_paff.ensure(np * aw * 4 + 16));
  // The partial records (98 B each for G2: 323 MB at 3.3M partials) come from pageable host memory. They cross in
  // chunks on the worker's tail stream, each chunk's repack + decode queued behind its copy on st, so the copy of
  // chunk c + 1 overlaps the decoding of chunk c instead of preceding all of it.
  const size_t pchunk = (w->tail && st == w->stream && np > ((size_t)1 << 19)) ? ((size_t)1 << 19) : np;
  for (size_t c0 = 0; c0 < np; c0 += pchunk) {
    const size_t cn = std::min(pchunk, np - c0);
    hipStream_t cs = pchunk < np ? w->tail : st;
    HIP_TRY(hipMemcpyAsync(w->r_raw.as<uint8_t>() + c0 * (2 + sl), partials + (size_t)(base + c0) * (2 + sl), cn * (2 + sl),
                           hipMemcpyHostToDevice, cs));
    if (cs != st) {
      HIP_TRY(hipEventRecord(w->handoff, cs));
      HIP_TRY(hipStreamWaitEvent(st, w->handoff, 0));
    }
    HIP_TRY(dh::launch_repack_partials(w->r_raw.as<uint8_t>() + c0 * (2 + sl), cn, sl, w->r_psigs.as<uint8_t>() + c0 * sl,
                                       w->r_pidx.as<uint32_t>() + c0, st));
    HIP_TRY(T.run(g2 ? "k_prep_sig<fp2>(partials)" : "k_prep_sig<fp>(partials)", [&] {
      return dh::launch_prep(g2, w->r_psigs.as<uint8_t>() + c0 * sl, sl, cn, w->r_pstatus.as<uint8_t>() + c0,
                             w->r_paff.as<uint32_t>() + c0 * aw, nullptr, st);
    }));
  }
  // 5. hash points of the round messages
  HIP_TRY(w->r_msgs.ensure(n_rounds * 32));
  HIP_TRY(w->r_q.ensure(n_rounds * jw * 4));
  HIP_TRY(hipMemcpyAsync(w->r_msgs.p, msgs32, n_rounds * 32, hipMemcpyHostToDevice, st));
  HIP_TRY(w->h2c_tmp.ensure(dh::hash_tmp_bytes(g2, n_rounds)));
  HIP_TRY(T.run(g2 ? "k_prep_msg32<fp2>" : "k_prep_msg32<fp>", [&] {
    return dh::launch_hash(g2, nullptr, nullptr, 0, nullptr, w->r_msgs.as<uint8_t>(), n_rounds, 0, dst_id(scheme), nullptr,
                           w->r_q.as<uint32_t>(), w->h2c_tmp.as<uint32_t>(), st);
  }));
  // 6. per-partial round and the group-membership rule, on the device (offsets relative to the first partial)
  std::vector<uint32_t> off_rel(n_rounds + 1);
  for (size_t j = 0; j <= n_rounds; j++) off_rel[j] = part_off[j] - base;
  HIP_TRY(w->r_off.ensure((n_rounds + 1) * 4));
  HIP_TRY(w->r_round_of.ensure(np * 4 + 4));
  HIP_TRY(hipMemcpyAsync(w->r_off.p, off_rel.data(), (n_rounds + 1) * 4, hipMemcpyHostToDevice, st));
  HIP_TRY(dh::launch_partial_meta(w->r_off.as<uint32_t>(), n_rounds, w->r_pidx.as<uint32_t>(), n_nodes,
                                  w->r_round_of.as<uint32_t>(), w->r_pstatus.as<uint8_t>(), st));
  // 7. RLC scalars per partial (0 for partials that failed decoding or lie outside the group), split as the 28-bit MSM
  // takes them: four 31-bit psi parts (G2 signatures) or two 63-bit phi halves (G1)
  const int parts = g2 ? 4 : 2;
  const size_t pw28 = g2 ? 64 : 32, wsw = g2 ? 96 : 48;  // words per 28-bit affine point / workspace Jacobian point
  uint32_t seedw[8];
  int rc = make_seed(0, seedw);
  if (rc) return rc;
  HIP_TRY(w->key_ok.ensure(64));
  uint32_t* d_seed = (uint32_t*)((uint8_t*)w->key_ok.p + 32);
  HIP_TRY(hipMemcpyAsync(d_seed, seedw, 32, hipMemcpyHostToDevice, st));
  HIP_TRY(w->r_scal.ensure(std::max(np, n_rounds) * 16 + 16));
  HIP_TRY(dh::launch_scalars(d_seed, np, w->r_pstatus.as<uint8_t>(), w->r_scal.as<uint4>(), parts, st));
  HIP_TRY(hipStreamSynchronize(st));
  for (int c = 0; c < t; c++)
    if (cst[c] != 1) return fail(DH_EKEY, "public polynomial commitment %d does not decode to a subgroup point", c);
  if (!pub_hit) w->r_pub_key = pub_key;  // r_caff / r_shares hold this polynomial until a call with another one
  // 8./9. MSMs: A = sum r sigma (one group), B_i = sum r Q_round per signer i: entry e -> point round_of[e], scalar e,
  // group min(share, n-1) (the sort keys by (group, window, digit), so the entries need no order; a zero scalar
  // contributes nothing)
  HIP_TRY(w->r_ok.ensure(np + 4));
  bool batch_ok = false;
  {
    HIP_TRY(w->entries.ensure(np * 4 + 4));
    HIP_TRY(dh::launch_iota(w->entries.as<uint32_t>(), np, st));
    HIP_TRY(w->r_e_grp.ensure(np * 4 + 4));
    HIP_TRY(dh::launch_clamp_group(w->r_pidx.as<uint32_t>(), np, (uint32_t)n_nodes - 1, w->r_e_grp.as<uint32_t>(), st));
    // the partials' sigmas and the rounds' hash points in the 28-bit form with their endomorphism images (a hash point
    // at infinity, probability ~2^-255, leaves its round's slot unwritten: the batch check then fails and the partials
    // get their leaf checks on the 32-bit points)
    HIP_TRY(w->s28.ensure(parts * std::max<size_t>(np, 1) * pw28 * 4));
    HIP_TRY(w->q28.ensure(parts * n_rounds * pw28 * 4));
    HIP_TRY(w->r_rstat.ensure(n_rounds));
    HIP_TRY(hipMemsetAsync(w->r_rstat.p, 1 /* DEC_OK */, n_rounds, st));
    HIP_TRY(dh::launch_msm_prep28(g2, np, w->r_pstatus.as<uint8_t>(), w->r_paff.as<uint32_t>(), nullptr, w->s28.as<uint32_t>(),
                                  nullptr, st, 1));
    HIP_TRY(dh::launch_msm_prep28(g2, n_rounds, w->r_rstat.as<uint8_t>(), nullptr, w->r_q.as<uint32_t>(), nullptr,
                                  w->q28.as<uint32_t>(), st, 2));
    dh::msm_geom gA = geom_for(std::max<size_t>(np, 1), parts);
    gA.half_stride = (uint32_t)np;
    // window geometry of the per-signer groups from the partials per signer that answered, the signers counted over
    // the first 65,536 records (np / n_nodes undercounted a group when the same t signers answer every round, and picked
    // 3 windows of c = 15 where 2 of c = 16 do a third fewer bucket additions: 43.1 -> 38.7 ms at n = 64, t = 33; with
    // every signer answering, np / t overcounted and c = 16 was slower, 39.4 -> 52.0 ms, profiles/r04/config_recover_*_r04p)
    size_t active = 0;
    {
      std::vector<uint8_t> seen((size_t)n_nodes, 0);
      const size_t ns = std::min<size_t>(np, 65536);
      for (size_t e = 0; e < ns; e++) {
        const uint8_t* r = partials + (size_t)(base + e) * (2 + sl);
        const size_t i = ((size_t)r[0] << 8) | r[1];
        if (i < (size_t)n_nodes && !seen[i]) {
          seen[i] = 1;
          active++;
        }
      }
    }
    size_t avg = std::max<size_t>(1, np / std::max<size_t>(1, active));
    dh::msm_geom gB = geom_for(avg, parts);
    while (gB.c > 3 && (size_t)n_nodes * gB.nwin * gB.nbuck > ((size_t)1 << 24))
      gB = geom_for(std::max<size_t>(1, ((size_t)1 << (gB.c + 1)) / parts), parts);
    gB.half_stride = (uint32_t)n_rounds;
    // one workspace for both (sized for each before anything is queued on it), used one MSM after the other
    dh::msm_ws wsA{}, wsB{};
    int rcw = msm_workspace(w, gA, np, 1, wsw, wsA);
    if (!rcw) rcw = msm_workspace(w, gB, np, n_nodes, wsw, wsB);
    if (!rcw) rcw = msm_workspace(w, gA, np, 1, wsw, wsA);
    if (rcw) return rcw;
    HIP_TRY(w->outA.ensure(jw * 4));
    HIP_TRY(w->outB.ensure((size_t)n_nodes * jw * 4));
    HIP_TRY(T.run("recover_msm_sigs", [&] {
      return dh::launch_msm28_set(g2, gA, w->entries.as<uint32_t>(), nullptr, nullptr, np, 1, w->r_scal.as<uint4>(),
                                  w->s28.as<uint32_t>(), wsA, w->outA.as<uint32_t>(), st);
    }));
    HIP_TRY(T.run("recover_msm_hash_by_signer", [&] {
      return dh::launch_msm28_set(g2, gB, w->r_round_of.as<uint32_t>(), w->entries.as<uint32_t>(), w->r_e_grp.as<uint32_t>(),
                                  np, n_nodes, w->r_scal.as<uint4>(), w->q28.as<uint32_t>(), wsB, w->outB.as<uint32_t>(), st);
    }));
    // 10. multi-pairing: n_nodes + 1 pairs
    const size_t npairs = (size_t)n_nodes + 1;
    HIP_TRY(w->r_P.ensure(npairs * JAC_WORDS_G1 * 4));
    HIP_TRY(w->r_Q.ensure(npairs * JAC_WORDS_G2 * 4));
    HIP_TRY(w->r_f.ensure(npairs * 192 * 4));  // k_vm.hip F12_WORDS (the one-lane path uses 144)
    HIP_TRY(w->r_skip.ensure(npairs + 4));
    HIP_TRY(w->pass.ensure(16));
    HIP_TRY(T.run("recover_pair_check", [&] {
      hipError_t e = dh::launch_recover_pairs(g2, w->r_shares.as<uint32_t>(), w->outB.as<uint32_t>(), w->outA.as<uint32_t>(),
                                              n_nodes, w->r_P.as<uint32_t>(), w->r_Q.as<uint32_t>(), st);
      if (e != hipSuccess) return e;
      if (lane_pairing())
        return dh::launch_pair_check(w->r_P.as<uint32_t>(), w->r_Q.as<uint32_t>(), npairs, 0, 0, nullptr,
                                     w->r_f.as<uint32_t>(), w->r_skip.as<uint8_t>(), w->pass.as<uint8_t>(), st);
      if ((e = w->vm_pairs.ensure(npairs * 72 * 4)) != hipSuccess) return e;
      if ((e = w->vm_live.ensure(npairs)) != hipSuccess) return e;
      return dh::launch_multi_pairing_vm(w->r_P.as<uint32_t>(), w->r_Q.as<uint32_t>(), npairs, w->vm_pairs.as<uint32_t>(),
                                         w->vm_live.as<uint8_t>(), w->r_f.as<uint32_t>(), w->pass.as<uint8_t>(), st);
    }));
    uint8_t pass = 0;
    HIP_TRY(hipMemcpyAsync(&pass, w->pass.p, 1, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    batch_ok = pass == 1;
  }
  // 11. per-partial validity, on the device
  if (batch_ok) {
    HIP_TRY(dh::launch_ok_from_status(w->r_pstatus.as<uint8_t>(), np, w->r_ok.as<uint8_t>(), st));
  } else {
    HIP_TRY(T.run("k_partial_leaf", [&] {
      return dh::launch_partial_leaf(g2, w->entries.as<uint32_t>(), np, w->r_paff.as<uint32_t>(), w->r_pstatus.as<uint8_t>(),
                                     w->r_pidx.as<uint32_t>(), w->r_round_of.as<uint32_t>(), w->r_q.as<uint32_t>(),
                                     w->r_shares.as<uint32_t>(), n_nodes, w->r_ok.as<uint8_t>(), st);
    }));
  }
  if (partial_ok_out) {  // dh_verify_partials_batch: per-partial VerifyPartial verdicts only
    HIP_TRY(hipMemcpyAsync(partial_ok_out, w->r_ok.p, np, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return DH_OK;
  }
  // 12. selection (first t valid in the given order; sorted by index; duplicates dropped) + Lagrange coefficients,
  // one lane per round
  HIP_TRY(w->r_sel.ensure(n_rounds * (size_t)t * 4));
  HIP_TRY(w->r_key.ensure(n_rounds * (size_t)t * 4));
  HIP_TRY(w->r_den.ensure(n_rounds * (size_t)t * 32));
  HIP_TRY(w->r_lam.ensure(n_rounds * (size_t)t * dh::lam_words() * 4));
  HIP_TRY(w->r_rok.ensure(n_rounds));
  HIP_TRY(w->r_lamset.ensure(n_rounds * 4));
  HIP_TRY(w->r_own.ensure(4));
  HIP_TRY(w->r_sig.ensure(n_rounds * jw * 4));
  HIP_TRY(T.run("k_select_lagrange", [&] {
    return dh::launch_select_lagrange(w->r_off.as<uint32_t>(), w->r_ok.as<uint8_t>(), w->r_pidx.as<uint32_t>(), t, n_rounds,
                                      w->r_sel.as<uint32_t>(), w->r_key.as<uint32_t>(), w->r_den.as<uint32_t>(),
                                      w->r_lam.as<uint32_t>(), w->r_lamset.as<uint32_t>(), w->r_rok.as<uint8_t>(),
                                      w->r_own.as<uint32_t>(), g2 ? 0 : 1, st);
  }));
  // tables of 8 odd multiples when some round has a Lagrange basis of its own (its wave then runs the regular windows
  // in k_lagrange), else of 4 for the width-4 NAF: one word back from the device. k_lagrange depends on this: k_lambda
  // writes width-4 NAF nibbles for round 0's basis only, so entries == 4 is valid only when every round uses basis 0
  // (own == 0); k_lagrange leaves a wave at infinity (not recovered) if that ever fails to hold
  int entries = 4;
  if (g2) {
    uint32_t own = 0;
    HIP_TRY(hipMemcpyAsync(&own, w->r_own.p, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (own) entries = 8;
  }
  // 13. interpolation on the device
  if (g2) {  // the selected partials' points in the 28-bit form and their tables of odd multiples, once per partial
    HIP_TRY(w->r_zs.ensure(dh::wnaf_table_scratch_bytes(np, entries) + 256));
    HIP_TRY(w->r_tbl.ensure(np * (size_t)entries * 64 * 4 + 1024));
    HIP_TRY(w->r_need.ensure(np + 4));
    HIP_TRY(dh::launch_mark_selected(w->r_sel.as<uint32_t>(), w->r_rok.as<uint8_t>(), t, n_rounds, np, w->r_need.as<uint8_t>(),
                                     st));
    HIP_TRY(T.run("k_wnaf_table", [&] {
      return dh::launch_wnaf_table_g2(w->r_paff.as<uint32_t>(), w->r_need.as<uint8_t>(), np, entries, w->r_tbl.as<uint32_t>(),
                                      w->r_zs.as<uint32_t>(), st);
    }));
  }
  HIP_TRY(w->r_ltmp.ensure(dh::lagrange_tmp_bytes(g2)));
  HIP_TRY(T.run("k_lagrange", [&] {
    return dh::launch_lagrange(g2, w->r_sel.as<uint32_t>(), w->r_lam.as<uint32_t>(), w->r_lamset.as<uint32_t>(),
                               w->r_rok.as<uint8_t>(), t,
                               n_rounds, w->r_paff.as<uint32_t>(), g2 ? w->r_tbl.as<uint32_t>() : nullptr, entries,
                               w->r_sig.as<uint32_t>(), w->r_ltmp.as<uint32_t>(), st);
  }));
  std::vector<uint8_t> rok(n_rounds, 0);
  HIP_TRY(hipMemcpyAsync(rok.data(), w->r_rok.p, n_rounds, hipMemcpyDeviceToHost, st));
  // 14./15. compress, then VerifyRecovered (chainstore.go:207) as one batch against the group key (commit 0)
  HIP_TRY(w->r_sigbytes.ensure(n_rounds * sl));
  HIP_TRY(w->r_status2.ensure(n_rounds));
  HIP_TRY(w->r_aff2.ensure(n_rounds * aw * 4));
  // the compression also leaves the affine points and decode statuses the VerifyRecovered batch takes (decoding the
  // bytes again — an Fp(2) square root and a subgroup test per round — would return the same points)
  HIP_TRY(dh::launch_compress(g2, w->r_sig.as<uint32_t>(), n_rounds, w->r_sigbytes.as<uint8_t>(), w->r_aff2.as<uint32_t>(),
                              w->r_status2.as<uint8_t>(), st));
  HIP_TRY(hipMemcpyAsync(sig_out, w->r_sigbytes.p, n_rounds * sl, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  // verify through the regular batch path (messages are given digests: use the per-round hash points)
  std::vector<uint8_t> vv(n_rounds, 0);
  {
    HIP_TRY(w->r_entries2.ensure(n_rounds * 4));
    HIP_TRY(w->r_scal.ensure(std::max(np, n_rounds) * 16 + 16));  // rounds may outnumber the partials
    HIP_TRY(dh::launch_scalars(d_seed, n_rounds, w->r_status2.as<uint8_t>(), w->r_scal.as<uint4>(), parts, st));
    HIP_TRY(dh::launch_iota(w->r_entries2.as<uint32_t>(), n_rounds, st));
    // group key = commit 0 (affine, key group) — staged where the group check expects it
    HIP_TRY(w->key_aff.ensure(96 * 4));
    HIP_TRY(hipMemcpyAsync(w->key_aff.p, w->r_caff.p, kaw * 4, hipMemcpyDeviceToDevice, st));
    dh::msm_geom g = geom_for(n_rounds, parts);
    g.half_stride = (uint32_t)n_rounds;
    dh::msm_ws ws{};
    int rcw = msm_workspace(w, g, n_rounds, 1, wsw, ws);
    if (rcw) return rcw;
    HIP_TRY(w->s28.ensure(parts * n_rounds * pw28 * 4));
    HIP_TRY(w->q28.ensure(parts * n_rounds * pw28 * 4));
    HIP_TRY(dh::launch_msm_prep28(g2, n_rounds, w->r_status2.as<uint8_t>(), w->r_aff2.as<uint32_t>(), w->r_q.as<uint32_t>(),
                                  w->s28.as<uint32_t>(), w->q28.as<uint32_t>(), st));
    HIP_TRY(T.run("recover_verify", [&] {
      hipError_t e = dh::launch_msm28(g2, g, w->r_entries2.as<uint32_t>(), n_rounds, 1, w->r_scal.as<uint4>(),
                                      w->s28.as<uint32_t>(), w->q28.as<uint32_t>(), ws, w->outA.as<uint32_t>(),
                                      w->outB.as<uint32_t>(), st, w->r_status2.as<uint8_t>(), false);
      if (e != hipSuccess) return e;
      return group_check(w, g2, w->outA.as<uint32_t>(), w->outB.as<uint32_t>(), 1, w->key_aff.as<uint32_t>(),
                         w->pass.as<uint8_t>(), st);
    }));
    uint8_t pass = 0, dummy = 0;
    (void)dummy;
    HIP_TRY(hipMemcpyAsync(&pass, w->pass.p, 1, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(w->r_ok.ensure(std::max(np, n_rounds) + 4));
    if (pass == 1) {
      HIP_TRY(hipMemcpyAsync(vv.data(), w->r_status2.p, n_rounds, hipMemcpyDeviceToHost, st));
    } else {
      HIP_TRY(hipMemsetAsync(w->r_ok.p, 0, n_rounds, st));
      HIP_TRY(leaf_check(w, g2, w->r_entries2.as<uint32_t>(), n_rounds, w->r_aff2.as<uint32_t>(), w->r_q.as<uint32_t>(),
                         w->key_aff.as<uint32_t>(), w->r_status2.as<uint8_t>(), w->r_ok.as<uint8_t>(), st));
      HIP_TRY(hipMemcpyAsync(vv.data(), w->r_ok.p, n_rounds, hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
  }
  for (size_t j = 0; j < n_rounds; j++) status_out[j] = (rok[j] && vv[j] == 1) ? 1 : 0;
  return DH_OK;
}

// ---- one call over several internal streams (the drop-in callers make ONE call per window)
// Off by default: measured on the MI355X (profiles/split_sweep_r02k_*.jsonl), one stream per call is the fastest
// form of a call (1M rounds 64.9 ms, 4M 225.8 ms = 92% of the 8-batches-in-flight rate) — a chunk's per-round
// kernels alone on the chip are no faster than one large launch, and the chunks' latency-bound tails, made of
// many small kernels, wait for wave slots the per-round kernels hold and slow them. When enabled
// (DRANDHIP_SPLIT="chunk,workers" or dh_set_split), a batch is cut into chunks, each a complete batch check (its own
// RLC scalars: seed + chunk index when the caller fixed a seed, fresh CSPRNG seeds otherwise, so verdicts stay
// bit-exact per round), verified by up to `workers` leased workers; the chunks' per-round kernels are chained in
// chunk order across the workers' streams (prep_gate) and each chunk's tail runs on its worker's high-priority
// stream. Streams share the process's hardware queues (GPU_MAX_HW_QUEUES, 4 by default per priority).
struct split_cfg {
  size_t chunk = 0;  // 0: one stream per call
  int workers = 3;
};
std::mutex g_split_mu;
split_cfg g_split = [] {
  split_cfg r;
  const char* e = getenv("DRANDHIP_SPLIT");
  if (e && *e) {
    char* end = nullptr;
    r.chunk = strtoull(e, &end, 10);
    if (end && *end == ',') r.workers = std::max(1, atoi(end + 1));
  }
  return r;
}();
static split_cfg split_config() {
  std::lock_guard<std::mutex> lk(g_split_mu);
  return g_split;
}

int ensure_device() {
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  int rc = ensure_init_locked(0);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(g_ctx.device));
  return DH_OK;
}

template <class F>
int run_split(size_t n, F&& fn, uint64_t seed) {
  const split_cfg cfg = split_config();
  size_t nchunks = 1;
  if (cfg.chunk && cfg.workers > 1 && n >= 2 * cfg.chunk) nchunks = (n + cfg.chunk - 1) / cfg.chunk;
  const size_t per = (n + nchunks - 1) / std::max<size_t>(nchunks, 1);
  const int nthreads = (int)std::min<size_t>(nchunks, (size_t)cfg.workers);
  std::atomic<size_t> next{0};
  std::atomic<int> first_rc{DH_OK};
  std::mutex err_mu;
  std::string err;
  // prep chain: chunk c's per-round kernels queue behind chunk c-1's (event ev[c-1], recorded by its thread)
  std::vector<hipEvent_t> ev(nchunks > 1 ? nchunks : 0, nullptr);
  std::vector<char> rec(nchunks, 0);
  std::mutex gate_mu;
  std::condition_variable gate_cv;
  for (auto& e : ev) {
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      for (auto& x : ev)
        if (x) (void)hipEventDestroy(x);
      return fail(DH_EDEVICE, "hipEventCreate failed");
    }
  }
  auto mark = [&](size_t c) {
    std::lock_guard<std::mutex> lk(gate_mu);
    rec[c] = 1;
    gate_cv.notify_all();
  };
  auto body = [&]() {
    lease L;
    int rc = L.rc ? L.rc : set_device_and_stream(L.w);
    for (size_t c; !rc && (c = next.fetch_add(1)) < nchunks;) {
      const size_t lo = c * per, hi = std::min(n, lo + per);
      prep_gate g;
      prep_gate* gp = nullptr;
      if (nchunks > 1) {
        if (c > 0) {  // chunk c-1 is held by a running thread that never waits on a later chunk: no deadlock
          std::unique_lock<std::mutex> lk(gate_mu);
          gate_cv.wait(lk, [&] { return rec[c - 1] != 0; });
          g.wait = ev[c - 1];
        }
        g.done = ev[c];
        g.recorded = [&mark, c] { mark(c); };
        gp = &g;
      }
      if (lo < hi) rc = fn(L.w, lo, hi, seed ? seed + 0x9e3779b97f4a7c15ULL * c : 0, gp);
      if (nchunks > 1) mark(c);  // also on failure: the next chunk must not wait forever
    }
    if (rc) {
      int expect = DH_OK;
      if (first_rc.compare_exchange_strong(expect, rc)) {
        std::lock_guard<std::mutex> lk(err_mu);
        err = g_err;  // the message lives in this thread's g_err: hand it to the caller's
      }
      next.store(nchunks);  // stop the other workers early
    }
  };
  if (nthreads <= 1) {
    body();
  } else {
    std::vector<std::thread> ths;
    for (int t = 1; t < nthreads; t++) ths.emplace_back(body);
    body();
    for (auto& th : ths) th.join();
  }
  for (auto& e : ev) (void)hipEventDestroy(e);
  const int rc = first_rc.load();
  if (rc) g_err = err;
  return rc;
}

}  // namespace

extern "C" {

int dh_init(uint32_t device_mask) {
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  return ensure_init_locked(device_mask);
}

void dh_shutdown(void) {
  // idle workers are freed now; a worker leased by a call still running on another thread is retired and freed
  // when that call returns, so the call never touches freed memory
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  for (worker* w : g_ctx.pool) {
    if (w->busy) {
      g_ctx.retired.push_back(w);
      continue;
    }
    w->release_all();
    delete w;
  }
  g_ctx.pool.clear();
  g_ctx.inited = false;
}

int dh_scheme_from_name(const char* name) {
  if (!name) return fail(DH_EINVAL, "null scheme name");
  static const char* names[4] = {"pedersen-bls-chained", "pedersen-bls-unchained", "bls-unchained-on-g1",
                                 "bls-unchained-g1-rfc9380"};
  for (int i = 0; i < 4; i++)
    if (!strcmp(name, names[i])) return i;
  return fail(DH_EINVAL, "invalid scheme name '%s'", name);
}

int dh_sig_len(int scheme) {
  if (scheme < 0 || scheme > 3) return fail(DH_EINVAL, "unknown scheme %d", scheme);
  return sig_on_g2(scheme) ? 96 : 48;
}
int dh_key_len(int scheme) {
  if (scheme < 0 || scheme > 3) return fail(DH_EINVAL, "unknown scheme %d", scheme);
  return sig_on_g2(scheme) ? 48 : 96;
}

int dh_verify_batch_device(int scheme, const uint8_t* pk, size_t pk_len, const uint64_t* d_rounds, const uint8_t* d_sigs,
                           size_t sig_stride, const uint8_t* d_prevs, size_t prev_stride, const uint32_t* d_prev_lens,
                           size_t n, uint8_t* d_verdict_out, uint8_t* d_rand_out, uint64_t seed, void* hip_stream,
                           uint64_t stats_out[4]) {
  if (scheme < 0 || scheme > 3) return fail(DH_EINVAL, "unknown scheme %d", scheme);
  if (!pk || (n && (!d_rounds || !d_sigs || !d_verdict_out))) return fail(DH_EINVAL, "null argument");
  if (stats_out) memset(stats_out, 0, 4 * sizeof(uint64_t));
  if (n && n <= small_batch_max()) {  // the small-batch path: every round its own check (stats: 0 levels, n leaves)
    lease L;
    if (L.rc) return L.rc;
    worker* w = L.w;
    int rc = set_device_and_stream(w);
    if (rc) return rc;
    hipStream_t st = w->stream;
    if (hip_stream) {
      HIP_TRY(hipEventRecord(w->part_ready, (hipStream_t)hip_stream));
      HIP_TRY(hipStreamWaitEvent(st, w->part_ready, 0));
    }
    const bool chained = scheme == DH_SCHEME_CHAINED && d_prevs;
    rc = verify_small(w, scheme, pk, pk_len, d_rounds, d_sigs, sig_stride, chained ? d_prevs : nullptr, prev_stride,
                      chained ? d_prev_lens : nullptr, n, d_verdict_out, d_rand_out, nullptr, st, false);
    if (rc) {
      (void)hipStreamSynchronize(st);
      if (w->tail) (void)hipStreamSynchronize(w->tail);
      return rc;
    }
    if (stats_out) {
      w->h_verdict.resize(n);
      HIP_TRY(hipMemcpyAsync(w->h_verdict.data(), d_verdict_out, n, hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(hipStreamSynchronize(st));
    if (stats_out) {
      size_t ok = 0;
      for (size_t i = 0; i < n; i++) ok += w->h_verdict[i] ? 1 : 0;
      stats_out[2] = n;
      stats_out[3] = n - ok;
    }
    return DH_OK;
  }
  // inputs produced on the caller's stream: every internal stream waits for that stream's work first
  hipEvent_t ready = nullptr;
  if (hip_stream) {
    int rc0 = ensure_device();
    if (rc0) return rc0;
    HIP_TRY(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(ready, (hipStream_t)hip_stream));
  }
  std::mutex stats_mu;
  int rc = run_split(n, [&](worker* w, size_t lo, size_t hi, uint64_t chunk_seed, prep_gate* gate) -> int {
    if (ready) HIP_TRY(hipStreamWaitEvent(w->stream, ready, 0));
    uint64_t st4[4];
    const bool chained = scheme == DH_SCHEME_CHAINED && d_prevs;
    int r = verify_core(w, scheme, pk, pk_len, d_rounds + lo, d_sigs + lo * sig_stride, sig_stride,
                        chained ? d_prevs + lo * prev_stride : nullptr,
                        prev_stride, chained && d_prev_lens ? d_prev_lens + lo : nullptr, hi - lo, d_verdict_out + lo,
                        d_rand_out ? d_rand_out + lo * 32 : nullptr, chunk_seed, w->stream, stats_out ? st4 : nullptr,
                        nullptr, VM_FULL, gate);
    if (!r && stats_out) {
      std::lock_guard<std::mutex> lk(stats_mu);
      stats_out[0] = std::max(stats_out[0], st4[0]);
      for (int k = 1; k < 4; k++) stats_out[k] += st4[k];
    }
    return r;
  }, seed);
  if (ready) (void)hipEventDestroy(ready);
  return rc;
}

int dh_verify_batch(int scheme, const uint8_t* pk, size_t pk_len, const uint64_t* rounds, const uint8_t* sigs,
                    size_t sig_stride, const uint8_t* prevs, size_t prev_stride, const uint32_t* prev_lens, size_t n,
                    uint8_t* verdict_out, uint8_t* rand_out, uint64_t seed) {
  if (scheme < 0 || scheme > 3) return fail(DH_EINVAL, "unknown scheme %d", scheme);
  if (!pk || (n && (!rounds || !sigs || !verdict_out))) return fail(DH_EINVAL, "null argument");
  if (n == 0) return DH_OK;
  const bool chained = scheme == DH_SCHEME_CHAINED && prevs;
  if (chained && prev_lens)
    for (size_t i = 0; i < n; i++)
      if (prev_lens[i] > prev_stride)
        return fail(DH_EINVAL, "previous signature %zu: length %u exceeds the record stride %zu", i, prev_lens[i], prev_stride);
  if (n <= small_batch_max()) return verify_small_host(scheme, pk, pk_len, rounds, sigs, sig_stride, chained ? prevs : nullptr,
                                                       prev_stride, chained ? prev_lens : nullptr, nullptr, n, verdict_out,
                                                       rand_out);
  // one chunk per worker at a time: its host->device copies overlap the other chunks' kernels
  return run_split(n, [&](worker* w, size_t lo, size_t hi, uint64_t chunk_seed, prep_gate* gate) -> int {
    const size_t m = hi - lo;
    hipStream_t st = w->stream;
    HIP_TRY(w->in_rounds.ensure(m * 8));
    HIP_TRY(w->in_sigs.ensure(m * sig_stride));
    HIP_TRY(w->out_verdict.ensure(m));
    if (rand_out) HIP_TRY(w->out_rand.ensure(m * 32));
    HIP_TRY(hipMemcpyAsync(w->in_rounds.p, rounds + lo, m * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(w->in_sigs.p, sigs + lo * sig_stride, m * sig_stride, hipMemcpyHostToDevice, st));
    if (chained) {
      HIP_TRY(w->in_prevs.ensure(m * prev_stride + 4));
      HIP_TRY(hipMemcpyAsync(w->in_prevs.p, prevs + lo * prev_stride, m * prev_stride, hipMemcpyHostToDevice, st));
      if (prev_lens) {
        HIP_TRY(w->in_prev_lens.ensure(m * 4));
        HIP_TRY(hipMemcpyAsync(w->in_prev_lens.p, prev_lens + lo, m * 4, hipMemcpyHostToDevice, st));
      }
    }
    int rc = verify_core(w, scheme, pk, pk_len, w->in_rounds.as<uint64_t>(), w->in_sigs.as<uint8_t>(), sig_stride,
                         chained ? w->in_prevs.as<uint8_t>() : nullptr, prev_stride,
                         chained && prev_lens ? w->in_prev_lens.as<uint32_t>() : nullptr, m, w->out_verdict.as<uint8_t>(),
                         rand_out ? w->out_rand.as<uint8_t>() : nullptr, chunk_seed, st, nullptr, nullptr, VM_FULL, gate);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(verdict_out + lo, w->out_verdict.p, m, hipMemcpyDeviceToHost, st));
    if (rand_out) HIP_TRY(hipMemcpyAsync(rand_out + lo * 32, w->out_rand.p, m * 32, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return DH_OK;
  }, seed);
}

// ---- node-wide batch check over several processes (one per GPU)
// A node batch holds ONE worker from dh_batch_begin to dh_batch_finish and runs everything on it: the per-round
// kernels on its stream, the level-0 MSM, the record, the node-wide check of the gathered records and the bisection
// on its high-priority tail stream (dh_batch_stream), where the caller also queues the collective. Nothing in begin
// or check waits on the host, and with one rank nothing crosses streams at all.
struct dh_batch {
  lease* L = nullptr;
  int scheme = 0;
  std::vector<uint8_t> pk;
  const uint64_t* d_rounds = nullptr;
  const uint8_t* d_sigs = nullptr;
  size_t sig_stride = 0;
  const uint8_t* d_prevs = nullptr;
  size_t prev_stride = 0;
  const uint32_t* d_prev_lens = nullptr;
  size_t n = 0;
  uint8_t* d_verdict = nullptr;
  uint8_t* d_rand = nullptr;
  hipStream_t st = nullptr;
  bool checked = false;  // dh_batch_check queued: its result is in the worker's node_res[2]
};

// one record: A, B (Jacobian AoS) + a status word (0 = this rank's batch began; nonzero = abandoned) + 3 pad words
static size_t partial_words(bool g2) { return 2 * (g2 ? JAC_WORDS_G2 : JAC_WORDS_G1) + 4; }

int dh_partial_bytes(int scheme) {
  if (scheme < 0 || scheme > 3) return fail(DH_EINVAL, "unknown scheme %d", scheme);
  return (int)(partial_words(sig_on_g2(scheme)) * 4);
}

// A node batch queues its level-0 tail, record, exchange and check on the worker's normal stream behind its per-round
// kernels, with the level-0 sort there too, instead of handing the tail to the high-priority stream behind an event
// wait: 8 batches in flight, one GPU (gpurun_out r04y, one box): 1M rounds 25.75 -> 26.36 M/s (local check 26.48),
// 131k rounds 18.09 -> 21.42 M/s. A high-priority queue holding a batch's pending wait for the whole of its per-round
// kernels cost the other batches' dispatch (the local path's host wait before queueing its tail is the same fix).
// DRANDHIP_NODE_ONE_STREAM=0 restores the tail-stream handoff (comparison runs).
static bool node_one_stream() {
  static const bool v = [] {
    const char* e = getenv("DRANDHIP_NODE_ONE_STREAM");
    return !(e && e[0] == '0');
  }();
  return v;
}
static hipStream_t batch_stream(worker* w) { return node_one_stream() ? w->stream : w->tail; }

int dh_batch_begin(int scheme, const uint8_t* pk, size_t pk_len, const uint64_t* d_rounds, const uint8_t* d_sigs,
                   size_t sig_stride, const uint8_t* d_prevs, size_t prev_stride, const uint32_t* d_prev_lens, size_t n,
                   uint8_t* d_verdict_out, uint8_t* d_rand_out, uint64_t seed, void* hip_stream, dh_batch** batch_out,
                   uint8_t* d_partials_out) {
  if (!batch_out) return fail(DH_EINVAL, "null batch handle");
  *batch_out = nullptr;
  if (scheme < 0 || scheme > 3) return fail(DH_EINVAL, "unknown scheme %d", scheme);
  if (!pk || !d_partials_out || (n && (!d_rounds || !d_sigs || !d_verdict_out))) return fail(DH_EINVAL, "null argument");
  std::unique_ptr<dh_batch> b(new dh_batch());
  b->L = new lease(false);  // the lease spans the collective: fail (DH_EBUSY) rather than wait for a worker
  if (b->L->rc) {
    int rc = b->L->rc;
    delete b->L;
    return rc;
  }
  worker* w = b->L->w;
  int rc = set_device_and_stream(w, !node_one_stream());
  if (!rc && hip_stream) {  // inputs produced on the caller's stream
    if (hipEventRecord(w->part_ready, (hipStream_t)hip_stream) != hipSuccess ||
        hipStreamWaitEvent(w->stream, w->part_ready, 0) != hipSuccess)
      rc = fail(DH_EDEVICE, "cannot order the batch after the caller's stream");
  }
  b->scheme = scheme;
  b->pk.assign(pk, pk + pk_len);
  b->d_rounds = d_rounds;
  b->d_sigs = d_sigs;
  b->sig_stride = sig_stride;
  b->d_prevs = d_prevs;
  b->prev_stride = prev_stride;
  b->d_prev_lens = d_prev_lens;
  b->n = n;
  b->d_verdict = d_verdict_out;
  b->d_rand = d_rand_out;
  b->st = w->stream;
  const size_t jw = sig_on_g2(scheme) ? JAC_WORDS_G2 : JAC_WORDS_G1;
  if (!rc) {
    w->begin_one_stream = node_one_stream();
    rc = verify_core(w, scheme, pk, pk_len, d_rounds, d_sigs, sig_stride, d_prevs, prev_stride, d_prev_lens, n, d_verdict_out,
                     d_rand_out, seed, b->st, nullptr, nullptr, VM_BEGIN);
    w->begin_one_stream = false;
  }
  if (!rc) {
    // the record (A, B, status 0) on the batch stream, where the level-0 MSM wrote the sums (an empty batch
    // contributes the identity, Z = 0)
    hipStream_t ts = batch_stream(w);
    const bool ok = (n ? hipMemcpyAsync(d_partials_out, w->outA.p, jw * 4, hipMemcpyDeviceToDevice, ts) == hipSuccess &&
                             hipMemcpyAsync(d_partials_out + jw * 4, w->outB.p, jw * 4, hipMemcpyDeviceToDevice, ts) == hipSuccess
                       : hipMemsetAsync(d_partials_out, 0, 2 * jw * 4, ts) == hipSuccess) &&
                    hipMemsetAsync(d_partials_out + 2 * jw * 4, 0, 16, ts) == hipSuccess;
    if (!ok) {
      rc = fail(DH_EDEVICE, "writing the partial sums failed");
    }
  }
  if (rc) {
    if (w->stream) (void)hipStreamSynchronize(w->stream);  // nothing queued may outlive the lease
    if (w->tail) (void)hipStreamSynchronize(w->tail);
    delete b->L;
    return rc;
  }
  *batch_out = b.release();
  return DH_OK;
}

// the node-wide check of k gathered records on the batch stream: sum, one pairing check, res = w->node_res
static int queue_node_check(worker* w, bool g2, const uint8_t* pk, size_t pk_len, const uint8_t* d_partials, size_t k,
                            hipStream_t ts) {
  int rc = ensure_key(w, g2, pk, pk_len, ts);
  if (rc) return rc;
  const size_t jw = g2 ? JAC_WORDS_G2 : JAC_WORDS_G1;
  HIP_TRY(w->node_sum.ensure(2 * jw * 4));
  HIP_TRY(w->node_res.ensure(16));
  HIP_TRY(hipMemsetAsync(w->node_res.p, 0, 16, ts));
  uint32_t* sA = w->node_sum.as<uint32_t>();
  uint8_t* res = w->node_res.as<uint8_t>();
  HIP_TRY(dh::launch_sum_partials(g2, (const uint32_t*)d_partials, k, partial_words(g2), sA, sA + jw, res, ts));
  HIP_TRY(group_check(w, g2, sA, sA + jw, 1, w->key_cur, res + 1, ts, w->key_cur + 48));
  return DH_OK;
}

void* dh_batch_stream(dh_batch* b) { return b ? (void*)batch_stream(b->L->w) : nullptr; }

int dh_batch_check(dh_batch* b, const uint8_t* d_partials, size_t k, void* hip_stream) {
  if (!b || !d_partials || !k) return fail(DH_EINVAL, "bad node-check arguments");
  worker* w = b->L->w;
  const bool g2 = sig_on_g2(b->scheme);
  hipStream_t bs = batch_stream(w);
  if (hip_stream && (hipStream_t)hip_stream != bs) {  // the gathered records are produced on the caller's stream
    HIP_TRY(hipEventRecord(w->gath_ready, (hipStream_t)hip_stream));
    HIP_TRY(hipStreamWaitEvent(bs, w->gath_ready, 0));
  }
  int rc = queue_node_check(w, g2, b->pk.data(), b->pk.size(), d_partials, k, bs);
  if (rc) return rc;
  // the node-wide result (node_res[2]) and, when it passed, every decoded round of this batch marked valid on the
  // device. A one-round batch put only the identity into the node-wide sums (verify_core VM_BEGIN, n < 2), so the check
  // says nothing about its round: none is marked here, and dh_batch_finish always gives it its leaf check.
  HIP_TRY(dh::launch_node_mark(b->n >= 2 ? b->n : 0, w->node_res.as<uint8_t>(), w->status.as<uint8_t>(), b->d_verdict, bs));
  b->checked = true;
  return DH_OK;
}

int dh_check_partials(int scheme, const uint8_t* pk, size_t pk_len, const uint8_t* d_partials, size_t k, int* pass_out) {
  if (scheme < 0 || scheme > 3) return fail(DH_EINVAL, "unknown scheme %d", scheme);
  if (!pk || !d_partials || !pass_out || !k) return fail(DH_EINVAL, "bad node-check arguments");
  const bool g2 = sig_on_g2(scheme);
  const size_t key_len = g2 ? 48 : 96;
  if (pk_len != key_len) return fail(DH_EINVAL, "public key must be %zu bytes for scheme %d", key_len, scheme);
  lease L;
  if (L.rc) return L.rc;
  worker* w = L.w;
  int rc = set_device_and_stream(w);
  if (rc) return rc;
  rc = queue_node_check(w, g2, pk, pk_len, d_partials, k, w->tail);
  if (rc) return rc;
  uint8_t res[2] = {0, 0};
  HIP_TRY(hipMemcpyAsync(res, w->node_res.p, 2, hipMemcpyDeviceToHost, w->tail));
  HIP_TRY(hipStreamSynchronize(w->tail));
  *pass_out = 0;
  if (res[0]) return fail(DH_EABANDONED, "a rank abandoned the node batch (nonzero status word)");
  *pass_out = res[1] == 1 ? 1 : 0;
  return DH_OK;
}

int dh_batch_finish(dh_batch* b, int node_pass, uint64_t stats_out[4]) {
  if (!b) return fail(DH_EINVAL, "null batch handle");
  worker* w = b->L->w;
  int rc = DH_OK, ret = DH_OK;
  if (stats_out) memset(stats_out, 0, 4 * sizeof(uint64_t));
  if (node_pass == DH_NODE_CHECKED) {
    uint8_t res = 0;
    if (!b->checked) {
      rc = fail(DH_EINVAL, "dh_batch_finish(DH_NODE_CHECKED) without dh_batch_check");
    } else if (hipMemcpyAsync(&res, w->node_res.as<uint8_t>() + 2, 1, hipMemcpyDeviceToHost, batch_stream(w)) != hipSuccess ||
               hipStreamSynchronize(batch_stream(w)) != hipSuccess) {
      rc = fail(DH_EDEVICE, "reading the node-wide check failed");
    } else if (res == 2) {
      rc = fail(DH_EABANDONED, "node batch abandoned: dh_batch_begin failed on another rank");
    } else {
      ret = res == 1 ? 1 : 0;
      // passed: the verdicts are already marked (dh_batch_check); the level bookkeeping only when stats are asked.
      // A one-round batch is never covered by the node check: its leaf check runs in every case.
      if (res != 1 || stats_out || b->n < 2)
        rc = verify_core(w, b->scheme, b->pk.data(), b->pk.size(), b->d_rounds, b->d_sigs, b->sig_stride, b->d_prevs,
                         b->prev_stride, b->d_prev_lens, b->n, b->d_verdict, b->d_rand, 0, b->st, stats_out, nullptr,
                         res == 1 ? VM_FINISH_PASS : VM_FINISH);
    }
  } else if (node_pass >= 0) {
    rc = verify_core(w, b->scheme, b->pk.data(), b->pk.size(), b->d_rounds, b->d_sigs, b->sig_stride, b->d_prevs,
                     b->prev_stride, b->d_prev_lens, b->n, b->d_verdict, b->d_rand, 0, b->st, stats_out, nullptr,
                     node_pass ? VM_FINISH_PASS : VM_FINISH);
  }
  // abandoned or failed: nothing this batch queued may outlive its lease
  if (w->stream) (void)hipStreamSynchronize(w->stream);
  if (w->tail) (void)hipStreamSynchronize(w->tail);
  delete b->L;
  delete b;
  return rc ? rc : ret;
}

int dh_verify_beacon(int scheme, const uint8_t* pk, size_t pk_len, uint64_t round, const uint8_t* sig, size_t sig_len,
                     const uint8_t* prev, size_t prev_len) {
  int sl = dh_sig_len(scheme);
  if (sl < 0) return sl;
  if (!sig || sig_len != (size_t)sl) return 0;  // kyber: wrong-length signature is an invalid signature
  uint8_t sbuf[96] __attribute__((aligned(16)));
  memcpy(sbuf, sig, sig_len);
  // the previous signature is hashed whatever its length (crypto/schemes.go:106-114)
  if (scheme == DH_SCHEME_CHAINED && prev_len > 0xffffffffu) return fail(DH_EINVAL, "previous signature too long");
  std::vector<uint8_t> pbuf(std::max<size_t>(96, (prev_len + 3) & ~(size_t)3), 0);
  uint32_t plen = 0;
  if (scheme == DH_SCHEME_CHAINED && prev && prev_len) {
    memcpy(pbuf.data(), prev, prev_len);
    plen = (uint32_t)prev_len;
  }
  uint8_t verdict = 0;
  int rc = dh_verify_batch(scheme, pk, pk_len, &round, sbuf, (size_t)sl, scheme == DH_SCHEME_CHAINED ? pbuf.data() : nullptr,
                           pbuf.size(), scheme == DH_SCHEME_CHAINED ? &plen : nullptr, 1, &verdict, nullptr, 0);
  return rc < 0 ? rc : verdict;
}

int dh_verify_recovered_batch(int scheme, const uint8_t* pk, size_t pk_len, const uint8_t* msgs32, const uint8_t* sigs,
                              size_t sig_stride, size_t n, uint8_t* verdict_out, uint64_t seed) {
  if (scheme < 0 || scheme > 3) return fail(DH_EINVAL, "unknown scheme %d", scheme);
  if (!pk || (n && (!msgs32 || !sigs || !verdict_out))) return fail(DH_EINVAL, "null argument");
  if (n == 0) return DH_OK;
  if (n <= small_batch_max())
    return verify_small_host(scheme, pk, pk_len, nullptr, sigs, sig_stride, nullptr, 0, nullptr, msgs32, n, verdict_out, nullptr);
  lease L;
  if (L.rc) return L.rc;
  worker* w = L.w;
  int rc = set_device_and_stream(w);
  if (rc) return rc;
  hipStream_t st = w->stream;
  HIP_TRY(w->in_sigs.ensure(n * sig_stride));
  HIP_TRY(w->r_msgs.ensure(n * 32));
  HIP_TRY(w->out_verdict.ensure(n));
  HIP_TRY(hipMemcpyAsync(w->in_sigs.p, sigs, n * sig_stride, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(w->r_msgs.p, msgs32, n * 32, hipMemcpyHostToDevice, st));
  rc = verify_core(w, scheme, pk, pk_len, nullptr, w->in_sigs.as<uint8_t>(), sig_stride, nullptr, 0, nullptr, n,
                   w->out_verdict.as<uint8_t>(), nullptr, seed, st, nullptr, w->r_msgs.as<uint8_t>());
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(verdict_out, w->out_verdict.p, n, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return DH_OK;
}

int dh_verify_recovered(int scheme, const uint8_t* pk, size_t pk_len, const uint8_t* msg32, const uint8_t* sig,
                        size_t sig_len) {
  int sl = dh_sig_len(scheme);
  if (sl < 0) return sl;
  if (!msg32) return fail(DH_EINVAL, "null argument");
  if (!sig || sig_len != (size_t)sl) return 0;  // kyber: wrong-length signature is an invalid signature
  uint8_t sbuf[96] __attribute__((aligned(16)));
  memcpy(sbuf, sig, sig_len);
  uint8_t verdict = 0;
  int rc = dh_verify_recovered_batch(scheme, pk, pk_len, msg32, sbuf, (size_t)sl, 1, &verdict, 0);
  return rc < 0 ? rc : verdict;
}

int dh_digest_batch(int scheme, const uint64_t* rounds, const uint8_t* prevs, size_t prev_stride,
                    const uint32_t* prev_lens, size_t n, uint8_t* out) {
  if (scheme < 0 || scheme > 3) return fail(DH_EINVAL, "unknown scheme %d", scheme);
  for (size_t i = 0; i < n; i++) {
    sha256_host s;
    s.init();
    if (scheme == DH_SCHEME_CHAINED && prevs) {
      size_t pl = prev_lens ? prev_lens[i] : prev_stride;
      if (pl > prev_stride) return fail(DH_EINVAL, "previous signature %zu: length %zu exceeds the record stride %zu", i, pl, prev_stride);
      s.update(prevs + i * prev_stride, pl);
    }
    uint8_t r[8];
    for (int k = 0; k < 8; k++) r[k] = (uint8_t)(rounds[i] >> (56 - 8 * k));
    s.update(r, 8);
    s.final(out + 32 * i);
  }
  return DH_OK;
}

int dh_randomness_batch(int scheme, const uint8_t* sigs, size_t sig_stride, size_t n, uint8_t* out) {
  int sl = dh_sig_len(scheme);
  if (sl < 0) return sl;
  if (n == 0) return DH_OK;
  if (sig_stride < (size_t)sl || sig_stride % 4) return fail(DH_EINVAL, "bad signature stride %zu", sig_stride);
  lease L;
  if (L.rc) return L.rc;
  worker* w = L.w;
  int rc = set_device_and_stream(w);
  if (rc) return rc;
  hipStream_t st = w->stream;
  HIP_TRY(w->in_sigs.ensure(n * sig_stride));
  HIP_TRY(w->out_rand.ensure(n * 32));
  HIP_TRY(w->status.ensure(n));
  HIP_TRY(w->sig_aff.ensure(n * (sl == 96 ? 48 : 24) * 4));
  HIP_TRY(hipMemcpyAsync(w->in_sigs.p, sigs, n * sig_stride, hipMemcpyHostToDevice, st));
  HIP_TRY(dh::launch_prep(sl == 96, w->in_sigs.as<uint8_t>(), sig_stride, n, w->status.as<uint8_t>(),
                          w->sig_aff.as<uint32_t>(), w->out_rand.as<uint8_t>(), st));
  HIP_TRY(hipMemcpyAsync(out, w->out_rand.p, n * 32, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return DH_OK;
}

int dh_recover_batch(int scheme, const uint8_t* commits, int t, int n_nodes, const uint8_t* msgs32,
                     const uint8_t* partials, const uint32_t* part_off, size_t n_rounds, uint8_t* sig_out,
                     uint8_t* status_out) {
  if (scheme < 0 || scheme > 3) return fail(DH_EINVAL, "unknown scheme %d", scheme);
  if (t < 1 || n_nodes < 1 || n_nodes > 65536 || !commits || (n_rounds && (!msgs32 || !partials || !part_off ||
                                                                          !sig_out || !status_out)))
    return fail(DH_EINVAL, "bad Recover arguments");
  for (size_t j = 0; j < n_rounds; j++)
    if (part_off[j + 1] < part_off[j]) return fail(DH_EINVAL, "part_off must be non-decreasing");
  lease L;
  if (L.rc) return L.rc;
  int rc = set_device_and_stream(L.w);
  if (rc) return rc;
  return recover_core(L.w, scheme, commits, t, n_nodes, msgs32, partials, part_off, n_rounds, sig_out, status_out,
                      L.w->stream);
}

int dh_verify_partials_batch(int scheme, const uint8_t* commits, int t, int n_nodes, const uint8_t* msgs32,
                             const uint8_t* partials, const uint32_t* part_off, size_t n_rounds, uint8_t* ok_out) {
  if (scheme < 0 || scheme > 3) return fail(DH_EINVAL, "unknown scheme %d", scheme);
  if (t < 1 || n_nodes < 1 || n_nodes > 65536 || !commits || (n_rounds && (!msgs32 || !partials || !part_off || !ok_out)))
    return fail(DH_EINVAL, "bad VerifyPartial arguments");
  for (size_t j = 0; j < n_rounds; j++)
    if (part_off[j + 1] < part_off[j]) return fail(DH_EINVAL, "part_off must be non-decreasing");
  if (n_rounds == 0 || part_off[n_rounds] == part_off[0]) return DH_OK;
  lease L;
  if (L.rc) return L.rc;
  int rc = set_device_and_stream(L.w);
  if (rc) return rc;
  std::vector<uint8_t> status(n_rounds);
  return recover_core(L.w, scheme, commits, t, n_nodes, msgs32, partials, part_off, n_rounds, nullptr, status.data(),
                      L.w->stream, ok_out);
}

static void sk_words(const uint8_t* sk32, uint32_t w[8]) {
  for (int i = 0; i < 8; i++) {
    const uint8_t* q = sk32 + 28 - 4 * i;
    w[i] = (uint32_t)q[0] << 24 | (uint32_t)q[1] << 16 | (uint32_t)q[2] << 8 | q[3];
  }
}

int dh_sign_batch(int scheme, const uint8_t* sk32, const uint64_t* rounds, const uint8_t* prevs, size_t n,
                  const uint32_t* prev_lens, size_t prev_stride, uint8_t* sigs_out) {
  int sl = dh_sig_len(scheme);
  if (sl < 0) return sl;
  if (!sk32 || (n && (!rounds || !sigs_out))) return fail(DH_EINVAL, "null argument");
  if (n == 0) return DH_OK;
  const bool chained = scheme == DH_SCHEME_CHAINED && prevs;
  lease L;
  if (L.rc) return L.rc;
  worker* w = L.w;
  int rc = set_device_and_stream(w);
  if (rc) return rc;
  hipStream_t st = w->stream;
  uint32_t skw[8];
  sk_words(sk32, skw);
  HIP_TRY(w->key_ok.ensure(64));
  HIP_TRY(w->in_rounds.ensure(n * 8));
  HIP_TRY(w->in_sigs.ensure(n * sl));
  HIP_TRY(hipMemcpyAsync(w->key_ok.p, skw, 32, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(w->in_rounds.p, rounds, n * 8, hipMemcpyHostToDevice, st));
  if (chained) {
    HIP_TRY(w->in_prevs.ensure(n * prev_stride + 4));
    HIP_TRY(hipMemcpyAsync(w->in_prevs.p, prevs, n * prev_stride, hipMemcpyHostToDevice, st));
    if (prev_lens) {
      for (size_t i = 0; i < n; i++)
        if (prev_lens[i] > prev_stride)
          return fail(DH_EINVAL, "previous signature %zu: length %u exceeds the record stride %zu", i, prev_lens[i], prev_stride);
      HIP_TRY(w->in_prev_lens.ensure(n * 4));
      HIP_TRY(hipMemcpyAsync(w->in_prev_lens.p, prev_lens, n * 4, hipMemcpyHostToDevice, st));
    }
  }
  if (sl == 96) {
    HIP_TRY(w->q_pts.ensure(n * JAC_WORDS_G2 * 4));
    HIP_TRY(w->h2c_tmp.ensure(dh::hash_tmp_bytes(1, n)));
  }
  HIP_TRY(dh::launch_sign(sl == 96, w->key_ok.as<uint32_t>(), w->in_rounds.as<uint64_t>(),
                          chained ? w->in_prevs.as<uint8_t>() : nullptr, prev_stride,
                          chained && prev_lens ? w->in_prev_lens.as<uint32_t>() : nullptr, nullptr, n, chained ? 1 : 0,
                          dst_id(scheme), w->in_sigs.as<uint8_t>(), w->q_pts.as<uint32_t>(), w->h2c_tmp.as<uint32_t>(), st));
  HIP_TRY(hipMemcpyAsync(sigs_out, w->in_sigs.p, n * sl, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return DH_OK;
}

int dh_hash_to_curve(int group, const uint8_t* msgs, const uint32_t* msg_off, size_t n, const uint8_t* dst, size_t dst_len,
                     uint8_t* out) {
  if (group != 1 && group != 2) return fail(DH_EINVAL, "group must be 1 (G1) or 2 (G2)");
  if (!msg_off || !out || (n && !msgs) || !dst || dst_len == 0 || dst_len > 255)
    return fail(DH_EINVAL, "bad hash_to_curve arguments (DST must be 1..255 bytes)");
  if (n == 0) return DH_OK;
  size_t maxm = 0;
  for (size_t i = 0; i < n; i++) {
    if (msg_off[i + 1] < msg_off[i]) return fail(DH_EINVAL, "msg_off must be non-decreasing");
    maxm = std::max<size_t>(maxm, msg_off[i + 1] - msg_off[i]);
  }
  const size_t total = msg_off[n] - msg_off[0];
  const size_t stride = (64 + maxm + 4 + dst_len + 63) & ~(size_t)63;
  const size_t outlen = group == 1 ? 48 : 96;
  std::vector<uint32_t> off(n + 1);
  for (size_t i = 0; i <= n; i++) off[i] = msg_off[i] - msg_off[0];
  lease L;
  if (L.rc) return L.rc;
  worker* w = L.w;
  int rc = set_device_and_stream(w);
  if (rc) return rc;
  hipStream_t st = w->stream;
  HIP_TRY(w->in_sigs.ensure(total + 4));
  HIP_TRY(w->in_prev_lens.ensure((n + 1) * 4));
  HIP_TRY(w->key_raw.ensure(256));
  HIP_TRY(w->h2c_tmp.ensure(n * stride));
  HIP_TRY(w->out_rand.ensure(n * outlen));
  if (total) HIP_TRY(hipMemcpyAsync(w->in_sigs.p, msgs + msg_off[0], total, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(w->in_prev_lens.p, off.data(), (n + 1) * 4, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(w->key_raw.p, dst, dst_len, hipMemcpyHostToDevice, st));
  HIP_TRY(dh::launch_h2c_generic(group == 2, w->in_sigs.as<uint8_t>(), w->in_prev_lens.as<uint32_t>(), n,
                                 w->key_raw.as<uint8_t>(), (uint32_t)dst_len, w->h2c_tmp.as<uint8_t>(), stride,
                                 w->out_rand.as<uint8_t>(), st));
  HIP_TRY(hipMemcpyAsync(out, w->out_rand.p, n * outlen, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return DH_OK;
}

int dh_public_key(int scheme, const uint8_t* sk32, uint8_t* key_out) {
  int kl = dh_key_len(scheme);
  if (kl < 0) return kl;
  if (!sk32 || !key_out) return fail(DH_EINVAL, "null argument");
  lease L;
  if (L.rc) return L.rc;
  worker* w = L.w;
  int rc = set_device_and_stream(w);
  if (rc) return rc;
  hipStream_t st = w->stream;
  uint32_t skw[8];
  sk_words(sk32, skw);
  HIP_TRY(w->key_ok.ensure(64));
  HIP_TRY(w->key_raw.ensure(96));
  HIP_TRY(hipMemcpyAsync(w->key_ok.p, skw, 32, hipMemcpyHostToDevice, st));
  HIP_TRY(dh::launch_pubkey(kl == 96, w->key_ok.as<uint32_t>(), w->key_raw.as<uint8_t>(), st));
  HIP_TRY(hipMemcpyAsync(key_out, w->key_raw.p, kl, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return DH_OK;
}

int dh_set_split(uint64_t chunk_rounds, int workers) {
  if (workers < 1) return fail(DH_EINVAL, "workers must be >= 1");
  std::lock_guard<std::mutex> lk(g_split_mu);
  g_split.chunk = (size_t)chunk_rounds;
  g_split.workers = workers;
  return DH_OK;
}

int dh_profile(int enable) {
  std::lock_guard<std::mutex> lk(g_prof.mu);
  prof_drain_locked();
  g_prof.on = enable != 0;
  g_prof.table.clear();
  return DH_OK;
}

int dh_profile_read(char* buf, size_t cap) {
  std::lock_guard<std::mutex> lk(g_prof.mu);
  prof_drain_locked();
  std::string out = "{";
  bool first = true;
  for (auto& e : g_prof.table) {
    char tmp[256];
    snprintf(tmp, sizeof tmp, "%s\"%s\": {\"count\": %llu, \"total_ms\": %.6f, \"products\": %llu}", first ? "" : ", ",
             e.first.c_str(), (unsigned long long)e.second.count, e.second.ms, e.second.prods);
    out += tmp;
    first = false;
  }
  out += "}";
  if (buf && cap) {
    size_t k = std::min(cap - 1, out.size());
    memcpy(buf, out.data(), k);
    buf[k] = 0;
  }
  return (int)out.size();
}

const char* dh_last_error_string(void) { return g_err.c_str(); }

const char* dh_version(void) { return "libdrandhip 0.1 gfx950 (BLS12-381 batch beacon verification)"; }

}  // extern "C"
