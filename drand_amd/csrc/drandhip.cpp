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
//   -> on failure, bisection levels with smaller groups (4096, 64 rounds) over the failing groups only
//   -> leaves: per-round 2-pairing checks. Verdict = decode ok AND (group passed OR leaf passed),
//   which is the per-round VerifyBeacon verdict of /root/reference/crypto/schemes.go:70-72.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <sys/random.h>

#include <algorithm>
#include <mutex>
#include <string>
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
  bool busy = false;
  // per-round state
  dbuf status, sig_aff, q_pts, scal, entries, verdict_tmp, rand_tmp;
  // host-API staging
  dbuf in_rounds, in_sigs, in_prevs, in_prev_lens, out_verdict, out_rand;
  // key
  dbuf key_raw, key_aff, key_ok;
  // MSM
  dbuf cnt, off, scan_tmp, list, buckets, segs, outA, outB, pass;
  std::vector<uint8_t> h_pass;
  // decoded group key cache: the same key is used for every batch of a chain
  uint8_t cached_key[96];
  size_t cached_key_len = 0;
  int cached_key_g2 = -1;
  uint8_t cached_key_ok = 0;
  std::vector<uint32_t> h_entries, h_next;
  void release_all() {
    dbuf* all[] = {&status, &sig_aff, &q_pts, &scal, &entries, &verdict_tmp, &rand_tmp, &in_rounds, &in_sigs,
                   &in_prevs, &in_prev_lens, &out_verdict, &out_rand, &key_raw, &key_aff, &key_ok, &cnt, &off,
                   &scan_tmp, &list, &buckets, &segs, &outA, &outB, &pass};
    for (dbuf* b : all) b->release();
    if (stream) (void)hipStreamDestroy(stream);
    stream = nullptr;
  }
};

struct context {
  std::mutex mu;
  bool inited = false;
  int device = 0;
  std::vector<worker*> pool;
};
context g_ctx;

int ensure_init_locked(uint32_t mask) {
  if (g_ctx.inited) return DH_OK;
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev <= 0) return fail(DH_EDEVICE, "no HIP device available (%s)", hipGetErrorString(e));
  int dev = 0;
  if (mask) dev = __builtin_ctz(mask);
  if (dev >= ndev) return fail(DH_EINVAL, "device %d not present (%d devices)", dev, ndev);
  g_ctx.device = dev;
  g_ctx.inited = true;
  return DH_OK;
}

struct lease {
  worker* w = nullptr;
  int rc = DH_OK;
  lease() {
    std::lock_guard<std::mutex> lk(g_ctx.mu);
    rc = ensure_init_locked(0);
    if (rc != DH_OK) return;
    for (worker* x : g_ctx.pool)
      if (!x->busy) {
        w = x;
        break;
      }
    if (!w) {
      w = new worker();
      g_ctx.pool.push_back(w);
    }
    w->busy = true;
  }
  ~lease() {
    if (!w) return;
    std::lock_guard<std::mutex> lk(g_ctx.mu);
    w->busy = false;
  }
};

int set_device_and_stream(worker* w) {
  HIP_TRY(hipSetDevice(g_ctx.device));
  if (!w->stream) HIP_TRY(hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking));
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

// MSM geometry for groups of gsize rounds
dh::msm_geom geom_for(size_t gsize) {
  int lg = 0;
  while (((size_t)1 << (lg + 1)) <= gsize) lg++;
  int c = std::max(3, std::min(16, lg - 2));
  dh::msm_geom g;
  g.gsize = (uint32_t)gsize;
  g.c = c;
  g.nwin = (128 + c - 1) / c;
  g.nbuck = 1u << c;
  uint32_t nseg = std::max(1u, std::min(2048u, g.nbuck / 32));
  g.nseg = nseg;
  g.seglen = (g.nbuck - 1 + nseg - 1) / nseg;
  return g;
}

constexpr size_t JAC_WORDS_G1 = 36, JAC_WORDS_G2 = 72;

// ---- live per-kernel timing with HIP events on the launching stream (dh_profile / dh_profile_read)
struct prof_entry {
  uint64_t count = 0;
  double ms = 0;
};
struct profiler {
  std::mutex mu;
  bool on = false;
  std::vector<std::pair<std::string, prof_entry>> table;
  void add(const char* name, float ms) {
    std::lock_guard<std::mutex> lk(mu);
    for (auto& e : table)
      if (e.first == name) {
        e.second.count++;
        e.second.ms += ms;
        return;
      }
    prof_entry pe;
    pe.count = 1;
    pe.ms = ms;
    table.emplace_back(name, pe);
  }
};
profiler g_prof;

// records a launch bracketed by events when profiling is on; resolved after the stream syncs
struct timed_launches {
  struct rec {
    const char* name;
    hipEvent_t a, b;
  };
  std::vector<rec> recs;
  hipStream_t st;
  explicit timed_launches(hipStream_t s) : st(s) {}
  template <class F>
  hipError_t run(const char* name, F&& f) {
    if (!g_prof.on) return f();
    rec r{name, nullptr, nullptr};
    (void)hipEventCreate(&r.a);
    (void)hipEventCreate(&r.b);
    (void)hipEventRecord(r.a, st);
    hipError_t e = f();
    (void)hipEventRecord(r.b, st);
    recs.push_back(r);
    return e;
  }
  void resolve() {
    for (auto& r : recs) {
      float ms = 0;
      if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) g_prof.add(r.name, ms);
      (void)hipEventDestroy(r.a);
      (void)hipEventDestroy(r.b);
    }
    recs.clear();
  }
  ~timed_launches() { resolve(); }
};

// core pipeline on device-resident inputs
int verify_core(worker* w, int scheme, const uint8_t* pk, size_t pk_len, const uint64_t* d_rounds, const uint8_t* d_sigs,
                size_t sig_stride, const uint8_t* d_prevs, size_t prev_stride, const uint32_t* d_prev_lens, size_t n,
                uint8_t* d_verdict, uint8_t* d_rand, uint64_t seed, hipStream_t st, uint64_t* stats) {
  const bool g2 = sig_on_g2(scheme);
  const int sig_len = g2 ? 96 : 48, key_len = g2 ? 48 : 96;
  if ((int)pk_len != key_len) return fail(DH_EINVAL, "public key must be %d bytes for scheme %d", key_len, scheme);
  if (sig_stride < (size_t)sig_len || sig_stride % 4) return fail(DH_EINVAL, "bad signature stride %zu", sig_stride);
  if (scheme == DH_SCHEME_CHAINED && d_prevs && (prev_stride % 4 || (!d_prev_lens && prev_stride > 96)))
    return fail(DH_EINVAL, "bad previous-signature stride %zu", prev_stride);
  if (stats) memset(stats, 0, 4 * sizeof(uint64_t));
  if (n == 0) return DH_OK;
  if (n > 0xffffffffu) return fail(DH_EINVAL, "batch too large");
  const size_t jw = g2 ? JAC_WORDS_G2 : JAC_WORDS_G1;
  const size_t aw = jw * 2 / 3;

  // key
  HIP_TRY(w->key_raw.ensure(96));
  HIP_TRY(w->key_aff.ensure(48 * 4));  // key-group affine point (G2: 48 words); fixed size keeps the key cache valid
  HIP_TRY(w->key_ok.ensure(64));  // [0] key status, [32..63] RLC seed
  uint8_t key_ok = 0;
  const bool key_hit = w->cached_key_len == pk_len && w->cached_key_g2 == (g2 ? 0 : 1) && !memcmp(w->cached_key, pk, pk_len);
  if (key_hit) {
    key_ok = w->cached_key_ok;
  } else {
    w->cached_key_len = 0;
    HIP_TRY(hipMemcpyAsync(w->key_raw.p, pk, pk_len, hipMemcpyHostToDevice, st));
    HIP_TRY(dh::launch_decode_key(g2 ? 0 : 1, w->key_raw.as<uint8_t>(), w->key_aff.as<uint32_t>(),
                                  w->key_ok.as<uint8_t>(), st));
    HIP_TRY(hipMemcpyAsync(&key_ok, w->key_ok.p, 1, hipMemcpyDeviceToHost, st));
  }

  // per-round prep
  HIP_TRY(w->status.ensure(n));
  HIP_TRY(w->sig_aff.ensure(n * aw * 4));
  HIP_TRY(w->q_pts.ensure(n * jw * 4));
  HIP_TRY(w->scal.ensure(n * 16));
  HIP_TRY(w->entries.ensure(n * 4));
  timed_launches T(st);
  HIP_TRY(T.run(g2 ? "k_prep_sig<fp2>" : "k_prep_sig<fp>", [&] {
    return dh::launch_prep(g2, d_sigs, sig_stride, n, w->status.as<uint8_t>(), w->sig_aff.as<uint32_t>(), d_rand, st);
  }));
  HIP_TRY(T.run(g2 ? "k_prep_msg<fp2>" : "k_prep_msg<fp>", [&] {
    return dh::launch_msg(g2, d_rounds, d_prevs, prev_stride, d_prev_lens, n, scheme == DH_SCHEME_CHAINED && d_prevs ? 1 : 0,
                          dst_id(scheme), w->q_pts.as<uint32_t>(), st);
  }));
  uint32_t seedw[8];
  int rc = make_seed(seed, seedw);
  if (rc) return rc;
  uint32_t* d_seed = (uint32_t*)((uint8_t*)w->key_ok.p + 32);
  HIP_TRY(hipMemcpyAsync(d_seed, seedw, 32, hipMemcpyHostToDevice, st));
  HIP_TRY(dh::launch_scalars(d_seed, n, w->status.as<uint8_t>(), w->scal.as<uint4>(), st));
  HIP_TRY(hipMemsetAsync(d_verdict, 0, n, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (!key_hit) {
    memcpy(w->cached_key, pk, pk_len);
    w->cached_key_len = pk_len;
    w->cached_key_g2 = g2 ? 0 : 1;
    w->cached_key_ok = key_ok;
  }
  if (key_ok != 1) return fail(DH_EKEY, "group public key is not a valid compressed subgroup point");
  HIP_TRY(dh::launch_iota(w->entries.as<uint32_t>(), n, st));

  // bisection levels: group sizes n, 4096, 64, then per-round leaves
  size_t m = n;
  std::vector<size_t> sizes = {n};
  if (n > 4096) sizes.push_back(4096);
  if (n > 64) sizes.push_back(64);
  int level = 0;
  for (size_t li = 0; li < sizes.size() && m > 0; li++) {
    const size_t gsize = std::min(sizes[li], m);
    const dh::msm_geom g = geom_for(gsize);
    const size_t ngroups = (m + gsize - 1) / gsize;
    const size_t nk = ngroups * g.nwin * (size_t)g.nbuck;
    HIP_TRY(w->cnt.ensure(nk * 4));
    HIP_TRY(w->off.ensure((nk + 1) * 4));
    HIP_TRY(w->scan_tmp.ensure(((nk + 4095) / 4096 + 1) * 4));
    HIP_TRY(w->list.ensure(m * g.nwin * 4));
    HIP_TRY(w->buckets.ensure(nk * jw * 4));
    HIP_TRY(w->segs.ensure(ngroups * g.nwin * g.nseg * jw * 4));
    HIP_TRY(w->outA.ensure(ngroups * jw * 4));
    HIP_TRY(w->outB.ensure(ngroups * jw * 4));
    HIP_TRY(w->pass.ensure(ngroups));
    dh::msm_ws ws{w->cnt.as<uint32_t>(), w->off.as<uint32_t>(), w->scan_tmp.as<uint32_t>(), w->list.as<uint32_t>(),
                  w->buckets.as<uint32_t>(), w->segs.as<uint32_t>()};
    HIP_TRY(T.run(level == 0 ? "msm_level0" : "msm_bisect", [&] {
      return dh::launch_msm(g2, g, w->entries.as<uint32_t>(), m, ngroups, w->scal.as<uint4>(), w->sig_aff.as<uint32_t>(),
                            w->q_pts.as<uint32_t>(), ws, w->outA.as<uint32_t>(), w->outB.as<uint32_t>(), st);
    }));
    HIP_TRY(T.run(level == 0 ? "k_group_check_level0" : "k_group_check_bisect", [&] {
      return dh::launch_group_check(g2, w->outA.as<uint32_t>(), w->outB.as<uint32_t>(), ngroups,
                                    w->key_aff.as<uint32_t>(), w->pass.as<uint8_t>(), st);
    }));
    HIP_TRY(dh::launch_mark_groups(w->entries.as<uint32_t>(), m, gsize, w->pass.as<uint8_t>(), w->status.as<uint8_t>(),
                                   d_verdict, st));
    w->h_pass.resize(ngroups);
    HIP_TRY(hipMemcpyAsync(w->h_pass.data(), w->pass.p, ngroups, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    level++;
    size_t nfail = 0;
    for (uint8_t p : w->h_pass) nfail += p ? 0 : 1;
    if (stats) stats[1] += nfail;
    if (nfail == 0) {
      m = 0;
      break;
    }
    // entries of failing groups, in order
    w->h_entries.resize(m);
    HIP_TRY(hipMemcpyAsync(w->h_entries.data(), w->entries.p, m * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    w->h_next.clear();
    for (size_t gi = 0; gi < ngroups; gi++)
      if (!w->h_pass[gi])
        for (size_t e = gi * gsize; e < std::min(m, (gi + 1) * gsize); e++) w->h_next.push_back(w->h_entries[e]);
    m = w->h_next.size();
    HIP_TRY(hipMemcpyAsync(w->entries.p, w->h_next.data(), m * 4, hipMemcpyHostToDevice, st));
  }
  if (m > 0) {
    HIP_TRY(T.run("k_leaf_check", [&] {
      return dh::launch_leaf_check(g2, w->entries.as<uint32_t>(), m, w->sig_aff.as<uint32_t>(), w->q_pts.as<uint32_t>(),
                                   w->key_aff.as<uint32_t>(), w->status.as<uint8_t>(), d_verdict, st);
    }));
    if (stats) stats[2] = m;
  }
  HIP_TRY(hipStreamSynchronize(st));
  if (stats) stats[0] = (uint64_t)level;
  return DH_OK;
}

}  // namespace

extern "C" {

int dh_init(uint32_t device_mask) {
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  return ensure_init_locked(device_mask);
}

void dh_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_ctx.mu);
  for (worker* w : g_ctx.pool) {
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
  lease L;
  if (L.rc) return L.rc;
  int rc = set_device_and_stream(L.w);
  if (rc) return rc;
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : L.w->stream;
  return verify_core(L.w, scheme, pk, pk_len, d_rounds, d_sigs, sig_stride, d_prevs, prev_stride, d_prev_lens, n,
                     d_verdict_out, d_rand_out, seed, st, stats_out);
}

int dh_verify_batch(int scheme, const uint8_t* pk, size_t pk_len, const uint64_t* rounds, const uint8_t* sigs,
                    size_t sig_stride, const uint8_t* prevs, size_t prev_stride, const uint32_t* prev_lens, size_t n,
                    uint8_t* verdict_out, uint8_t* rand_out, uint64_t seed) {
  if (scheme < 0 || scheme > 3) return fail(DH_EINVAL, "unknown scheme %d", scheme);
  if (!pk || (n && (!rounds || !sigs || !verdict_out))) return fail(DH_EINVAL, "null argument");
  if (n == 0) return DH_OK;
  lease L;
  if (L.rc) return L.rc;
  worker* w = L.w;
  int rc = set_device_and_stream(w);
  if (rc) return rc;
  hipStream_t st = w->stream;
  const bool chained = scheme == DH_SCHEME_CHAINED && prevs;
  HIP_TRY(w->in_rounds.ensure(n * 8));
  HIP_TRY(w->in_sigs.ensure(n * sig_stride));
  HIP_TRY(w->out_verdict.ensure(n));
  if (rand_out) HIP_TRY(w->out_rand.ensure(n * 32));
  HIP_TRY(hipMemcpyAsync(w->in_rounds.p, rounds, n * 8, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(w->in_sigs.p, sigs, n * sig_stride, hipMemcpyHostToDevice, st));
  if (chained) {
    HIP_TRY(w->in_prevs.ensure(n * prev_stride + 4));
    HIP_TRY(hipMemcpyAsync(w->in_prevs.p, prevs, n * prev_stride, hipMemcpyHostToDevice, st));
    if (prev_lens) {
      for (size_t i = 0; i < n; i++)
        if (prev_lens[i] % 4 || prev_lens[i] > 96 || prev_lens[i] > prev_stride)
          return fail(DH_EINVAL, "previous signature %zu has unsupported length %u", i, prev_lens[i]);
      HIP_TRY(w->in_prev_lens.ensure(n * 4));
      HIP_TRY(hipMemcpyAsync(w->in_prev_lens.p, prev_lens, n * 4, hipMemcpyHostToDevice, st));
    }
  }
  rc = verify_core(w, scheme, pk, pk_len, w->in_rounds.as<uint64_t>(), w->in_sigs.as<uint8_t>(), sig_stride,
                   chained ? w->in_prevs.as<uint8_t>() : nullptr, prev_stride,
                   chained && prev_lens ? w->in_prev_lens.as<uint32_t>() : nullptr, n, w->out_verdict.as<uint8_t>(),
                   rand_out ? w->out_rand.as<uint8_t>() : nullptr, seed, st, nullptr);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(verdict_out, w->out_verdict.p, n, hipMemcpyDeviceToHost, st));
  if (rand_out) HIP_TRY(hipMemcpyAsync(rand_out, w->out_rand.p, n * 32, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return DH_OK;
}

int dh_verify_beacon(int scheme, const uint8_t* pk, size_t pk_len, uint64_t round, const uint8_t* sig, size_t sig_len,
                     const uint8_t* prev, size_t prev_len) {
  int sl = dh_sig_len(scheme);
  if (sl < 0) return sl;
  if (!sig || sig_len != (size_t)sl) return 0;  // kyber: wrong-length signature is an invalid signature
  uint8_t sbuf[96] __attribute__((aligned(16)));
  uint8_t pbuf[96] __attribute__((aligned(16)));
  memcpy(sbuf, sig, sig_len);
  uint32_t plen = 0;
  if (scheme == DH_SCHEME_CHAINED && prev && prev_len) {
    if (prev_len % 4 || prev_len > 96) return fail(DH_EINVAL, "unsupported previous-signature length %zu", prev_len);
    memcpy(pbuf, prev, prev_len);
    plen = (uint32_t)prev_len;
  }
  uint8_t verdict = 0;
  int rc = dh_verify_batch(scheme, pk, pk_len, &round, sbuf, (size_t)sl, scheme == DH_SCHEME_CHAINED ? pbuf : nullptr, 96,
                           scheme == DH_SCHEME_CHAINED ? &plen : nullptr, 1, &verdict, nullptr, 0);
  return rc < 0 ? rc : verdict;
}

int dh_verify_recovered(int scheme, const uint8_t* pk, size_t pk_len, const uint8_t* msg32, const uint8_t* sig,
                        size_t sig_len) {
  (void)scheme; (void)pk; (void)pk_len; (void)msg32; (void)sig; (void)sig_len;
  return fail(DH_EINVAL, "dh_verify_recovered: not yet implemented on the device path");
}

int dh_digest_batch(int scheme, const uint64_t* rounds, const uint8_t* prevs, size_t prev_stride,
                    const uint32_t* prev_lens, size_t n, uint8_t* out) {
  if (scheme < 0 || scheme > 3) return fail(DH_EINVAL, "unknown scheme %d", scheme);
  for (size_t i = 0; i < n; i++) {
    sha256_host s;
    s.init();
    if (scheme == DH_SCHEME_CHAINED && prevs) {
      size_t pl = prev_lens ? prev_lens[i] : prev_stride;
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
  (void)scheme; (void)commits; (void)t; (void)n_nodes; (void)msgs32; (void)partials; (void)part_off; (void)n_rounds;
  (void)sig_out; (void)status_out;
  return fail(DH_EINVAL, "dh_recover_batch: not yet implemented on the device path");
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
  if (chained && (prev_stride % 4 || (!prev_lens && prev_stride > 96)))
    return fail(DH_EINVAL, "bad previous-signature stride %zu", prev_stride);
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
        if (prev_lens[i] % 4 || prev_lens[i] > 96 || prev_lens[i] > prev_stride)
          return fail(DH_EINVAL, "previous signature %zu has unsupported length %u", i, prev_lens[i]);
      HIP_TRY(w->in_prev_lens.ensure(n * 4));
      HIP_TRY(hipMemcpyAsync(w->in_prev_lens.p, prev_lens, n * 4, hipMemcpyHostToDevice, st));
    }
  }
  HIP_TRY(dh::launch_sign(sl == 96, w->key_ok.as<uint32_t>(), w->in_rounds.as<uint64_t>(),
                          chained ? w->in_prevs.as<uint8_t>() : nullptr, prev_stride,
                          chained && prev_lens ? w->in_prev_lens.as<uint32_t>() : nullptr, n, chained ? 1 : 0,
                          dst_id(scheme), w->in_sigs.as<uint8_t>(), st));
  HIP_TRY(hipMemcpyAsync(sigs_out, w->in_sigs.p, n * sl, hipMemcpyDeviceToHost, st));
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

int dh_profile(int enable) {
  std::lock_guard<std::mutex> lk(g_prof.mu);
  g_prof.on = enable != 0;
  g_prof.table.clear();
  return DH_OK;
}

int dh_profile_read(char* buf, size_t cap) {
  std::lock_guard<std::mutex> lk(g_prof.mu);
  std::string out = "{";
  bool first = true;
  for (auto& e : g_prof.table) {
    char tmp[256];
    snprintf(tmp, sizeof tmp, "%s\"%s\": {\"count\": %llu, \"total_ms\": %.6f}", first ? "" : ", ", e.first.c_str(),
             (unsigned long long)e.second.count, e.second.ms);
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
