"""GPU parity at the BASELINE.json configs' own sizes (the bench measures them; these tests certify the verdicts):
  * configs[1] quicknet: 1,048,576 device-signed rounds, 0.1% corrupted in the three Cfg5 classes (sigma + g1, a
    flipped bit, an on-curve point outside the subgroup) at splitmix64(0xD5A11D) positions;
  * configs[2] pedersen-bls-unchained: 1,048,576 rounds through the node-wide check (dh_batch_begin on two shards,
    one pairing check of both shards' records per batch, dh_batch_finish — the protocol dist.begin_node_batch drives
    on each rank) and through the local path, clean and 0.1% corrupted;
  * configs[3] tbls Recover n = 64, t = 33 x 100,000 rounds, the first 33 signers every round and random signer
    subsets (with invalid partials and rounds short of t valid ones), pinned by [f(0)] H(m).
The rejected set must be exactly the corrupted one; the CPU oracle (oracle/, test infrastructure) re-verifies every
rejected round and a sample of accepted ones (crypto/schemes.go:70-72 restated), and Recover on a sample of rounds
(chain/beacon/chainstore.go:202-207 restated). configs[4] (4M chained replay at 0.1%) runs here at 262,144 rounds,
twice, so the second call takes the dense-fault shape (level 0 skipped, the 256 -> 32 -> 4 ladder); the 16k-round
1% real-chain test (test_gpu_paths.py::test_chained_replay_real_chain) stays beside it; signing a sequential 4M chain
takes minutes, so the full size is the bench's (bench/bench_configs.py chained).
"""
import ctypes
import hashlib
import os
import random
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bench"))
R_ORDER = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
N_1M = 1 << 20

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dh():
    import torch
    import drand_amd
    from drand_amd import _lib
    torch.zeros(1, device="cuda")
    assert _lib.load().dh_init(0) == 0, _lib.last_error()
    return drand_amd


def _secret(name):
    """The bench's key (bench.py, bench/bench_configs.py): SHA-256("drandhip-sk-" || scheme) mod r."""
    return (int.from_bytes(hashlib.sha256(b"drandhip-sk-" + name.encode()).digest(), "big") % R_ORDER).to_bytes(32, "big")


def _oracle_agrees(oracle, name, pk, rounds, sigs, verdict, rejected, n_sample, seed):
    """The oracle's per-round VerifyBeacon on every rejected round and n_sample random accepted ones (16 threads)."""
    acc = np.flatnonzero(verdict)
    samp = np.unique(np.concatenate([rejected, np.random.default_rng(seed).choice(acc, n_sample, replace=False)]))
    ov, _ = oracle.verify_batch(name, pk, rounds[samp], sigs[samp], nthreads=16, want_rand=False)
    assert np.array_equal(ov.astype(bool), verdict[samp].astype(bool))
    return len(samp)


def _randomness_spot_check(rand, sigs, seed, k=512):
    for i in np.random.default_rng(seed).choice(len(sigs), k, replace=False):
        assert rand[i].tobytes() == hashlib.sha256(sigs[i].tobytes()).digest(), i


def test_config2_quicknet_1m(dh, oracle):
    """BASELINE configs[1] at its size: 1,048,576 quicknet rounds. Clean: every round verifies (one level-0 group
    check, no bisection). 0.1% corrupted (1,048 rounds): exactly those rounds are rejected, the oracle agrees on all of
    them and on 2,000 sampled accepted rounds, and randomness = SHA-256(signature) on a sample."""
    import chainsynth
    import g1_synth
    name = "bls-unchained-g1-rfc9380"
    s = dh.scheme_from_name(name)
    sk = _secret(name)
    pk = s.public_key(sk)
    rounds = np.arange(1, N_1M + 1, dtype=np.uint64)
    sigs = s.sign_beacons(sk, rounds)
    v, rand = s.verify_beacons(pk, rounds, sigs, seed=101)
    assert v.all()
    _randomness_spot_check(rand, sigs, 1)
    bad = chainsynth.corrupted_rounds(N_1M, N_1M // 1000)
    sigs2 = sigs.copy()
    g1_synth.corrupt(sigs2, bad, random.Random(41))
    v2, rand2 = s.verify_beacons(pk, rounds, sigs2, seed=102)
    rejected = np.flatnonzero(~v2)
    assert rejected.tolist() == bad.tolist()
    _oracle_agrees(oracle, name, pk, rounds, sigs2, v2, rejected, 2000, 2)
    _randomness_spot_check(rand2, sigs2, 3)
    assert all(rand2[i].tobytes() == hashlib.sha256(sigs2[i].tobytes()).digest() for i in bad[:30])


def test_config3_unchained_1m_node_and_local(dh, oracle):
    """BASELINE configs[2] at its size: 1,048,576 pedersen-bls-unchained rounds (G2 signatures, hash-to-G2), as two
    shards under the node-wide check — each shard a dh_batch_begin (per-round kernels + level-0 MSM, its record
    written), dh_batch_check of BOTH records (the all-gather of two ranks is their concatenation on one device) and
    dh_batch_finish(DH_NODE_CHECKED) — and as one local call. Clean: the node check passes. 0.1% corrupted in the
    Cfg5 classes: the node check fails, each shard bisects, and both paths reject exactly the corrupted rounds; the
    oracle agrees on every rejected round and 2,000 sampled accepted ones."""
    import torch
    import chainsynth
    from drand_amd import _lib
    lib = _lib.load()
    name = "pedersen-bls-unchained"
    s = dh.scheme_from_name(name)
    sk = _secret(name)
    pk = s.public_key(sk)
    n = N_1M
    rounds = np.arange(1, n + 1, dtype=np.uint64)
    sigs = s.sign_beacons(sk, rounds)
    dev = torch.device("cuda", 0)
    d_r = torch.from_numpy(rounds.view(np.int64)).to(dev)
    pb = lib.dh_partial_bytes(s.id)
    shards = [(0, n // 2), (n // 2, n)]

    def node(sig_arr, seed):
        d_s = torch.from_numpy(np.ascontiguousarray(sig_arr)).to(dev)
        d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
        d_rand = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
        parts = torch.zeros(len(shards) * pb, dtype=torch.uint8, device=dev)
        cur = torch.cuda.Stream(device=dev)  # explicit: the default stream is the NULL stream ("no stream")
        cur.wait_stream(torch.cuda.current_stream(dev))
        sp = ctypes.c_void_p(cur.cuda_stream)
        handles = []
        for k, (lo, hi) in enumerate(shards):
            b = ctypes.c_void_p()
            rc = lib.dh_batch_begin(s.id, pk, len(pk), ctypes.c_void_p(d_r.data_ptr() + 8 * lo),
                                    ctypes.c_void_p(d_s.data_ptr() + 96 * lo), 96, None, 0, None, hi - lo,
                                    ctypes.c_void_p(d_v.data_ptr() + lo), ctypes.c_void_p(d_rand.data_ptr() + 32 * lo),
                                    seed + 7 * k, sp, ctypes.byref(b), ctypes.c_void_p(parts.data_ptr() + k * pb))
            assert rc == 0, _lib.last_error()
            handles.append(b)
        for b in handles:  # both records complete before either check reads them
            cur.wait_stream(torch.cuda.ExternalStream(lib.dh_batch_stream(b), device=dev))
        for b in handles:
            assert lib.dh_batch_check(b, ctypes.c_void_p(parts.data_ptr()), len(shards), sp) == 0, _lib.last_error()
        res = []
        for b in handles:
            r = lib.dh_batch_finish(b, _lib.DH_NODE_CHECKED, None)
            assert r in (0, 1), _lib.last_error()
            res.append(r)
        torch.cuda.synchronize()
        assert res[0] == res[1]
        return res[0], d_v.cpu().numpy().astype(bool), d_rand.cpu().numpy()

    passed, v, rand = node(sigs, 11)
    assert passed == 1 and v.all()
    _randomness_spot_check(rand, sigs, 4)
    vl, _ = s.verify_beacons(pk, rounds, sigs, seed=12, want_randomness=False)
    assert vl.all()
    bad = chainsynth.corrupted_rounds(n, n // 1000)
    sigs2 = sigs.copy()
    chainsynth.corrupt(sigs2, bad, random.Random(43))
    passed, v2, rand2 = node(sigs2, 13)
    assert passed == 0
    rejected = np.flatnonzero(~v2)
    assert rejected.tolist() == bad.tolist()
    vl2, _ = s.verify_beacons(pk, rounds, sigs2, seed=14, want_randomness=False)
    assert np.array_equal(vl2, v2)
    _oracle_agrees(oracle, name, pk, rounds, sigs2, v2, rejected, 2000, 5)
    _randomness_spot_check(rand2, sigs2, 6)


def _dealer(s, t, tag):
    coeffs = [int.from_bytes(hashlib.sha256(b"%s-%d" % (tag, j)).digest(), "big") % R_ORDER for j in range(t)]
    return coeffs, [s.public_key(cf.to_bytes(32, "big")) for cf in coeffs]


def _share(coeffs, i):
    x, acc = i + 1, 0
    for cf in reversed(coeffs):
        acc = (acc * x + cf) % R_ORDER
    return acc.to_bytes(32, "big")


@pytest.mark.parametrize("subsets", ["first", "random"])
def test_config4_tbls_recover_100k(dh, oracle, subsets):
    """BASELINE configs[3] at its size: tbls Recover, n = 64 signers, threshold t = 33, 100,000 rounds (VerifyPartial
    batch check, selection of the first t valid partials in arrival order, Lagrange interpolation in G2, VerifyRecovered
    of the result). "first": the signers 0..32 every round (the bench's default shape); "random": a random t-subset of
    the 64 per round in random arrival order, every 97th round with another round's signature in front (still t valid,
    recovered), every 1,009th round one of its t partials bit-flipped (t - 1 valid: not recovered). Recovered rounds
    equal the group signature [f(0)] H(m) (chain/beacon/node_test.go:60-109 pattern); 16 sampled rounds, the odd ones
    among them, equal the oracle's Recover."""
    from concurrent.futures import ThreadPoolExecutor
    s = dh.scheme_from_name("pedersen-bls-unchained")
    n, t, nr = 64, 33, 100000
    coeffs, commits = _dealer(s, t, b"cfg4-%s" % subsets.encode())
    rounds = np.arange(1, nr + 1, dtype=np.uint64)
    rng = np.random.default_rng(71)
    if subsets == "first":
        ids = np.tile(np.arange(t, dtype=np.int64), (nr, 1))
    else:
        ids = np.argsort(rng.random((nr, n)), axis=1)[:, :t]
    shares = np.zeros((n, nr, 96), dtype=np.uint8)
    for i in np.unique(ids):
        shares[i] = s.sign_beacons(_share(coeffs, int(i)), rounds)
    per = t + 1  # a slot for the invalid partial in front; the other rounds leave it empty
    raw = np.zeros((nr, per, 98), dtype=np.uint8)
    raw[:, 1:, 0] = (ids >> 8).astype(np.uint8)
    raw[:, 1:, 1] = (ids & 0xff).astype(np.uint8)
    raw[:, 1:, 2:] = shares[ids, np.arange(nr)[:, None]]
    cnt = np.full(nr, t, dtype=np.int64)
    front = np.arange(0, nr, 97) if subsets == "random" else np.array([], dtype=np.int64)
    raw[front, 0, 0] = (ids[front, 0] >> 8).astype(np.uint8)
    raw[front, 0, 1] = (ids[front, 0] & 0xff).astype(np.uint8)
    raw[front, 0, 2:] = shares[ids[front, 0], (front + 1) % nr]
    cnt[front] = t + 1
    short = np.arange(500, nr, 1009) if subsets == "random" else np.array([], dtype=np.int64)
    raw[short, 1 + t // 2, 2 + 50] ^= 0x02
    # pack each round's records (the in-front slot only where it is used) into one contiguous buffer
    keep = np.ones((nr, per), dtype=bool)
    keep[:, 0] = False
    keep[front, 0] = True
    flat = np.ascontiguousarray(raw[keep])
    off = np.zeros(nr + 1, dtype=np.uint32)
    off[1:] = np.cumsum(cnt)
    assert off[-1] == len(flat)
    msgs = np.stack([np.frombuffer(s.digest_beacon(int(r)), np.uint8) for r in rounds])
    sigs, ok = s.recover_batch_packed(commits, t, n, msgs, flat, off)
    want_ok = np.ones(nr, dtype=bool)
    want_ok[short] = False
    assert np.array_equal(ok, want_ok)
    group = s.sign_beacons(coeffs[0].to_bytes(32, "big"), rounds)
    assert np.array_equal(sigs[ok], group[ok])
    sample = sorted(set(np.random.default_rng(8).choice(nr, 12, replace=False).tolist()) |
                    set(front[:2].tolist()) | set(short[:2].tolist()))

    def orc(j):
        parts = [flat[k].tobytes() for k in range(int(off[j]), int(off[j + 1]))]
        return oracle.recover(s.name, commits, t, n, msgs[j].tobytes(), parts)

    with ThreadPoolExecutor(16) as ex:
        want = list(ex.map(orc, sample))
    for j, w in zip(sample, want):
        assert (w is not None) == bool(ok[j]), j
        if w is not None:
            assert w == sigs[j].tobytes(), j


def test_config5_chained_replay_262k_dense(dh, oracle):
    """BASELINE configs[4]'s shape at 262,144 rounds (a quarter of one 1M window; the 4M chain's signing takes ~3.5
    minutes and stays in the bench, profiles/r06/config_chained_*.json): a sequential pedersen-bls-chained chain, 0.1%
    of its rounds corrupted in the three Cfg5 classes, replayed twice through dh_verify_batch_device as
    CheckPastBeacons does, one call per window. The first call fails level 0 and bisects 1024 -> ...; its first level's
    failure rate (~1 fault per 1000 rounds) marks the worker dense, so the second call skips level 0 and runs the
    dense ladder 256 -> 32 -> 4 -> leaves (drandhip.cpp skip0, next_group_size) — the shape the 16k-round 1% test
    never reaches. Both calls must reject exactly U{k, k+1} (/root/reference/chain/beacon/sync_manager.go:191-225;
    core/drand_test.go:1105-1111's faulty-round contract), which the oracle confirms on every rejected round and 2,000
    accepted ones."""
    import torch
    import chainsynth
    from drand_amd import _lib
    lib = _lib.load()
    name = "pedersen-bls-chained"
    s = dh.scheme_from_name(name)
    sk = _secret(name)
    pk = s.public_key(sk)
    n = 1 << 18
    genesis = hashlib.sha256(b"drandhip-genesis").digest()
    bad = chainsynth.corrupted_rounds(n, n // 1000)
    sigs = chainsynth.sign_chain(s, sk, 1, n, genesis, bad, np.random.default_rng(0xC5))
    chainsynth.corrupt(sigs, bad, random.Random(31))
    prev, plen = chainsynth.stored_prevs(sigs, genesis)
    rounds = np.arange(1, n + 1, dtype=np.uint64)
    expected = chainsynth.expected_faulty(bad, n)
    dev = torch.device("cuda")
    d_r = torch.from_numpy(rounds.view(np.int64)).to(dev)
    d_s = torch.from_numpy(sigs).to(dev)
    d_p = torch.from_numpy(np.concatenate([prev.reshape(-1), np.zeros(4, np.uint8)])).to(dev)
    d_l = torch.from_numpy(plen.astype(np.uint32).view(np.int32)).to(dev)
    d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    levels = []
    for seed in (91, 92):
        st = (ctypes.c_uint64 * 4)()
        rc = lib.dh_verify_batch_device(s.id, pk, len(pk), ctypes.c_void_p(d_r.data_ptr()), ctypes.c_void_p(d_s.data_ptr()),
                                        96, ctypes.c_void_p(d_p.data_ptr()), prev.shape[1], ctypes.c_void_p(d_l.data_ptr()),
                                        n, ctypes.c_void_p(d_v.data_ptr()), None, seed, None, st)
        assert rc == 0, _lib.last_error()
        v = d_v.cpu().numpy().astype(bool)
        assert np.flatnonzero(~v).tolist() == expected.tolist()
        assert st[3] == len(expected)
        levels.append(list(st))
    # call 1: level 0 + at least the 1024-group level; call 2: no level 0 (the dense worker's hint), >= 3 levels
    assert levels[0][0] >= 3 and levels[0][1] >= 1 and levels[1][0] >= 3 and levels[1][2] > 0, levels
    ov = np.zeros(0)
    samp = np.unique(np.concatenate([expected, np.random.default_rng(5).choice(np.flatnonzero(v), 2000, replace=False)]))
    ov = np.zeros(len(samp), np.uint8)
    rs, ss = np.ascontiguousarray(rounds[samp]), np.ascontiguousarray(sigs[samp])
    ps, ls = np.ascontiguousarray(prev[samp]), np.ascontiguousarray(plen[samp].astype(np.uint32))
    oracle.lib().or_verify_batch(oracle.sid(name), pk, len(pk), rs.ctypes.data, ss.ctypes.data, 96, ps.ctypes.data,
                                 prev.shape[1], ls.ctypes.data, len(samp), 16, ov.ctypes.data, None)
    assert ov.astype(bool).tolist() == v[samp].tolist()
    print("bisection stats per call:", levels)
