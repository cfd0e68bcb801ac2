"""GPU parity for the round-2 paths, through the C ABI against the CPU oracle (test infrastructure):
  * chained DigestBeacon over previous signatures of any length (crypto/schemes.go:106-114,
    chain/boltdb/trimmed.go:183-189) and CheckPastBeacons marking only the affected rounds faulty
    (chain/beacon/sync_manager.go:215-217);
  * tbls Recover / VerifyPartial at the BASELINE config shape n = 64, t = 33 (chain/beacon/chainstore.go:202-207);
  * a real sequential chained replay (prev = stored signature of round-1) with the three Cfg5 corruption
    classes, faulty set = U{k, k+1} (core/drand_test.go:1105-1111);
  * concurrent callers (SURVEY.md §8b threading contract) and one-call multi-stream splitting;
  * the stream-sync micro-batcher on the device (chain/beacon/sync_manager.go:376-445).
"""
import hashlib
import json
import os
import queue
import random
import subprocess
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bench"))

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
R_ORDER = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
CHAINED = "pedersen-bls-chained"


@pytest.fixture(scope="module")
def dh():
    import torch
    import drand_amd
    from drand_amd import _lib
    # torch carries its own HIP runtime: bring it up before the library's runtime has created its streams
    torch.zeros(1, device="cuda")
    assert _lib.load().dh_init(0) == 0, _lib.last_error()
    return drand_amd


def _secret(tag):
    return (int.from_bytes(hashlib.sha256(tag).digest(), "big") % R_ORDER).to_bytes(32, "big")


# ---------------------------------------------------------------- chained digests of any length
def test_chained_prev_any_length(dh, oracle):
    """Previous signatures of 0/1/4/31/32/95/96/97/100/300 and 5000 bytes: the device hashes exactly what it is
    given (valid when the round was signed over that record, invalid otherwise), matching the oracle per round."""
    s = dh.scheme_from_name(CHAINED)
    sk = _secret(b"anylen")
    pk = s.public_key(sk)
    rng = np.random.default_rng(3)
    lengths = [0, 1, 4, 31, 32, 95, 96, 97, 100, 300, 5000]
    rounds = np.arange(1000, 1000 + 2 * len(lengths), dtype=np.uint64)
    prevs = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in lengths for _ in range(2)]
    signed_over = list(prevs)
    for k in range(1, len(prevs), 2):  # every second round was signed over a different record
        signed_over[k] = prevs[k][:-1] + bytes([prevs[k][-1] ^ 1]) if prevs[k] else b"\x00" * 7
    small = [k for k in range(len(prevs)) if len(signed_over[k]) <= 4096]
    sigs = np.zeros((len(rounds), 96), np.uint8)
    sigs[small] = s.sign_beacons(sk, rounds[small], [signed_over[k] for k in small])
    for k in range(len(prevs)):
        want_sig = oracle.sign(CHAINED, sk, oracle.digest_beacon(CHAINED, int(rounds[k]), signed_over[k]))
        if k in small:  # the device signer hashes odd-length records exactly as the oracle does
            assert sigs[k].tobytes() == want_sig, k
        else:
            sigs[k] = np.frombuffer(want_sig, np.uint8)
    v, rand = s.verify_beacons(pk, rounds, sigs, prevs, seed=21)
    want = [oracle.verify_beacon(CHAINED, pk, int(r), sigs[k].tobytes(), prevs[k]) for k, r in enumerate(rounds)]
    assert v.tolist() == want
    assert want == [k % 2 == 0 for k in range(len(prevs))]
    assert rand[5].tobytes() == hashlib.sha256(sigs[5].tobytes()).digest()
    for k in (2, 3, 16):  # single-beacon path
        b = dh.Beacon(int(rounds[k]), sigs[k].tobytes(), prevs[k])
        if want[k]:
            s.verify_beacon(b, pk)
        else:
            with pytest.raises(dh.SchemeError):
                s.verify_beacon(b, pk)


def _serial_check(oracle, pk, sig_of, n, up_to):
    """CheckPastBeacons (chain/beacon/sync_manager.go:191-225) serially on the oracle over a trimmed store."""
    faulty = []
    for r in range(1, n):
        sig, prev = sig_of.get(r), sig_of.get(r - 1)
        if sig is None or prev is None:
            faulty.append(r)
        elif len(sig) != 96 or not oracle.verify_beacon(CHAINED, pk, r, sig, prev):
            faulty.append(r)
        if r >= up_to:
            break
    return faulty


def test_check_past_beacons_odd_records(dh, oracle):
    """A trimmed store whose records at some rounds are 0/31/95/97/100 bytes: CheckPastBeacons reports exactly
    the oracle's faulty rounds (the odd record's round and the next one, whose previous signature is that record)
    instead of aborting the window."""
    from drand_amd.sync import TrimmedMemStore, check_past_beacons
    c = json.load(open(os.path.join(GOLD, "chains.json")))[CHAINED]
    s = dh.scheme_from_name(CHAINED)
    pk = bytes.fromhex(c["pk"])
    st = TrimmedMemStore(True)
    sig_of = {0: bytes.fromhex(c["prevs"][0])}
    for r, sig in zip(c["rounds"], c["sigs"]):
        sig_of[r] = bytes.fromhex(sig)
    rng = random.Random(9)
    for r, L in zip((3, 7, 11, 15, 19), (0, 31, 95, 97, 100)):
        sig_of[r] = bytes(rng.randrange(256) for _ in range(L))
    for r, sig in sig_of.items():
        st.put(r, sig)
    n = st.len()
    got = check_past_beacons(st, s, pk, 1000, window=9)
    assert got == _serial_check(oracle, pk, sig_of, n, 1000)
    assert got == [3, 4, 7, 8, 11, 12, 15, 16, 19, 20]


# ---------------------------------------------------------------- tbls at n = 64, t = 33
def _dealer(s, t, tag):
    coeffs = [int.from_bytes(hashlib.sha256(b"%s-%d" % (tag, j)).digest(), "big") % R_ORDER for j in range(t)]
    commits = [s.public_key(cf.to_bytes(32, "big")) for cf in coeffs]
    return coeffs, commits


def _share(coeffs, i):
    x, acc = i + 1, 0
    for cf in reversed(coeffs):
        acc = (acc * x + cf) % R_ORDER
    return acc.to_bytes(32, "big")


def test_recover_config4_n64_t33(dh, oracle):
    """chain/beacon/chainstore.go:202-207 at the BASELINE shape: 64 signers, threshold 33, 160 rounds with random
    signer subsets in random arrival order, invalid partials (another round's signature, a flipped bit), duplicate
    indices, an index outside the group, and rounds with fewer than t valid partials. Recover bytes + status and
    VerifyPartial per partial are compared with the oracle (kyber sign/tbls restated)."""
    s = dh.scheme_from_name("pedersen-bls-unchained")
    n, t, nr = 64, 33, 160
    coeffs, commits = _dealer(s, t, b"cfg4")
    rounds = np.arange(7000, 7000 + nr, dtype=np.uint64)
    shares = [s.sign_beacons(_share(coeffs, i), rounds) for i in range(n)]
    msgs = [s.digest_beacon(int(r)) for r in rounds]
    rng = random.Random(2024)
    parts = []
    for j in range(nr):
        kind = j % 8
        k = rng.randrange(t - 3, t) if kind == 7 else rng.randrange(t, n + 1)  # kind 7: fewer than t signers
        ids = rng.sample(range(n), k)
        ps = [i.to_bytes(2, "big") + shares[i][j].tobytes() for i in ids]
        if kind in (1, 4):  # invalid partials in front: another round's signature, a flipped bit
            i = ids[0]
            ps.insert(0, i.to_bytes(2, "big") + shares[i][(j + 1) % nr].tobytes())
            bad = bytearray(ps[-1])
            bad[40] ^= 0x08
            ps.insert(1, bytes(bad))
        if kind == 2:  # duplicate index (same partial twice) early in the arrival order
            ps.insert(3, ps[0])
        if kind == 3:  # an index outside the group (kyber evaluates any index; node.go:138-141 filters them)
            ps.insert(0, (n + 6).to_bytes(2, "big") + shares[5][j].tobytes())
        rng.shuffle(ps) if kind == 5 else None
        parts.append(ps)
    sigs, ok = s.recover_batch(commits, t, n, msgs, parts)

    def oracle_round(j):
        return oracle.recover(s.name, commits, t, n, msgs[j], parts[j])

    with ThreadPoolExecutor(16) as ex:
        want = list(ex.map(oracle_round, range(nr)))
    for j in range(nr):
        assert bool(ok[j]) == (want[j] is not None), j
        if want[j] is not None:
            assert sigs[j].tobytes() == want[j], j
    assert ok.sum() >= nr * 3 // 4 and not ok.all()
    group_sig = s.sign_beacons(coeffs[0].to_bytes(32, "big"), rounds)
    assert np.array_equal(sigs[ok], group_sig[ok])  # the property pin: [f(0)] H(m)
    # VerifyPartial per partial on a subset of rounds (each oracle check is a full pairing)
    sub = list(range(0, nr, 5))  # every kind of round (j % 8) appears
    got = s.verify_partials_batch(commits, t, n, [msgs[j] for j in sub], [parts[j] for j in sub])
    evals = {}

    def oracle_partial(jk):
        j, p = jk
        i = s.index_of(p)
        if i >= n:
            return False  # documented: indices outside the group are rejected (include/drandhip.h)
        if i not in evals:
            evals[i] = oracle.pubpoly_eval(s.name, commits, i)
        return oracle.verify(s.name, evals[i], msgs[j], p[2:])

    jobs = [(j, p) for j in sub for p in parts[j]]
    with ThreadPoolExecutor(16) as ex:
        want_p = list(ex.map(oracle_partial, jobs))
    flat = [bool(x) for g in got for x in g]
    assert flat == want_p
    assert not all(want_p)


def test_recover_mostly_empty_rounds(dh):
    """1000 rounds of which only 3 have t partials (most have none or fewer than t): the VerifyRecovered batch over
    all rounds must size its scalars for the rounds, not the partials (r_scal overflow)."""
    s = dh.scheme_from_name("bls-unchained-g1-rfc9380")
    n, t, nr = 7, 4, 1000
    coeffs, commits = _dealer(s, t, b"sparse")
    rounds = np.arange(1, nr + 1, dtype=np.uint64)
    good = {17, 500, 999}
    shares = {i: s.sign_beacons(_share(coeffs, i), rounds[sorted(good)]) for i in range(n)}
    msgs = [s.digest_beacon(int(r)) for r in rounds]
    parts = []
    for j in range(nr):
        if j in good:
            g = sorted(good).index(j)
            parts.append([i.to_bytes(2, "big") + shares[i][g].tobytes() for i in (6, 1, 3, 0, 2)])
        elif j % 3 == 0:
            parts.append([i.to_bytes(2, "big") + shares[i][0].tobytes() for i in (0, 1)])
        else:
            parts.append([])
    sigs, ok = s.recover_batch(commits, t, n, msgs, parts)
    assert np.flatnonzero(ok).tolist() == sorted(good)
    want = s.sign_beacons(coeffs[0].to_bytes(32, "big"), rounds[sorted(good)])
    assert np.array_equal(sigs[sorted(good)], want)


def test_recover_large_batch_sliced_and_chunked(dh, oracle):
    """A Recover batch big enough for the paths a 160-round test never takes: 18,944 rounds are 296 blocks of 64, so
    k_lagrange's last 40 blocks (past 256 CUs) run sliced over 6 workgroups each and are summed by k_lagrange_sum;
    551k partial records cross to the device in two chunks overlapped with their decoding. Rounds carry t + 1 partials
    of a random signer subset (every second round the signers of round 0, whose Lagrange rows it then shares, the others a basis of
    their own), every 7th round one invalid partial in front (still t valid, a different basis), every 101st two more
    (fewer than t valid: not recovered). Recovered = the group signature [f(0)] H(m);
    a few rounds against the oracle."""
    s = dh.scheme_from_name("pedersen-bls-unchained")
    n, t, nr = 30, 28, 18944
    coeffs, commits = _dealer(s, t, b"large")
    rounds = np.arange(1, nr + 1, dtype=np.uint64)
    shares = np.stack([s.sign_beacons(_share(coeffs, i), rounds) for i in range(n)])  # (n, nr, 96)
    rng = np.random.default_rng(55)
    ids = np.argsort(rng.random((nr, n)), axis=1)[:, :t + 1]
    ids[::2] = ids[0]  # every second round the signers (and arrival order) of round 0: their lambda rows are round 0's
    raw = np.zeros((nr, t + 1, 98), dtype=np.uint8)
    raw[:, :, 0] = (ids >> 8).astype(np.uint8)
    raw[:, :, 1] = (ids & 0xff).astype(np.uint8)
    raw[:, :, 2:] = shares[ids, np.arange(nr)[:, None]]
    bad1 = np.arange(3, nr, 7)
    raw[bad1, 0, 2 + 40] ^= 0x08
    bad2 = np.arange(5, nr, 101)
    raw[bad2, 1, 2:] = shares[ids[bad2, 1], (bad2 + 1) % nr]  # another round's signature
    raw[bad2, 2, 2 + 60] ^= 0x01
    raw = raw.reshape(nr * (t + 1), 98)
    off = (np.arange(nr + 1) * (t + 1)).astype(np.uint32)
    msgs = np.stack([np.frombuffer(s.digest_beacon(int(r)), np.uint8) for r in rounds])
    sigs, ok = s.recover_batch_packed(commits, t, n, msgs, raw, off)
    want_ok = np.ones(nr, dtype=bool)
    want_ok[bad2] = False
    assert np.array_equal(ok, want_ok)
    group = s.sign_beacons(coeffs[0].to_bytes(32, "big"), rounds)
    assert np.array_equal(sigs[ok], group[ok])
    for j in [0, 1, 2, 10, 3, 5, nr - 1]:
        parts = [raw[j * (t + 1) + k].tobytes() for k in range(t + 1)]
        got = oracle.recover(s.name, commits, t, n, msgs[j].tobytes(), parts)
        assert (got is not None) == bool(ok[j]) and (got is None or got == sigs[j].tobytes()), j


# ---------------------------------------------------------------- real sequential chained replay (Cfg5 shape)
def test_chained_replay_real_chain(dh, oracle):
    """16 384 rounds of a sequential chain (each round signed over the stored signature of the round before,
    genesis seed for round 1), 1% of the rounds corrupted in the three Cfg5 classes (sigma + g2, a flipped bit, an
    on-curve point outside the subgroup): the batch replay rejects exactly U{k, k+1}, which the oracle confirms on
    every faulty round and a sample of the valid ones; check_past_beacons over the store reports the same rounds."""
    import chainsynth
    from drand_amd.sync import TrimmedMemStore, check_past_beacons
    s = dh.scheme_from_name(CHAINED)
    sk = _secret(b"drandhip-sk-" + CHAINED.encode())
    pk = s.public_key(sk)
    n = 1 << 14
    genesis = hashlib.sha256(b"drandhip-genesis").digest()
    bad = chainsynth.corrupted_rounds(n, n // 100)
    rng = np.random.default_rng(0xC5)
    t0 = time.time()
    sigs = chainsynth.sign_chain(s, sk, 1, n, genesis, bad, rng)
    t_sign = time.time() - t0
    prev, plen = chainsynth.stored_prevs(sigs, genesis)
    rounds = np.arange(1, n + 1, dtype=np.uint64)
    v, _ = s.verify_beacons(pk, rounds, sigs, prev, seed=77, previous_lengths=plen)
    heads = sorted(int(k) + 1 for k in bad if k + 1 < n)  # segment heads: signed over a stand-in for sigma_k
    assert np.flatnonzero(~v).tolist() == heads  # every other round is a verified link of the chain
    prng = random.Random(31)
    chainsynth.corrupt(sigs, bad, prng)
    prev, plen = chainsynth.stored_prevs(sigs, genesis)
    v, _ = s.verify_beacons(pk, rounds, sigs, [prev[i, :plen[i]].tobytes() for i in range(n)], seed=78)
    expected = chainsynth.expected_faulty(bad, n)
    assert np.flatnonzero(~v).tolist() == expected.tolist()
    # oracle: every rejected round and 1500 sampled accepted rounds
    sample = np.sort(np.concatenate([expected, np.random.default_rng(1).choice(n, 1500, replace=False)]))
    sample = np.unique(sample)
    ov = np.zeros(len(sample), np.uint8)
    import ctypes
    lib = oracle.lib()
    rs = np.ascontiguousarray(rounds[sample])
    ss = np.ascontiguousarray(sigs[sample])
    ps = np.ascontiguousarray(prev[sample])
    ls = np.ascontiguousarray(plen[sample])
    lib.or_verify_batch(oracle.sid(CHAINED), pk, len(pk), rs.ctypes.data, ss.ctypes.data, 96, ps.ctypes.data, 96,
                        ls.ctypes.data, len(sample), 16, ov.ctypes.data, None)
    assert ov.astype(bool).tolist() == v[sample].tolist()
    st = TrimmedMemStore(True)
    st.put(0, genesis)
    for i in range(n):
        st.put(i + 1, sigs[i].tobytes())
    assert check_past_beacons(st, s, pk, n) == (expected + 1).tolist()
    print("chain of %d rounds signed in %.1f s" % (n, t_sign))


# ---------------------------------------------------------------- threading contract
def test_concurrent_callers(dh):
    """8 threads call the C ABI at once on mixed schemes (batch verify, single verify, Recover, VerifyPartial), one
    of them calling dh_shutdown midway (leased workers are retired, not freed under a running call); every result
    matches the golden fixtures."""
    from drand_amd import _lib
    chains = json.load(open(os.path.join(GOLD, "chains.json")))
    neg = json.load(open(os.path.join(GOLD, "negatives.json")))
    rec = json.load(open(os.path.join(GOLD, "recover.json")))["pedersen-bls-unchained"]
    errors = []

    def job(tid):
        try:
            for it in range(4):
                name = list(chains)[(tid + it) % 4]
                c = chains[name]
                s = dh.scheme_from_name(name)
                sigs = np.array([np.frombuffer(bytes.fromhex(x), np.uint8) for x in c["sigs"]])
                prevs = [bytes.fromhex(p) for p in c["prevs"]] if s.chained else None
                v, rand = s.verify_beacons(bytes.fromhex(c["pk"]), c["rounds"], sigs, prevs, seed=tid + 1)
                assert v.tolist() == c["valid"] and [r.tobytes().hex() for r in rand] == c["randomness"]
                cases = neg[name]["cases"]
                sg = np.array([np.frombuffer(bytes.fromhex(x["sig"]), np.uint8) for x in cases])
                pv = [bytes.fromhex(x["prev"]) for x in cases] if s.chained else None
                v2, _ = s.verify_beacons(bytes.fromhex(neg[name]["pk"]), [x["round"] for x in cases], sg, pv)
                assert v2.tolist() == [x["valid"] for x in cases]
                if tid % 2 == 0:
                    rs = dh.scheme_from_name("pedersen-bls-unchained")
                    commits = [bytes.fromhex(x) for x in rec["commits"]]
                    msgs = [bytes.fromhex(x["msg"]) for x in rec["cases"]]
                    parts = [[bytes.fromhex(p) for p in x["partials"]] for x in rec["cases"]]
                    got, ok = rs.recover_batch(commits, rec["t"], rec["n"], msgs, parts)
                    for k, x in enumerate(rec["cases"]):
                        assert bool(ok[k]) == (x["expected"] is not None)
                        if x["expected"]:
                            assert got[k].tobytes().hex() == x["expected"]
                if tid == 3 and it == 1:
                    _lib.load().dh_shutdown()
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append((tid, repr(e)))

    ths = [threading.Thread(target=job, args=(t,)) for t in range(8)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=240)
    assert not errors, errors
    assert _lib.load().dh_init(0) == 0


def test_single_call_split():
    """One dh_verify_batch / dh_verify_batch_device call over 60 000 quicknet rounds, split by the library over
    4 internal streams in 6 000-round chunks (DRANDHIP_SPLIT), with corrupted rounds in several chunks: verdicts,
    randomness and stats are those of the unsplit call."""
    env = dict(os.environ, DRANDHIP_SPLIT="6000,4")
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "split_check.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    got = json.loads(r.stdout.strip().splitlines()[-1])
    assert got["rejected"] == got["expected"] and got["device_rejected"] == got["expected"]
    assert got["rand_ok"] and got["stats"][3] == len(got["expected"])


# ---------------------------------------------------------------- stream sync on the device
def test_sync_from_stream_device(dh):
    """tryNode's receive loop (chain/beacon/sync_manager.go:376-445) over a live queue: packets that arrive and then
    a quiet stream are verified and stored without waiting for a full window; an invalid packet stops the peer
    after everything before it is stored."""
    from drand_amd.sync import END, TrimmedMemStore, sync_from_stream
    c = json.load(open(os.path.join(GOLD, "chains.json")))[CHAINED]
    s = dh.scheme_from_name(CHAINED)
    pk = bytes.fromhex(c["pk"])
    pkts = [{"round": r, "signature": bytes.fromhex(x), "previous_signature": bytes.fromhex(p)}
            for r, x, p in zip(c["rounds"], c["sigs"], c["prevs"])]
    q = queue.Queue()
    st = TrimmedMemStore(True)
    st.put(0, bytes.fromhex(c["prevs"][0]))  # the genesis record: tryNode starts from the store's Last()
    out = {}
    th = threading.Thread(target=lambda: out.update(res=sync_from_stream(q, s, pk, st, up_to=20, window=500,
                                                                         idle=0.05, max_delay=0.5)))
    th.start()
    for p in pkts[:5]:
        q.put(p)
    deadline = time.time() + 60
    while st.len() < 6 and time.time() < deadline:  # the live follow stores them with the window far from full
        time.sleep(0.02)
    assert st.len() == 6
    for p in pkts[5:]:
        q.put(p)
    q.put(END)
    th.join(timeout=120)
    done, stored = out["res"]
    assert done and stored == list(range(1, 21))
    bad = [dict(p) for p in pkts]
    bad[12]["signature"] = bad[13]["signature"]
    q2 = queue.Queue()
    for p in bad:
        q2.put(p)
    q2.put(END)
    st2 = TrimmedMemStore(True)
    st2.put(0, bytes.fromhex(c["prevs"][0]))
    done, stored = sync_from_stream(q2, s, pk, st2, up_to=24, window=8)
    assert not done and stored == list(range(1, 13))


# ---------------------------------------------------------------- node-wide check (dh_batch_begin / check / finish)
def test_node_wide_check_protocol(dh):
    """The multi-GPU protocol of SURVEY.md §8e on one device: two shards begun as two batches, their level-0 sums
    combined by dh_check_partials (one pairing check), then finished. All-valid shards pass the node check and are
    accepted without a local check; with a corrupted round in one shard the node check fails and each shard's own
    check and bisection give exact verdicts (the clean shard passes its local check)."""
    import ctypes
    import torch
    from drand_amd import _lib
    from drand_amd.dist import gather_partials  # noqa: F401  (the exchange is a concatenation on one device)
    lib = _lib.load()
    s = dh.scheme_from_name("bls-unchained-g1-rfc9380")
    sk = hashlib.sha256(b"node").digest()
    n = 12000
    rounds = np.arange(1, n + 1, dtype=np.uint64)
    sigs = s.sign_beacons(sk, rounds)
    pk = s.public_key(sk)
    dev = torch.device("cuda", 0)
    pb = lib.dh_partial_bytes(s.id)
    assert pb == 2 * 36 * 4 + 16  # A, B, status word, padding

    def run(sig_arr):
        half = [(0, 5000), (5000, n)]
        d_r = torch.from_numpy(rounds.view(np.int64)).to(dev)
        d_s = torch.from_numpy(sig_arr).to(dev)
        d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
        parts = torch.zeros(2 * pb, dtype=torch.uint8, device=dev)
        handles = []
        for k, (lo, hi) in enumerate(half):
            b = ctypes.c_void_p()
            rc = lib.dh_batch_begin(s.id, pk, len(pk), ctypes.c_void_p(d_r.data_ptr() + 8 * lo),
                                    ctypes.c_void_p(d_s.data_ptr() + 48 * lo), 48, None, 0, None, hi - lo,
                                    ctypes.c_void_p(d_v.data_ptr() + lo), None, 0, None, ctypes.byref(b),
                                    ctypes.c_void_p(parts.data_ptr() + k * pb))
            assert rc == 0, _lib.last_error()
            handles.append(b)
        torch.cuda.synchronize()
        ok = ctypes.c_int(-1)
        assert lib.dh_check_partials(s.id, pk, len(pk), ctypes.c_void_p(parts.data_ptr()), 2, ctypes.byref(ok)) == 0
        stats = []
        for b in handles:
            st = (ctypes.c_uint64 * 4)()
            assert lib.dh_batch_finish(b, ok.value, st) == 0, _lib.last_error()
            stats.append(list(st))
        torch.cuda.synchronize()
        return ok.value, d_v.cpu().numpy(), stats

    ok, v, stats = run(sigs)
    assert ok == 1 and v.all()
    bad = sigs.copy()
    bad[7000] = bad[7001]
    bad[11999, 0] ^= 0x20
    ok, v, stats = run(bad)
    assert ok == 0 and np.flatnonzero(v == 0).tolist() == [7000, 11999]
    assert stats[0][1] == 0 and stats[1][1] >= 1  # the clean shard passed its own level-0 check
    ref, _ = s.verify_beacons(pk, rounds, bad, seed=5)
    assert np.array_equal(ref, v.astype(bool))


# ---------------------------------------------------------------- RFC 9380 hash_to_curve on the device
def test_hash_to_curve_rfc9380_device(dh):
    """dh_hash_to_curve (arbitrary message and DST) reproduces the RFC 9380 J.9.1 (G1) / J.10.1 (G2) vectors exactly
    — the quicknet hash path up to its DST — and agrees with the batch kernels' fixed-shape hashing on the drand
    DSTs (hash of a 32-byte digest, as in a signature of the device signer)."""
    import bls_py
    from kat import H2C_DST_G1, H2C_DST_G2, H2C_G1, H2C_G2
    pts = dh.hash_to_curve(1, [m for m, _, _ in H2C_G1], H2C_DST_G1)
    for (m, x, y), c in zip(H2C_G1, pts):
        assert bls_py.g1_decompress(c) == (int(x, 16), int(y, 16)), m[:8]
    pts = dh.hash_to_curve(2, [v[0] for v in H2C_G2], H2C_DST_G2)
    for (m, x0, x1, y0, y1), c in zip(H2C_G2, pts):
        (px0, px1), (py0, py1) = bls_py.g2_decompress(c)
        assert (px0, px1, py0) == (int(x0, 16), int(x1, 16), int(y0, 16)), m
        if y1 is not None:
            assert py1 == int(y1, 16)
    # [1] H(m) from the signer = H(m) of the generic path, for both drand DSTs
    one = (1).to_bytes(32, "big")
    for name, group, dst in (("bls-unchained-g1-rfc9380", 1, b"BLS_SIG_BLS12381G1_XMD:SHA-256_SSWU_RO_NUL_"),
                             ("bls-unchained-on-g1", 1, b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"),
                             ("pedersen-bls-unchained", 2, b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_")):
        s = dh.scheme_from_name(name)
        rounds = np.array([1, 77, 2 ** 40 + 3], dtype=np.uint64)
        sig = s.sign_beacons(one, rounds)
        gen = dh.hash_to_curve(group, [s.digest_beacon(int(r)) for r in rounds], dst)
        assert [x.tobytes() for x in sig] == gen, name


# ---------------------------------------------------------------- the batch check itself, not only the verdicts
@pytest.mark.parametrize("scheme", ["bls-unchained-g1-rfc9380", "bls-unchained-on-g1", "pedersen-bls-unchained",
                                    CHAINED])
def test_group_checks_pass_on_clean_batches(dh, scheme):
    """Verdicts alone cannot show a broken MSM: bisection down to per-round leaves still gets every verdict right.
    So the batch statistics are checked: a clean batch (with one undecodable round, scalar 0) passes its single
    level-0 group check, and a batch with one forged round fails exactly one group per bisection level and sends
    at most a handful of rounds to leaves. This pins the random-linear-combination sums, including the
    endomorphism split (scalars a + b*mu with endo(P) images, k_msm_prep28) at every level."""
    import ctypes
    import torch
    from drand_amd import _lib
    lib = _lib.load()
    s = dh.scheme_from_name(scheme)
    sk = _secret(b"clean-" + scheme.encode())
    n = 6000 if s.sig_len == 48 else 3000
    rounds = np.arange(1, n + 1, dtype=np.uint64)
    prevs = None
    if s.chained:
        rng = np.random.default_rng(11)
        prevs = rng.integers(0, 256, (n, 96), dtype=np.uint8)
        sigs = s.sign_beacons(sk, rounds, [p.tobytes() for p in prevs])
    else:
        sigs = s.sign_beacons(sk, rounds)
    pk = s.public_key(sk)
    sigs[77, 9] ^= 0x01  # off the curve (or at least not this round's point): rejected, its scalar never counts
    dev = torch.device("cuda", 0)
    d_r = torch.from_numpy(rounds.view(np.int64)).to(dev)
    d_p = torch.from_numpy(np.ascontiguousarray(prevs)).to(dev) if prevs is not None else None

    def run(sg, seed):
        d_s = torch.from_numpy(sg).to(dev)
        d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
        stats = (ctypes.c_uint64 * 4)()
        rc = lib.dh_verify_batch_device(s.id, pk, len(pk), ctypes.c_void_p(d_r.data_ptr()), ctypes.c_void_p(d_s.data_ptr()),
                                        s.sig_len, ctypes.c_void_p(d_p.data_ptr()) if d_p is not None else None,
                                        96 if d_p is not None else 0, None, n, ctypes.c_void_p(d_v.data_ptr()), None,
                                        seed, None, stats)
        assert rc == 0, _lib.last_error()
        torch.cuda.synchronize()
        return d_v.cpu().numpy(), list(stats)

    # a worker whose last bisection saw dense faults (an earlier test's ladder) starts its next batch at 256-round groups
    # (drandhip.cpp skip0); a batch whose groups all pass clears that hint, so the second call runs level 0
    run(sigs, 5)
    v, st = run(sigs, 5)
    assert np.flatnonzero(v == 0).tolist() == [77], st  # rejected at decode (off the curve or off the subgroup)
    assert st[:3] == [1, 0, 0], st  # one level, no failed group, no leaf
    forged = sigs.copy()
    k = 4321 % n
    forged[k] = forged[k + 1]  # a valid point of another round
    v2, st2 = run(forged, 6)
    assert sorted(np.flatnonzero(v2 == 0).tolist()) == sorted({77, k}), st2
    # exactly one failing group per level (the forged round's): every other group's sums check out at every level
    # (the cost model may also go from the failed level 0 straight to leaves; tests/fixed_ladder_check.py forces
    # bisection levels on G1 and G2)
    assert st2[1] == st2[0], st2
    assert 1 <= st2[2] <= (n if st2[0] == 1 else 1024), st2


# ---------------------------------------------------------------- the MSM's exact path for exceptional additions
@pytest.mark.parametrize("scheme", ["bls-unchained-g1-rfc9380", "pedersen-bls-unchained"])
def test_msm_exceptional_cases(dh, scheme):
    """Thousands of copies of ONE valid beacon: every bucket of every window receives the same signature point (and
    the same hash point) with both signs, so the bucket pass meets P + P and P - P, and the bucket sums, being small
    multiples of one point, collide again in the segment sums, the tree and the window Horner. Each such addition
    leaves Z = 0 in the fast formulas and must be recomputed on the exact path (k_msm.hip MSM28). The batch must still
    pass its single level-0 check — stats [1 level, 0 failed groups, 0 leaf rounds] — since a broken exact path would
    fail the check and show up only as bisection levels (the verdicts would still be right)."""
    import ctypes
    import torch
    from drand_amd import _lib
    lib = _lib.load()
    s = dh.scheme_from_name(scheme)
    sk = _secret(b"exceptional-" + scheme.encode())
    pk = s.public_key(sk)
    n = 20000 if s.sig_len == 48 else 8000
    rounds = np.full(n, 123457, dtype=np.uint64)
    sigs = np.ascontiguousarray(np.repeat(s.sign_beacons(sk, rounds[:1]), n, axis=0))
    dev = torch.device("cuda", 0)
    d_r = torch.from_numpy(rounds.view(np.int64)).to(dev)
    d_s = torch.from_numpy(sigs).to(dev)
    for seed in (3, 4):
        d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
        st = (ctypes.c_uint64 * 4)()
        rc = lib.dh_verify_batch_device(s.id, pk, len(pk), ctypes.c_void_p(d_r.data_ptr()), ctypes.c_void_p(d_s.data_ptr()),
                                        s.sig_len, None, 0, None, n, ctypes.c_void_p(d_v.data_ptr()), None, seed, None, st)
        assert rc == 0, _lib.last_error()
        torch.cuda.synchronize()
        assert d_v.cpu().numpy().all()
        assert list(st) == [1, 0, 0, 0], list(st)


# ---------------------------------------------------------------- the Go sign.ThresholdScheme drop-in, call by call
@pytest.mark.parametrize("scheme", ["pedersen-bls-unchained", "bls-unchained-g1-rfc9380"])
def test_threshold_scheme_dropin_shapes(dh, oracle, scheme):
    """drand_amd.scheme.ThresholdScheme makes exactly the C calls of the cgo gpuThresholdScheme
    — dh_verify_recovered with one digest, dh_verify_partials_batch with one partial and n_nodes = index + 1,
    dh_recover_batch with one round and n_nodes = max(n, largest index + 1) — and each result equals kyber sign/tbls
    restated by the oracle: any index is evaluated (a valid partial of index 11 in a group of n = 8 verifies and counts
    toward Recover, as in kyber), wrong-length records are never kept, fewer than t valid partials is an error."""
    from drand_amd.scheme import SchemeError, ThresholdScheme
    s = dh.scheme_from_name(scheme)
    ts = ThresholdScheme(s)
    n, t = 8, 5
    coeffs, commits = _dealer(s, t, b"dropin-" + scheme.encode())
    pk = commits[0]
    rounds = np.array([424242, 424243], dtype=np.uint64)
    msgs = [s.digest_beacon(int(r)) for r in rounds]
    idx = list(range(n)) + [11]
    share_sigs = {i: s.sign_beacons(_share(coeffs, i), rounds) for i in idx}
    part = {i: i.to_bytes(2, "big") + share_sigs[i][0].tobytes() for i in idx}
    other = 3 .to_bytes(2, "big") + share_sigs[3][1].tobytes()  # index 3, the other round's signature
    # IndexOf
    assert ts.index_of(part[11]) == 11 and ts.index_of(b"\x01\x02") == 258
    with pytest.raises(SchemeError):
        ts.index_of(b"\x01")
    # VerifyRecovered: the group signature [f(0)] H(m)
    group = s.sign_beacons(coeffs[0].to_bytes(32, "big"), rounds)[0].tobytes()
    assert oracle.verify(s.name, pk, msgs[0], group)
    ts.verify_recovered(pk, msgs[0], group)
    bad = bytearray(group)
    bad[-1] ^= 1
    with pytest.raises(SchemeError):
        ts.verify_recovered(pk, msgs[0], bytes(bad))
    with pytest.raises(SchemeError):
        ts.verify_recovered(pk, msgs[1], group)
    # VerifyPartial, any index (kyber evaluates PubPoly.Eval(i) for every i)
    for i in (0, 5, 7, 11):
        assert oracle.verify(s.name, oracle.pubpoly_eval(s.name, commits, i), msgs[0], part[i][2:])
        ts.verify_partial(commits, msgs[0], part[i])
    for p in (other, part[4][:-1], part[2][:2] + part[6][2:]):  # wrong round, short record, another share's sig
        with pytest.raises(SchemeError):
            ts.verify_partial(commits, msgs[0], p)
    # Recover: arrival order with an invalid partial, a wrong-length record and the index-11 share among the first t
    arrivals = [other, part[11], part[0][:-3], part[6], part[2], part[9 % n], part[4], part[7], part[3]]
    got = ts.recover(commits, msgs[0], arrivals, t, n)
    want = oracle.recover(s.name, commits, t, n, msgs[0], [p for p in arrivals if len(p) == 2 + s.sig_len])
    assert want is not None and got == want == group
    with pytest.raises(SchemeError, match="not enough good public shares"):
        ts.recover(commits, msgs[0], [other, part[1], part[2], part[11], part[5][:-1]], t, n)
    assert oracle.recover(s.name, commits, t, n, msgs[0], [other, part[1], part[2], part[11]]) is None


# ---------------------------------------------------------------- the Go batch methods' C calls, buffer by buffer
def test_go_batch_call_shapes(dh, oracle):
    """The exact C calls of INTEGRATION.md §2.4 against the oracle. Scheme.VerifyBeacons: dh_verify_batch over host
    buffers built as the Go code builds them — a chained window whose previous signatures have the lengths a trimmed
    store yields (the 32-byte genesis seed, 96-byte signatures, an empty and a 100-byte corrupted record), packed at
    stride = max(4, the longest rounded up to 4) with a u32 length per round, and a wrong-length signature replaced by
    an all-zero record (kyber rejects it); verdict bytes only (rand_out NULL, seed 0). RecoverBatch: dh_recover_batch
    with the wrong-length partial records dropped, the messages back to back, u32 offsets per round and one zero
    record of padding. Each verdict / recovered signature equals the oracle's (kyber restated)."""
    import ctypes
    import chainsynth
    from drand_amd import _lib
    lib = _lib.load()
    s = dh.scheme_from_name(CHAINED)
    sk = _secret(b"go-shapes")
    pk = s.public_key(sk)
    n = 40
    genesis = hashlib.sha256(b"drandhip-genesis").digest()
    sigs = chainsynth.sign_chain(s, sk, 1, n, genesis, [], np.random.default_rng(2))
    recs = [(r + 1, sigs[r].tobytes(), genesis if r == 0 else sigs[r - 1].tobytes()) for r in range(n)]
    recs[7] = (8, recs[7][1], b"")                           # empty previous record
    recs[12] = (13, recs[12][1], bytes(range(100)))          # corrupted 100-byte record
    recs[20] = (21, recs[20][1][:-1], recs[20][2])           # wrong-length signature
    recs[30] = (31, recs[31][1], recs[30][2])                # another round's signature
    stride = 4
    for _, _, p in recs:
        stride = max(stride, (len(p) + 3) & ~3)
    rounds = np.array([r for r, _, _ in recs], dtype=np.uint64)
    sbuf = np.zeros((n, 96), np.uint8)
    pbuf = np.zeros((n, stride), np.uint8)
    plen = np.zeros(n, np.uint32)
    for i, (_, sg, p) in enumerate(recs):
        if len(sg) == 96:
            sbuf[i] = np.frombuffer(sg, np.uint8)
        pbuf[i, :len(p)] = np.frombuffer(p, np.uint8)
        plen[i] = len(p)
    verdict = np.zeros(n, np.uint8)
    rc = lib.dh_verify_batch(s.id, pk, len(pk), rounds.ctypes.data, sbuf.ctypes.data, 96, pbuf.ctypes.data, stride,
                             plen.ctypes.data, n, verdict.ctypes.data, None, 0)
    assert rc == 0, _lib.last_error()
    want = [len(sg) == 96 and oracle.verify_beacon(CHAINED, pk, r, sg, p) for r, sg, p in recs]
    assert verdict.astype(bool).tolist() == want
    assert [i + 1 for i in range(n) if not want[i]] == [8, 13, 21, 31]
    # RecoverBatch
    name = "pedersen-bls-unchained"
    u = dh.scheme_from_name(name)
    t, nn, nr = 5, 9, 6
    coeffs, commits = _dealer(u, t, b"go-recover")
    rr = np.arange(50, 50 + nr, dtype=np.uint64)
    shares = {i: u.sign_beacons(_share(coeffs, i), rr) for i in range(nn)}
    msgs = [u.digest_beacon(int(r)) for r in rr]
    parts = []
    for j in range(nr):
        ps = [i.to_bytes(2, "big") + shares[i][j].tobytes() for i in ((j + k) % nn for k in range(t + 1))]
        if j == 2:
            ps.insert(0, ps[1][:-4])                         # wrong length: dropped before the call
        if j == 4:
            ps = ps[:t - 1] + [ps[t][:50]]                   # t - 1 well-sized: not enough good shares
        parts.append(ps)
    rec = 98
    raw, off = b"", [0]
    for ps in parts:
        raw += b"".join(p for p in ps if len(p) == rec)
        off.append(len(raw) // rec)
    raw += bytes(rec)
    offa = np.array(off, dtype=np.uint32)
    rawa = np.frombuffer(raw, np.uint8).copy()
    ma = np.frombuffer(b"".join(msgs), np.uint8).copy()
    out = np.zeros((nr, 96), np.uint8)
    st = np.zeros(nr, np.uint8)
    rc = lib.dh_recover_batch(u.id, b"".join(commits), t, nn, ma.ctypes.data, rawa.ctypes.data, offa.ctypes.data, nr,
                              out.ctypes.data, st.ctypes.data)
    assert rc == 0, _lib.last_error()
    for j in range(nr):
        w = oracle.recover(name, commits, t, nn, msgs[j], [p for p in parts[j] if len(p) == rec])
        assert (w is not None) == (st[j] == 1), j
        if w is not None:
            assert out[j].tobytes() == w, j
    assert st.tolist() == [1, 1, 1, 1, 0, 1]
