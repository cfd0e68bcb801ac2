"""GPU parity: libdrandhip (gfx950 kernels, through the C ABI) against the CPU oracle, the reference's
known-answer tests and the committed golden fixtures. Bit-exact verdicts and randomness are required.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from kat import VERIFY_KATS

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
SCHEMES = ["pedersen-bls-chained", "pedersen-bls-unchained", "bls-unchained-on-g1", "bls-unchained-g1-rfc9380"]


@pytest.fixture(scope="module")
def dh():
    import torch
    import drand_amd
    from drand_amd import _lib
    # torch carries its own HIP runtime: bring it up before the library's runtime has created its streams
    torch.zeros(1, device="cuda")
    lib = _lib.load()
    assert lib.dh_init(0) == 0, _lib.last_error()
    return drand_amd


def _prev_array(prevs):
    return [bytes.fromhex(p) if isinstance(p, str) else p for p in prevs]


@pytest.mark.parametrize("kat", VERIFY_KATS, ids=[k[0] + "-" + str(k[2]) for k in VERIFY_KATS])
def test_reference_kats(dh, kat):
    scheme, pk, rnd, sig, prev = kat
    s = dh.scheme_from_name(scheme)
    s.verify_beacon(dh.Beacon(rnd, sig, prev), pk)  # raises on failure
    with pytest.raises(dh.SchemeError):
        s.verify_beacon(dh.Beacon(rnd + 1, sig, prev), pk)
    v, rand = s.verify_beacons(pk, [rnd, rnd + 1], np.frombuffer(sig * 2, np.uint8).reshape(2, -1),
                               [prev, prev] if s.chained else None, seed=7)
    assert v.tolist() == [True, False]
    assert rand[0].tobytes() == hashlib.sha256(sig).digest()


@pytest.mark.parametrize("scheme", SCHEMES)
def test_golden_chain(dh, scheme):
    c = json.load(open(os.path.join(GOLD, "chains.json")))[scheme]
    s = dh.scheme_from_name(scheme)
    sigs = np.array([np.frombuffer(bytes.fromhex(x), np.uint8) for x in c["sigs"]])
    v, rand = s.verify_beacons(bytes.fromhex(c["pk"]), c["rounds"], sigs,
                               _prev_array(c["prevs"]) if s.chained else None, seed=1)
    assert v.tolist() == c["valid"]
    assert [r.tobytes().hex() for r in rand] == c["randomness"]


@pytest.mark.parametrize("scheme", SCHEMES)
def test_golden_negatives(dh, scheme, oracle):
    c = json.load(open(os.path.join(GOLD, "negatives.json")))[scheme]
    s = dh.scheme_from_name(scheme)
    pk = bytes.fromhex(c["pk"])
    cases = c["cases"]
    sigs = np.array([np.frombuffer(bytes.fromhex(x["sig"]), np.uint8) for x in cases])
    rounds = [x["round"] for x in cases]
    prevs = [bytes.fromhex(x["prev"]) for x in cases] if s.chained else None
    v, _ = s.verify_beacons(pk, rounds, sigs, prevs, seed=3)
    assert v.tolist() == [x["valid"] for x in cases], [x["name"] for x in cases]
    for x in cases:  # single-beacon path
        b = dh.Beacon(x["round"], bytes.fromhex(x["sig"]), bytes.fromhex(x["prev"]))
        if x["valid"]:
            s.verify_beacon(b, pk)
        else:
            with pytest.raises(dh.SchemeError):
                s.verify_beacon(b, pk)


def test_chained_replay_faulty_rounds(dh):
    """CheckPastBeacons semantics (chain/beacon/sync_manager.go:170-235): prev = stored sig of round-1."""
    rp = json.load(open(os.path.join(GOLD, "replay.json")))
    s = dh.scheme_from_name("pedersen-bls-chained")
    stored = [bytes.fromhex(x) for x in rp["stored_sigs"]]
    prevs = [bytes.fromhex(rp["genesis_seed"])] + stored[:-1]
    v, _ = s.verify_beacons(bytes.fromhex(rp["pk"]), rp["rounds"], np.array([np.frombuffer(x, np.uint8) for x in stored]),
                            prevs, seed=11)
    assert [r for r, ok in zip(rp["rounds"], v) if not ok] == rp["faulty"]


@pytest.mark.parametrize("scheme", SCHEMES)
def test_device_signer_matches_oracle(dh, scheme, oracle):
    c = json.load(open(os.path.join(GOLD, "chains.json")))[scheme]
    s = dh.scheme_from_name(scheme)
    sk = bytes.fromhex(c["sk"])
    assert s.public_key(sk).hex() == c["pk"]
    sigs = s.sign_beacons(sk, c["rounds"], _prev_array(c["prevs"]) if s.chained else None)
    assert [x.tobytes().hex() for x in sigs] == c["sigs"]


@pytest.mark.parametrize("scheme", ["bls-unchained-g1-rfc9380", "pedersen-bls-unchained"])
def test_large_batch_with_corruption(dh, scheme, oracle):
    """n rounds signed on the device, a seeded set corrupted: exactly those rounds are rejected; the
    bisection levels the expected-cost ladder picks run. Corrupted rows are cross-checked on the oracle."""
    n = 20000 if scheme == "bls-unchained-g1-rfc9380" else 6000
    s = dh.scheme_from_name(scheme)
    sk = hashlib.sha256(b"large-" + scheme.encode()).digest()
    rounds = np.arange(1, n + 1, dtype=np.uint64)
    sigs = s.sign_beacons(sk, rounds)
    pk = s.public_key(sk)
    v, rand = s.verify_beacons(pk, rounds, sigs, seed=5)
    assert v.all()
    rng = np.random.default_rng(12345)
    bad = np.sort(rng.choice(n, size=9, replace=False))
    sigs2 = sigs.copy()
    for k, i in enumerate(bad):
        if k % 3 == 0:
            sigs2[i] = sigs[(i + 1) % n]              # valid point, wrong signature
        elif k % 3 == 1:
            sigs2[i, s.sig_len // 2] ^= 0x04          # bit flip (usually not on the curve)
        else:
            sigs2[i, 0] ^= 0x20                       # negated point
    v2, rand2 = s.verify_beacons(pk, rounds, sigs2, seed=6)
    assert np.flatnonzero(~v2).tolist() == bad.tolist()
    for i in bad[:3]:
        assert not oracle.verify_beacon(scheme, pk, int(rounds[i]), sigs2[i].tobytes())
    for i in [0, n // 2, n - 1]:
        assert rand2[i].tobytes() == hashlib.sha256(sigs2[i].tobytes()).digest()


def test_dense_corruption_every_window_geometry(dh):
    """131 195 quicknet rounds (level 0 at c = 13, whose top window must stay populated) with 0.5% corrupted
    rounds in three classes, then a small batch where EVERY round is bad: the signed-digit MSM runs at every
    window geometry the expected-cost ladder picks (c = 13 at level 0, 8 for 1024-round groups, 5/4/3 for
    the small ones) and the rejected set is exactly the corrupted one."""
    s = dh.scheme_from_name("bls-unchained-g1-rfc9380")
    sk = hashlib.sha256(b"dense").digest()
    n = (1 << 17) + 123
    rounds = np.arange(7, n + 7, dtype=np.uint64)
    sigs = s.sign_beacons(sk, rounds)
    pk = s.public_key(sk)
    rng = np.random.default_rng(777)
    bad = np.sort(rng.choice(n, size=n // 200, replace=False))
    sigs2 = sigs.copy()
    for k, i in enumerate(bad):
        if k % 3 == 0:
            sigs2[i] = sigs[(i + 5) % n]
        elif k % 3 == 1:
            sigs2[i, 17] ^= 0x10
        else:
            sigs2[i, 0] ^= 0x20
    v, rand = s.verify_beacons(pk, rounds, sigs2, seed=11)
    assert np.flatnonzero(~v).tolist() == bad.tolist()
    for i in [0, int(bad[0]), n - 1]:
        assert rand[i].tobytes() == hashlib.sha256(sigs2[i].tobytes()).digest()
    # again: the worker's last bisection saw dense faults, so this batch skips level 0 and starts at 256-round
    # groups (drandhip.cpp skip0); then a clean batch on the dense hint, whose 256-groups all pass
    v, _ = s.verify_beacons(pk, rounds, sigs2, seed=13)
    assert np.flatnonzero(~v).tolist() == bad.tolist()
    s.verify_beacons(pk, rounds, sigs2, seed=14)
    v, _ = s.verify_beacons(pk, rounds, sigs, seed=15)
    assert v.all()
    m = 300
    sigs3 = np.ascontiguousarray(np.roll(sigs[:m], 1, axis=0))  # every signature belongs to another round
    v3, _ = s.verify_beacons(pk, rounds[:m], sigs3, seed=12)
    assert not v3.any()


def test_seed_independence(dh):
    c = json.load(open(os.path.join(GOLD, "negatives.json")))["bls-unchained-g1-rfc9380"]
    s = dh.scheme_from_name("bls-unchained-g1-rfc9380")
    sigs = np.array([np.frombuffer(bytes.fromhex(x["sig"]), np.uint8) for x in c["cases"]])
    rounds = [x["round"] for x in c["cases"]]
    out = [s.verify_beacons(bytes.fromhex(c["pk"]), rounds, sigs, seed=sd)[0].tolist() for sd in (0, 1, 99)]
    assert out[0] == out[1] == out[2]


def test_bad_key_and_arguments(dh):
    s = dh.scheme_from_name("bls-unchained-g1-rfc9380")
    with pytest.raises(dh.SchemeError):
        s.verify_beacons(b"\x00" * 96, [1], np.zeros((1, 48), np.uint8))
    with pytest.raises(dh.SchemeError):
        s.verify_beacons(b"\x00" * 95, [1], np.zeros((1, 48), np.uint8))
    v, _ = s.verify_beacons(VERIFY_KATS[3][1], [], np.zeros((0, 48), np.uint8))
    assert len(v) == 0


@pytest.mark.parametrize("scheme", ["pedersen-bls-unchained", "bls-unchained-g1-rfc9380"])
def test_recover_golden(dh, scheme):
    """tbls Recover (chain/beacon/chainstore.go:202) vs the oracle: invalid partials skipped in arrival
    order, duplicate / out-of-range indices, too few valid partials -> error."""
    c = json.load(open(os.path.join(GOLD, "recover.json")))[scheme]
    s = dh.scheme_from_name(scheme)
    commits = [bytes.fromhex(x) for x in c["commits"]]
    msgs = [bytes.fromhex(x["msg"]) for x in c["cases"]]
    parts = [[bytes.fromhex(p) for p in x["partials"]] for x in c["cases"]]
    sigs, ok = s.recover_batch(commits, c["t"], c["n"], msgs, parts)
    for k, x in enumerate(c["cases"]):
        if x["expected"] is None:
            assert not ok[k], k
        else:
            assert ok[k], k
            assert sigs[k].tobytes().hex() == x["expected"], k
    with pytest.raises(dh.SchemeError):
        s.recover(commits, msgs[3], parts[3], c["t"], c["n"])
    assert s.recover(commits, msgs[0], parts[0], c["t"], c["n"]).hex() == c["cases"][0]["expected"]


def test_recover_threshold_property(dh):
    """n = 16 signers, t = 9, 40 rounds, random signer subsets per round (partials signed on the device):
    the recovered signature equals [f(0)] H(m) and verifies under the group key (dealer pattern
    /root/reference/chain/beacon/node_test.go:60-109)."""
    import random
    s = dh.scheme_from_name("pedersen-bls-unchained")
    R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
    t, n, nr = 9, 16, 40
    coeffs = [int.from_bytes(hashlib.sha256(b"prop-%d" % j).digest(), "big") % R for j in range(t)]
    commits = [s.public_key(cf.to_bytes(32, "big")) for cf in coeffs]
    rounds = np.arange(500, 500 + nr, dtype=np.uint64)
    shares = []
    for i in range(n):
        x, acc = i + 1, 0
        for cf in reversed(coeffs):
            acc = (acc * x + cf) % R
        shares.append(s.sign_beacons(acc.to_bytes(32, "big"), rounds))
    rng = random.Random(7)
    parts = []
    for j in range(nr):
        ids = rng.sample(range(n), t + rng.randrange(0, 3))
        parts.append([i.to_bytes(2, "big") + shares[i][j].tobytes() for i in ids])
    msgs = [s.digest_beacon(int(r)) for r in rounds]
    sigs, ok = s.recover_batch(commits, t, n, msgs, parts)
    assert ok.all()
    want = s.sign_beacons(coeffs[0].to_bytes(32, "big"), rounds)
    assert np.array_equal(sigs, want)
    v, _ = s.verify_beacons(commits[0], rounds, sigs, seed=2)
    assert v.all()


def test_check_past_beacons_batch_caller(dh):
    """SyncManager.CheckPastBeacons semantics (chain/beacon/sync_manager.go:170-235) over a trimmed store
    (chain/boltdb/trimmed.go:156-193); TestDrandCheckChain (core/drand_test.go:1105-1111) expects 2 faulty
    rounds for a deleted chained beacon and 1 for unchained."""
    from drand_amd.sync import TrimmedMemStore, check_past_beacons
    chains = json.load(open(os.path.join(GOLD, "chains.json")))
    for name, per_delete in (("pedersen-bls-chained", [4, 5]), ("pedersen-bls-unchained", [4])):
        c = chains[name]
        s = dh.scheme_from_name(name)
        st = TrimmedMemStore(s.chained)
        st.put(0, bytes.fromhex(c["prevs"][0]) if s.chained else b"\x00" * 32)  # genesis
        for r, sig in zip(c["rounds"], c["sigs"]):
            st.put(r, bytes.fromhex(sig))
        pk = bytes.fromhex(c["pk"])
        seen = []
        assert check_past_beacons(st, s, pk, 24, cb=lambda i, u: seen.append(i), window=7) == []
        assert seen == list(range(1, 25))
        st.delete(4)
        assert check_past_beacons(st, s, pk, 24, window=5) == per_delete
        st.put(10, bytes.fromhex(c["sigs"][8]))  # round 10 now stores round 9's signature
        want = sorted(per_delete + ([10, 11] if s.chained else [10]))
        assert check_past_beacons(st, s, pk, 24, window=3) == want
        assert check_past_beacons(st, s, pk, 9) == [x for x in per_delete if x <= 9]


def test_readers_and_client_walk_on_device(dh, tmp_path):
    """Chain readers feeding the device path: a bbolt trimmed file (tests/boltwrite.py) replayed by
    check_past_beacons, and the batched strict-client trust walk (client/verify.go:109-168)."""
    from boltwrite import write_bolt
    from drand_amd.chain import Info
    from drand_amd.client import BatchVerifyingClient, ClientError
    from drand_amd.store import BoltTrimmedStore
    from drand_amd.sync import check_past_beacons
    c = json.load(open(os.path.join(GOLD, "chains.json")))["pedersen-bls-chained"]
    s = dh.scheme_from_name("pedersen-bls-chained")
    sigs = {r: bytes.fromhex(x) for r, x in zip(c["rounds"], c["sigs"])}
    kv = {int(0).to_bytes(8, "big"): bytes.fromhex(c["prevs"][0])}
    kv.update({int(r).to_bytes(8, "big"): sg for r, sg in sigs.items() if r != 7})
    path = str(tmp_path / "chain.db")
    write_bolt(path, b"beacons", kv)
    assert check_past_beacons(BoltTrimmedStore(path, True), s, bytes.fromhex(c["pk"]), 1000, window=8) == [7, 8]
    info = Info(bytes.fromhex(c["pk"]), 30, s.name, 0, bytes.fromhex(c["prevs"][0]))
    cl = BatchVerifyingClient(info, s, get_signature=lambda r: sigs[r], strict=True)
    cl.point_of_trust = (3, sigs[3])
    assert cl.trusted_previous_signature(20) == sigs[19] and cl.point_of_trust == (19, sigs[19])
    bad = dict(sigs)
    bad[15] = sigs[16]
    cl2 = BatchVerifyingClient(info, s, get_signature=lambda r: bad[r], strict=True)
    cl2.point_of_trust = (11, sigs[11])
    with pytest.raises(ClientError):
        cl2.trusted_previous_signature(20)


@pytest.mark.parametrize("scheme", ["pedersen-bls-unchained", "bls-unchained-g1-rfc9380"])
def test_verify_partials_and_recovered(dh, scheme, oracle):
    """Batch VerifyPartial (chain/beacon/node.go:150) per partial against the oracle's
    Verify(PubPoly.Eval(i), msg, sig), and VerifyRecovered (chainstore.go:207) on the golden recovered
    signatures, a swapped message and a wrong-length signature."""
    c = json.load(open(os.path.join(GOLD, "recover.json")))[scheme]
    s = dh.scheme_from_name(scheme)
    commits = [bytes.fromhex(x) for x in c["commits"]]
    msgs = [bytes.fromhex(x["msg"]) for x in c["cases"]]
    parts = [[bytes.fromhex(p) for p in x["partials"]] for x in c["cases"]]
    got = s.verify_partials_batch(commits, c["t"], c["n"], msgs, parts)
    n_bad = 0
    for j, ps in enumerate(parts):
        for k, p in enumerate(ps):
            i = s.index_of(p)
            want = i < c["n"] and oracle.verify(scheme, oracle.pubpoly_eval(scheme, commits, i), msgs[j], p[2:])
            assert bool(got[j][k]) == bool(want), (j, k)
            n_bad += not want
    assert n_bad > 0
    good = [(bytes.fromhex(x["msg"]), bytes.fromhex(x["expected"])) for x in c["cases"] if x["expected"]]
    for m, sig in good:
        s.verify_recovered(commits[0], m, sig)
    with pytest.raises(dh.SchemeError):
        s.verify_recovered(commits[0], good[1][0], good[0][1])
    with pytest.raises(dh.SchemeError):
        s.verify_recovered(commits[0], good[0][0], good[0][1][:-1])
    ms = [m for m, _ in good] + [good[1][0]]
    sg = np.array([np.frombuffer(x, np.uint8) for _, x in good] + [np.frombuffer(good[0][1], np.uint8)])
    assert s.verify_recovered_batch(commits[0], ms, sg, seed=4).tolist() == [True] * len(good) + [False]


def test_one_lane_pairing_path(dh):
    """The one-lane tower pairing (k_check.hip, DRANDHIP_LANE_PAIRING=1) stays correct: same verdicts as the
    fixtures on the negative sets (group checks fail, bisection reaches per-round leaves); the child process also
    runs tbls Recover as its very first library call."""
    import subprocess
    import sys
    env = dict(os.environ, DRANDHIP_LANE_PAIRING="1")
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "lane_pairing_check.py")],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    got = json.loads(r.stdout.strip().splitlines()[-1])
    rc = json.load(open(os.path.join(GOLD, "recover.json")))["pedersen-bls-unchained"]
    assert got.pop("recover") == [x["expected"] for x in rc["cases"]]
    neg = json.load(open(os.path.join(GOLD, "negatives.json")))
    for name, v in got.items():
        assert v == [x["valid"] for x in neg[name]["cases"]], name


@pytest.mark.parametrize("skip0", ["1", "0"])
@pytest.mark.parametrize("ladder", ["4096,256,16,2", "64"])
def test_fixed_bisection_ladder(dh, ladder, skip0):
    """The bisection is exact whatever the group sizes: a fixed ladder (DRANDHIP_BISECT, the r01 sizes with the
    c = 10 window geometry, and a single level of 64 before leaves) rejects exactly the corrupted rounds, as the
    default expected-cost ladder does in the tests above. The second quicknet call comes after a dense first one, so
    with skip0 "1" (the default) it starts at the ladder's first size without a level-0 check, with "0" it runs level 0
    first. The G2 statistics pin the sums themselves: exactly one failing group per level."""
    import subprocess
    import sys
    env = dict(os.environ, DRANDHIP_BISECT=ladder, DRANDHIP_SKIP_LEVEL0=skip0)
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "fixed_ladder_check.py")],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    got = json.loads(r.stdout.strip().splitlines()[-1])
    assert got["rejected"] == got["expected"] == got["rejected_again"] and len(got["expected"]) == 200
    # G2 with one forged round: every level of the ladder fails exactly its group, leaves = the last size
    levels, failed, leaves, rejected = got["g2_stats"]
    last = int(ladder.split(",")[-1])
    assert got["g2_rejected"] == [1234] and rejected == 1
    assert levels >= 2 and failed == levels and leaves == last, got["g2_stats"]


def test_device_entry_stats(dh):
    """dh_verify_batch_device on HBM-resident inputs fills stats_out = {levels, groups_failed, leaf_rounds,
    rounds_rejected} (include/drandhip.h): rounds_rejected counts decode failures and failed leaves alike."""
    import ctypes
    import torch
    from drand_amd import _lib
    lib = _lib.load()
    s = dh.scheme_from_name("bls-unchained-g1-rfc9380")
    sk = hashlib.sha256(b"stats").digest()
    n = 5000
    rounds = np.arange(1, n + 1, dtype=np.uint64)
    sigs = s.sign_beacons(sk, rounds)
    pk = s.public_key(sk)
    sigs[10] = sigs[11]          # valid point, wrong round: fails its group, then its leaf
    sigs[4000, 0] ^= 0x20        # negated point: also a leaf failure
    sigs[2500, 5] ^= 0x01        # usually off the curve: rejected at decode, scalar 0
    dev = torch.device("cuda", 0)
    d_r = torch.from_numpy(rounds.view(np.int64)).to(dev)
    d_s = torch.from_numpy(sigs).to(dev)
    d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_rand = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
    stats = (ctypes.c_uint64 * 4)()
    rc = lib.dh_verify_batch_device(s.id, pk, len(pk), ctypes.c_void_p(d_r.data_ptr()), ctypes.c_void_p(d_s.data_ptr()),
                                    s.sig_len, None, 0, None, n, ctypes.c_void_p(d_v.data_ptr()),
                                    ctypes.c_void_p(d_rand.data_ptr()), 9, None, stats)
    assert rc == 0, _lib.last_error()
    torch.cuda.synchronize()
    v = d_v.cpu().numpy()
    assert np.flatnonzero(v == 0).tolist() == [10, 2500, 4000]
    assert stats[0] >= 2 and stats[1] >= 3 and stats[2] >= 2 and stats[3] == 3
    host_v, _ = s.verify_beacons(pk, rounds, sigs, seed=9)
    assert np.array_equal(host_v, v.astype(bool))
