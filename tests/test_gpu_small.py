"""The small-batch path (drandhip.cpp verify_small): the drop-in's one-beacon calls — VerifyBeacon from the gossip
validator (/root/reference/lp2p/client/validator.go:62) and the client (client/verify.go:192), VerifyRecovered from the
aggregator (chain/beacon/chainstore.go:207) — and every batch of at most DRANDHIP_SMALL_N (64) rounds: per-round
2-pairing checks, no MSM. Verdicts and randomness must equal the batch path's and the oracle's bit for bit.

Also the G2 group check with the cofactor clearing inside the pairing program (k_vm_pairing_c, NP2C) on the branches a
real batch never reaches: A at infinity with B finite, B at infinity with A finite, and a B whose cleared
point is the identity (a small-order point of E'(Fp2): [h_eff] kills the whole cofactor), driven through
dh_check_partials with hand-built records and checked against bls_py's pairing and the one-lane path (DRANDHIP_NP2C=0).
"""
import ctypes
import hashlib
import json
import os
import random
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCHEMES = ["pedersen-bls-chained", "pedersen-bls-unchained", "bls-unchained-on-g1", "bls-unchained-g1-rfc9380"]
R_ORDER = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
SMALL_N = 64


@pytest.fixture(scope="module")
def dh():
    import torch
    import drand_amd
    from drand_amd import _lib
    torch.zeros(1, device="cuda")
    lib = _lib.load()
    assert lib.dh_init(0) == 0, _lib.last_error()
    return drand_amd


def _sk(tag):
    return (int.from_bytes(hashlib.sha256(tag).digest(), "big") % R_ORDER).to_bytes(32, "big")


def _corrupt(s, sigs, rounds, sk, prevs):
    """A batch with every fault class of the negatives fixture: bit flips, another round's signature, a signature of
    another key, an on-curve non-subgroup point (G1: a point of E(Fp) of order 3 ... via the oracle's decoder is not
    needed: a flipped x bit mostly gives off-curve or non-subgroup points), the point at infinity, a wrong prefix."""
    bad = sigs.copy()
    n = len(bad)
    bad[1, 20] ^= 0x01                      # bit flip (decodes to another point or fails)
    bad[3] = sigs[4]                        # another round's signature
    other = s.sign_beacons(_sk(b"other-key"), rounds[5:6], prevs[5:6] if prevs is not None else None)
    bad[5] = other[0]                       # another key's signature
    bad[7] = 0
    bad[7, 0] = 0xc0                        # the compressed point at infinity (rejected)
    bad[9, 0] ^= 0x20                       # sign bit flipped: -sigma
    bad[11, 0] &= 0x7f                      # compression flag cleared
    bad[n - 1, s.sig_len - 1] ^= 0x80       # last round, last byte
    return bad


@pytest.mark.parametrize("scheme", SCHEMES)
def test_small_path_matches_batch_path_and_oracle(dh, scheme, oracle):
    s = dh.scheme_from_name(scheme)
    sk = _sk(b"small-" + scheme.encode())
    pk = s.public_key(sk)
    n = SMALL_N
    rounds = np.arange(500, 500 + n + 1, dtype=np.uint64)
    prevs = None
    if s.chained:
        rng = np.random.default_rng(5)
        prevs = rng.integers(0, 256, (n + 1, 96), dtype=np.uint8)
    sigs = s.sign_beacons(sk, rounds, prevs)
    bad = _corrupt(s, sigs, rounds, sk, prevs)
    # n rounds: the small path; the same rounds plus one: the batch path (RLC + bisection)
    v_small, r_small = s.verify_beacons(pk, rounds[:n], bad[:n], prevs[:n] if prevs is not None else None, seed=3)
    v_batch, r_batch = s.verify_beacons(pk, rounds, bad, prevs, seed=4)
    assert np.array_equal(v_small, v_batch[:n])
    assert np.array_equal(r_small, r_batch[:n])
    want = [oracle.verify_beacon(scheme, pk, int(rounds[i]), bad[i].tobytes(),
                                 prevs[i].tobytes() if prevs is not None else b"") for i in range(n)]
    assert v_small.tolist() == want
    assert not all(want) and sum(want) >= n - 10
    for i in range(n):
        assert r_small[i].tobytes() == hashlib.sha256(bad[i].tobytes()).digest()
    # one round at a time (VerifyBeacon), valid and faulty
    for i in (0, 1, 3, 5, 7, 9, 11, n - 1):
        b = dh.Beacon(int(rounds[i]), bad[i].tobytes(), prevs[i].tobytes() if prevs is not None else b"")
        if want[i]:
            s.verify_beacon(b, pk)
        else:
            with pytest.raises(dh.SchemeError):
                s.verify_beacon(b, pk)


@pytest.mark.parametrize("scheme", SCHEMES)
def test_small_verify_recovered(dh, scheme, oracle):
    """VerifyRecovered one at a time and as a small batch, against the oracle's Verify of the 32-byte digest."""
    s = dh.scheme_from_name(scheme)
    sk = _sk(b"rec-" + scheme.encode())
    pk = s.public_key(sk)
    rounds = np.arange(1, 9, dtype=np.uint64)
    prevs = np.full((8, 96), 7, np.uint8) if s.chained else None
    sigs = s.sign_beacons(sk, rounds, prevs)
    msgs = [s.digest_beacon(int(r), prevs[k].tobytes() if prevs is not None else b"") for k, r in enumerate(rounds)]
    bad = sigs.copy()
    bad[2, 10] ^= 4
    bad[5] = sigs[6]
    v = s.verify_recovered_batch(pk, msgs, bad)
    want = [oracle.verify(scheme, pk, msgs[k], bad[k].tobytes()) for k in range(8)]
    assert v.tolist() == want and want.count(False) == 2
    for k in range(8):
        if want[k]:
            s.verify_recovered(pk, msgs[k], bad[k].tobytes())
        else:
            with pytest.raises(dh.SchemeError):
                s.verify_recovered(pk, msgs[k], bad[k].tobytes())


def test_small_device_entry_stats_and_unchecked_lengths(dh, oracle):
    """dh_verify_batch_device below the threshold: stats = {0 levels, 0 failed groups, n leaves, rejected}; chained
    lengths in device memory (not checked by the host) keep the hash kernels behind the signature kernels, and a
    length beyond the record stride rejects its round, as in the batch path."""
    import torch
    from drand_amd import _lib
    lib = _lib.load()
    s = dh.scheme_from_name("pedersen-bls-chained")
    sk = _sk(b"dev-small")
    pk = s.public_key(sk)
    n = 12
    rounds = np.arange(40, 40 + n, dtype=np.uint64)
    prevs = np.random.default_rng(9).integers(0, 256, (n, 96), dtype=np.uint8)
    lens = np.full(n, 96, np.uint32)
    lens[4] = 60
    sigs = s.sign_beacons(sk, rounds, prevs, lens)
    bad = sigs.copy()
    bad[2, 30] ^= 1
    lens_dev = lens.copy()
    lens_dev[8] = 200  # longer than the 96-byte stride: rejected
    dev = torch.device("cuda")
    d_r = torch.from_numpy(rounds.view(np.int64)).to(dev)
    d_s = torch.from_numpy(bad).to(dev)
    d_p = torch.from_numpy(np.concatenate([prevs.reshape(-1), np.zeros(4, np.uint8)])).to(dev)
    d_l = torch.from_numpy(lens_dev.view(np.int32)).to(dev)
    d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
    d_rand = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
    stats = (ctypes.c_uint64 * 4)()
    torch.cuda.synchronize()
    rc = lib.dh_verify_batch_device(s.id, pk, len(pk), ctypes.c_void_p(d_r.data_ptr()), ctypes.c_void_p(d_s.data_ptr()),
                                    96, ctypes.c_void_p(d_p.data_ptr()), 96, ctypes.c_void_p(d_l.data_ptr()), n,
                                    ctypes.c_void_p(d_v.data_ptr()), ctypes.c_void_p(d_rand.data_ptr()), 5, None, stats)
    assert rc == 0, _lib.last_error()
    v = d_v.cpu().numpy().astype(bool)
    want = [oracle.verify_beacon(s.name, pk, int(rounds[i]), bad[i].tobytes(), prevs[i, :lens[i]].tobytes()) for i in range(n)]
    want[8] = False
    assert v.tolist() == want and want.count(False) == 2
    assert list(stats) == [0, 0, n, 2]
    rr = d_rand.cpu().numpy()
    assert all(rr[i].tobytes() == hashlib.sha256(bad[i].tobytes()).digest() for i in range(n))


# ---------------------------------------------------------------- NP2C branches
P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
H2 = 0x5d543a95414e7f1091d50792876a202cd91de4547085abaa68a205b2e5a7ddfa628f1cb4d9e82ef21537e293a6691ae1616ec6e786f0c70cf1c38e31c7238e5


def _words(v):
    m = v * (1 << 384) % P
    return [(m >> (32 * i)) & 0xffffffff for i in range(12)]


def _jac_words(B, pt, rng):
    """a G2 point (affine pair of Fp2, or None) as 72 Jacobian words with a random Z (Z = 0 for the identity)"""
    if pt is None:
        return [0] * 72
    z = (rng.randrange(1, P), rng.randrange(P))
    z2 = B.f2mul(z, z)
    x, y = B.f2mul(pt[0], z2), B.f2mul(pt[1], B.f2mul(z2, z))
    out = []
    for c in (x, y, z):
        out += _words(c[0]) + _words(c[1])
    return out


def _np2c_cases():
    """(name, A, B, want): A = the signature sum, B = the uncleared hash sum (affine G2 points or None), want = kilic's
    e(pk, [h_eff] B) e(-g1, A) == 1 with pairs at infinity skipped."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bls_py as B
    rng = random.Random(13)
    sk = rng.randrange(2, B.R)
    h = B.iso_map_g2(B.sswu_g2((rng.randrange(P), rng.randrange(P))))
    hh = B.ec_mul(B.FP2, h, B.H_EFF_G2)
    sig = B.ec_mul(B.FP2, hh, sk)
    r2 = B.iso_map_g2(B.sswu_g2((rng.randrange(P), rng.randrange(P))))
    # the 13-part of E'(Fp2) is Z13 x Z13 (13^2 | h2): [h2 r / 13^2] R has order 13, and [h_eff] T = O (h2 | h_eff)
    t13 = B.ec_mul(B.FP2, r2, H2 * B.R // 169)
    assert t13 is not None and B.ec_mul(B.FP2, t13, 13) is None
    pk = B.ec_mul(B.FP, B.G1_GEN, sk)
    cases = [
        ("clean", sig, h, True),
        ("A_inf_B_finite", None, h, False),                    # f == 1: the exact one-lane path
        ("A_inf_B_small_order", None, t13, True),              # f == 1, [h]B = O: both pairs skipped
        ("B_inf_A_finite", sig, None, False),                  # f == 2: NP1 on the signature pair
        ("B_inf_A_inf", None, None, True),                     # f == 0: the empty product
        ("B_small_order_A_finite", sig, t13, False),           # f == 3, cleared Z = 0: the exact path
        ("B_plus_torsion", sig, B.ec_add(B.FP2, h, t13), True),  # cleared [h](H + T) = [h] H
        ("wrong_sig", B.ec_add(B.FP2, sig, B.G2_GEN), h, False),
    ]
    return B, pk, cases


def _run_np2c_cases(records_hex, pk_hex):
    """dh_check_partials over each record (one rank's record each); returns the pass flags"""
    import torch
    from drand_amd import _lib
    lib = _lib.load()
    out = []
    for rec in records_hex:
        raw = np.frombuffer(bytes.fromhex(rec), np.uint8).copy()
        d = torch.from_numpy(raw).to("cuda")
        torch.cuda.synchronize()
        ok = ctypes.c_int(-1)
        pk = bytes.fromhex(pk_hex)
        rc = lib.dh_check_partials(1, pk, len(pk), ctypes.c_void_p(d.data_ptr()), 1, ctypes.byref(ok))
        assert rc == 0, _lib.last_error()
        out.append(ok.value)
    return out


def test_np2c_group_check_branches(dh):
    from drand_amd import _lib
    lib = _lib.load()
    B, pk, cases = _np2c_cases()
    rng = random.Random(21)
    assert lib.dh_partial_bytes(1) == (72 * 2 + 4) * 4
    recs = []
    for _, a, b, _ in cases:
        w = _jac_words(B, a, rng) + _jac_words(B, b, rng) + [0, 0, 0, 0]
        recs.append(np.array(w, dtype=np.uint32).tobytes().hex())
    pk_b = B.g1_compress(pk).hex()
    got = _run_np2c_cases(recs, pk_b)
    assert got == [int(c[3]) for c in cases], list(zip([c[0] for c in cases], got))
    # the same records through the one-lane clearing path (k_vm_prep_groups<fp2> + k_vm_pairing) in a fresh process
    env = dict(os.environ, DRANDHIP_NP2C="0")
    code = ("import sys, json; sys.path.insert(0, %r); sys.path.insert(0, %r); import torch; torch.zeros(1, device='cuda');"
            "from drand_amd import _lib; assert _lib.load().dh_init(0) == 0;"
            "import test_gpu_small as t; print(json.dumps(t._run_np2c_cases(%r, %r)))") % (
        ROOT, os.path.join(ROOT, "tests"), recs, pk_b)
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    assert json.loads(p.stdout.strip().splitlines()[-1]) == got


# ---------------------------------------------------------------- DH_EBUSY from a blocking call
_BUSY_CHILD = r"""
import ctypes, sys
sys.path.insert(0, %(root)r)
import numpy as np, torch
torch.zeros(1, device="cuda")
import drand_amd
from drand_amd import _lib
lib = _lib.load()
assert lib.dh_init(0) == 0
s = drand_amd.scheme_from_name("bls-unchained-g1-rfc9380")
sk = bytes(31) + b"\x05"
pk = s.public_key(sk)
rounds = np.arange(1, 101, dtype=np.uint64)
sigs = s.sign_beacons(sk, rounds)
d_r = torch.from_numpy(rounds.view(np.int64)).cuda()
d_s = torch.from_numpy(sigs).cuda()
d_v = torch.zeros(100, dtype=torch.uint8, device="cuda")
part = torch.zeros(lib.dh_partial_bytes(s.id), dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
b = ctypes.c_void_p()
ptr = lambda t: ctypes.c_void_p(t.data_ptr())
assert lib.dh_batch_begin(s.id, pk, len(pk), ptr(d_r), ptr(d_s), 48, None, 0, None, 100, ptr(d_v), None, 1, None,
                          ctypes.byref(b), ptr(part)) == 0, _lib.last_error()
# the only worker is held by the node batch: a blocking call waits DRANDHIP_LEASE_TIMEOUT_MS, then DH_EBUSY
try:
    s.verify_beacons(pk, rounds[:3], sigs[:3])
    print("NOT-BUSY")
except drand_amd.DeviceBusy as e:
    print("BUSY", e)
assert lib.dh_batch_finish(b, 1, None) >= 0, _lib.last_error()
v, _ = s.verify_beacons(pk, rounds[:3], sigs[:3])
print("AFTER", bool(v.all()))
"""


def test_blocking_call_busy_then_succeeds():
    env = dict(os.environ, DRANDHIP_MAX_WORKERS="1", DRANDHIP_LEASE_TIMEOUT_MS="200")
    p = subprocess.run([sys.executable, "-c", _BUSY_CHILD % {"root": ROOT}], env=env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    out = p.stdout.split("\n")
    assert any(line.startswith("BUSY libdrandhip error -6") for line in out), p.stdout
    assert "AFTER True" in out, p.stdout
