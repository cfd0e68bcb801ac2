"""CPU: the oracle (test infrastructure) against the reference's known-answer tests and the golden
fixtures. Oracle pinning gate of the build plan."""
import hashlib
import json
import os

import pytest

from kat import SIGN_KAT, VERIFY_KATS, XMD_DST, XMD_KATS

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("kat", VERIFY_KATS, ids=[k[0] + "-" + str(k[2]) for k in VERIFY_KATS])
def test_verify_kats(oracle, kat):
    scheme, pk, rnd, sig, prev = kat
    assert oracle.verify_beacon(scheme, pk, rnd, sig, prev)
    # negative: wrong round must fail (pattern test/mock/grpcserver.go:175-177)
    assert not oracle.verify_beacon(scheme, pk, rnd + 1, sig, prev)


def test_sign_kat(oracle):
    sk, msg, want = SIGN_KAT
    assert oracle.sign("pedersen-bls-chained", sk, msg) == want


@pytest.mark.parametrize("msg,want", XMD_KATS)
def test_xmd_rfc9380(oracle, msg, want):
    assert oracle.expand_message_xmd(msg, XMD_DST, 32) == want


def test_fast_subgroup_agrees(oracle):
    """The endomorphism subgroup tests the GPU uses agree with kilic's r*P == O test on the KAT points."""
    for scheme, pk, _, sig, _ in VERIFY_KATS:
        g2sig = scheme in ("pedersen-bls-chained", "pedersen-bls-unchained")
        L = oracle.lib(True)
        fast = (L.or_decode(1 if g2sig else 0, sig), L.or_decode(0 if g2sig else 1, pk))
        L = oracle.lib(False)
        slow = (L.or_decode(1 if g2sig else 0, sig), L.or_decode(0 if g2sig else 1, pk))
        assert fast == slow == (1, 1)


def test_mainnet_chain_hash():
    """chain.Info.Hash (/root/reference/chain/info.go:48-67) reproduces the documented mainnet chain hash
    (/root/reference/client/doc.go:16) for the KAT public key."""
    pk = VERIFY_KATS[0][1]
    h = hashlib.sha256()
    h.update((30).to_bytes(4, "big"))
    h.update((1595431050).to_bytes(8, "big"))
    h.update(pk)
    h.update(bytes.fromhex("176f93498eac9ca337150b46d21dd58673ea4e3581185f869672e59fa4cb390a"))
    assert h.hexdigest() == "8990e7a9aaed2ffed73dbd7092123d6f289930540d7651336225dc172e51b2ce"


def test_golden_chains(oracle):
    chains = json.load(open(os.path.join(GOLD, "chains.json")))
    for scheme, c in chains.items():
        pk = bytes.fromhex(c["pk"])
        for r, s, p, v, rnd in zip(c["rounds"], c["sigs"], c["prevs"], c["valid"], c["randomness"]):
            s = bytes.fromhex(s)
            assert oracle.verify_beacon(scheme, pk, r, s, bytes.fromhex(p)) == v
            assert hashlib.sha256(s).hexdigest() == rnd


def test_golden_negatives(oracle):
    negs = json.load(open(os.path.join(GOLD, "negatives.json")))
    for scheme, c in negs.items():
        pk = bytes.fromhex(c["pk"])
        for case in c["cases"]:
            got = oracle.verify_beacon(scheme, pk, case["round"], bytes.fromhex(case["sig"]), bytes.fromhex(case["prev"]))
            assert got == case["valid"], (scheme, case["name"])


def test_golden_replay(oracle):
    rp = json.load(open(os.path.join(GOLD, "replay.json")))
    pk = bytes.fromhex(rp["pk"])
    stored = [bytes.fromhex(s) for s in rp["stored_sigs"]]
    prevs = [bytes.fromhex(rp["genesis_seed"])] + stored[:-1]
    faulty = [r for r, s, p in zip(rp["rounds"], stored, prevs)
              if not oracle.verify_beacon("pedersen-bls-chained", pk, r, s, p)]
    assert faulty == rp["faulty"] == [10, 11]


def test_hash_to_curve_rfc9380_vectors(oracle):
    """RFC 9380 J.9.1 (G1) and J.10.1 (G2) vectors: the oracle's hash_to_curve with the QUUX test DSTs. With the
    quicknet DST this is the whole quicknet hash path, so quicknet is pinned up to its DST string."""
    import bls_py
    from kat import H2C_DST_G1, H2C_DST_G2, H2C_G1, H2C_G2
    for msg, x, y in H2C_G1:
        pt = bls_py.g1_decompress(oracle.hash_to_curve(False, msg, H2C_DST_G1))
        assert pt == (int(x, 16), int(y, 16)), msg[:8]
    for msg, x0, x1, y0, y1 in H2C_G2:
        (px0, px1), (py0, py1) = bls_py.g2_decompress(oracle.hash_to_curve(True, msg, H2C_DST_G2))
        assert (px0, px1, py0) == (int(x0, 16), int(x1, 16), int(y0, 16)), msg
        if y1 is not None:
            assert py1 == int(y1, 16)


def test_cofactor_moves_to_the_key_side():
    """The G1-signature batch check reads e([h_eff] B, pk) as e(B, [h_eff] pk) with B = sum r_i Q_i the unreduced
    RLC sum of hash points (NOT in G1; k_vm.hip k_vm_prep_groups). Pinned here with the oracle's generic pairing on
    a point of E1(Fp) off the subgroup, with a negative control."""
    import random
    import bls_py as B
    rng = random.Random(7)
    Q = B.iso_map_g1(B.sswu_g1(rng.randrange(B.P)))
    assert B.ec_mul(B.FP, Q, B.R) is not None  # off G1
    pk = B.ec_mul(B.FP2, B.G2_GEN, rng.randrange(1, B.R))
    h = B.H_EFF_G1
    hQ, hpk, negQ = B.ec_mul(B.FP, Q, h), B.ec_mul(B.FP2, pk, h), B.ec_neg(B.FP, Q)
    assert B.pairing_check([(hQ, pk), (negQ, hpk)])
    assert not B.pairing_check([(hQ, pk), (negQ, pk)])
