"""CPU: the chained-replay data synthesis (bench/g2_synth.py, bench/chainsynth.py) against the oracle — the three
Cfg5 corruption classes produce what they claim, and the expected faulty set follows the replay rule."""
import json
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bench"))

import chainsynth  # noqa: E402
import g2_synth  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_g2_codec_round_trip_and_classes(oracle):
    c = json.load(open(os.path.join(GOLD, "chains.json")))["pedersen-bls-chained"]
    rng = random.Random(5)
    pk = bytes.fromhex(c["pk"])
    for r, sig_hex, prev_hex in list(zip(c["rounds"], c["sigs"], c["prevs"]))[:4]:
        sig = bytes.fromhex(sig_hex)
        assert g2_synth.compress(g2_synth.decompress(sig)) == sig
        moved = g2_synth.plus_generator(sig)
        assert oracle.decode(True, moved) == 1  # a valid subgroup point ...
        assert not oracle.verify_beacon("pedersen-bls-chained", pk, r, moved, bytes.fromhex(prev_hex))  # ... wrong sig
        assert oracle.verify_beacon("pedersen-bls-chained", pk, r, sig, bytes.fromhex(prev_hex))
        flipped = g2_synth.flip_bit(sig, rng)
        assert sum(bin(a ^ b).count("1") for a, b in zip(flipped, sig)) == 1
        assert not oracle.verify_beacon("pedersen-bls-chained", pk, r, flipped, bytes.fromhex(prev_hex))
    off = g2_synth.off_subgroup(rng)
    pt = g2_synth.decompress(off)  # on E2 (decompress solves the curve equation) ...
    assert g2_synth.compress(pt) == off
    assert oracle.decode(True, off) != 1  # ... but rejected by the subgroup check


def test_corrupted_rounds_and_expected_set():
    bad = chainsynth.corrupted_rounds(1 << 20, 1000)
    assert len(bad) == 1000 and len(np.unique(bad)) == 1000 and bad.min() >= 0 and bad.max() < (1 << 20)
    assert np.array_equal(bad, chainsynth.corrupted_rounds(1 << 20, 1000))  # seeded
    exp = chainsynth.expected_faulty(np.array([0, 5, 6, 9]), 10)
    assert exp.tolist() == [0, 1, 5, 6, 7, 9]


def test_g1_codec_round_trip_and_classes(oracle):
    """The G1 variant (bench/g1_synth.py) used by the quicknet config-size GPU test."""
    import g1_synth
    name = "bls-unchained-g1-rfc9380"
    c = json.load(open(os.path.join(GOLD, "chains.json")))[name]
    rng = random.Random(6)
    pk = bytes.fromhex(c["pk"])
    for r, sig_hex in list(zip(c["rounds"], c["sigs"]))[:4]:
        sig = bytes.fromhex(sig_hex)
        assert g1_synth.compress(g1_synth.decompress(sig)) == sig
        moved = g1_synth.plus_generator(sig)
        assert oracle.decode(False, moved) == 1  # a valid subgroup point ...
        assert not oracle.verify_beacon(name, pk, r, moved)  # ... not the signature
        assert oracle.verify_beacon(name, pk, r, sig)
        flipped = g1_synth.flip_bit(sig, rng)
        assert sum(bin(a ^ b).count("1") for a, b in zip(flipped, sig)) == 1
        assert not oracle.verify_beacon(name, pk, r, flipped)
    for _ in range(3):
        off = g1_synth.off_subgroup(rng)
        assert g1_synth.compress(g1_synth.decompress(off)) == off  # on E1 ...
        assert oracle.decode(False, off) != 1  # ... but rejected by the subgroup check
