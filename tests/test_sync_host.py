"""CPU: the CheckPastBeacons batch caller's host logic (drand_amd/sync.py) against the reference semantics
(/root/reference/chain/beacon/sync_manager.go:170-235, trimmed store /root/reference/chain/boltdb/trimmed.go:156-193),
with verification delegated to the CPU oracle so no GPU is needed. The GPU path of the same function is
covered in tests/test_gpu_parity.py::test_check_past_beacons_batch_caller."""
import json
import os

import numpy as np

from drand_amd.sync import NoBeaconStored, TrimmedMemStore, check_past_beacons

GOLD = os.path.join(os.path.dirname(__file__), "golden")


class OracleScheme:
    def __init__(self, oracle, name, sig_len, chained):
        self.o, self.name, self.sig_len, self.chained = oracle, name, sig_len, chained
        self.calls = []

    def verify_beacons(self, pk, rounds, sigs, prevs=None, seed=0, want_randomness=True):
        self.calls.append(len(rounds))
        v = [self.o.verify_beacon(self.name, pk, int(r), bytes(s), bytes(prevs[k]) if prevs else b"")
             for k, (r, s) in enumerate(zip(rounds, sigs))]
        return np.array(v, dtype=bool), None


def test_trimmed_store_semantics():
    st = TrimmedMemStore(True)
    st.put(0, b"seed")
    st.put(1, b"s1")
    st.put(3, b"s3")
    assert st.get(1).previous_signature == b"seed"
    try:
        st.get(3)
        raise AssertionError("missing previous must raise")
    except NoBeaconStored:
        pass
    try:
        st.last()  # Last() rebuilds round 3 and needs round 2, like trimmed.go's Last
        raise AssertionError("last with a missing previous must raise")
    except NoBeaconStored:
        pass
    st.put(2, b"s2")
    assert st.last().round == 3 and st.last().previous_signature == b"s2" and st.len() == 4
    assert TrimmedMemStore(False).put(5, b"x") is None


def test_check_past_beacons_host_logic(oracle):
    chains = json.load(open(os.path.join(GOLD, "chains.json")))
    for name, per_delete in (("pedersen-bls-chained", [4, 5]), ("bls-unchained-g1-rfc9380", [4])):
        c = chains[name]
        s = OracleScheme(oracle, name, 96 if "pedersen" in name else 48, name == "pedersen-bls-chained")
        st = TrimmedMemStore(s.chained)
        st.put(0, bytes.fromhex(c["prevs"][0]) if s.chained else b"\x00" * 32)
        for r, sig in zip(c["rounds"], c["sigs"]):
            st.put(r, bytes.fromhex(sig))
        pk = bytes.fromhex(c["pk"])
        assert check_past_beacons(st, s, pk, 1000, window=10) == []  # up_to clamped to the last round
        assert s.calls == [10, 10, 4]
        st.delete(4)
        assert check_past_beacons(st, s, pk, 24, window=6) == per_delete
        st.put(12, b"\x01" * 7)  # wrong-length stored signature -> faulty, like kyber's length check
        want = sorted(per_delete + ([12, 13] if s.chained else [12]))
        assert check_past_beacons(st, s, pk, 24, window=6) == want
