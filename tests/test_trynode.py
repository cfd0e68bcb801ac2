"""tryNode's stream verify + chain-store Put (/root/reference/chain/beacon/sync_manager.go:376-445,
chain/beacon/store.go:55-124): drand_amd.sync.sync_from_stream over ChainStore against a serial restatement of the
reference loop (tests/trynode_cases.py) on every case: a valid chained beacon whose previous signature is not the
last stored signature, an out-of-order round, duplicates of the last stored round (at and before up_to), a
duplicate carrying another signature, unchained previous signatures dropped on Put, an invalid signature, a wrong
beacon ID, and a resync through the insecure store. The CPU test verifies with the oracle standing in for the
device; the GPU test runs the same cases through libdrandhip."""
import queue
import threading
import time

import numpy as np
import pytest

import trynode_cases as tc

SCHEMES = ["pedersen-bls-chained", "pedersen-bls-unchained", "bls-unchained-g1-rfc9380"]


class OracleScheme:
    """The verification half of drand_amd.scheme.Scheme on the CPU oracle (test stand-in for the device)."""

    def __init__(self, oracle, name):
        self.o, self.name = oracle, name
        self.sig_len = 96 if name.startswith("pedersen") else 48
        self.chained = name == "pedersen-bls-chained"

    def verify_beacons(self, pk, rounds, sigs, prevs=None, seed=0, want_randomness=True):
        v = [self.o.verify_beacon(self.name, pk, int(r), bytes(s), bytes(prevs[k]) if prevs else b"")
             for k, (r, s) in enumerate(zip(rounds, sigs))]
        return np.array(v, dtype=bool), None


def _run_cases(oracle, scheme, name, windows=(1, 3, 500)):
    from drand_amd.sync import ChainStore, TrimmedMemStore, sync_from_stream
    sig, cs = tc.cases(oracle, name)
    pk = oracle.public_key(name, tc.secret(name))
    checked = 0
    for label, base, pkts, up_to, resync in cs:
        want_done, want_stored, want_store = tc.serial_trynode(oracle, name, pk, tc.base_items(sig, base), pkts, up_to,
                                                               resync)
        for w in windows:
            st = TrimmedMemStore(name == "pedersen-bls-chained")
            for r, s in tc.base_items(sig, base):
                st.put(r, s)
            target = st if resync else ChainStore(st, scheme)
            done, stored = sync_from_stream(iter([dict(p) for p in pkts]), scheme, pk, target, up_to, window=w,
                                            resync=resync)
            assert (done, stored) == (want_done, want_stored), (name, label, w)
            assert {r: st._sigs[r] for r in st._sigs} == want_store, (name, label, w)
            checked += 1
    return checked


@pytest.mark.parametrize("name", SCHEMES)
def test_trynode_put_semantics_oracle(oracle, name):
    assert _run_cases(oracle, OracleScheme(oracle, name), name) >= 27


def test_chain_store_put_checks(oracle):
    """ChainStore alone: appendStore / schemeStore errors and ErrBeaconAlreadyStored (store.go:55-124)."""
    from drand_amd.chain import Beacon
    from drand_amd.scheme import scheme_from_name
    from drand_amd.sync import BeaconAlreadyStored, ChainStore, NoBeaconStored, PutError, TrimmedMemStore
    st = TrimmedMemStore(True)
    with pytest.raises(NoBeaconStored):
        ChainStore(st, scheme_from_name("pedersen-bls-chained"))  # newAppendStore needs Last()
    st.put(0, b"g" * 32)
    st.put(1, b"a" * 96)
    cs = ChainStore(st, scheme_from_name("pedersen-bls-chained"))
    with pytest.raises(BeaconAlreadyStored):
        cs.put(Beacon(1, b"a" * 96, b"g" * 32))
    with pytest.raises(PutError, match="previous signature was different"):
        cs.put(Beacon(1, b"a" * 96, b"x" * 32))
    with pytest.raises(PutError, match="signature was different"):
        cs.put(Beacon(1, b"b" * 96, b"g" * 32))
    with pytest.raises(PutError, match="invalid round"):
        cs.put(Beacon(3, b"c" * 96, b"a" * 96))
    with pytest.raises(PutError, match="invalid previous signature"):
        cs.put(Beacon(2, b"c" * 96, b"z" * 96))
    cs.put(Beacon(2, b"c" * 96, b"a" * 96))
    assert st.get(2).previous_signature == b"a" * 96 and cs.last().round == 2
    u = TrimmedMemStore(False)
    u.put(0, b"g")
    cu = ChainStore(u, scheme_from_name("pedersen-bls-unchained"))
    cu.put(Beacon(1, b"s" * 96, b"p" * 96))  # unchained: previous signature not checked, dropped on Put
    with pytest.raises(PutError, match="previous signature was different"):
        cu.put(Beacon(1, b"s" * 96, b"p" * 96))
    with pytest.raises(BeaconAlreadyStored):
        cu.put(Beacon(1, b"s" * 96, b""))


def test_stream_reader_stops_on_early_return(oracle):
    """A sync that returns early (invalid beacon) stops the reader thread and closes the packet stream (tryNode's
    deferred cancel), even when the stream would go on forever."""
    from drand_amd.sync import TrimmedMemStore, sync_from_stream
    name = "pedersen-bls-unchained"
    _, sig = tc.build_chain(oracle, name, 3)
    pk = oracle.public_key(name, tc.secret(name))
    closed = threading.Event()
    produced = [0]

    def endless():
        try:
            r = 1
            while True:
                produced[0] += 1
                yield tc.packet(name, sig, 1 + (r - 1) % 3) if r <= 2 else dict(tc.packet(name, sig, 3), signature=sig[1])
                r += 1
        finally:
            closed.set()

    st = TrimmedMemStore(False)
    st.put(0, b"genesis")
    before = threading.active_count()
    done, stored = sync_from_stream(endless(), OracleScheme(oracle, name), pk, st, up_to=50, window=2)
    assert (done, stored) == (False, [1, 2])
    assert closed.wait(5), "the packet stream was not closed"
    time.sleep(0.2)
    assert threading.active_count() <= before
    n = produced[0]
    time.sleep(0.3)
    assert produced[0] == n  # nothing keeps reading from the stream


@pytest.mark.gpu
@pytest.mark.parametrize("name", SCHEMES)
def test_trynode_put_semantics_device(oracle, name):
    """The same cases through libdrandhip (verify-ahead windows of 1, 3 and 500 packets), and the stream fed live
    through a queue for the chained scheme."""
    import torch
    import drand_amd
    from drand_amd import _lib
    from drand_amd.sync import END, ChainStore, TrimmedMemStore, sync_from_stream
    torch.zeros(1, device="cuda")
    assert _lib.load().dh_init(0) == 0, _lib.last_error()
    s = drand_amd.scheme_from_name(name)
    assert _run_cases(oracle, s, name) >= 27
    if name != "pedersen-bls-chained":
        return
    sig, _ = tc.cases(oracle, name)
    pk = oracle.public_key(name, tc.secret(name))
    st = TrimmedMemStore(True)
    for r, x in tc.base_items(sig, 5):
        st.put(r, x)
    q = queue.Queue()
    out = {}
    th = threading.Thread(target=lambda: out.update(r=sync_from_stream(q, s, pk, ChainStore(st, s), 12, window=500,
                                                                       idle=0.05, max_delay=0.5)))
    th.start()
    for r in range(6, 13):
        q.put(tc.packet(name, sig, r))
        time.sleep(0.01)
    q.put(END)
    th.join(timeout=120)
    assert out["r"] == (True, list(range(6, 13))) and st.last().round == 12
