"""CPU: chain readers and client/sync batch callers.

* bbolt readers against the reference's own store fixtures (/root/reference/chain/boltdb/testdata, copied as
  data to tests/golden/boltdb/): the trimmed file's reconstructed PreviousSig must equal the PreviousSig the
  untrimmed (legacy JSON) file stores for the same chain;
* a bbolt file written by tests/boltwrite.py from the golden chain drives check_past_beacons end to end;
* chain.Info.Hash against the documented mainnet chain hash (/root/reference/client/doc.go:16);
* the batched client trust walk and stream sync against a serial restatement of the reference loops, with
  verification delegated to the CPU oracle."""
import json
import os

import numpy as np
import pytest

from boltwrite import write_bolt
from drand_amd.chain import Info, info_from_json
from drand_amd.client import BatchVerifyingClient, ClientError
from drand_amd.store import (BoltTrimmedStore, BoltUntrimmedStore, beacon_from_hexjson, random_data_columns,
                             read_random_data)
from drand_amd.sync import TrimmedMemStore, check_past_beacons, sync_from_stream

GOLD = os.path.join(os.path.dirname(__file__), "golden")


class OracleScheme:
    def __init__(self, oracle, name):
        self.o, self.name = oracle, name
        self.sig_len = 96 if name.startswith("pedersen") else 48
        self.chained = name == "pedersen-bls-chained"
        self.calls = []

    def verify_beacons(self, pk, rounds, sigs, prevs=None, seed=0, want_randomness=True):
        self.calls.append(len(rounds))
        v = [self.o.verify_beacon(self.name, pk, int(r), bytes(s), bytes(prevs[k]) if prevs else b"")
             for k, (r, s) in enumerate(zip(rounds, sigs))]
        return np.array(v, dtype=bool), None


def test_reference_bolt_fixtures():
    t = BoltTrimmedStore(os.path.join(GOLD, "boltdb", "trimmed.db"), True)
    u = BoltUntrimmedStore(os.path.join(GOLD, "boltdb", "untrimmed.db"), True)
    assert t.rounds() == list(range(46)) and u.rounds() == list(range(27))
    assert t.get(0).signature == u.get(0).signature  # genesis seed record
    for r in range(1, 27):
        bt, bu = t.get(r), u.get(r)
        assert bt.signature == bu.signature and len(bt.signature) == 96
        assert bt.previous_signature == bu.previous_signature  # trimmed.go:183 == legacy stored PreviousSig
    assert t.last().round == 45 and t.len() == 46
    rounds, sigs, prevs, missing = t.columns(1, 45, 96)
    assert rounds.tolist() == list(range(1, 46)) and missing == [] and sigs.shape == (45, 96)
    assert prevs[0] == t.get(0).signature and prevs[5] == sigs[4].tobytes()


def test_bolt_store_drives_check_past_beacons(tmp_path, oracle):
    c = json.load(open(os.path.join(GOLD, "chains.json")))["pedersen-bls-chained"]
    kv = {int(0).to_bytes(8, "big"): bytes.fromhex(c["prevs"][0])}
    for r, sig in zip(c["rounds"], c["sigs"]):
        if r != 7:  # a missing record: rounds 7 and 8 are faulty (TestDrandCheckChain pattern)
            kv[int(r).to_bytes(8, "big")] = bytes.fromhex(sig)
    path = str(tmp_path / "chain.db")
    write_bolt(path, b"beacons", kv)
    st = BoltTrimmedStore(path, True)
    s = OracleScheme(oracle, "pedersen-bls-chained")
    assert check_past_beacons(st, s, bytes.fromhex(c["pk"]), 1000, window=8) == [7, 8]
    mem = TrimmedMemStore(True)
    for k, v in kv.items():
        mem.put(int.from_bytes(k, "big"), v)
    assert check_past_beacons(mem, s, bytes.fromhex(c["pk"]), 1000, window=5) == [7, 8]
    # many records: branch page + several leaves
    big = {int(r).to_bytes(8, "big"): bytes([r % 251]) * 96 for r in range(300)}
    write_bolt(path, b"beacons", big)
    st = BoltTrimmedStore(path, False)
    assert st.rounds() == list(range(300)) and st.get(299).signature == bytes([299 % 251]) * 96


def test_hexjson_records():
    text = "\n".join(json.dumps({"round": r, "randomness": "ab" * 32, "signature": ("%02x" % r) * 48,
                                 "previous_signature": ""}) for r in (5, 6))
    recs = read_random_data(text)
    assert [r["round"] for r in recs] == [5, 6] and recs[0]["signature"] == bytes([5]) * 48
    rounds, sigs, prevs, rand = random_data_columns(recs + [{"round": 7, "signature": b"\x01", "randomness": b"",
                                                             "previous_signature": b""}], 48)
    assert rounds.tolist() == [5, 6, 7] and sigs[2].sum() == 0 and rand[0] == bytes([0xab]) * 32
    assert read_random_data(json.dumps([json.loads(l) for l in text.splitlines()]))[1]["round"] == 6
    b = beacon_from_hexjson('{"PreviousSig":null,"Round":3,"Signature":"0102"}')
    assert (b.round, b.signature, b.previous_signature) == (3, b"\x01\x02", b"")


def test_chain_info_hash():
    mainnet = Info(public_key=bytes.fromhex(
        "868f005eb8e6e4ca0a47c8a77ceaa5309a47978a7c71bc5cce96366b5d7a569937c529eeda66c7293784a9402801af31"),
        period=30, scheme="pedersen-bls-chained", genesis_time=1595431050,
        genesis_seed=bytes.fromhex("176f93498eac9ca337150b46d21dd58673ea4e3581185f869672e59fa4cb390a"))
    assert mainnet.hash_string() == "8990e7a9aaed2ffed73dbd7092123d6f289930540d7651336225dc172e51b2ce"
    again = info_from_json(mainnet.to_json())
    assert again.hash() == mainnet.hash() and again.scheme == "pedersen-bls-chained"
    named = Info(mainnet.public_key, 30, mainnet.scheme, mainnet.genesis_time, mainnet.genesis_seed, id="x")
    assert named.hash() != mainnet.hash()  # non-default beacon IDs are hashed in (info.go:61-64)
    with pytest.raises(ValueError):
        info_from_json(json.dumps({"public_key": "00" * 10, "period": 3, "schemeID": "pedersen-bls-chained"}))


def _serial_trusted_prev(scheme, info, get, pot, round_):
    """Serial restatement of getTrustedPreviousSignature (client/verify.go:109-168) for the test."""
    if round_ == 1:
        return info.genesis_seed, pot
    if pot is None or pot[0] > round_:
        tr, tp = 1, info.genesis_seed
    else:
        tr, tp = pot
    init = tr
    nxt = None
    while tr < round_ - 1:
        tr += 1
        nxt = get(tr)
        ok, _ = scheme.verify_beacons(info.public_key, [tr], [nxt], [tp] if scheme.chained else None)
        if not ok[0]:
            raise ClientError("verifying beacon")
        tp = nxt
    if tr == round_ - 1 and tr > init:
        pot = (tr, nxt)
    return tp, pot


def test_batched_client_trust_walk(oracle):
    c = json.load(open(os.path.join(GOLD, "chains.json")))["pedersen-bls-chained"]
    sigs = {r: bytes.fromhex(s) for r, s in zip(c["rounds"], c["sigs"])}
    info = Info(bytes.fromhex(c["pk"]), 30, "pedersen-bls-chained", 0, bytes.fromhex(c["prevs"][0]))
    s = OracleScheme(oracle, "pedersen-bls-chained")
    cl = BatchVerifyingClient(info, s, get_signature=lambda r: sigs[r], strict=True)
    # point of trust at round 3: rounds 4..11 verified in one batch
    cl.point_of_trust = (3, sigs[3])
    assert cl.trusted_previous_signature(12) == sigs[11]
    assert cl.point_of_trust == (11, sigs[11]) and s.calls[-1] == 8
    rec = {"round": 12, "signature": sigs[12], "previous_signature": b""}
    cl.verify(rec)
    assert rec["randomness"] == __import__("hashlib").sha256(sigs[12]).digest()
    # a corrupted round inside the walk: same outcome as the serial loop, point of trust unchanged
    bad = dict(sigs)
    bad[15] = sigs[16]
    cl2 = BatchVerifyingClient(info, s, get_signature=lambda r: bad[r], strict=True)
    cl2.point_of_trust = (11, sigs[11])
    with pytest.raises(ClientError):
        cl2.trusted_previous_signature(20)
    with pytest.raises(ClientError):
        _serial_trusted_prev(s, info, lambda r: bad[r], (11, sigs[11]), 20)
    assert cl2.point_of_trust == (11, sigs[11])
    # slow path (no point of trust) follows the reference: round 2 is paired with the genesis seed
    cl3 = BatchVerifyingClient(info, s, get_signature=lambda r: sigs[r], strict=True)
    try:
        got = cl3.trusted_previous_signature(5)
        want = _serial_trusted_prev(s, info, lambda r: sigs[r], None, 5)[0]
        assert got == want
    except ClientError:
        with pytest.raises(ClientError):
            _serial_trusted_prev(s, info, lambda r: sigs[r], None, 5)
    # non-strict batch: one verify call for all results
    cl4 = BatchVerifyingClient(info, s)
    recs = [{"round": r, "signature": sigs[r], "previous_signature": bytes.fromhex(c["prevs"][r - 1])} for r in (2, 3, 4)]
    recs[1]["signature"] = sigs[5]
    n0 = len(s.calls)
    errs = cl4.verify_many(recs)
    assert [e is None for e in errs] == [True, False, True] and len(s.calls) == n0 + 1


def test_stream_sync_windows(oracle):
    c = json.load(open(os.path.join(GOLD, "chains.json")))["pedersen-bls-unchained"]
    s = OracleScheme(oracle, "pedersen-bls-unchained")
    pk = bytes.fromhex(c["pk"])
    pk_packets = [{"round": r, "signature": bytes.fromhex(x), "previous_signature": b""}
                  for r, x in zip(c["rounds"], c["sigs"])]

    def genesis_store():
        st = TrimmedMemStore(False)
        st.put(0, b"genesis seed")  # a chain store always holds the genesis beacon (tryNode starts from Last())
        return st

    st = genesis_store()
    done, stored = sync_from_stream(pk_packets, s, pk, st, up_to=20, window=6)
    assert done and stored == list(range(1, 21))
    bad = [dict(p) for p in pk_packets]
    bad[9]["signature"] = bad[10]["signature"]  # round 10 invalid: rounds 1..9 stored, then the peer is dropped
    done, stored = sync_from_stream(bad, s, pk, genesis_store(), up_to=24, window=4)
    assert not done and stored == list(range(1, 10))
    wrong_id = [dict(p) for p in pk_packets]
    wrong_id[5]["beacon_id"] = "other"
    done, stored = sync_from_stream(wrong_id, s, pk, genesis_store(), up_to=24, window=4)
    assert not done and stored == list(range(1, 6))
    # an empty store has no Last(): tryNode gives up before asking the peer (sync_manager.go:338-342)
    assert sync_from_stream(pk_packets, s, pk, TrimmedMemStore(False), up_to=20) == (False, [])


def _serial_relay_s3(scheme, pk, get, begin, end):
    """cmd/relay-s3/main.go:182-195 serially: Get (fetch + verifyingClient.verify), upload, log-and-continue."""
    out = []
    for rnd in range(begin, end + 1):
        try:
            r = get(rnd)
        except KeyError:
            continue
        prev = r["previous_signature"] if scheme.chained else b""
        if len(r["signature"]) != scheme.sig_len or not scheme.verify_beacons(pk, [rnd], [r["signature"]], [prev])[0][0]:
            continue
        out.append(rnd)
    return out


def test_relay_s3_range_sync(oracle):
    """relay-s3 sync batched per window: the same uploaded rounds as the serial loop (missing rounds and a round
    whose signature belongs to another round are skipped), bodies = encoding/json of client.RandomData
    (base64 []byte, omitempty) with randomness = SHA-256(signature)."""
    import base64
    import hashlib
    from drand_amd.client import marshal_random_data, relay_s3_sync
    c = json.load(open(os.path.join(GOLD, "chains.json")))["pedersen-bls-chained"]
    s = OracleScheme(oracle, "pedersen-bls-chained")
    info = Info(bytes.fromhex(c["pk"]), 30, s.name, 0, bytes.fromhex(c["prevs"][0]))
    recs = {r: {"round": r, "signature": bytes.fromhex(x), "previous_signature": bytes.fromhex(p)}
            for r, x, p in zip(c["rounds"], c["sigs"], c["prevs"])}
    del recs[6]
    recs[9] = dict(recs[9], signature=recs[10]["signature"])

    def get(r):
        return dict(recs[r])

    bucket = {}
    cl = BatchVerifyingClient(info, s)
    up = relay_s3_sync(cl, get, lambda k, b: bucket.__setitem__(k, b), 1, 24, window=5)
    assert len(s.calls) == 5  # one verification batch per window
    assert up == _serial_relay_s3(s, info.public_key, get, 1, 24)
    assert 6 not in up and 9 not in up and len(up) == 22
    body = json.loads(bucket["public/3"])
    assert list(body) == ["round", "randomness", "signature", "previous_signature"]
    assert body["round"] == 3 and base64.b64decode(body["signature"]) == recs[3]["signature"]
    assert base64.b64decode(body["randomness"]) == hashlib.sha256(recs[3]["signature"]).digest()
    assert marshal_random_data({"round": 0, "signature": b"\x01"}) == b'{"signature":"AQ=="}'
