#!/usr/bin/env python3
"""One-beacon latency of the drop-in calls (VERDICT r05 Next #1): the calls the cgo scheme makes for every live
beacon — VerifyBeacon (gossip validator lp2p/client/validator.go:62, client/verify.go:192), VerifyRecovered
(chain/beacon/chainstore.go:207) and a one-round Recover (the aggregator, chainstore.go:202) — timed one at a time
from the host, per scheme, with the group key cached on the worker ("warm") and with a key-cache miss on every call
("cold": six keys cycled, more than a worker's 4-slot key cache holds; "two_keys": two chains' keys alternating,
both cached). Beside them, the CPU oracle's per-verify time on one core (context only: a C
restatement, not kyber).

    python bench/single_beacon.py [--reps 40] [--out gpurun_out/single_beacon.json]

measure() is also what bench.py calls for its "single_beacon_ms" field.
"""
import argparse
import hashlib
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
R_ORDER = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
SCHEMES = ["pedersen-bls-chained", "pedersen-bls-unchained", "bls-unchained-on-g1", "bls-unchained-g1-rfc9380"]


def _sk(tag):
    return (int.from_bytes(hashlib.sha256(tag).digest(), "big") % R_ORDER).to_bytes(32, "big")


def _share(coeffs, i):
    x, acc = i + 1, 0
    for cf in reversed(coeffs):
        acc = (acc * x + cf) % R_ORDER
    return acc.to_bytes(32, "big")


def _stats(ts):
    ms = sorted(t * 1000.0 for t in ts)
    return {"p50": round(statistics.median(ms), 3), "min": round(ms[0], 3),
            "p90": round(ms[min(len(ms) - 1, int(0.9 * len(ms)))], 3), "n": len(ms)}


def _time(fn, reps):
    out = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        out.append(time.perf_counter() - t0)
    return out


def measure(schemes=SCHEMES, reps=40, recover_nt=(64, 33), with_oracle=True):
    """-> {scheme: {"verify_beacon_warm": stats, "verify_beacon_cold": stats, "verify_recovered_warm": stats,
    "recover_one_round": stats, "oracle_verify_1core_ms": x, "verdicts_ok": bool}} (milliseconds)."""
    from drand_amd import _lib, scheme_from_name
    lib = _lib.load()
    orc = None
    if with_oracle:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_ctypes as orc
    res = {}
    for name in schemes:
        s = scheme_from_name(name)
        sk1, sk2 = _sk(b"single-1-" + name.encode()), _sk(b"single-2-" + name.encode())
        pk1, pk2 = s.public_key(sk1), s.public_key(sk2)
        # cold: more keys than a worker's key cache holds (drandhip.cpp KEY_SLOTS = 4), cycled, so every call misses
        cold_keys = [(s.public_key(_sk(b"single-c%d-" % c + name.encode())), _sk(b"single-c%d-" % c + name.encode()))
                     for c in range(6)]
        rounds = np.arange(1000, 1000 + reps + 1, dtype=np.uint64)
        prevs = None
        if s.chained:
            prevs = np.frombuffer(hashlib.sha256(b"prev").digest() * 3, np.uint8)[:96].reshape(1, 96).repeat(len(rounds), 0).copy()
            prevs[:, 0] = np.arange(len(rounds), dtype=np.uint8)
        sig1 = s.sign_beacons(sk1, rounds, prevs)
        sig2 = s.sign_beacons(sk2, rounds, prevs)
        prev_b = [prevs[k].tobytes() if prevs is not None else b"" for k in range(len(rounds))]

        def vb(pk, sig, k):
            pb = prev_b[k]
            return lib.dh_verify_beacon(s.id, pk, len(pk), int(rounds[k]), sig[k].tobytes(), s.sig_len, pb, len(pb))

        ok = True
        vb(pk1, sig1, 0)  # worker, key cache, code objects
        k_it = iter(range(10 ** 9))
        warm = _time(lambda: vb(pk1, sig1, next(k_it) % len(rounds)), reps)
        ok &= all(vb(pk1, sig1, k) == 1 for k in range(3))
        bad = bytearray(sig1[1].tobytes())
        bad[20] ^= 1
        ok &= lib.dh_verify_beacon(s.id, pk1, len(pk1), int(rounds[1]), bytes(bad), s.sig_len, prev_b[1], len(prev_b[1])) == 0
        ok &= vb(pk1, sig1, 2) == 1 and vb(pk2, sig1, 2) == 0  # a key switch (cold) rejects the other key's signature
        two_t = []  # two keys alternating (a node serving two chains): both stay cached
        for k in range(max(6, reps // 4)):
            pk, sg = (pk2, sig2) if k % 2 == 0 else (pk1, sig1)
            t0 = time.perf_counter()
            r = vb(pk, sg, k % len(rounds))
            two_t.append(time.perf_counter() - t0)
            ok &= r == 1
        cold_sigs = [s.sign_beacons(csk, rounds[:1], prevs[:1] if prevs is not None else None) for _, csk in cold_keys]
        cold_t = []
        for k in range(12):
            cpk, _ = cold_keys[k % len(cold_keys)]
            t0 = time.perf_counter()
            r = vb(cpk, cold_sigs[k % len(cold_keys)], 0)
            cold_t.append(time.perf_counter() - t0)
            ok &= r == 1
        vb(pk1, sig1, 0)
        msgs = [s.digest_beacon(int(rounds[k]), prev_b[k]) for k in range(len(rounds))]

        def vr(k):
            return lib.dh_verify_recovered(s.id, pk1, len(pk1), msgs[k], sig1[k].tobytes(), s.sig_len)

        vr(0)
        k_it2 = iter(range(10 ** 9))
        rec_v = _time(lambda: vr(next(k_it2) % len(rounds)), reps)
        ok &= vr(3) == 1
        entry = {"verify_beacon_warm": _stats(warm), "verify_beacon_cold": _stats(cold_t),
                 "verify_beacon_two_keys": _stats(two_t),
                 "verify_recovered_warm": _stats(rec_v)}
        # one-round Recover as the aggregator makes it: n signers, threshold t, the first t partials of the round
        n, t = recover_nt
        coeffs = [int.from_bytes(hashlib.sha256(b"sb-%s-%d" % (name.encode(), j)).digest(), "big") % R_ORDER for j in range(t)]
        commits = [s.public_key(cf.to_bytes(32, "big")) for cf in coeffs]
        r1 = rounds[:1]
        parts = [(i).to_bytes(2, "big") + s.sign_beacons(_share(coeffs, i), r1, prevs[:1] if prevs is not None else None)[0].tobytes()
                 for i in range(t)]
        msg = msgs[0]
        s.recover_batch(commits, t, n, [msg], [parts])
        rec_t = []
        for _ in range(max(6, reps // 4)):
            t0 = time.perf_counter()
            sigs_out, okr = s.recover_batch(commits, t, n, [msg], [parts])
            rec_t.append(time.perf_counter() - t0)
            ok &= bool(okr[0])
        group = s.sign_beacons(coeffs[0].to_bytes(32, "big"), r1, prevs[:1] if prevs is not None else None)
        ok &= bool(np.array_equal(sigs_out[0], group[0]))
        entry["recover_one_round"] = _stats(rec_t)
        entry["recover_shape"] = "n = %d, t = %d, the first t partials (PubPoly cached after the first call)" % (n, t)
        if orc is not None:
            m = max(3, min(12, reps // 4))
            t0 = time.perf_counter()
            for k in range(m):
                ok &= orc.verify_beacon(name, pk1, int(rounds[k]), sig1[k].tobytes(), prev_b[k])
            entry["oracle_verify_1core_ms"] = round((time.perf_counter() - t0) * 1000.0 / m, 3)
        entry["verdicts_ok"] = bool(ok)
        res[name] = entry
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--schemes", default=",".join(SCHEMES))
    ap.add_argument("--out", default="")
    ap.add_argument("--no-oracle", action="store_true")
    a = ap.parse_args()
    from drand_amd import _lib
    lib = _lib.load()
    if lib.dh_init(1) != 0:
        raise SystemExit("dh_init: %s" % _lib.last_error())
    r = measure(a.schemes.split(","), a.reps, with_oracle=not a.no_oracle)
    txt = json.dumps(r, indent=1)
    print(txt, flush=True)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(txt + "\n")
    if not all(v["verdicts_ok"] for v in r.values()):
        raise SystemExit("single-beacon verdicts wrong")


if __name__ == "__main__":
    main()
