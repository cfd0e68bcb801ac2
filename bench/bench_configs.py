#!/usr/bin/env python3
"""Secondary BASELINE.json configs (the headline is bench.py = configs[1], quicknet 1M).

    python bench/bench_configs.py unchained   [--rounds 1048576 --corrupt 0]   # configs[2] on one GPU
    python bench/bench_configs.py chained     [--rounds 1048576 --corrupt 0.001]   # configs[4] shape, one GPU
    python bench/bench_configs.py recover     [--rounds 2048 --n 64 --t 33]        # configs[3], scaled rounds

Each prints one JSON line: rounds/s (or recovered signatures/s), ms per batch, stage times from the
library's HIP-event profiler, the verdict check against the expected faulty set, and a bounded CPU-oracle
sample for comparison. Data is synthetic and signed on the GPU (dh_sign_batch), outside the timed region.
For the chained replay, previous signatures are random 96-byte strings rather than a true sequential chain
(signing a real 1M chain is inherently serial); the verification work per round is identical and the
replay semantics (prev = stored signature of round-1) are covered by tests/golden/replay.json.
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
R_ORDER = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001


def secret(name):
    return (int.from_bytes(hashlib.sha256(b"drandhip-sk-" + name.encode()).digest(), "big") % R_ORDER).to_bytes(32, "big")


def profile_read(lib):
    buf = ctypes.create_string_buffer(1 << 16)
    lib.dh_profile_read(buf, len(buf))
    return json.loads(buf.value.decode())


def run_batches(lib, fn, steps, streams):
    errs = []

    def worker(t):
        try:
            for k in range(t, steps, streams):
                fn(t)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(min(streams, steps))]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    if errs:
        raise errs[0]
    return time.perf_counter() - t0


def cfg_verify(args, scheme_name, corrupt):
    import torch
    from drand_amd import _lib, scheme_from_name
    import oracle_ctypes as orc
    lib = _lib.load()
    assert lib.dh_init(1) == 0
    s = scheme_from_name(scheme_name)
    n = args.rounds
    sk = secret(scheme_name)
    pk = s.public_key(sk)
    rounds = np.arange(1, n + 1, dtype=np.uint64)
    prevs = None
    if s.chained:
        rng = np.random.default_rng(99)
        prevs = rng.integers(0, 256, (n, 96), dtype=np.uint8)
    t0 = time.perf_counter()
    sigs = s.sign_beacons(sk, rounds, prevs)
    t_sign = time.perf_counter() - t0
    bad = np.array([], dtype=np.int64)
    if corrupt > 0:
        rng = np.random.default_rng(0xD5A11D)
        bad = np.sort(rng.choice(n, size=max(1, int(n * corrupt)), replace=False))
        for k, i in enumerate(bad):
            if k % 2 == 0:
                sigs[i] = sigs[(i + 1) % n]          # valid point, wrong signature
            else:
                sigs[i, 40] ^= 0x01                   # bit flip
    dev = torch.device("cuda", 0)
    d_rounds = torch.from_numpy(rounds.view(np.int64)).to(dev)
    d_sigs = torch.from_numpy(sigs).to(dev)
    d_prev = torch.from_numpy(prevs).to(dev) if prevs is not None else None
    S = args.streams
    d_v = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(S)]
    d_r = [torch.zeros((n, 32), dtype=torch.uint8, device=dev) for _ in range(S)]
    stats = [(ctypes.c_uint64 * 4)() for _ in range(S)]

    def one(slot):
        rc = lib.dh_verify_batch_device(s.id, pk, len(pk), ctypes.c_void_p(d_rounds.data_ptr()),
                                        ctypes.c_void_p(d_sigs.data_ptr()), s.sig_len,
                                        ctypes.c_void_p(d_prev.data_ptr()) if d_prev is not None else None,
                                        96 if d_prev is not None else 0, None, n,
                                        ctypes.c_void_p(d_v[slot].data_ptr()), ctypes.c_void_p(d_r[slot].data_ptr()),
                                        0, None, stats[slot])
        if rc != 0:
            raise RuntimeError(_lib.last_error())

    run_batches(lib, one, args.warmup, S)
    torch.cuda.synchronize()
    lib.dh_profile(1)
    el = run_batches(lib, one, args.steps, S)
    torch.cuda.synchronize()
    prof = profile_read(lib)
    lib.dh_profile(0)
    v = d_v[0].cpu().numpy()
    faulty = np.flatnonzero(v == 0)
    ok = np.array_equal(faulty, bad)
    # CPU oracle sample (16 threads, bounded)
    m = min(n, args.cpu_sample)
    t0 = time.perf_counter()
    cv, _ = orc.verify_batch(scheme_name, pk, rounds[:m], sigs[:m], prevs[:m] if prevs is not None else None,
                             nthreads=args.cpu_threads)
    cdt = time.perf_counter() - t0
    ok = ok and np.array_equal(cv.astype(bool), v[:m].astype(bool))
    return {
        "config": scheme_name + (" replay %.2f%% corrupted" % (100 * corrupt) if corrupt else ""),
        "rounds_per_batch": n, "steps": args.steps, "streams": S,
        "value": round(n * args.steps / el, 1), "unit": "beacons/s (1 GPU)", "ms_per_batch": round(el * 1000 / args.steps, 2),
        "verdicts_match_expected_and_oracle_sample": bool(ok), "faulty_found": int(len(faulty)),
        "bisection_stats_last_batch": list(stats[0]),
        "stages_ms_per_batch": {k: round(x["total_ms"] / args.steps, 3) for k, x in prof.items()},
        "cpu_baseline": {"value": round(m / cdt, 1), "unit": "beacons/s", "cores": args.cpu_threads, "kind": "port",
                         "sample": "%d rounds" % m},
        "sign_seconds": round(t_sign, 1),
    }


def cfg_recover(args):
    from drand_amd import _lib, scheme_from_name
    import oracle_ctypes as orc
    lib = _lib.load()
    assert lib.dh_init(1) == 0
    s = scheme_from_name("pedersen-bls-unchained")
    t, n, nr = args.t, args.n, args.rounds
    coeffs = [int.from_bytes(hashlib.sha256(b"bench-tbls-%d" % j).digest(), "big") % R_ORDER for j in range(t)]
    commits = [s.public_key(c.to_bytes(32, "big")) for c in coeffs]
    rounds = np.arange(1, nr + 1, dtype=np.uint64)
    signers = list(range(t))  # configs[3] default: the same first t indices every round
    t0 = time.perf_counter()
    shares = {}
    for i in signers:
        x, acc = i + 1, 0
        for c in reversed(coeffs):
            acc = (acc * x + c) % R_ORDER
        shares[i] = s.sign_beacons(acc.to_bytes(32, "big"), rounds)
    t_sign = time.perf_counter() - t0
    msgs = [s.digest_beacon(int(r)) for r in rounds]
    parts = [[i.to_bytes(2, "big") + shares[i][j].tobytes() for i in signers] for j in range(nr)]
    s.recover_batch(commits, t, n, msgs[:64], parts[:64])  # warm-up
    lib.dh_profile(1)
    t0 = time.perf_counter()
    sigs, ok = s.recover_batch(commits, t, n, msgs, parts)
    el = time.perf_counter() - t0
    prof = profile_read(lib)
    lib.dh_profile(0)
    want = s.sign_beacons(coeffs[0].to_bytes(32, "big"), rounds)
    good = bool(ok.all() and np.array_equal(sigs, want))
    m = min(nr, 4)
    t0 = time.perf_counter()
    for j in range(m):
        got = orc.recover(s.name, commits, t, n, msgs[j], parts[j])
        good = good and got == sigs[j].tobytes()
    cdt = time.perf_counter() - t0
    return {"config": "tbls Recover n=%d t=%d (pedersen-bls-unchained), %d rounds" % (n, t, nr),
            "value": round(nr / el, 1), "unit": "recovered+verified signatures/s (1 GPU, host API incl. PCIe)",
            "seconds": round(el, 3), "recovered_equal_to_group_signature_and_oracle": good,
            "stages_ms": {k: round(x["total_ms"], 3) for k, x in prof.items()},
            "cpu_baseline": {"value": round(m / cdt, 3), "unit": "signatures/s", "cores": 1, "kind": "port",
                             "sample": "%d rounds, single thread (oracle or_recover)" % m},
            "sign_seconds": round(t_sign, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", choices=["unchained", "chained", "recover", "quicknet"])
    ap.add_argument("--rounds", type=int, default=None)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--corrupt", type=float, default=None, help="fraction of corrupted rounds (chained: 0.001)")
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--t", type=int, default=33)
    ap.add_argument("--cpu-sample", type=int, default=2000)
    ap.add_argument("--cpu-threads", type=int, default=16)
    args = ap.parse_args()
    if args.config == "recover":
        args.rounds = args.rounds or 2048
        out = cfg_recover(args)
    else:
        args.rounds = args.rounds or (1 << 20)
        name = {"unchained": "pedersen-bls-unchained", "chained": "pedersen-bls-chained",
                "quicknet": "bls-unchained-g1-rfc9380"}[args.config]
        corrupt = args.corrupt if args.corrupt is not None else (0.001 if args.config == "chained" else 0.0)
        out = cfg_verify(args, name, corrupt)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
