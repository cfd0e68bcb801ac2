#!/usr/bin/env python3
"""Secondary BASELINE.json configs (the headline is bench.py = configs[1], quicknet 1M).

    python bench/bench_configs.py unchained  [--rounds 1048576]                  # configs[2] on one GPU
    python bench/bench_configs.py chained    [--rounds 4194304 --window 0]        # configs[4]: replay of a real chain
    python bench/bench_configs.py recover    [--rounds 100000 --n 64 --t 33]      # configs[3]
(configs[2] over 1/2/4/8 GPUs is bench.py --scheme pedersen-bls-unchained under torch.distributed.run.)

Each prints one JSON line: rounds/s (or recovered signatures/s), ms per batch, stage times from the library's
HIP-event profiler, the verdict check against the expected faulty set, and a bounded CPU-oracle sample.
Data is synthetic and signed on the GPU (dh_sign_batch), outside the timed region.

chained (Cfg5): a sequential chain (every round signed over the stored signature of the round before,
bench/chainsynth.py), 0.1% of the rounds corrupted in the three classes (sigma + g2, a flipped bit, an on-curve point
outside the subgroup) at splitmix64(0xD5A11D) positions; the replay verifies the store in one call over the whole chain
(CheckPastBeacons' shape; --window w cuts it into windows, --streams of them in flight; r04 measured one 4M call at
6.00 M/s against 5.89 for 2 x 2M and 5.68 for 4 x 1M, profiles/r04/config_chained_w*_r04s.json), prev = stored
signature of round-1 (chain/boltdb/trimmed.go:183), and must reject exactly U{k, k+1}.
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
sys.path.insert(0, os.path.join(ROOT, "bench"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
R_ORDER = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001

# as bench.py: 16 hardware queues per process, so one batch's latency-bound tail does not block the others
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("DRANDHIP_BENCH_HW_QUEUES", "16")


def secret(name):
    return (int.from_bytes(hashlib.sha256(b"drandhip-sk-" + name.encode()).digest(), "big") % R_ORDER).to_bytes(32, "big")


def profile_read(lib):
    buf = ctypes.create_string_buffer(1 << 16)
    lib.dh_profile_read(buf, len(buf))
    return json.loads(buf.value.decode())


def run_batches(fn, jobs, streams):
    """Run fn(slot, job) over the jobs with `streams` host threads (one library stream each)."""
    errs = []

    def worker(t):
        try:
            for k in range(t, len(jobs), streams):
                fn(t, jobs[k])
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(min(streams, len(jobs)))]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    if errs:
        raise errs[0]
    return time.perf_counter() - t0


def workmodel():
    return json.load(open(os.path.join(ROOT, "bench", "workmodel.json")))


def roofline(prof1, n_units, names, wm):
    """Dominant kernel among `names` in a single-stream profile: its credited mul32 over its average launch time."""
    kern = {k: v for k, v in prof1.items() if k in names}
    if not kern:
        return None
    dom = max(kern, key=lambda k: kern[k]["total_ms"])
    avg_s = kern[dom]["total_ms"] / kern[dom]["count"] / 1000.0
    achieved = names[dom] * wm["mul32_per_M"] * n_units / avg_s
    return {"bound": "valu", "kernel": dom, "achieved": round(achieved / 1e12, 3),
            "peak": round(wm["peak_mul32_per_s_measured"] / 1e12, 3), "unit": "Tmul32/s",
            "frac": round(achieved / wm["peak_mul32_per_s_measured"], 4), "avg_launch_ms": round(avg_s * 1000, 3),
            "work_per_launch": "%d M x %d mul32 x %d" % (names[dom], wm["mul32_per_M"], n_units)}


def cfg_unchained(args):
    import torch
    from drand_amd import _lib, scheme_from_name
    import oracle_ctypes as orc
    lib = _lib.load()
    torch.zeros(1, device="cuda")
    assert lib.dh_init(1) == 0
    name = "pedersen-bls-unchained"
    s = scheme_from_name(name)
    n = args.rounds
    sk = secret(name)
    pk = s.public_key(sk)
    rounds = np.arange(1, n + 1, dtype=np.uint64)
    t0 = time.perf_counter()
    sigs = s.sign_beacons(sk, rounds)
    t_sign = time.perf_counter() - t0
    dev = torch.device("cuda", 0)
    d_rounds = torch.from_numpy(rounds.view(np.int64)).to(dev)
    d_sigs = torch.from_numpy(sigs).to(dev)
    S = args.streams
    d_v = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(S)]
    d_r = [torch.zeros((n, 32), dtype=torch.uint8, device=dev) for _ in range(S)]

    def one(slot, _):
        rc = lib.dh_verify_batch_device(s.id, pk, len(pk), ctypes.c_void_p(d_rounds.data_ptr()),
                                        ctypes.c_void_p(d_sigs.data_ptr()), s.sig_len, None, 0, None, n,
                                        ctypes.c_void_p(d_v[slot].data_ptr()), ctypes.c_void_p(d_r[slot].data_ptr()),
                                        0, None, None)
        if rc != 0:
            raise RuntimeError(_lib.last_error())

    run_batches(one, list(range(max(args.warmup, S))), S)
    torch.cuda.synchronize()
    lib.dh_profile(1)
    el = run_batches(one, list(range(args.steps)), S)
    torch.cuda.synchronize()
    prof = profile_read(lib)
    lib.dh_profile(1)
    run_batches(one, [0], 1)
    prof1 = profile_read(lib)
    lib.dh_profile(0)
    v = d_v[0].cpu().numpy()
    ok = bool(v.all())
    m = min(n, args.cpu_sample)
    t0 = time.perf_counter()
    cv, _ = orc.verify_batch(name, pk, rounds[:m], sigs[:m], nthreads=args.cpu_threads)
    cdt = time.perf_counter() - t0
    ok = ok and bool(cv.all())
    wm = workmodel()
    return {
        "config": name, "rounds_per_batch": n, "steps": args.steps, "streams": S,
        "value": round(n * args.steps / el, 1), "unit": "beacons/s (1 GPU)", "ms_per_batch": round(el * 1000 / args.steps, 2),
        "verdicts_ok": ok, "roofline": roofline(prof1, n, {k: wm["kernel_units_M_per_round"][k] for k in
                                                           ("k_prep_sig<fp2>", "k_prep_msg<fp2>")}, wm),
        "stages_ms_per_batch": {k: round(x["total_ms"] / args.steps, 3) for k, x in prof.items()},
        "stages_ms_single_stream": {k: round(x["total_ms"] / max(1, x["count"]), 3) for k, x in prof1.items()},
        "cpu_baseline": {"value": round(m / cdt, 1), "unit": "beacons/s", "cores": args.cpu_threads, "kind": "port",
                         "sample": "%d rounds" % m},
        "sign_seconds": round(t_sign, 1),
    }


def cfg_chained(args):
    import torch
    import chainsynth
    from drand_amd import _lib, scheme_from_name
    import oracle_ctypes as orc
    lib = _lib.load()
    torch.zeros(1, device="cuda")
    assert lib.dh_init(1) == 0
    name = "pedersen-bls-chained"
    s = scheme_from_name(name)
    n = args.rounds
    W = args.window or n  # 0: one call over the whole chain
    sk = secret(name)
    pk = s.public_key(sk)
    genesis = hashlib.sha256(b"drandhip-genesis").digest()
    n_bad = max(1, int(round(n * args.corrupt)))
    bad = chainsynth.corrupted_rounds(n, n_bad)
    rng = np.random.default_rng(0xC5)
    t0 = time.perf_counter()
    cache = os.path.join(args.chain_cache, "chain_%d_%d.npy" % (n, n_bad)) if args.chain_cache else None
    if cache and os.path.exists(cache):  # the same seeded chain, signed by an earlier run (ladder sweeps)
        sigs = np.load(cache)
    else:
        sigs = chainsynth.sign_chain(s, sk, 1, n, genesis, bad, rng,
                                     progress=lambda p, m: print("chain: step %d / %d (%.0f s)" % (
                                         p, m, time.perf_counter() - t0), file=sys.stderr, flush=True))
        if cache:
            os.makedirs(args.chain_cache, exist_ok=True)
            np.save(cache, sigs)
    t_sign = time.perf_counter() - t0
    import random
    chainsynth.corrupt(sigs, bad, random.Random(31))
    prev, plen = chainsynth.stored_prevs(sigs, genesis)
    expected = chainsynth.expected_faulty(bad, n)
    dev = torch.device("cuda", 0)
    rounds = np.arange(1, n + 1, dtype=np.uint64)
    d_rounds = torch.from_numpy(rounds.view(np.int64)).to(dev)
    d_sigs = torch.from_numpy(sigs).to(dev)
    d_prev = torch.from_numpy(prev).to(dev)
    d_plen = torch.from_numpy(plen.view(np.int32)).to(dev)
    d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
    windows = [(lo, min(n, lo + W)) for lo in range(0, n, W)]
    stats = [(ctypes.c_uint64 * 4)() for _ in windows]

    def one(slot, w):
        lo, hi = windows[w]
        rc = lib.dh_verify_batch_device(s.id, pk, len(pk), ctypes.c_void_p(d_rounds.data_ptr() + 8 * lo),
                                        ctypes.c_void_p(d_sigs.data_ptr() + 96 * lo), 96,
                                        ctypes.c_void_p(d_prev.data_ptr() + 96 * lo), 96,
                                        ctypes.c_void_p(d_plen.data_ptr() + 4 * lo), hi - lo,
                                        ctypes.c_void_p(d_v.data_ptr() + lo), None, 0, None, stats[w])
        if rc != 0:
            raise RuntimeError(_lib.last_error())

    S = min(args.streams, len(windows))
    run_batches(one, list(range(len(windows))), S)  # warm-up: one replay
    torch.cuda.synchronize()
    lib.dh_profile(1)
    el = run_batches(one, [w for _ in range(args.steps) for w in range(len(windows))], S)
    torch.cuda.synchronize()
    prof = profile_read(lib)
    lib.dh_profile(0)
    v = d_v.cpu().numpy()
    faulty = np.flatnonzero(v == 0)
    exact = bool(np.array_equal(faulty, expected))
    # oracle on every faulty round and a sample of the accepted ones (bounded CPU time)
    samp = np.unique(np.concatenate([expected, np.random.default_rng(1).choice(n, args.cpu_sample, replace=False)]))
    ov = np.zeros(len(samp), np.uint8)
    lib_o = orc.lib()
    rs, ss, ps, ls = (np.ascontiguousarray(a[samp]) for a in (rounds, sigs, prev, plen))
    t0 = time.perf_counter()
    lib_o.or_verify_batch(orc.sid(name), pk, len(pk), rs.ctypes.data, ss.ctypes.data, 96, ps.ctypes.data, 96, ls.ctypes.data,
                          len(samp), args.cpu_threads, ov.ctypes.data, None)
    cdt = time.perf_counter() - t0
    oracle_ok = bool(np.array_equal(ov.astype(bool), v[samp].astype(bool)))
    return {
        "config": "%s replay of a %d-round sequential chain, %.2f%% corrupted (Cfg5 classes), %d x %d-round windows" % (
            name, n, 100 * args.corrupt, len(windows), W),
        "rounds": n, "steps": args.steps, "streams": S,
        "value": round(n * args.steps / el, 1), "unit": "beacons/s (1 GPU)", "ms_per_replay": round(el * 1000 / args.steps, 2),
        "faulty_expected": int(len(expected)), "faulty_found": int(len(faulty)), "exact_faulty_set": exact,
        "oracle_sample_agrees": oracle_ok, "oracle_sample": int(len(samp)),
        "bisection_stats_per_window_last": [list(x) for x in stats],
        "stages_ms_per_replay": {k: round(x["total_ms"] / args.steps, 3) for k, x in prof.items()},
        "cpu_baseline": {"value": round(len(samp) / cdt, 1), "unit": "beacons/s", "cores": args.cpu_threads, "kind": "port",
                         "sample": "%d rounds (all faulty + random accepted)" % len(samp)},
        "chain_sign_seconds": round(t_sign, 1),
    }


def cfg_recover(args):
    import torch
    from drand_amd import _lib, scheme_from_name
    import oracle_ctypes as orc
    lib = _lib.load()
    torch.zeros(1, device="cuda")
    assert lib.dh_init(1) == 0
    s = scheme_from_name("pedersen-bls-unchained")
    t, n, nr = args.t, args.n, args.rounds
    coeffs = [int.from_bytes(hashlib.sha256(b"bench-tbls-%d" % j).digest(), "big") % R_ORDER for j in range(t)]
    commits = [s.public_key(c.to_bytes(32, "big")) for c in coeffs]
    rounds = np.arange(1, nr + 1, dtype=np.uint64)
    rng = np.random.default_rng(33)
    if args.subsets == "first":  # configs[3] default: the same first t indices every round
        ids = np.tile(np.arange(t, dtype=np.int64), (nr, 1))
    else:  # a random t-subset of the n signers per round, in random arrival order
        ids = np.argsort(rng.random((nr, n)), axis=1)[:, :t]
    t0 = time.perf_counter()
    shares = np.zeros((n, nr, 96), dtype=np.uint8)
    for i in np.unique(ids):
        x, acc = int(i) + 1, 0
        for c in reversed(coeffs):
            acc = (acc * x + c) % R_ORDER
        shares[i] = s.sign_beacons(acc.to_bytes(32, "big"), rounds)
    t_sign = time.perf_counter() - t0
    msgs = np.zeros((nr, 32), dtype=np.uint8)
    for j in range(nr):
        msgs[j] = np.frombuffer(s.digest_beacon(int(rounds[j])), np.uint8)
    raw = np.zeros((nr * t, 98), dtype=np.uint8)
    flat = ids.reshape(-1)
    raw[:, 0] = (flat >> 8).astype(np.uint8)
    raw[:, 1] = (flat & 0xff).astype(np.uint8)
    raw[:, 2:] = shares[flat, np.repeat(np.arange(nr), t)]
    off = (np.arange(nr + 1) * t).astype(np.uint32)
    s.recover_batch_packed(commits, t, n, msgs[:64], raw[:64 * t], off[:65])  # warm-up
    lib.dh_profile(1)
    t0 = time.perf_counter()
    sigs, ok = s.recover_batch_packed(commits, t, n, msgs, raw, off)
    el = time.perf_counter() - t0
    prof = profile_read(lib)
    lib.dh_profile(0)
    want = s.sign_beacons(coeffs[0].to_bytes(32, "big"), rounds)
    good = bool(ok.all() and np.array_equal(sigs, want))
    m = min(nr, 4)
    t0 = time.perf_counter()
    for j in range(m):
        parts = [raw[j * t + k].tobytes() for k in range(t)]
        got = orc.recover(s.name, commits, t, n, msgs[j].tobytes(), parts)
        good = good and got == sigs[j].tobytes()
    cdt = time.perf_counter() - t0
    wm = workmodel()
    dev_ms = sum(x["total_ms"] for x in prof.values())
    ku = wm["kernel_units_M_per_round"]
    lag = ku.get("k_lagrange_t33_random", ku.get("k_lagrange_t33")) if args.subsets == "random" else ku.get("k_lagrange_t33")
    units = {"k_lagrange": lag or 97700,
             "k_prep_sig<fp2>(partials)": wm["kernel_units_M_per_round"]["k_prep_sig<fp2>"]}
    roof = None
    if "k_lagrange" in prof and "k_prep_sig<fp2>(partials)" in prof:
        la = prof["k_lagrange"]["total_ms"] / 1000.0
        ps = prof["k_prep_sig<fp2>(partials)"]["total_ms"] / 1000.0
        cand = {"k_lagrange": (units["k_lagrange"] * nr, la),
                "k_prep_sig<fp2>(partials)": (units["k_prep_sig<fp2>(partials)"] * nr * t, ps)}
        dom = max(cand, key=lambda k: cand[k][1])
        ach = cand[dom][0] * wm["mul32_per_M"] / cand[dom][1]
        roof = {"bound": "valu", "kernel": dom, "achieved": round(ach / 1e12, 3),
                "peak": round(wm["peak_mul32_per_s_measured"] / 1e12, 3), "unit": "Tmul32/s",
                "frac": round(ach / wm["peak_mul32_per_s_measured"], 4), "avg_launch_ms": round(cand[dom][1] * 1000, 3)}
    return {"config": "tbls Recover n=%d t=%d (pedersen-bls-unchained), %d rounds, %s signer subsets" % (n, t, nr, args.subsets),
            "value": round(nr / el, 1), "unit": "recovered+verified signatures/s (1 GPU, host API incl. PCIe)",
            "seconds": round(el, 3), "device_stage_ms": round(dev_ms, 1),
            "recovered_equal_to_group_signature_and_oracle": good, "roofline": roof,
            "node_roofline_frac_W_T": round(nr / el * wm["W_M_per_beacon"]["tbls_round_t33"] * wm["mul32_per_M"] /
                                            wm["peak_mul32_per_s_measured"], 4),
            "stages_ms": {k: round(x["total_ms"], 3) for k, x in prof.items()},
            "cpu_baseline": {"value": round(m / cdt, 3), "unit": "signatures/s", "cores": 1, "kind": "port",
                             "sample": "%d rounds, single thread (oracle or_recover)" % m},
            "sign_seconds": round(t_sign, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", choices=["unchained", "chained", "recover"])
    ap.add_argument("--rounds", type=int, default=None)
    ap.add_argument("--window", type=int, default=0, help="chained: rounds per call (0: the whole chain in one call)")
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--streams", type=int, default=8)
    ap.add_argument("--corrupt", type=float, default=0.001)
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--t", type=int, default=33)
    ap.add_argument("--subsets", choices=["first", "random"], default="first")
    ap.add_argument("--cpu-sample", type=int, default=2000)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--chain-cache", default=None, help="directory for the signed chained chain (reused by later runs)")
    ap.add_argument("--split", default="0", help="the library's one-call split (DRANDHIP_SPLIT): off, so each of the "
                    "--streams batches in flight is one stream")
    args = ap.parse_args()
    os.environ["DRANDHIP_SPLIT"] = args.split  # read when the library loads
    if args.config == "recover":
        args.rounds = args.rounds or 100000
        out = cfg_recover(args)
    elif args.config == "chained":
        args.rounds = args.rounds or (4 << 20)
        args.steps = args.steps or 2
        out = cfg_chained(args)
    else:
        args.rounds = args.rounds or (1 << 20)
        args.steps = args.steps or 8
        out = cfg_unchained(args)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
