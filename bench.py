#!/usr/bin/env python3
"""bench.py — verified beacons/sec on MI355X for the quicknet scheme (bls-unchained-g1-rfc9380).

Workload (BASELINE.json configs[1]): batch-verify 1M synthetic quicknet rounds per GPU — G1 signatures,
G2 group key, RFC 9380 hash-to-G1 — with per-round verdicts and SHA-256 randomness, inputs resident in
HBM before the timed region. One "step" = one dh_verify_batch_device call over the GPU's 1M rounds (fresh
CSPRNG seed each step), followed, for N > 1, by an all-gather of the per-GPU verdict bitmaps over RCCL.
Rounds shard across GPUs (rank r owns rounds r*n+1 .. (r+1)*n): weak scaling, no data-path collective.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rounds n] [--scheme name]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Prints ONE JSON line on rank 0 (contract in the task statement): value = rounds verified by all ranks /
max-over-ranks wall time of the K timed steps. "roofline" reports the dominant kernel's achieved
integer-multiply rate (algorithmic work of bench/workmodel.json / its HIP-event-measured duration on its
own stream) against the measured v_mad_u64_u32 peak. "cpu_baseline" times the CPU oracle (a C port of
the reference's per-round algorithm, oracle/bls_oracle.c) on a bounded sample on the host cores.
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=1 << 20, help="rounds per GPU per step")
    ap.add_argument("--scheme", default="bls-unchained-g1-rfc9380")
    ap.add_argument("--cpu-sample-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stage-times", action="store_true",
                    help="leave the library's HIP-event stage timing off inside the timed region")
    ap.add_argument("--roofline-steps", type=int, default=2, help="single-stream batches timed for the roofline")
    ap.add_argument("--streams", type=int, default=8,
                    help="batches in flight per GPU (host threads, each with its own HIP stream in libdrandhip)")
    ap.add_argument("--split", default="0",
                    help="DRANDHIP_SPLIT for the timed calls ('chunk,workers'; 0 = each call on one stream: the bench "
                         "already keeps --streams calls in flight)")
    return ap.parse_args()


def load_workmodel():
    with open(os.path.join(ROOT, "bench", "workmodel.json")) as f:
        return json.load(f)


def cpu_baseline(scheme, pk, rounds, sigs, seconds, threads):
    """Oracle (port of the reference per-round VerifyBeacon) on `threads` host threads, bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ctypes as orc
    lib = orc.lib()
    probe = max(threads, 16)
    t0 = time.perf_counter()
    v, _ = orc.verify_batch(scheme, pk, rounds[:probe], sigs[:probe], nthreads=threads)
    dt = time.perf_counter() - t0
    per = dt / probe
    n = int(min(len(rounds), max(probe, seconds / max(per, 1e-9))))
    t0 = time.perf_counter()
    v, _ = orc.verify_batch(scheme, pk, rounds[:n], sigs[:n], nthreads=threads)
    dt = time.perf_counter() - t0
    assert v.all(), "oracle rejected a valid synthetic round"
    del lib
    return {"value": n / dt, "unit": "beacons/s", "cores": threads, "kind": "port",
            "sample": "%d quicknet rounds (first of the 1M synthetic chain), per-round decode+subgroup(r*P)+hash+"
                      "2-pairing VerifyBeacon, %d threads, %.1f s" % (n, threads, dt)}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ["DRANDHIP_SPLIT"] = args.split  # read once, when the library first splits a call
    import torch
    import torch.distributed as dist
    from drand_amd import _lib, scheme_from_name
    from drand_amd.dist import gather_verdicts, pack_bits, shard_rounds

    lib = _lib.load()
    rc = lib.dh_init(1 << local)
    if rc != 0:
        raise SystemExit("dh_init failed: %s" % _lib.last_error())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    sch = scheme_from_name(args.scheme)
    n = args.rounds
    sk = (int.from_bytes(hashlib.sha256(b"drandhip-sk-" + args.scheme.encode()).digest(), "big") %
          0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001).to_bytes(32, "big")
    pk = sch.public_key(sk)
    rounds = shard_rounds(rank, world, n)
    t0 = time.perf_counter()
    sigs = sch.sign_beacons(sk, rounds)  # synthetic chain, signed on the GPU (not timed)
    t_sign = time.perf_counter() - t0

    d_rounds = torch.from_numpy(rounds.view(np.int64)).to(dev)
    d_sigs = torch.from_numpy(sigs).to(dev)
    S = max(1, args.streams)
    d_verdict = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(S)]
    d_rand = [torch.zeros((n, 32), dtype=torch.uint8, device=dev) for _ in range(S)]
    torch.cuda.synchronize()

    def verify(slot):
        rc = lib.dh_verify_batch_device(sch.id, pk, len(pk), ctypes.c_void_p(d_rounds.data_ptr()),
                                        ctypes.c_void_p(d_sigs.data_ptr()), sch.sig_len, None, 0, None, n,
                                        ctypes.c_void_p(d_verdict[slot].data_ptr()),
                                        ctypes.c_void_p(d_rand[slot].data_ptr()), 0, None, None)
        if rc != 0:
            raise RuntimeError("dh_verify_batch_device: %s" % _lib.last_error())

    def run_steps(k_steps, streams):
        """k_steps batches, `streams` in flight: thread t runs steps t, t+streams, ... on its own output slot."""
        import threading
        errs = []
        bits = [None] * k_steps

        def worker(t):
            try:
                torch.cuda.set_device(local)
                for k in range(t, k_steps, streams):
                    verify(t)
                    bits[k] = pack_bits(d_verdict[t])
            except Exception as e:  # surfaced below
                errs.append(e)

        ths = [threading.Thread(target=worker, args=(t,)) for t in range(min(streams, k_steps))]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        if errs:
            raise errs[0]
        if world > 1:  # whole-node verdict bitmaps: one all-gather over RCCL at the end of the batches
            gather_verdicts(torch.cat(bits), world)
        torch.cuda.synchronize()

    def profile_read():
        buf = ctypes.create_string_buffer(1 << 16)
        lib.dh_profile_read(buf, len(buf))
        return json.loads(buf.value.decode())

    # warm-up: at least one batch per stream, so every library worker (stream + device workspace) exists before
    # the timed region; W < S would leave workspace allocation inside it
    warm_batches = max(args.warmup, S) if args.warmup else 0
    run_steps(warm_batches, S)
    lib.dh_profile(0 if args.no_stage_times else 1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(args.steps, S)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    prof = profile_read()
    # Roofline pass (after the timed region, not counted in `value`): with S batches in flight the kernels of
    # different batches share the CUs, so per-launch durations measured there are not one kernel's speed.
    # Two more batches on ONE stream give each kernel the whole GPU; the dominant kernel's roofline is
    # computed from their HIP events (recorded on the library's stream). bench/profile.sh collects the
    # rocprofv3 kernel-trace of the same single-stream batches.
    lib.dh_profile(1)
    run_steps(args.roofline_steps, 1)
    prof1 = profile_read()
    lib.dh_profile(0)

    # sanity (outside the timed region): every synthetic round verifies, randomness = SHA-256(sig)
    ok = all(bool(d.cpu().numpy().all()) for d in d_verdict[:min(S, args.steps)])
    r0 = d_rand[0].cpu().numpy()[0].tobytes()
    ok = ok and r0 == hashlib.sha256(sigs[0].tobytes()).digest()

    if world > 1:
        t = torch.tensor([elapsed, 0.0 if ok else 1.0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, bad = float(t[0]), float(t[1])
        ok = bad == 0.0
    if rank != 0:
        dist.destroy_process_group()
        return

    wm = load_workmodel()
    ms_per_step = elapsed * 1000.0 / args.steps
    value = world * n * args.steps / elapsed
    peak = wm["peak_mul32_per_s_measured"]
    kern = {k: v for k, v in prof1.items() if k.startswith("k_prep")}
    dom = max(kern, key=lambda k: kern[k]["total_ms"]) if kern else None
    roof = None
    if dom:
        avg_s = kern[dom]["total_ms"] / kern[dom]["count"] / 1000.0
        units = wm["kernel_units_M_per_round"][dom] * wm["mul32_per_M"] * n
        achieved = units / avg_s / 1e12
        traffic = None  # HBM bytes per launch from the committed PMC passes (bench/profile.sh, pmc_summary.py)
        pmc = os.path.join(ROOT, "profiles", "pmc_r01.json")
        if os.path.exists(pmc):
            per_round = json.load(open(pmc)).get(dom, {}).get("hbm_bytes_per_round")
            traffic = round(per_round * n) if per_round is not None else None
        roof = {"bound": "valu", "kernel": dom, "achieved": round(achieved, 3), "peak": round(peak / 1e12, 3),
                "unit": "Tmul32/s", "frac": round(achieved * 1e12 / peak, 4), "traffic": traffic,
                "traffic_unit": "bytes per launch (FETCH+WRITE, PMC)",
                "avg_launch_ms": round(avg_s * 1000, 3),
                "work_per_launch": "%d M x %d mul32 x %d rounds" % (wm["kernel_units_M_per_round"][dom],
                                                                   wm["mul32_per_M"], n),
                "measured": "HIP events, %d single-stream batches after the timed region" % args.roofline_steps}
    w_beacon = wm["W_M_per_beacon"]["g2_sig" if sch.sig_len == 96 else "g1_sig"] * wm["mul32_per_M"]
    out = {
        "metric": "verified beacons/sec (whole node), quicknet G1 scheme" if sch.id == 3 else
                  "verified beacons/sec (whole node), %s" % sch.name,
        "value": round(value, 1), "unit": "beacons/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u32 (12x32-bit Montgomery limbs)", "data": "synthetic (GPU-signed chain, seeded key)",
        "config": {"workload": "%s batch verify, %d rounds per GPU per step" % (sch.name, n), "scheme": sch.name,
                   "rounds_per_gpu": n, "global_batch": world * n, "parallelism": "round-shard x%d" % world},
        "roofline": roof,
        "node_roofline_frac": round(value * w_beacon / (peak * world), 4),
        "verdicts_ok": ok,
        "streams": S, "warmup_batches": warm_batches,
        "stages_ms_per_step": {k: round(v["total_ms"] / args.steps, 3) for k, v in prof.items()},
        "stages_ms_single_stream": {k: round(v["total_ms"] / max(1, v["count"]), 3) for k, v in prof1.items()},
        "sign_seconds": round(t_sign, 2),
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(sch.name, pk, rounds, sigs, args.cpu_sample_seconds, args.cpu_threads)
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
