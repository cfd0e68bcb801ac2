#!/usr/bin/env python3
"""bench.py — verified beacons/sec on MI355X for the quicknet scheme (bls-unchained-g1-rfc9380).

Workload (BASELINE.json configs[1]): batch-verify a 1M-round synthetic quicknet chain per GPU — G1 signatures, G2
group key, RFC 9380 hash-to-G1 — with per-round verdicts and SHA-256 randomness, inputs resident in HBM before the
timed region. Weak scaling by default (rounds are independent objects): every rank owns its own
contiguous 1M-round range of the chain, so N GPUs verify N x 1M rounds per step; --total-rounds n splits one n-round
chain over the N GPUs instead (strong scaling, e.g. the north_star's 1M-round chain on 8 GPUs). One "step" = every
rank verifies its rounds once (fresh CSPRNG seed); with N > 1 each batch runs under the node-wide check: the ranks'
level-0 RLC sums are all-gathered over RCCL and ONE pairing check covers the node (drand_amd/dist.py), queued
without a host wait; the verdict bitmaps are all-gathered at the end of the timed steps. With N > 1 under weak scaling
the line also carries "strong_scaling": the north_star's shape, ONE 1,048,576-round chain split over the N ranks
(--strong-total-rounds), timed the same way after the weak leg.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--total-rounds n | --rounds-per-gpu n] [--scheme name]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

`--gpus N` with N > 1 and no WORLD_SIZE in the environment launches the N ranks itself (a child
`python -m torch.distributed.run`, started before this process touches the GPU) and exits with its status; rank 0's
JSON line is the output. Under a launcher, WORLD_SIZE must equal --gpus.

Rank 0 prints ONE JSON line: value = rounds verified by all ranks / max-over-ranks wall time of the K steps.
"roofline": the dominant kernel's integer-multiply rate (its algorithmic mul32 per launch, bench/workmodel.json, over
its HIP-event duration on its own stream) against the measured v_mad_u64_u32 peak (bench/microbench_mul.hip).
"cpu_baseline": the CPU oracle (a C restatement of the reference's per-round VerifyBeacon, oracle/bls_oracle.c) on a
bounded sample, on the host cores this process may use. "single_call": one dh_verify_batch_device call at a time
(the drop-in callers' shape), split by the library over its internal streams.
"""
import argparse
import collections
import ctypes
import datetime
import hashlib
import json
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
R_ORDER = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 steps: ~8 s of timed GPU work at 1M rounds per step, long enough for an outside utilisation sampler
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--total-rounds", type=int, default=0,
                    help="strong scaling: one chain of this many rounds split over the GPUs")
    ap.add_argument("--rounds-per-gpu", type=int, default=0,
                    help="weak scaling: rounds per GPU (default 1048576 when --total-rounds is not given)")
    ap.add_argument("--strong-total-rounds", type=int, default=1 << 20,
                    help="N > 1, weak scaling: also time ONE chain of this many rounds split over the N ranks and report "
                         "it as strong_scaling (0: skip)")
    ap.add_argument("--scheme", default="bls-unchained-g1-rfc9380")
    ap.add_argument("--cpu-sample-seconds", type=float, default=8.0,
                    help="wall time of the bounded CPU-baseline sample (after the GPU legs; kept short so the GPU work is "
                         "not a small share of the run)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stage-times", action="store_true",
                    help="leave the library's HIP-event stage timing off inside the timed region")
    ap.add_argument("--roofline-steps", type=int, default=2, help="single-stream batches timed for the roofline")
    ap.add_argument("--single-call-steps", type=int, default=4, help="one-call-at-a-time batches timed after")
    ap.add_argument("--single-call-split", default="0,1", help="chunk rounds,workers of the one-call split (library "
                    "default: none)")
    ap.add_argument("--single-beacon-reps", type=int, default=20,
                    help="one-beacon latency calls per scheme (bench/single_beacon.py); 0: skip")
    ap.add_argument("--streams", type=int, default=8,
                    help="batches in flight per GPU (local check: host threads, each with its own library worker; "
                         "node-wide check: one host thread keeping this many batches queued)")
    ap.add_argument("--split", default="0",
                    help="one-call split inside the timed region ('chunk,workers'; 0 = each call on one stream: "
                         "the bench already keeps --streams calls in flight)")
    ap.add_argument("--node-check", choices=["auto", "on", "off"], default="auto",
                    help="node-wide RLC check with an all-gather of partial sums (auto: when N > 1)")
    ap.add_argument("--hw-queues", type=int, default=16,
                    help="GPU_MAX_HW_QUEUES for this process (0: keep the environment's)")
    ap.add_argument("--collective-timeout", type=float, default=300.0,
                    help="process-group timeout in seconds (init_process_group(timeout=...)): a collective blocked "
                         "longer than this fails instead of hanging")
    ap.add_argument("--batch-deadline", type=float, default=120.0,
                    help="N > 1: seconds a node batch may stay unfinished before its rank reports the stall (rank, "
                         "batch) and exits with status 3 (dist.BatchWatchdog); 0: off")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="gloo: rehearse N ranks on one GPU with host-staged collectives")
    ap.add_argument("--exchange", choices=["auto", "always"], default="auto",
                    help="always: run the node step's collectives at N = 1 too, over a one-rank process group (the "
                         "RCCL branch rehearsed on one GPU; RCCL takes one rank per GPU)")
    return ap.parse_args()


def load_workmodel():
    with open(os.path.join(ROOT, "bench", "workmodel.json")) as f:
        return json.load(f)


def host_cores():
    """Threads this process may really run: the CPU affinity mask, capped by the cgroup CPU quota (the GPU box
    shows the whole machine's CPUs but grants a share of them); plus the CPU model."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return (min(n, quota) if quota else n), n, quota, model


def cpu_baseline(scheme, pk, rounds, sigs, seconds):
    """Oracle (C restatement of the reference per-round VerifyBeacon) on the usable host cores, bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ctypes as orc
    threads, affinity, quota, model = host_cores()
    # probe with 4 rounds per thread (one round per thread mostly timed the threads' start-up), then size the
    # sample so the timed run takes about `seconds`
    probe = 4 * threads
    t0 = time.perf_counter()
    orc.verify_batch(scheme, pk, rounds[:probe], sigs[:probe], nthreads=threads)
    per = (time.perf_counter() - t0) / probe
    n = int(min(len(rounds), max(probe, seconds / max(per, 1e-9))))
    n -= n % threads if n > threads else 0  # whole rounds per thread
    t0 = time.perf_counter()
    v, _ = orc.verify_batch(scheme, pk, rounds[:n], sigs[:n], nthreads=threads)
    dt = time.perf_counter() - t0
    assert v.all(), "oracle rejected a valid synthetic round"
    return {"value": round(n / dt, 1), "unit": "beacons/s", "cores": threads, "kind": "port",
            "cpu_model": model, "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
            "sample": "%d quicknet rounds (the first of the synthetic chain): per-round decode + subgroup (r*P) + "
                      "hash + 2-pairing VerifyBeacon (CPU restatement, not kyber), %d threads, %.1f s" % (n, threads, dt)}


def launch_ranks(args):
    """--gpus N without a launcher: run this script as N ranks under torch.distributed.run (one process per GPU) in a
    child process; this process never touches the GPU. Rank 0 prints the JSON line; the exit status is the child's."""
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("WORLD_SIZE=%d but --gpus %d: launch one rank per GPU" % (world, args.gpus))
    os.environ["DRANDHIP_SPLIT"] = args.split  # the library's default one-call split, read when it loads
    # 16 hardware queues per process instead of the 4 the environment sets: with 8 batches in flight (16 library
    # streams), a batch's latency-bound tail (MSM reduction, pairing check) no longer holds up another batch's
    # per-round kernels queued behind it on a shared queue (131k-round shard 19.0 -> 20.7 M/s, profiles/r03j); HIP
    # reads it when it initialises, below
    if args.hw_queues > 0:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    import torch
    import torch.distributed as dist
    from drand_amd import _lib, scheme_from_name
    from drand_amd.dist import BatchWatchdog, begin_node_batch, gather_verdicts, pack_bits, shard_rounds, strong_shard

    gloo = args.backend == "gloo"
    dev_index = 0 if gloo else local  # gloo rehearsal: every rank on GPU 0
    lib = _lib.load()
    rc = lib.dh_init(1 << dev_index)
    if rc != 0:
        raise SystemExit("dh_init failed: %s" % _lib.last_error())
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    pg = world > 1 or args.exchange == "always"  # a process group runs the collectives
    xchg = True if args.exchange == "always" else None  # dist._exchanges: collectives at world 1 too
    if pg:
        if "MASTER_ADDR" not in os.environ:  # a one-rank group without a launcher
            so = socket.socket()
            so.bind(("127.0.0.1", 0))
            os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(so.getsockname()[1])
            so.close()
        tmo = datetime.timedelta(seconds=args.collective_timeout)
        if gloo:
            dist.init_process_group("gloo", rank=rank, world_size=world, timeout=tmo)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev, timeout=tmo)
    node_check = args.node_check == "on" or (args.node_check == "auto" and world > 1)

    sch = scheme_from_name(args.scheme)
    weak = args.total_rounds <= 0
    if weak:
        per_gpu = args.rounds_per_gpu or (1 << 20)
        total = world * per_gpu
    else:
        total = args.total_rounds
    sk = (int.from_bytes(hashlib.sha256(b"drandhip-sk-" + args.scheme.encode()).digest(), "big") % R_ORDER).to_bytes(32, "big")
    pk = sch.public_key(sk)
    S = max(1, args.streams)
    pbytes = lib.dh_partial_bytes(sch.id)

    class Work:
        """One rank's rounds resident in HBM, with 2 x S output slots: a slot's verdicts are packed (pack_bits, on
        torch's stream) after its batch finished, and the slot is not handed to another batch before that packing has
        run (its event; ADVICE r04: the next begin's memset on the library stream raced the packing). With 2 x S slots
        the packing of a slot finished long before the slot comes round again, so the wait is a formality."""

        def __init__(self, rnds):
            self.rounds = rnds
            self.n = len(rnds)
            t0 = time.perf_counter()
            self.sigs = sch.sign_beacons(sk, rnds)  # synthetic chain, signed on the GPU (not timed)
            self.sign_s = time.perf_counter() - t0
            self.d_rounds = torch.from_numpy(rnds.view(np.int64)).to(dev)
            self.d_sigs = torch.from_numpy(self.sigs).to(dev)
            self.d_verdict = [torch.zeros(self.n, dtype=torch.uint8, device=dev) for _ in range(2 * S)]
            self.d_rand = [torch.zeros((self.n, 32), dtype=torch.uint8, device=dev) for _ in range(2 * S)]
            self.d_part = [torch.zeros(pbytes, dtype=torch.uint8, device=dev) for _ in range(2 * S)]
            self.packed = [None] * (2 * S)
            self.used = set()

        def take(self, slot):
            ev = self.packed[slot]
            if ev is not None:
                ev.synchronize()
            self.used.add(slot)
            return slot

        def pack(self, slot):
            bits = pack_bits(self.d_verdict[slot])
            ev = torch.cuda.Event()
            ev.record()
            self.packed[slot] = ev
            return bits

        def all_valid(self):
            return all(bool(self.d_verdict[k].cpu().numpy().all()) for k in sorted(self.used))

    if weak:
        work = Work(shard_rounds(rank, world, per_gpu))
    else:
        work = Work(strong_shard(rank, world, args.total_rounds))
    n = work.n
    rounds, sigs, t_sign = work.rounds, work.sigs, work.sign_s
    d_rounds, d_sigs = work.d_rounds, work.d_sigs
    torch.cuda.synchronize()
    state = {"node_check": node_check,
             "watchdog": BatchWatchdog(args.batch_deadline, rank) if pg and args.batch_deadline > 0 else None}

    def verify(wk, slot):
        rc = lib.dh_verify_batch_device(sch.id, pk, len(pk), ctypes.c_void_p(wk.d_rounds.data_ptr()),
                                        ctypes.c_void_p(wk.d_sigs.data_ptr()), sch.sig_len, None, 0, None, wk.n,
                                        ctypes.c_void_p(wk.d_verdict[slot].data_ptr()),
                                        ctypes.c_void_p(wk.d_rand[slot].data_ptr()), 0, None, None)
        if rc != 0:
            raise RuntimeError("dh_verify_batch_device: %s" % _lib.last_error())

    def run_node_steps(wk, k_steps, streams, gather=True):
        """k_steps batches under the node-wide check, `streams` in flight, driven by ONE host thread: batch k is begun,
        its record all-gathered and its check queued (no host wait under nccl), and the oldest batch is finished once
        `streams` are queued. One thread issues every rank's collectives in the same order over one process group."""
        pending = collections.deque()
        bits = []
        ht = state.setdefault("node_host_s", collections.Counter())
        # a batch whose collective or check never completes (a dead or hung peer) ends this rank with a message naming
        # the rank and the batch instead of a silent hang (dist.BatchWatchdog)
        wd = state.get("watchdog")

        def retire():
            slot, h, key = pending.popleft()
            t0 = time.perf_counter()
            h.finish()
            if wd is not None:
                wd.end(key)
            t1 = time.perf_counter()
            bits.append(wk.pack(slot))
            ht["finish_wait"] += t1 - t0
            ht["pack"] += time.perf_counter() - t1
            ht["batches"] += 1

        for k in range(k_steps):
            if len(pending) == streams:
                retire()
            slot = wk.take(k % (2 * streams))
            # the record, the collective and the check of a batch run on that batch's own library stream
            # (dist.begin_node_batch): no stream shared by the batches carries a wait for another batch's record (r04a
            # ordered them all through torch's current stream and chained every batch's per-round kernels behind the
            # previous batch's MSM: 14.2 M/s at 131k rounds, 8 slots)
            t0 = time.perf_counter()
            state["batch_seq"] = key = state.get("batch_seq", 0) + 1
            if wd is not None:
                wd.begin(key, "%d rounds, slot %d" % (wk.n, slot))
            pending.append((slot, begin_node_batch(lib, sch, pk, wk.d_rounds, wk.d_sigs, wk.n, wk.d_verdict[slot],
                                                   wk.d_rand[slot], wk.d_part[slot], world, None, stage_host=gloo,
                                                   rank=rank, inputs_ready=True, exchange=xchg), key))
            ht["begin_exchange_check"] += time.perf_counter() - t0
        while pending:
            retire()
        torch.cuda.synchronize()
        if pg and gather and k_steps:
            b = torch.cat(bits)
            gather_verdicts(b.cpu() if gloo else b, world, exchange=xchg)
        torch.cuda.synchronize()

    def run_steps(wk, k_steps, streams, gather=True):
        """k_steps batches, `streams` in flight: thread t runs steps t, t+streams, ... alternating over its two slots."""
        if state["node_check"]:
            return run_node_steps(wk, k_steps, streams, gather)
        errs = []
        bits = [None] * k_steps

        def worker(t):
            try:
                torch.cuda.set_device(dev_index)
                for j, k in enumerate(range(t, k_steps, streams)):
                    slot = wk.take(2 * t + (j & 1))
                    verify(wk, slot)
                    bits[k] = wk.pack(slot)
            except Exception as e:  # surfaced below
                errs.append(e)

        ths = [threading.Thread(target=worker, args=(t,)) for t in range(min(streams, k_steps))]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        if errs:
            raise errs[0]
        if pg and gather and k_steps:  # whole-node verdict bitmaps: one all-gather after the batches
            b = torch.cat(bits)
            gather_verdicts(b.cpu() if gloo else b, world, exchange=xchg)
        torch.cuda.synchronize()

    def timed(wk, k_steps):
        """Barrier + synchronize on both sides of k_steps batches; the max over ranks of the wall time."""
        if pg:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run_steps(wk, k_steps, S)
        torch.cuda.synchronize()
        if pg:
            dist.barrier()
        return time.perf_counter() - t0

    def profile_read():
        buf = ctypes.create_string_buffer(1 << 16)
        lib.dh_profile_read(buf, len(buf))
        return json.loads(buf.value.decode())

    # warm-up: at least one batch per stream, so every library worker (stream + device workspace) exists before
    # the timed region; W < S would leave workspace allocation inside it
    warm_batches = max(args.warmup, 2 * S) if args.warmup else 0
    run_steps(work, warm_batches, S)
    lib.dh_profile(0 if args.no_stage_times else 1)
    state["node_host_s"] = collections.Counter()  # the timed region's host time per pipeline phase
    elapsed = timed(work, args.steps)
    prof = profile_read()
    # sanity (outside the timed region): every synthetic round verifies, randomness = SHA-256(sig)
    ok = work.all_valid()
    r0 = work.d_rand[min(work.used)].cpu().numpy()[0].tobytes()
    ok = ok and r0 == hashlib.sha256(sigs[0].tobytes()).digest()
    node_host = dict(state.get("node_host_s", {}))

    # The north_star's shape beside the weak-scaling value: ONE --strong-total-rounds chain (1M) split over the N
    # ranks, each rank's shard under the node-wide check, timed the same way (after the weak leg, same workers).
    strong = None
    if weak and world > 1 and args.strong_total_rounds > 0:
        swork = Work(strong_shard(rank, world, args.strong_total_rounds))
        torch.cuda.synchronize()
        run_steps(swork, 2 * S, S)
        s_el = timed(swork, args.steps)
        s_ok = swork.all_valid()
        t = torch.tensor([s_el, 0.0 if s_ok else 1.0], dtype=torch.float64, device="cpu" if gloo else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        s_el, s_ok = float(t[0]), float(t[1]) == 0.0
        strong = {"scaling": "strong", "rounds_total": args.strong_total_rounds, "rounds_per_gpu": swork.n,
                  "steps": args.steps, "value": round(args.strong_total_rounds * args.steps / s_el, 1),
                  "unit": "beacons/s", "ms_per_step": round(s_el * 1000.0 / args.steps, 3), "verdicts_ok": s_ok,
                  "what": "one %d-round %s chain split over the %d ranks per step (node-wide RLC check), max-over-"
                          "ranks wall time of the steps" % (args.strong_total_rounds, sch.name, world)}
        del swork

    # Roofline pass (after the timed region, not counted in `value`): with S batches in flight the kernels of
    # different batches share the CUs, so per-launch durations there are not one kernel's speed. Single-stream
    # local batches give each kernel the whole GPU; the dominant kernel's roofline comes from their HIP events (on
    # the library's stream). bench/profile.sh records the rocprofv3 kernel trace of the same batches.
    state["node_check"] = False
    prof1 = {}
    if args.roofline_steps:
        lib.dh_profile(1)
        run_steps(work, args.roofline_steps, 1, gather=False)
        prof1 = profile_read()
        lib.dh_profile(0)
    single = None
    if args.single_call_steps and world == 1:  # the drop-in shape: ONE call at a time, split internally
        chunk, workers = (int(x) for x in args.single_call_split.split(","))
        lib.dh_set_split(chunk, workers)
        run_steps(work, 1, 1, gather=False)  # warm the split workers
        t1 = time.perf_counter()
        run_steps(work, args.single_call_steps, 1, gather=False)
        dt = time.perf_counter() - t1
        single = {"value": round(n * args.single_call_steps / dt, 1), "unit": "beacons/s",
                  "ms_per_call": round(dt * 1000 / args.single_call_steps, 3),
                  "split": ("%d-round chunks x %d streams" % (chunk, workers)) if chunk else "none (library default)",
                  "calls": args.single_call_steps}
        # the CheckPastBeacons shape: one call over a whole stored chain (4 x the bench window, the same signed
        # rounds repeated); the call's one exposed tail is amortised over 4x the rounds
        reps = 4
        d_r4, d_s4 = d_rounds.repeat(reps), d_sigs.repeat(reps, 1)
        d_v4 = torch.zeros(n * reps, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()

        def call4():
            rc = lib.dh_verify_batch_device(sch.id, pk, len(pk), ctypes.c_void_p(d_r4.data_ptr()),
                                            ctypes.c_void_p(d_s4.data_ptr()), sch.sig_len, None, 0, None, n * reps,
                                            ctypes.c_void_p(d_v4.data_ptr()), None, 0, None, None)
            if rc != 0:
                raise RuntimeError("dh_verify_batch_device: %s" % _lib.last_error())

        call4()
        t1 = time.perf_counter()
        for _ in range(2):
            call4()
        dt4 = (time.perf_counter() - t1) / 2
        ok = ok and bool(d_v4.cpu().numpy().all())
        single["whole_chain_call"] = {"rounds": n * reps, "value": round(n * reps / dt4, 1), "ms_per_call": round(dt4 * 1000, 3),
                                      "calls": 2}
        del d_r4, d_s4, d_v4
        lib.dh_set_split(0, 1)

    # the drop-in's one-beacon calls (VerifyBeacon / VerifyRecovered / one-round Recover), one at a time from the host,
    # every scheme, warm and cold key cache, beside the CPU restatement's per-verify time on one core
    # (bench/single_beacon.py; the small-batch path of drandhip.cpp verify_small)
    single_beacon = None
    if world == 1 and args.single_beacon_reps > 0:
        sys.path.insert(0, os.path.join(ROOT, "bench"))
        import single_beacon as sbm
        sb = sbm.measure(reps=args.single_beacon_reps, with_oracle=not args.no_cpu_baseline)
        ok = ok and all(v["verdicts_ok"] for v in sb.values())
        single_beacon = {name: {k: (v["p50"] if isinstance(v, dict) else v) for k, v in e.items()
                                if k not in ("recover_shape", "verdicts_ok")} for name, e in sb.items()}
        single_beacon["what"] = ("p50 ms of one host call at a time (%d calls; cold = key-cache miss on every call (6 keys cycled), two_keys = two keys alternating; "
                                 "recover = n 64 / t 33, one round); oracle = the C restatement on one core"
                                 % args.single_beacon_reps)

    if pg:
        t = torch.tensor([elapsed, 0.0 if ok else 1.0], dtype=torch.float64, device="cpu" if gloo else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, bad = float(t[0]), float(t[1])
        ok = bad == 0.0
    if rank != 0:
        if state["watchdog"] is not None:
            state["watchdog"].stop()
        dist.destroy_process_group()
        return

    wm = load_workmodel()
    ms_per_step = elapsed * 1000.0 / args.steps
    value = total * args.steps / elapsed
    peak = wm["peak_mul32_per_s_measured"]
    units = wm["kernel_units_M_per_round"]
    kern = {k: v for k, v in prof1.items() if k in units}
    dom = max(kern, key=lambda k: kern[k]["total_ms"]) if kern else None
    roof = None
    if dom:
        avg_s = kern[dom]["total_ms"] / kern[dom]["count"] / 1000.0
        achieved = units[dom] * wm["mul32_per_M"] * n / avg_s
        # HBM bytes per launch from the committed PMC passes (bench/profile.sh, pmc_summary.py); the summary is kept
        # under bench/ (profiles/ does not travel to the GPU box) with the same file in profiles/
        traffic = None
        pmc = os.path.join(ROOT, wm.get("pmc_file", "bench/pmc_r02h.json"))
        if os.path.exists(pmc):
            per_round = json.load(open(pmc)).get(dom, {}).get("hbm_bytes_per_round")
            traffic = round(per_round * n) if per_round is not None else None
        roof = {"bound": "valu", "kernel": dom, "achieved": round(achieved / 1e12, 3), "peak": round(peak / 1e12, 3),
                "unit": "Tmul32/s", "frac": round(achieved / peak, 4), "traffic": traffic,
                "traffic_unit": "bytes per launch (WRITE_SIZE + FETCH_SIZE, PMC; FETCH doubled for this streaming-read "
                                "kernel per MI355X_MICROARCH.md)",
                "avg_launch_ms": round(avg_s * 1000, 3),
                "work_per_launch": "%d M x %d mul32 x %d rounds" % (units[dom], wm["mul32_per_M"], n),
                "peak_source": wm["peak_source"],
                "measured": "HIP events, %d single-stream batches after the timed region" % args.roofline_steps}
    ex_key = "g2_sig" if sch.sig_len == 96 else "g1_sig"
    executed = wm["executed_M_per_beacon"][ex_key] * wm["mul32_per_M"]
    out = {
        "metric": "verified beacons/sec (whole node), quicknet G1 scheme" if sch.id == 3 else
                  "verified beacons/sec (whole node), %s" % sch.name,
        "value": round(value, 1), "unit": "beacons/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3), "higher_is_better": True, "scaling": "weak" if weak else "strong",
        "vs_baseline": None, "dtype": "u32 (Fp products on 14x28-bit limbs, 64-bit MAD accumulators; 12x32-bit Montgomery storage)", "data": "synthetic (GPU-signed chain, seeded key)",
        "config": {"workload": "%s batch verify of a %d-round chain, %s" % (
                       sch.name, total, "%d rounds per GPU" % n if weak else "split over %d GPU(s)" % world),
                   "scheme": sch.name, "rounds_total": total, "rounds_per_gpu": n, "global_batch": total,
                   "parallelism": "round-shard x%d%s" % (world, (", node-wide RLC check (%s)" % (
                       ("%s all-gather%s" % ("gloo, host-staged" if gloo else "RCCL", ", one-rank group" if world == 1
                                             else "")) if pg else "one rank, no exchange")) if node_check else "")},
        "roofline": roof,
        "node_roofline_frac": round(value * executed / (peak * world), 4),
        "node_roofline_basis": "executed kernel work %d M/beacon (prep_sig + prep_msg + MSM, bench/workmodel.json "
                               "executed_M_per_beacon) at the measured peak" % wm["executed_M_per_beacon"][ex_key],
        "verdicts_ok": ok,
        "streams": S, "warmup_batches": warm_batches, "hip_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
        "stages_ms_per_step": {k: round(v["total_ms"] / args.steps, 3) for k, v in prof.items()},
        "stages_ms_single_stream": {k: round(v["total_ms"] / max(1, v["count"]), 3) for k, v in prof1.items()},
        "single_call": single,
        "single_beacon_ms": single_beacon,
        "strong_scaling": strong,
        "node_host_ms_per_batch": ({k: round(v * 1000 / node_host["batches"], 3) for k, v in node_host.items()
                                    if k != "batches"} if node_host.get("batches") else None),
        "sign_seconds": round(t_sign, 2),
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(sch.name, pk, rounds, sigs, args.cpu_sample_seconds)
    print(json.dumps(out), flush=True)
    if state["watchdog"] is not None:
        state["watchdog"].stop()
    if pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
