"""GPU tests of the multi-GPU protocol and the device-backed range sync:
  * the node-wide check (dh_batch_begin -> dh_check_partials -> dh_batch_finish) on every scheme, G2 included,
    with a one-round shard (identity partial sums) and a corruption on a shard boundary of a real chained chain;
  * two fresh processes (spawn, gloo, both on GPU 0, the rehearsal shape of bench.py --backend gloo) running
    drand_amd.dist.replay_shard — exchange_halo + verify_node_batch + gather_verdicts with the real library — on a
    sequential chained chain with a fault on the shard boundary, and with the boundary round missing from the store;
    the whole-node faulty set equals the serial oracle replay (chain/beacon/sync_manager.go:191-225);
  * relay-s3 sync (/root/reference/cmd/relay-s3/main.go:182-195) verified through the device.
The CPU oracle (oracle/, test infrastructure) is the checker."""
import ctypes
import hashlib
import json
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bench"))
GOLD = os.path.join(ROOT, "tests", "golden")
R_ORDER = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
CHAINED = "pedersen-bls-chained"
GENESIS = hashlib.sha256(b"drandhip-genesis").digest()

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dh():
    import torch
    import drand_amd
    from drand_amd import _lib
    torch.zeros(1, device="cuda")
    assert _lib.load().dh_init(0) == 0, _lib.last_error()
    return drand_amd


def _secret(tag):
    return (int.from_bytes(hashlib.sha256(tag).digest(), "big") % R_ORDER).to_bytes(32, "big")


def _chain(s, n, every=64, seed=5):
    """A sequential chained chain of n rounds (round k signed over the stored signature of k-1, genesis seed before
    round 1) signed on the device; cut into segments of `every` rounds so signing takes `every` steps (segment heads
    are signed over a random record and so fail, as in chainsynth)."""
    import chainsynth
    sk = _secret(b"node-" + s.name.encode())
    breaks = np.arange(every - 1, n - 1, every, dtype=np.int64)
    sigs = chainsynth.sign_chain(s, sk, 1, n, GENESIS, breaks, np.random.default_rng(seed))
    return sk, s.public_key(sk), sigs


def _oracle_replay(oracle, name, pk, sig_of, first, last):
    """Serial CheckPastBeacons verdicts over a trimmed store {round: sig} (Get error or VerifyBeacon error ->
    faulty), the oracle's batch entry point on 16 threads."""
    faulty, todo = [], []
    for r in range(first, last + 1):
        if r not in sig_of or (name == CHAINED and (r - 1) not in sig_of):
            faulty.append(r)
        else:
            todo.append(r)
    lib = oracle.lib()
    sl = 96 if name.startswith("pedersen") else 48
    rs = np.array(todo, dtype=np.uint64)
    ss = np.zeros((len(todo), sl), np.uint8)
    ps = np.zeros((len(todo), 96), np.uint8)
    ls = np.zeros(len(todo), np.uint32)
    ok = np.ones(len(todo), bool)
    for k, r in enumerate(todo):
        if len(sig_of[r]) != sl:
            ok[k] = False
            continue
        ss[k] = np.frombuffer(sig_of[r], np.uint8)
        if name == CHAINED:
            p = sig_of[r - 1]
            ps[k, :len(p)] = np.frombuffer(p, np.uint8)
            ls[k] = len(p)
    ov = np.zeros(len(todo), np.uint8)
    lib.or_verify_batch(oracle.sid(name), pk, len(pk), rs.ctypes.data, ss.ctypes.data, sl,
                        ps.ctypes.data if name == CHAINED else None, 96, ls.ctypes.data if name == CHAINED else None,
                        len(todo), 16, ov.ctypes.data, None)
    faulty += [r for r, o, k in zip(todo, ov, ok) if not (o and k)]
    return sorted(faulty)


# ---------------------------------------------------------------- node-wide check, in one process
@pytest.mark.parametrize("mode", ["device", "host"])
@pytest.mark.parametrize("name", ["bls-unchained-g1-rfc9380", "pedersen-bls-unchained", CHAINED, "bls-unchained-on-g1"])
def test_node_wide_check_all_schemes(dh, oracle, name, mode):
    """Three shards begun as three batches — one of them a single round, which contributes the identity — their
    level-0 sums combined by ONE pairing check, then finished. mode "device": the protocol the multi-GPU bench and
    replay run — dh_batch_begin ordered onto torch's stream, then per batch dh_batch_check of the three records on its
    own worker (no host wait) and dh_batch_finish(DH_NODE_CHECKED), which returns 1 / 0; mode "host": the standalone
    dh_check_partials and an explicit node_pass. A clean chain passes the node check and every round is accepted; with
    a corruption on the shard boundary (chained: the last round of shard 0 stores another round's signature, so round k
    and k+1 fail, k+1 being the one-round shard) the node check fails and each shard's own check + bisection gives the
    oracle's verdicts."""
    import torch
    from drand_amd import _lib
    lib = _lib.load()
    s = dh.scheme_from_name(name)
    n = 2400 if s.sig_len == 96 else 6000
    b0 = n // 2
    shards = [(0, b0 - 1), (b0 - 1, b0), (b0, n)]  # the middle shard holds ONE round
    if s.chained:
        sk, pk, sigs = _chain(s, n, every=n)  # one segment: every round is a real link
    else:
        sk = _secret(b"node-" + name.encode())
        pk = s.public_key(sk)
        sigs = s.sign_beacons(sk, np.arange(1, n + 1, dtype=np.uint64))
    rounds = np.arange(1, n + 1, dtype=np.uint64)
    dev = torch.device("cuda", 0)
    pb = lib.dh_partial_bytes(s.id)
    assert pb == 2 * (72 if s.sig_len == 96 else 36) * 4 + 16

    def run(sig_arr, seed, with_stats=True):
        prev = np.zeros((n, 96), np.uint8)
        plen = np.full(n, 96, np.uint32)
        if s.chained:  # the stored column: prev of round k = stored sig of k-1 (halo across shards included)
            prev[1:] = sig_arr[:-1]
            prev[0, :32] = np.frombuffer(GENESIS, np.uint8)
            plen[0] = 32
        d_r = torch.from_numpy(rounds.view(np.int64)).to(dev)
        d_s = torch.from_numpy(np.ascontiguousarray(sig_arr)).to(dev)
        d_p = torch.from_numpy(prev).to(dev)
        d_l = torch.from_numpy(plen.view(np.int32)).to(dev)
        d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
        parts = torch.zeros(len(shards) * pb, dtype=torch.uint8, device=dev)
        handles = []
        sl = s.sig_len
        # an explicit stream: torch's default stream is the NULL stream, which the library reads as "no stream"
        cur = torch.cuda.Stream(device=dev)
        cur.wait_stream(torch.cuda.current_stream(dev))  # the inputs above
        sp = ctypes.c_void_p(cur.cuda_stream) if mode == "device" else None
        if mode == "host":
            torch.cuda.synchronize()
        for k, (lo, hi) in enumerate(shards):
            b = ctypes.c_void_p()
            rc = lib.dh_batch_begin(s.id, pk, len(pk), ctypes.c_void_p(d_r.data_ptr() + 8 * lo),
                                    ctypes.c_void_p(d_s.data_ptr() + sl * lo), sl,
                                    ctypes.c_void_p(d_p.data_ptr() + 96 * lo) if s.chained else None,
                                    96 if s.chained else 0,
                                    ctypes.c_void_p(d_l.data_ptr() + 4 * lo) if s.chained else None, hi - lo,
                                    ctypes.c_void_p(d_v.data_ptr() + lo), None, seed + 101 * k, sp, ctypes.byref(b),
                                    ctypes.c_void_p(parts.data_ptr() + k * pb))
            assert rc == 0, _lib.last_error()
            handles.append(b)
        if mode == "device":
            # each record is complete in its batch's stream order (dh_batch_stream): the current stream waits for all
            # three, and each check is ordered after the current stream's work
            for b in handles:
                cur.wait_stream(torch.cuda.ExternalStream(lib.dh_batch_stream(b), device=dev))
            with torch.cuda.stream(cur):
                snap = parts.clone()
            results, stats = [], []
            for b in handles:
                assert lib.dh_batch_check(b, ctypes.c_void_p(parts.data_ptr()), len(shards), sp) == 0, _lib.last_error()
            for b in handles:
                st = (ctypes.c_uint64 * 4)()
                r = lib.dh_batch_finish(b, _lib.DH_NODE_CHECKED, st if with_stats else None)
                assert r in (0, 1), _lib.last_error()
                results.append(r)
                stats.append(list(st))
            torch.cuda.synchronize()
            assert not snap[pb:2 * pb].cpu().numpy().any(), "a one-round shard must contribute the identity"
            assert len(set(results)) == 1  # every batch saw the same node-wide result
            return results[0], d_v.cpu().numpy().astype(bool), stats
        torch.cuda.synchronize()
        one = parts[pb:2 * pb].cpu().numpy()
        assert not one.any(), "a one-round shard must contribute the identity"
        ok = ctypes.c_int(-1)
        assert lib.dh_check_partials(s.id, pk, len(pk), ctypes.c_void_p(parts.data_ptr()), len(shards),
                                     ctypes.byref(ok)) == 0, _lib.last_error()
        stats = []
        for b in handles:
            st = (ctypes.c_uint64 * 4)()
            assert lib.dh_batch_finish(b, ok.value, st) == 0, _lib.last_error()
            stats.append(list(st))
        torch.cuda.synchronize()
        return ok.value, d_v.cpu().numpy().astype(bool), stats

    sig_of = {r + 1: sigs[r].tobytes() for r in range(n)}
    sig_of[0] = GENESIS
    want_clean = _oracle_replay(oracle, name, pk, sig_of, 1, n)
    ok, v, stats = run(sigs, 7)
    assert [int(r) + 1 for r in np.flatnonzero(~v)] == want_clean
    assert want_clean == [] and ok == 1 and v.all()  # node check passed: no shard ran its own level-0 check
    assert stats[0][1] == 0 and stats[2][1] == 0
    bad = sigs.copy()
    bad[b0 - 2] = bad[b0 - 3]  # the last round of shard 0 stores another round's signature
    bad[n - 1, 5] ^= 0x10
    ok, v, stats = run(bad, 8)
    assert ok == 0
    sig_of = {r + 1: bad[r].tobytes() for r in range(n)}
    sig_of[0] = GENESIS
    want = _oracle_replay(oracle, name, pk, sig_of, 1, n)
    assert [int(r) + 1 for r in np.flatnonzero(~v)] == want
    assert {b0 - 1, n} <= set(want) and (not s.chained or b0 in want)
    ref, _ = s.verify_beacons(pk, rounds, bad, [p for p in ([GENESIS] + [x.tobytes() for x in bad[:-1]])]
                              if s.chained else None, seed=5)
    assert np.array_equal(ref, v)
    if mode == "device":
        # only the one-round shard is bad, finished without stats (NodeBatch.finish()): its identity record lets the
        # node check pass on the other shards' sums (unchained schemes), and the round must still get its own check
        # (it used to be marked valid by the node check)
        lone = sigs.copy()
        lone[b0 - 1] = lone[b0 + 3]
        ok, v, _ = run(lone, 9, with_stats=False)
        sig_of = {r + 1: lone[r].tobytes() for r in range(n)}
        sig_of[0] = GENESIS
        want = _oracle_replay(oracle, name, pk, sig_of, 1, n)
        assert [int(r) + 1 for r in np.flatnonzero(~v)] == want
        assert b0 in want and ok == (0 if s.chained else 1)


def test_node_batch_abandoned(dh):
    """A gathered record whose status word is nonzero (a rank whose dh_batch_begin failed) makes the node-wide check
    abandon the batch: dh_batch_finish(DH_NODE_CHECKED) returns DH_EABANDONED and marks no round valid, and
    dh_check_partials returns DH_EABANDONED too."""
    import torch
    from drand_amd import _lib
    lib = _lib.load()
    s = dh.scheme_from_name("bls-unchained-g1-rfc9380")
    sk = _secret(b"abandon")
    pk = s.public_key(sk)
    n = 2048
    rounds = np.arange(1, n + 1, dtype=np.uint64)
    dev = torch.device("cuda", 0)
    d_r = torch.from_numpy(rounds.view(np.int64)).to(dev)
    d_s = torch.from_numpy(s.sign_beacons(sk, rounds)).to(dev)
    d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
    pb = lib.dh_partial_bytes(s.id)
    parts = torch.zeros(2 * pb, dtype=torch.uint8, device=dev)
    parts[2 * pb - 16] = 1  # the second rank's record: began nothing, status 1
    cur = torch.cuda.Stream(device=dev)  # explicit: the default stream is the NULL stream ("no stream" to the library)
    cur.wait_stream(torch.cuda.current_stream(dev))
    sp = ctypes.c_void_p(cur.cuda_stream)
    b = ctypes.c_void_p()
    assert lib.dh_batch_begin(s.id, pk, len(pk), ctypes.c_void_p(d_r.data_ptr()), ctypes.c_void_p(d_s.data_ptr()), 48,
                              None, 0, None, n, ctypes.c_void_p(d_v.data_ptr()), None, 3, sp, ctypes.byref(b),
                              ctypes.c_void_p(parts.data_ptr())) == 0, _lib.last_error()
    # the status byte was written on the current stream, the record on the batch's stream: the check is queued on the
    # batch's stream after the current stream's work
    assert lib.dh_batch_check(b, ctypes.c_void_p(parts.data_ptr()), 2, sp) == 0, _lib.last_error()
    assert lib.dh_batch_finish(b, _lib.DH_NODE_CHECKED, None) == _lib.DH_EABANDONED
    torch.cuda.synchronize()
    assert not d_v.cpu().numpy().any()
    ok = ctypes.c_int(-1)
    assert lib.dh_check_partials(s.id, pk, len(pk), ctypes.c_void_p(parts.data_ptr()), 2, ctypes.byref(ok)) == \
        _lib.DH_EABANDONED
    parts[2 * pb - 16] = 0  # the same records with status 0: the node check passes (identity + the batch's sums)
    assert lib.dh_check_partials(s.id, pk, len(pk), ctypes.c_void_p(parts.data_ptr()), 2, ctypes.byref(ok)) == 0
    assert ok.value == 1


# ---------------------------------------------------------------- two processes, gloo, one GPU
def _free_port():
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    p = so.getsockname()[1]
    so.close()
    return p


def _replay_worker(rank, world, port, name, pk, first, last, local, genesis, q, stage_host=None, backend="gloo",
                   exchange=None):
    try:
        import torch
        import torch.distributed as dist
        sys.path.insert(0, ROOT)
        from drand_amd import _lib, scheme_from_name
        from drand_amd.dist import replay_shard
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        lib = _lib.load()
        assert lib.dh_init(1) == 0, _lib.last_error()
        torch.cuda.set_device(0)
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        s = scheme_from_name(name)
        res = []
        for case_local in local:
            res.append(replay_shard(lib, s, pk, first, last, case_local, rank, world, prev_of_first=genesis, seed=0,
                                    stage_host=stage_host, exchange=exchange))
        q.put({"rank": rank, "faulty": res})
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 - reported to the parent
        import traceback
        q.put({"rank": rank, "error": repr(e) + traceback.format_exc()})


@pytest.mark.parametrize("stage_host", [None, False])
def test_replay_shard_two_processes(dh, oracle, stage_host):
    """dist.replay_shard in two spawned processes (gloo, both on GPU 0): a sequential chained chain of 3000 rounds,
    (a) round hi0 (the last round of rank 0) stores round hi0-1's signature: hi0 fails and so does hi0+1, the
    first round of rank 1, whose previous signature reaches it only through exchange_halo; (b) round hi0 is missing:
    hi0 and hi0+1 are reported missing (Get error) through MISSING_HALO; (c) the clean chain. Each whole-node faulty
    set equals the serial oracle replay over the unsharded store. stage_host=False keeps the records on the device
    (gloo's CUDA all-gather): the device-ordered branch of begin_node_batch — the library orders torch's stream after
    the record and its check after the collective — which the nccl backend takes on a multi-GPU node."""
    import torch.multiprocessing as mp
    from drand_amd.dist import shard_range
    s = dh.scheme_from_name(CHAINED)
    n, world = 3000, 2
    sk, pk, sigs = _chain(s, n, every=100, seed=9)
    store = {r + 1: sigs[r].tobytes() for r in range(n)}
    store[0] = GENESIS
    _, hi0 = shard_range(0, world, n)  # rank 0 owns rounds 1..hi0
    case_a = dict(store)
    case_a[hi0] = store[hi0 - 1]
    case_b = dict(store)
    del case_b[hi0]
    cases = [case_a, case_b, store]
    local = {}
    for rank in range(world):
        lo, hi = shard_range(rank, world, n)
        local[rank] = [{r: c[r] for r in range(lo + 1, hi + 1) if r in c} for c in cases]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_replay_worker, args=(r, world, port, CHAINED, pk, 1, n, local[r], GENESIS, q,
                                                      stage_host))
             for r in range(world)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    errs = [m["error"] for m in msgs if "error" in m]
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs)
    by_rank = {m["rank"]: m["faulty"] for m in msgs}
    assert by_rank[0] == by_rank[1]  # every rank returns the whole node's faulty set
    for c, got in zip(cases, by_rank[0]):
        want = _oracle_replay(oracle, CHAINED, pk, c, 1, n)
        assert got == want
    heads = [k + 1 for k in range(100, n, 100)]  # segment heads of the signer (see _chain)
    assert by_rank[0][2] == heads
    assert {hi0, hi0 + 1} <= set(by_rank[0][0]) and {hi0, hi0 + 1} <= set(by_rank[0][1])


def test_replay_rccl_one_rank_group(dh, oracle):
    """The RCCL branch on one GPU: dist.replay_shard in a spawned process over a one-rank `nccl` process group with
    exchange=True, so the halo exchange, the all-gather of the partial record on the batch's library stream
    (torch ExternalStream -> RCCL's stream -> dh_batch_check) and the verdict gather all run through RCCL, as on a
    multi-GPU node (RCCL takes one rank per GPU, so two ranks cannot share this box's GPU). A chained chain with a
    swapped and a missing record, and the clean chain: the faulty sets equal the serial oracle replay."""
    import torch.multiprocessing as mp
    s = dh.scheme_from_name(CHAINED)
    n = 2000
    sk, pk, sigs = _chain(s, n, every=250, seed=11)
    store = {r + 1: sigs[r].tobytes() for r in range(n)}
    store[0] = GENESIS
    case_a = dict(store)
    case_a[700] = store[699]
    case_b = dict(store)
    del case_b[1500]
    cases = [case_a, case_b, store]
    local = [{r: c[r] for r in range(1, n + 1) if r in c} for c in cases]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_replay_worker, args=(0, 1, _free_port(), CHAINED, pk, 1, n, local, GENESIS, q, False,
                                                 "nccl", True))
    p.start()
    msg = q.get(timeout=240)
    p.join(timeout=60)
    assert "error" not in msg, msg.get("error")
    assert p.exitcode == 0
    for c, got in zip(cases, msg["faulty"]):
        assert got == _oracle_replay(oracle, CHAINED, pk, c, 1, n)
    assert {700, 701} <= set(msg["faulty"][0]) and {1500, 1501} <= set(msg["faulty"][1])
    assert msg["faulty"][2] == [k + 1 for k in range(250, n, 250)]


def test_bench_rccl_one_rank_group():
    """bench.py --exchange always at N = 1: the node-wide batches of the multi-GPU bench (record all-gathered over RCCL
    on each batch's stream, check queued after it, verdict bitmaps gathered) on a one-rank nccl group; every verdict
    valid and the line names the RCCL all-gather."""
    import subprocess
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--exchange", "always", "--node-check", "on",
           "--rounds-per-gpu", "131072", "--steps", "4", "--warmup", "2", "--streams", "4", "--no-cpu-baseline",
           "--roofline-steps", "0", "--single-call-steps", "0"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, out.stdout[-2000:]
    res = json.loads(line[0])
    assert res["n_gpus"] == 1 and res["verdicts_ok"] is True
    assert "RCCL all-gather, one-rank group" in res["config"]["parallelism"]


# ---------------------------------------------------------------- relay-s3 through the device
def test_relay_s3_sync_device(dh, oracle):
    """relay-s3 `sync` batched per window with the verifying client on the device: the uploaded rounds equal the
    serial loop's on the oracle (a missing round and a round carrying another round's signature are skipped), and
    every body is the Go encoding/json of RandomData with randomness = SHA-256(signature)."""
    import base64
    from drand_amd.chain import Info
    from drand_amd.client import BatchVerifyingClient, relay_s3_sync
    for name in (CHAINED, "bls-unchained-g1-rfc9380"):
        c = json.load(open(os.path.join(GOLD, "chains.json")))[name]
        s = dh.scheme_from_name(name)
        info = Info(bytes.fromhex(c["pk"]), 30, s.name, 0, bytes.fromhex(c["prevs"][0]))
        recs = {r: {"round": r, "signature": bytes.fromhex(x), "previous_signature": bytes.fromhex(p) if s.chained else b""}
                for r, x, p in zip(c["rounds"], c["sigs"], c["prevs"])}
        del recs[6]
        recs[9] = dict(recs[9], signature=recs[10]["signature"])
        recs[17] = dict(recs[17], signature=recs[17]["signature"][:-1])  # wrong length
        bucket = {}
        up = relay_s3_sync(BatchVerifyingClient(info, s), lambda r: dict(recs[r]),
                           lambda k, b: bucket.__setitem__(k, b), 1, 24, window=7)
        want = [r for r in range(1, 25) if r in recs and len(recs[r]["signature"]) == s.sig_len and
                oracle.verify_beacon(name, info.public_key, r, recs[r]["signature"], recs[r]["previous_signature"])]
        assert up == want and 6 not in up and 9 not in up and 17 not in up
        for r in up:
            body = json.loads(bucket["public/%d" % r])
            assert base64.b64decode(body["randomness"]) == hashlib.sha256(recs[r]["signature"]).digest()


# ---------------------------------------------------------------- bench.py --gpus N launches N ranks
def test_bench_launches_ranks():
    """`python bench.py --gpus 2` with no launcher spawns the two ranks itself (torch.distributed.run in a child
    process, before any HIP call) and prints rank 0's line: n_gpus 2, the node-wide check as the parallelism, every
    verdict valid. gloo rehearsal: both ranks on GPU 0, strong scaling of a 262,144-round chain; then weak scaling,
    whose line also carries the strong_scaling field (one chain split over the ranks, the north_star's shape)."""
    import subprocess
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    base = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--steps", "2",
            "--warmup", "1", "--streams", "4", "--no-cpu-baseline", "--roofline-steps", "0", "--single-call-steps", "0"]
    out = subprocess.run(base + ["--total-rounds", "262144"], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, out.stdout[-2000:]
    res = json.loads(line[0])
    assert res["n_gpus"] == 2 and res["verdicts_ok"] is True and res["scaling"] == "strong"
    assert "node-wide RLC check" in res["config"]["parallelism"] and res["config"]["rounds_per_gpu"] == 131072
    assert res["strong_scaling"] is None  # the value itself is the strong figure
    out = subprocess.run(base + ["--rounds-per-gpu", "65536", "--strong-total-rounds", "131072"], env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][0])
    assert res["scaling"] == "weak" and res["verdicts_ok"] is True and res["config"]["rounds_total"] == 131072
    st = res["strong_scaling"]
    assert st["scaling"] == "strong" and st["rounds_total"] == 131072 and st["rounds_per_gpu"] == 65536
    assert st["verdicts_ok"] is True and st["value"] > 0
    # under a launcher WORLD_SIZE must match --gpus
    bad = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True, text=True,
                         env=dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), timeout=120)
    assert bad.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in bad.stderr


# ---------------------------------------------------------------- sharded tbls Recover, two processes
def _recover_shard_worker(rank, world, port, name, commits, t, n, msgs, parts, q):
    try:
        import torch
        import torch.distributed as dist
        sys.path.insert(0, ROOT)
        from drand_amd import _lib, scheme_from_name
        from drand_amd.dist import recover_shard
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        assert _lib.load().dh_init(1) == 0, _lib.last_error()
        torch.cuda.set_device(0)
        sigs, ok = recover_shard(scheme_from_name(name), commits, t, n, msgs, parts, rank, world)
        q.put({"rank": rank, "sigs": sigs.tobytes(), "ok": ok.tolist()})
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 - reported to the parent
        import traceback
        q.put({"rank": rank, "error": repr(e) + traceback.format_exc()})


def test_recover_shard_two_processes(dh, oracle):
    """drand_amd.dist.recover_shard in two spawned processes (gloo, both on GPU 0, the real library): 40 rounds of a
    16-signer, threshold-9 group split over the ranks, with rounds short of t valid partials and an invalid partial in
    front; both ranks return the whole node's recovered signatures and flags, equal to the oracle's Recover per
    round (kyber sign/tbls restated) and to the group signature [f(0)] H(m)."""
    import random
    import torch.multiprocessing as mp
    name = "pedersen-bls-unchained"
    s = dh.scheme_from_name(name)
    n, t, nr, world = 16, 9, 40, 2
    coeffs = [int.from_bytes(hashlib.sha256(b"rshard-%d" % j).digest(), "big") % R_ORDER for j in range(t)]
    commits = [s.public_key(c.to_bytes(32, "big")) for c in coeffs]

    def share(i):
        x, acc = i + 1, 0
        for cf in reversed(coeffs):
            acc = (acc * x + cf) % R_ORDER
        return acc.to_bytes(32, "big")

    rounds = np.arange(900, 900 + nr, dtype=np.uint64)
    shares = [s.sign_beacons(share(i), rounds) for i in range(n)]
    msgs = [s.digest_beacon(int(r)) for r in rounds]
    rng = random.Random(77)
    parts = []
    for j in range(nr):
        ids = rng.sample(range(n), t - 1 if j % 5 == 0 else rng.randrange(t, n + 1))
        ps = [i.to_bytes(2, "big") + shares[i][j].tobytes() for i in ids]
        if j % 4 == 1:  # another round's signature in front
            ps.insert(0, ids[0].to_bytes(2, "big") + shares[ids[0]][(j + 1) % nr].tobytes())
        parts.append(ps)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_recover_shard_worker, args=(r, world, port, name, commits, t, n, msgs, parts, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    errs = [m["error"] for m in res if "error" in m]
    assert not errs, errs
    want = [oracle.recover(name, commits, t, n, m, ps) for m, ps in zip(msgs, parts)]
    group = s.sign_beacons(coeffs[0].to_bytes(32, "big"), rounds)
    for m in res:
        assert m["ok"] == [w is not None for w in want]
        got = np.frombuffer(m["sigs"], np.uint8).reshape(nr, 96)
        for j, w in enumerate(want):
            if w is not None:
                assert got[j].tobytes() == w == group[j].tobytes()
    assert sum(res[0]["ok"]) == nr - nr // 5
