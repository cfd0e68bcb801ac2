"""CPU, world_size 2 and 3 over gloo: the multi-GPU layer of drand_amd/dist.py that bench.py and the chained replay
use — strong-scaling shards, the chained halo (host-supplied from the store, and exchanged rank to rank), the
all-gather of per-rank partial-sum bytes in rank order, and the whole-node verdict bitmaps (ranks of unequal size).
Verification itself runs on the CPU oracle here (test infrastructure standing in for the device, same verdict
semantics); a corruption sits on the shard boundary, so the next rank's first round must fail through the halo."""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from drand_amd.dist import (MISSING_HALO, exchange_halo, gather_partials, gather_verdicts, pack_bits, rank_seed,
                            shard_beacons, shard_range, shard_rounds, strong_shard, verify_node_batch)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
CHAINED = "pedersen-bls-chained"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _store_with_boundary_fault(boundary):
    from drand_amd.sync import TrimmedMemStore
    c = json.load(open(os.path.join(GOLD, "chains.json")))[CHAINED]
    st = TrimmedMemStore(True)
    st.put(0, bytes.fromhex(c["prevs"][0]))
    for r, sig in zip(c["rounds"], c["sigs"]):
        st.put(r, bytes.fromhex(sig))
    st.put(boundary, bytes.fromhex(c["sigs"][boundary - 2]))  # round `boundary` stores round boundary-1's signature
    return st, bytes.fromhex(c["pk"]), c["rounds"][-1]


def sigs_prev_rank_last(st, rank, world, last):
    lo, _ = shard_range(rank, world, last)
    return st.get(lo).signature  # the last round of rank-1 is round lo (rounds start at 1)


def _worker(rank, world, port, boundary, q):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ctypes as orc
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    st, pk, last = _store_with_boundary_fault(boundary)
    rounds, sigs, prevs, missing = shard_beacons(st, rank, world, 1, last)
    halo = exchange_halo(sigs[-1] if sigs else b"", rank, world)  # rank r-1's last stored signature
    halo_ok = rank == 0 or halo == prevs[0] == st.get(rounds[0] - 1).signature
    # a shard whose last round is missing from the store hands the next rank MISSING_HALO (trimmed.go:183-187)
    gone = exchange_halo(None if rank == 0 else sigs[-1], rank, world)
    halo_ok = halo_ok and gone is (None if rank == 0 else MISSING_HALO if rank == 1 else gone)
    halo_ok = halo_ok and (rank < 2 or gone == sigs_prev_rank_last(st, rank, world, last))
    verdict = torch.tensor([orc.verify_beacon(CHAINED, pk, r, s, p) for r, s, p in zip(rounds, sigs, prevs)],
                           dtype=torch.uint8)
    parts = gather_verdicts(pack_bits(verdict), world)
    allp = gather_partials(torch.full((24,), rank + 1, dtype=torch.uint8), world)
    if rank == 0:
        faulty = []
        for r_, bits in enumerate(parts):
            lo, hi = shard_range(r_, world, last)
            v = np.unpackbits(bits.numpy())[:hi - lo]
            faulty += [lo + 1 + i for i in np.flatnonzero(v == 0)]
        q.put({"faulty": faulty, "partials": allp.numpy().tolist()})
    q.put({"rank": rank, "halo_ok": bool(halo_ok), "missing": missing})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,boundary", [(2, 12), (3, 16)])
def test_sharded_chained_replay_gloo(world, boundary, oracle):
    """Round `boundary` (the last round of a shard) stores the previous round's signature: it fails, and the next
    shard's first round fails too because its previous signature is that record — visible only through the halo.
    The whole-node faulty set equals the serial oracle replay over the unsharded store."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, boundary, q)) for r in range(world)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=180) for _ in range(world + 1)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res = next(m for m in msgs if "faulty" in m)
    assert all(m["halo_ok"] for m in msgs if "rank" in m)
    assert res["faulty"] == [boundary, boundary + 1]
    st, pk, last = _store_with_boundary_fault(boundary)
    serial = [r for r in range(1, last + 1)
              if not oracle.verify_beacon(CHAINED, pk, r, st.get(r).signature, st.get(r).previous_signature)]
    assert res["faulty"] == serial
    lo0, hi0 = shard_range(0, world, last)
    assert hi0 == boundary or world == 3  # world 2: the fault sits exactly on the shard boundary
    assert res["partials"] == sum(([r + 1] * 24 for r in range(world)), [])


def test_shards_partition_rounds():
    n = 1000
    seen = np.concatenate([shard_rounds(r, 4, n) for r in range(4)])
    assert np.array_equal(seen, np.arange(1, 4 * n + 1, dtype=np.uint64))
    for total in (10, 11, 1 << 20):
        spans = [shard_range(r, 3, total) for r in range(3)]
        assert spans[0][0] == 0 and spans[-1][1] == total
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        strong = np.concatenate([strong_shard(r, 3, total) for r in range(3)])
        assert np.array_equal(strong, np.arange(1, total + 1, dtype=np.uint64))
    with pytest.raises(ValueError):
        shard_rounds(2, 2, 5)


def test_pack_bits_matches_numpy():
    v = (np.arange(29) % 3 == 0).astype(np.uint8)
    assert np.array_equal(pack_bits(torch.from_numpy(v)).numpy(), np.packbits(v))


class _FakeLib:
    """The node-check entry points of libdrandhip, on the host: dh_batch_begin writes a rank-specific record (or
    fails on `fail_rank`), dh_batch_check records what the all-gather delivered and whether a status word was set,
    dh_batch_finish(DH_NODE_CHECKED) reports it like the library (1 passed, DH_EABANDONED)."""

    def __init__(self, rank, fail_rank, pb):
        self.rank, self.fail_rank, self.pb = rank, fail_rank, pb
        self.seed, self.seen, self.finished, self.abandoned = None, None, [], False

    def dh_batch_begin(self, sid, pk, pklen, r, s, sl, p, ps, pl, n, v, rnd, seed, stream, bref, parts):
        import ctypes
        self.seed = seed
        if self.rank == self.fail_rank:
            return -2
        ctypes.memmove(parts.value, bytes([self.rank + 1]) * (self.pb - 16) + bytes(16), self.pb)
        bref._obj.value = 1000 + self.rank
        return 0

    def dh_batch_check(self, b, allp, k, stream):
        import ctypes
        self.seen = ctypes.string_at(allp.value, k * self.pb)
        self.abandoned = any(self.seen[i * self.pb + self.pb - 16] for i in range(k))
        return 0

    def dh_batch_finish(self, b, mode, st):
        self.finished.append(mode)
        return -7 if self.abandoned else 1


def _node_worker(rank, world, port, fail_rank, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drand_amd.scheme import scheme_from_name
    s = scheme_from_name("pedersen-bls-unchained")
    pb = 2 * 72 * 4 + 16
    lib = _FakeLib(rank, fail_rank, pb)
    parts = torch.zeros(pb, dtype=torch.uint8)
    out = {"rank": rank}
    try:
        out["pass"] = verify_node_batch(lib, s, b"k" * 48, None, None, 10, None, None, parts, world, seed=5)
    except RuntimeError as e:
        out["error"] = str(e)
    # a rank that failed after the node check still joins the verdict gather, and every rank raises
    try:
        gather_verdicts(torch.zeros(2, dtype=torch.uint8), world, failed="boom" if rank == 2 else None)
        out["gather"] = "ok"
    except RuntimeError as e:
        out["gather"] = str(e)
    out.update(seed=lib.seed, seen=lib.seen, finished=lib.finished)
    q.put(out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("fail_rank", [None, 1])
def test_node_batch_protocol_gloo(fail_rank):
    """verify_node_batch's collective protocol at world 3 over gloo (library entry points faked on the host): the
    partial records arrive in rank order at every rank, each rank's RLC seed is distinct (rank_seed); when
    dh_batch_begin fails on one rank, its record carries status 1, every other rank's check sees it and its finish
    reports the batch abandoned, so every rank raises instead of blocking in the all-gather; and a failure flagged
    in the verdict gather raises on every rank."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_node_worker, args=(r, world, port, fail_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=120) for _ in range(world)), key=lambda m: m["rank"])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len({m["seed"] for m in res}) == world and res[0]["seed"] == rank_seed(5, 0) != 5
    pb = 2 * 72 * 4 + 16
    recs = [bytes([r + 1]) * (pb - 16) + bytes(16) for r in range(world)]
    if fail_rank is None:
        assert all(m["pass"] is True and m["finished"] == [2] for m in res)
        assert all(m["seen"] == b"".join(recs) for m in res)
    else:
        assert all("error" in m for m in res)
        assert "dh_batch_begin" in res[fail_rank]["error"] and "abandoned" in res[0]["error"]
        assert [m["finished"] for m in res] == [[2], [], [2]]
        recs[fail_rank] = bytes(pb - 16) + bytes([1]) + bytes(15)
        assert res[0]["seen"] == b"".join(recs) and res[fail_rank]["seen"] is None
    assert res[2]["gather"] == "boom" and all("rank(s) [2]" in m["gather"] for m in res[:2])
    assert rank_seed(0, 3) == 0


class _StallLib(_FakeLib):
    """rank `stall_rank`'s dh_batch_begin never returns in time (a hung peer): it sleeps for `secs`"""

    def __init__(self, rank, stall_rank, pb, secs):
        super().__init__(rank, None, pb)
        self.stall_rank, self.secs = stall_rank, secs

    def dh_batch_begin(self, *a):
        import time
        if self.rank == self.stall_rank:
            time.sleep(self.secs)
        return super().dh_batch_begin(*a)


def _stall_worker(rank, world, port, out_dir):
    import datetime
    from drand_amd.dist import BatchWatchdog, STALL_EXIT
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # the process group's own timeout is the second line: longer than the watchdog's deadline
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    from drand_amd.scheme import scheme_from_name
    s = scheme_from_name("pedersen-bls-unchained")
    pb = 2 * 72 * 4 + 16
    lib = _StallLib(rank, 1, pb, 600)

    def on_stall(msg):
        with open(os.path.join(out_dir, "stall_%d.txt" % rank), "w") as f:
            f.write(msg)
        os._exit(STALL_EXIT)

    wd = BatchWatchdog(2.0, rank, on_stall=on_stall, poll=0.2)
    for k in range(3):
        wd.begin(k, "test batch")
        verify_node_batch(lib, s, b"k" * 48, None, None, 10, None, None, torch.zeros(pb, dtype=torch.uint8), world, seed=5)
        wd.end(k)
    os._exit(0)


def test_node_batch_stall_exits_with_message(tmp_path):
    """a rank whose peer hangs (rank 1 never returns from dh_batch_begin) must not wait in the
    all-gather for ever. Every rank's BatchWatchdog names the rank and the stalled batch and the rank exits with
    STALL_EXIT (3): rank 0 from inside the blocked all-gather, rank 1 from inside its stalled begin."""
    from drand_amd.dist import STALL_EXIT
    world = 2
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_stall_worker, args=(r, world, port, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=90)
        if p.exitcode is None:
            p.kill()
    assert [p.exitcode for p in procs] == [STALL_EXIT, STALL_EXIT]
    for r in range(world):
        msg = open(os.path.join(str(tmp_path), "stall_%d.txt" % r)).read()
        assert msg.startswith("rank %d: node batch 0 stalled" % r), msg


def test_watchdog_quiet_when_batches_finish():
    from drand_amd.dist import BatchWatchdog
    fired = []
    wd = BatchWatchdog(0.5, 0, on_stall=fired.append, poll=0.05)
    import time
    for k in range(5):
        wd.begin(k)
        time.sleep(0.05)
        wd.end(k)
    time.sleep(0.8)
    wd.stop()
    assert fired == [] and wd.fired is None
    wd = BatchWatchdog(0.3, 4, on_stall=fired.append, poll=0.05)
    wd.begin("b7")
    time.sleep(1.0)
    wd.stop()
    assert len(fired) == 1 and fired[0].startswith("rank 4: node batch b7 stalled")


# ---------------------------------------------------------------- sharded tbls Recover (config 4 over the node)
class _OracleRecoverScheme:
    """Stands in for drand_amd.scheme.Scheme.recover_batch on the CPU: the oracle's per-round Recover (kyber sign/tbls
    restated), so recover_shard's sharding and gather run here without a GPU."""

    def __init__(self, name, orc):
        self.name, self.orc = name, orc
        self.sig_len = 96 if name.startswith("pedersen") else 48

    def recover_batch(self, commits, t, n, msgs, parts):
        sigs = np.zeros((len(msgs), self.sig_len), np.uint8)
        ok = np.zeros(len(msgs), bool)
        for j, (m, ps) in enumerate(zip(msgs, parts)):
            r = self.orc.recover(self.name, commits, t, n, m, ps)
            if r is not None:
                sigs[j] = np.frombuffer(r, np.uint8)
                ok[j] = True
        return sigs, ok


def _tbls_case(orc, name, t, n, nr):
    import hashlib
    R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
    coeffs = [int.from_bytes(hashlib.sha256(b"shard-rec-%d" % j).digest(), "big") % R for j in range(t)]
    commits = [orc.public_key(name, c.to_bytes(32, "big")) for c in coeffs]

    def share(i):
        x, acc = i + 1, 0
        for cf in reversed(coeffs):
            acc = (acc * x + cf) % R
        return acc.to_bytes(32, "big")

    msgs = [orc.digest_beacon(name, 100 + j) for j in range(nr)]
    parts = []
    for j in range(nr):
        ids = [(j + k) % n for k in range(t if j % 3 else t - 1)]  # every third round: one partial short
        parts.append([i.to_bytes(2, "big") + orc.sign(name, share(i), msgs[j]) for i in ids])
    return commits, msgs, parts


def _recover_worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ctypes as orc
    from drand_amd.dist import recover_shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    name = "pedersen-bls-unchained"
    commits, msgs, parts = _tbls_case(orc, name, 3, 5, 7)
    sigs, ok = recover_shard(_OracleRecoverScheme(name, orc), commits, 3, 5, msgs, parts, rank, world)
    q.put({"rank": rank, "sigs": sigs.tobytes(), "ok": ok.tolist()})
    dist.barrier()
    dist.destroy_process_group()


def test_recover_shard_gloo(oracle):
    """recover_shard at world 3 (gloo, CPU; Recover itself on the oracle): every rank returns the whole node's
    recovered signatures and status flags in round order, equal to a serial Recover of every round."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_recover_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    name = "pedersen-bls-unchained"
    commits, msgs, parts = _tbls_case(oracle, name, 3, 5, 7)
    want = [oracle.recover(name, commits, 3, 5, m, ps) for m, ps in zip(msgs, parts)]
    for m in res:
        assert m["ok"] == [w is not None for w in want]
        got = np.frombuffer(m["sigs"], np.uint8).reshape(7, 96)
        for j, w in enumerate(want):
            if w is not None:
                assert got[j].tobytes() == w
    assert sum(m["ok"]) == 4  # rounds 0, 3, 6 are one partial short
