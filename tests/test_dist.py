"""CPU, world_size 2 over gloo: the multi-GPU sharding and the whole-node verdict all-gather used by
bench.py (drand_amd/dist.py). The verification itself is replaced by a deterministic stand-in verdict so
this runs without a GPU; the exchange is the same code path as on RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from drand_amd.dist import gather_verdicts, pack_bits, shard_range, shard_rounds


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rounds = shard_rounds(rank, world, n)
    verdict = torch.from_numpy((rounds % 7 != 0).astype(np.uint8))  # stand-in for the device verdicts
    parts = gather_verdicts(pack_bits(verdict), world)
    if rank == 0:
        bits = np.concatenate([p.numpy() for p in parts])
        q.put(np.unpackbits(bits).tolist())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [64, 1000])
def test_gather_verdicts_world2(n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    per = (n + 7) // 8 * 8
    expect = []
    for r in range(2):
        rounds = shard_rounds(r, 2, n)
        expect += (rounds % 7 != 0).astype(int).tolist() + [0] * (per - n)
    assert got == expect


def test_shards_partition_rounds():
    n = 1000
    seen = np.concatenate([shard_rounds(r, 4, n) for r in range(4)])
    assert np.array_equal(seen, np.arange(1, 4 * n + 1, dtype=np.uint64))
    for total in (10, 11, 1 << 20):
        spans = [shard_range(r, 3, total) for r in range(3)]
        assert spans[0][0] == 0 and spans[-1][1] == total
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    with pytest.raises(ValueError):
        shard_rounds(2, 2, 5)


def test_pack_bits_matches_numpy():
    v = (np.arange(29) % 3 == 0).astype(np.uint8)
    assert np.array_equal(pack_bits(torch.from_numpy(v)).numpy(), np.packbits(v))
