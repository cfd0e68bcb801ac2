"""Multi-GPU layout of the batch verifier: one process per GPU, rounds sharded across ranks.

* Sharding: contiguous round ranges (shard_range). Strong scaling splits one chain (e.g. 1M quicknet rounds) over
  the node; weak scaling gives every rank its own n rounds (shard_rounds).
* Chained halo: a chained shard's first round needs the STORED signature of round start-1
  (/root/reference/chain/boltdb/trimmed.go:183), which lives in the previous rank's shard. shard_beacons reads it
  from the shared store (host-supplied halo); exchange_halo passes it rank to rank when each rank only holds its
  own shard (e.g. each streams its range from a different peer).
* Node-wide check: every rank computes its level-0 RLC sums (A_g, B_g) with dh_batch_begin; one all-gather of
  those 2 points per rank over RCCL (xGMI), then ONE pairing check of the sums for the whole node
  (dh_check_partials) and dh_batch_finish: all ranks accept, or each bisects its own shard. No data-path collective
  besides that (the per-round data never leaves its GPU).
* Verdicts: packed bitmaps all-gathered once at the end (gather_verdicts).
The collectives use torch.distributed: backend "nccl" (= RCCL) on the GPUs, "gloo" in the CPU tests.
"""
import ctypes

import numpy as np


def shard_rounds(rank, world, n_per_rank, first_round=1):
    """Weak scaling: round numbers owned by `rank`: [first + rank*n, first + (rank+1)*n)."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    lo = first_round + rank * n_per_rank
    return np.arange(lo, lo + n_per_rank, dtype=np.uint64)


def shard_range(rank, world, total):
    """Contiguous split of `total` items over `world` ranks (sizes differ by at most one): [lo, hi)."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def strong_shard(rank, world, total, first_round=1):
    """Strong scaling: this rank's part of rounds first_round .. first_round + total - 1."""
    lo, hi = shard_range(rank, world, total)
    return np.arange(first_round + lo, first_round + hi, dtype=np.uint64)


def shard_beacons(store, rank, world, first, last):
    """The beacons of this rank's part of rounds first..last from a shared trimmed store (TrimmedMemStore,
    store.BoltTrimmedStore): (rounds, signatures, previous signatures, missing rounds). The previous signature of
    the shard's first round is the store's record of the round before it: the halo comes from the host."""
    from .sync import NoBeaconStored
    lo, hi = shard_range(rank, world, last - first + 1)
    rounds, sigs, prevs, missing = [], [], [], []
    for r in range(first + lo, first + hi):
        try:
            b = store.get(r)
        except NoBeaconStored:
            missing.append(r)
            continue
        rounds.append(r)
        sigs.append(bytes(b.signature))
        prevs.append(bytes(b.previous_signature or b""))
    return rounds, sigs, prevs, missing


def exchange_halo(last_signature, rank, world, group=None, max_len=96):
    """Rank r receives rank r-1's last stored signature (rank 0 gets None): one all-gather of a fixed-size slot
    (length + bytes) per rank. Used when each rank holds only its own shard of the chain."""
    import torch
    import torch.distributed as dist
    slot = torch.zeros(max_len + 4, dtype=torch.uint8)
    sig = bytes(last_signature or b"")
    if len(sig) > max_len:
        raise ValueError("signature longer than the halo slot")
    slot[:4] = torch.tensor(list(len(sig).to_bytes(4, "little")), dtype=torch.uint8)
    if sig:
        slot[4:4 + len(sig)] = torch.tensor(list(sig), dtype=torch.uint8)
    if world == 1:
        return None
    out = [torch.zeros_like(slot) for _ in range(world)]
    dist.all_gather(out, slot, group=group)
    if rank == 0:
        return None
    prev = out[rank - 1].numpy().tobytes()
    n = int.from_bytes(prev[:4], "little")
    return prev[4:4 + n]


def pack_bits(verdict):
    """(n,) uint8 0/1 torch tensor -> (ceil(n/8),) uint8 bitmap, MSB first (np.packbits order), on its device."""
    import torch
    n = verdict.numel()
    pad = (-n) % 8
    v = torch.nn.functional.pad(verdict.to(torch.uint8), (0, pad)).view(-1, 8).to(torch.int32)
    w = torch.tensor([128, 64, 32, 16, 8, 4, 2, 1], dtype=torch.int32, device=verdict.device)
    return (v * w).sum(dim=1).to(torch.uint8)


def gather_verdicts(bits, world, group=None):
    """All-gather the ranks' bitmaps (sizes may differ by one byte under strong scaling); returns them in rank
    order, each trimmed to its own length."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return [bits]
    size = torch.tensor([bits.numel()], dtype=torch.int64, device=bits.device)
    sizes = [torch.zeros_like(size) for _ in range(world)]
    dist.all_gather(sizes, size, group=group)
    m = int(max(int(x) for x in sizes))
    padded = torch.zeros(m, dtype=bits.dtype, device=bits.device)
    padded[:bits.numel()] = bits
    out = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(out, padded, group=group)
    return [o[:int(k)] for o, k in zip(out, sizes)]


def gather_partials(local, world, group=None):
    """All-gather each rank's level-0 partial sums (dh_partial_bytes bytes, uint8 tensor) into one
    (world * bytes) tensor in rank order: the input of dh_check_partials."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return local
    out = torch.empty(world * local.numel(), dtype=local.dtype, device=local.device)
    if local.is_cuda:
        dist.all_gather_into_tensor(out, local, group=group)
    else:
        parts = list(out.view(world, -1).unbind(0))
        dist.all_gather(parts, local, group=group)
    return out


def verify_node_batch(lib, scheme, pk, d_rounds, d_sigs, n, d_verdict, d_rand, partials, world, group=None,
                      d_prevs=None, prev_stride=0, d_prev_lens=None, seed=0, stage_host=False):
    """One batch of this rank's shard under the node-wide check: dh_batch_begin -> all-gather of the (A, B) sums
    -> dh_check_partials (one pairing check for the whole node) -> dh_batch_finish. `partials` is a uint8 device
    tensor of dh_partial_bytes(scheme) bytes; with stage_host the exchange goes through host memory (gloo).
    Returns the node-wide pass flag."""
    import torch
    from . import _lib

    def ptr(t):
        return ctypes.c_void_p(t.data_ptr()) if t is not None else None

    b = ctypes.c_void_p()
    rc = lib.dh_batch_begin(scheme.id, pk, len(pk), ptr(d_rounds), ptr(d_sigs), scheme.sig_len, ptr(d_prevs),
                            prev_stride, ptr(d_prev_lens), n, ptr(d_verdict), ptr(d_rand), seed, None,
                            ctypes.byref(b), ptr(partials))
    if rc != 0:
        raise RuntimeError("dh_batch_begin: %s" % _lib.last_error())
    try:
        if stage_host:
            allp = gather_partials(partials.cpu(), world, group).to(partials.device)
        else:
            allp = gather_partials(partials, world, group)
        torch.cuda.current_stream(partials.device).synchronize()  # the library reads it from its own streams
        ok = ctypes.c_int(0)
        rc = lib.dh_check_partials(scheme.id, pk, len(pk), ptr(allp), world, ctypes.byref(ok))
        if rc != 0:
            raise RuntimeError("dh_check_partials: %s" % _lib.last_error())
    except Exception:
        lib.dh_batch_finish(b, -1, None)
        raise
    rc = lib.dh_batch_finish(b, ok.value, None)
    if rc != 0:
        raise RuntimeError("dh_batch_finish: %s" % _lib.last_error())
    return bool(ok.value)
