"""Round sharding and the whole-node verdict exchange for multi-GPU runs.

Rounds are independent given the group key, so rank r of `world` verifies a contiguous shard with no
data-path collective; the only exchange is one all-gather of packed verdict bitmaps at the end of a
batch sequence (RCCL over xGMI with backend "nccl"; gloo on CPU in the tests).
"""
import numpy as np


def shard_rounds(rank, world, n_per_rank, first_round=1):
    """Round numbers owned by `rank`: [first + rank*n, first + (rank+1)*n)."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    lo = first_round + rank * n_per_rank
    return np.arange(lo, lo + n_per_rank, dtype=np.uint64)


def shard_range(rank, world, total):
    """Contiguous split of `total` rounds over `world` ranks (sizes differ by at most one)."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def pack_bits(verdict):
    """(n,) uint8 0/1 torch tensor -> (ceil(n/8),) uint8 bitmap, MSB first (np.packbits order), on its device."""
    import torch
    n = verdict.numel()
    pad = (-n) % 8
    v = torch.nn.functional.pad(verdict.to(torch.uint8), (0, pad)).view(-1, 8).to(torch.int32)
    w = torch.tensor([128, 64, 32, 16, 8, 4, 2, 1], dtype=torch.int32, device=verdict.device)
    return (v * w).sum(dim=1).to(torch.uint8)


def gather_verdicts(bits, world, group=None):
    """All-gather equal-size bitmaps from every rank; returns the list in rank order."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return [bits]
    out = [torch.empty_like(bits) for _ in range(world)]
    dist.all_gather(out, bits, group=group)
    return out
