"""Multi-GPU layout of the batch verifier: one process per GPU, rounds sharded across ranks.

* Sharding: contiguous round ranges (shard_range). Strong scaling splits one chain (e.g. 1M quicknet rounds) over
  the node; weak scaling gives every rank its own n rounds (shard_rounds).
* Chained halo: a chained shard's first round needs the STORED signature of round start-1
  (/root/reference/chain/boltdb/trimmed.go:183), which lives in the previous rank's shard. shard_beacons reads it
  from the shared store (host-supplied halo); exchange_halo passes it rank to rank when each rank only holds its
  own shard (e.g. each streams its range from a different peer). A missing round start-1 travels as MISSING_HALO,
  and the next rank reports its first round missing, as the trimmed store's Get would (trimmed.go:183-187).
* Node-wide check: every rank computes its level-0 RLC sums (A_g, B_g) with dh_batch_begin; one all-gather of
  those 2 points (plus a status word) per rank over RCCL (xGMI) on the batch's own library stream, then ONE pairing
  check of the sums for the whole node (dh_batch_check, queued on that stream) and dh_batch_finish, the batch's one
  host wait: all ranks accept, or each bisects its own shard. A rank whose
  dh_batch_begin failed still takes part in the exchange (identity sums, status 1), so every rank abandons the
  batch together instead of blocking in the collective. No data-path collective besides that (the per-round data
  never leaves its GPU).
* Verdicts: packed bitmaps all-gathered once at the end (gather_verdicts).
* Stalls: a rank whose peer died or hangs would wait in the collective (or in the batch's host wait behind it) for
  ever. BatchWatchdog gives every in-flight node batch a deadline: past it the rank names itself, the batch and how
  long it has waited on stderr and exits with STALL_EXIT (a child process exit, never an exec), so the launcher tears
  the job down instead of hanging; the process group's own collective timeout (init_process_group(timeout=...)) is the
  second line behind it.
* replay_shard: the sharded CheckPastBeacons (chain/beacon/sync_manager.go:170-235) built from the pieces above;
  recover_shard: tbls Recover with its rounds sharded (no exchange before the gather).
The collectives use torch.distributed: backend "nccl" (= RCCL) with device tensors, "gloo" with host tensors
(the CPU tests, and N ranks rehearsed on one GPU).
"""
import ctypes
import hashlib
import os
import sys
import threading
import time

import numpy as np

PREV_SLOT_MAX = 4096  # as scheme.PREV_SLOT_MAX: longer stored records only come from a corrupted store


class _MissingHalo:
    def __repr__(self):
        return "MISSING_HALO"


MISSING_HALO = _MissingHalo()


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


def _exchanges(world, exchange):
    """Whether a node step runs its collective: with more than one rank, or at world 1 when the caller asks for it
    (exchange=True: the all-gathers run over a one-rank process group, which rehearses the device-side RCCL branch on
    one GPU — two ranks cannot share a GPU under RCCL)."""
    return world > 1 if exchange is None else bool(exchange)


def _collective_device(group):
    """Where the collective's tensors live: the current GPU under nccl (RCCL), the host under gloo."""
    import torch
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def exchange_halo(last_signature, rank, world, group=None, exchange=None):
    """Rank r receives rank r-1's last stored signature (a stored record may have any length): an all-gather of
    the record lengths, then one of slots that fit the longest, on the device under nccl. `last_signature` is None
    when this shard's last round is missing from the store: the next rank then gets MISSING_HALO. Rank 0 (and
    world 1) gets None."""
    import torch
    import torch.distributed as dist
    if not _exchanges(world, exchange):
        return None
    dev = _collective_device(group)
    missing = last_signature is None
    sig = b"" if missing else bytes(last_signature)
    ln = torch.tensor([-1 if missing else len(sig)], dtype=torch.int64, device=dev)
    lens = [torch.zeros_like(ln) for _ in range(world)]
    dist.all_gather(lens, ln, group=group)
    width = max(1, max(int(x) for x in lens))
    host = np.zeros(width, dtype=np.uint8)
    host[:len(sig)] = np.frombuffer(sig, np.uint8)
    slot = torch.from_numpy(host).to(dev)
    out = [torch.zeros_like(slot) for _ in range(world)]
    dist.all_gather(out, slot, group=group)
    if rank == 0:
        return None
    n = int(lens[rank - 1])
    if n < 0:
        return MISSING_HALO
    return out[rank - 1].cpu().numpy().tobytes()[:n]


def pack_bits(verdict):
    """(n,) uint8 0/1 torch tensor -> (ceil(n/8),) uint8 bitmap, MSB first (np.packbits order), on its device."""
    import torch
    n = verdict.numel()
    pad = (-n) % 8
    v = torch.nn.functional.pad(verdict.to(torch.uint8), (0, pad)).view(-1, 8).to(torch.int32)
    # bit weights made on the device (arange): a host-built tensor is a pageable copy that waits for the queue
    sh = torch.arange(7, -1, -1, dtype=torch.int32, device=verdict.device)
    return (v << sh).sum(dim=1).to(torch.uint8)


class NodeFailure(RuntimeError):
    """Some rank failed its part of a node-wide step; raised on every rank after the collective."""


def gather_verdicts(bits, world, group=None, failed=None, exchange=None):
    """All-gather the ranks' bitmaps (sizes may differ by one byte under strong scaling); returns them in rank
    order, each trimmed to its own length. `failed` (a message, or None) marks this rank's part as failed: the flag
    travels with the sizes, so a rank that failed after the node check still joins the collective and every rank
    raises NodeFailure instead of waiting for it."""
    import torch
    import torch.distributed as dist
    if not _exchanges(world, exchange):
        if failed:
            raise NodeFailure(failed)
        return [bits]
    size = torch.tensor([bits.numel(), 1 if failed else 0], dtype=torch.int64, device=bits.device)
    sizes = [torch.zeros_like(size) for _ in range(world)]
    dist.all_gather(sizes, size, group=group)
    bad = [r for r, x in enumerate(sizes) if int(x[1])]
    if bad:
        raise NodeFailure(failed or "node step failed on rank(s) %s" % bad)
    m = int(max(int(x[0]) for x in sizes))
    padded = torch.zeros(m, dtype=bits.dtype, device=bits.device)
    padded[:bits.numel()] = bits
    out = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(out, padded, group=group)
    return [o[:int(k[0])] for o, k in zip(out, sizes)]


def gather_partials(local, world, group=None, exchange=None):
    """All-gather each rank's level-0 partial sums (dh_partial_bytes bytes, uint8 tensor) into one
    (world * bytes) tensor in rank order: the input of dh_batch_check (or of the standalone dh_check_partials)."""
    import torch
    import torch.distributed as dist
    if not _exchanges(world, exchange):
        return local
    out = torch.empty(world * local.numel(), dtype=local.dtype, device=local.device)
    if local.is_cuda:
        dist.all_gather_into_tensor(out, local, group=group)
    else:
        parts = list(out.view(world, -1).unbind(0))
        dist.all_gather(parts, local, group=group)
    return out


def rank_seed(seed, rank):
    """A caller-fixed RLC seed made distinct per rank: the scalars are SHA-256(seed || local index), so equal
    seeds would give every rank the same scalar at the same index, and errors planted at one index on two ranks
    could cancel in the node-wide sums. 0 stays 0 (fresh CSPRNG seed per call in the library)."""
    if not seed:
        return 0
    h = hashlib.sha256(b"drandhip-rank-seed" + int(seed).to_bytes(8, "little") + int(rank).to_bytes(4, "little"))
    return int.from_bytes(h.digest()[:8], "little") or 1


class _nullcontext:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


STALL_EXIT = 3


class BatchWatchdog:
    """Deadline per in-flight node batch. begin(key, what) when a batch is begun, end(key) when its finish() returned;
    a daemon thread checks the oldest in-flight batch every `poll` seconds, and once it is older than `deadline`
    seconds reports "rank R: node batch K stalled ..." on stderr and calls on_stall(message) — by default
    os._exit(STALL_EXIT): the thread that would report is blocked in a collective or in the library's host wait (ctypes
    and the collectives release the GIL), so raising in it is not possible. A deadline <= 0 disables the watchdog."""

    def __init__(self, deadline, rank, on_stall=None, poll=None):
        self.deadline, self.rank = float(deadline), rank
        self.on_stall = on_stall or self._exit
        self.poll = poll if poll is not None else max(0.05, min(1.0, self.deadline / 8))
        self._live = {}
        self._mu = threading.Lock()
        self._stop = threading.Event()
        self.fired = None
        self._th = None
        if self.deadline > 0:
            self._th = threading.Thread(target=self._run, name="node-batch-watchdog", daemon=True)
            self._th.start()

    @staticmethod
    def _exit(msg):
        sys.stderr.flush()
        os._exit(STALL_EXIT)

    def begin(self, key, what=""):
        with self._mu:
            self._live[key] = (time.monotonic(), what)

    def end(self, key):
        with self._mu:
            self._live.pop(key, None)

    def stop(self):
        self._stop.set()
        if self._th is not None:
            self._th.join(timeout=5)

    def _run(self):
        while not self._stop.wait(self.poll):
            with self._mu:
                old = min(self._live.items(), key=lambda kv: kv[1][0]) if self._live else None
            if old is None:
                continue
            key, (t0, what) = old
            waited = time.monotonic() - t0
            if waited > self.deadline:
                msg = ("rank %d: node batch %s stalled: not finished %.1f s after it began (deadline %.1f s; %s) -- its "
                       "all-gather or node check never completed, a peer rank has likely died or hangs; exiting with "
                       "status %d" % (self.rank, key, waited, self.deadline, what or "node-wide check", STALL_EXIT))
                print(msg, file=sys.stderr, flush=True)
                self.fired = msg
                self.on_stall(msg)
                return


def _status_offset(pb):
    """Byte offset of the status word in a partial record of pb bytes: [A | B | status | 3 pad words]."""
    return pb - 16


class NodeBatch:
    """One batch of this rank's shard under the node-wide check, begun and queued: dh_batch_begin -> all-gather of
    the partial records -> dh_batch_check, none of which waits on the host under nccl (the collective and the
    library are ordered through events on torch's current stream). finish() is the batch's one host wait."""

    def __init__(self, lib, b, gathered, err, rank):
        self.lib, self.b, self.gathered, self.err, self.rank = lib, b, gathered, err, rank

    def finish(self, stats=None):
        """Wait for the node-wide verdict: True when the node check passed, False when this shard was checked and
        bisected on its own (verdicts are exact either way). Raises when the batch was abandoned by any rank."""
        from . import _lib
        if self.err is not None:
            raise RuntimeError(self.err)
        rc = self.lib.dh_batch_finish(self.b, _lib.DH_NODE_CHECKED, stats)
        self.gathered = None  # the check has read it (finish waited for the batch's streams)
        if rc == _lib.DH_EABANDONED:
            raise RuntimeError("node batch abandoned: dh_batch_begin failed on another rank")
        if rc < 0:
            raise RuntimeError("rank %d: dh_batch_finish: %s" % (self.rank, _lib.last_error()))
        return rc == 1


def begin_node_batch(lib, scheme, pk, d_rounds, d_sigs, n, d_verdict, d_rand, partials, world, group=None,
                     d_prevs=None, prev_stride=0, d_prev_lens=None, seed=0, stage_host=None, rank=None,
                     inputs_ready=False, exchange=None):
    """Begin one batch under the node-wide check and queue its exchange and check: dh_batch_begin
    (per-round kernels + level-0 MSM, record written into `partials`, a uint8 device tensor of dh_partial_bytes) ->
    all-gather of the records -> dh_batch_check (ONE pairing check of the summed records, on this batch's worker).
    The record, the collective and the check are queued in the order of the batch's own library stream
    (dh_batch_stream, as a torch ExternalStream): under nccl nothing waits on the host, and with one rank nothing
    crosses streams; the inputs are ordered after torch's current stream (unless inputs_ready). Under gloo
    (stage_host) the records go through host memory. A rank whose dh_batch_begin failed still takes part in the exchange with a record whose
    status word is 1, so every rank's check sees it and abandons the batch (finish raises everywhere) instead of
    blocking in the collective. exchange=True runs the all-gather at world 1 too (_exchanges). Returns a NodeBatch;
    its finish() waits for the verdicts."""
    import torch
    import torch.distributed as dist
    from . import _lib

    if rank is None:
        rank = dist.get_rank(group) if world > 1 else 0

    def ptr(t):
        return ctypes.c_void_p(t.data_ptr()) if t is not None else None

    stream = torch.cuda.current_stream(partials.device) if partials.is_cuda else None
    # inputs still in production on the current stream are waited for; resident inputs (inputs_ready: the bench) are
    # not, since the current stream also carries the earlier batches' verdict packing, queued behind other batches'
    # saturating kernels (r04c: ordering on it cost the 131k-round node shape ~20%). torch's default stream is the
    # NULL stream, whose handle the library reads as "no stream": its work is waited for on the host instead.
    sp = None
    if stream is not None and not inputs_ready:
        if stream.cuda_stream:
            sp = ctypes.c_void_p(stream.cuda_stream)
        else:
            stream.synchronize()
    b = ctypes.c_void_p()
    rc = lib.dh_batch_begin(scheme.id, pk, len(pk), ptr(d_rounds), ptr(d_sigs), scheme.sig_len, ptr(d_prevs),
                            prev_stride, ptr(d_prev_lens), n, ptr(d_verdict), ptr(d_rand), rank_seed(seed, rank), sp,
                            ctypes.byref(b), ptr(partials))
    err = None if rc == 0 else "rank %d: dh_batch_begin: %s" % (rank, _lib.last_error())
    pb = partials.numel()
    # the record, the collective and the check in the order of the batch's own library stream (dh_batch_stream);
    # a rank whose begin failed writes its record (identity sums, status word 1) on its current stream instead
    ctx = stream
    if err is None and partials.is_cuda:
        ctx = torch.cuda.ExternalStream(lib.dh_batch_stream(b), device=partials.device)
    with torch.cuda.stream(ctx) if ctx is not None else _nullcontext():
        if err is not None:
            partials.zero_()
            partials[_status_offset(pb)] = 1
        if not _exchanges(world, exchange):
            gathered = partials
        else:
            if stage_host is None:
                stage_host = not dist.get_backend(group) == "nccl"
            slot = partials.cpu() if stage_host else partials
            gathered = gather_partials(slot, world, group, exchange)
            if stage_host:
                gathered = gathered.to(partials.device)
    if err is not None:
        return NodeBatch(lib, None, None, err, rank)
    rc = lib.dh_batch_check(b, ptr(gathered), world, None)  # queued on the batch's stream, after the gather
    if rc != 0:
        e = "rank %d: dh_batch_check: %s" % (rank, _lib.last_error())
        lib.dh_batch_finish(b, -1, None)
        return NodeBatch(lib, None, None, e, rank)
    return NodeBatch(lib, b, gathered, None, rank)


def verify_node_batch(lib, scheme, pk, d_rounds, d_sigs, n, d_verdict, d_rand, partials, world, group=None,
                      d_prevs=None, prev_stride=0, d_prev_lens=None, seed=0, stage_host=None, rank=None, exchange=None):
    """One batch of this rank's shard under the node-wide check, to completion (begin_node_batch + finish). Returns
    the node-wide pass flag; raises on every rank if any rank's dh_batch_begin failed."""
    return begin_node_batch(lib, scheme, pk, d_rounds, d_sigs, n, d_verdict, d_rand, partials, world, group,
                            d_prevs=d_prevs, prev_stride=prev_stride, d_prev_lens=d_prev_lens, seed=seed,
                            stage_host=stage_host, rank=rank, exchange=exchange).finish()


def replay_shard(lib, scheme, pk, first, last, sig_of, rank, world, group=None, prev_of_first=None, seed=0,
                 device=None, stage_host=None, exchange=None):
    """This rank's part of a sharded chain replay (CheckPastBeacons' verification over the node,
    /root/reference/chain/beacon/sync_manager.go:191-225, sharded as SURVEY.md §8e): rounds first..last are split
    with shard_range, and `sig_of` maps each round of this rank's range to its stored signature (a round absent
    from it is missing from the store). Chained: the previous signature of round k is the stored signature of
    k-1 (chain/boltdb/trimmed.go:183); the one before this rank's first round comes from the previous rank
    (exchange_halo), or from `prev_of_first` on rank 0 (the stored record of round first-1: the genesis seed when
    first = 1). A round is faulty when it is missing, its previous record is missing (chained), or it fails
    VerifyBeacon. The present rounds are verified in one batch under the node-wide check (verify_node_batch) and
    the ranks' verdicts all-gathered: every rank returns the whole node's faulty rounds, ascending. exchange=True
    runs every collective at world 1 too (_exchanges)."""
    import torch
    from .sync import NoBeaconStored  # noqa: F401  (the store error this mirrors)

    lo, hi = shard_range(rank, world, last - first + 1)
    lo, hi = first + lo, first + hi
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    halo = None
    xchg = _exchanges(world, exchange)
    if scheme.chained and xchg:
        # only trailing ranks can be empty (shard_range gives the extra rounds to the lower ranks): they need no halo
        halo = exchange_halo(sig_of.get(hi - 1) if hi > lo else None, rank, world, group, exchange)
    prev_first = prev_of_first if rank == 0 else halo
    if prev_first is MISSING_HALO:
        prev_first = None
    ok_range = np.zeros(hi - lo, dtype=np.uint8)
    idx, prevs = [], []
    for k, r in enumerate(range(lo, hi)):
        sig = sig_of.get(r)
        if sig is None:
            continue
        if scheme.chained:
            p = prev_first if r == lo else sig_of.get(r - 1)
            if p is None:
                continue  # Get fails: previous record missing (trimmed.go:183-187)
            prevs.append(bytes(p))
        idx.append(k)
    # a previous record longer than the device slot (only a corrupted store holds one) stays out of the device batch
    # (hashing a truncated record would fail the node-wide sums and bisect every rank's whole shard): those rounds
    # are verified on their own below
    oversize = [j for j, p in enumerate(prevs) if len(p) > PREV_SLOT_MAX] if scheme.chained else []
    host_j = set(oversize)
    dev_j = [j for j in range(len(idx)) if j not in host_j]
    n = len(dev_j)
    sigs = np.zeros((max(len(idx), 1), scheme.sig_len), dtype=np.uint8)
    bad_len = np.zeros(max(len(idx), 1), dtype=bool)
    for j, k in enumerate(idx):
        s_ = bytes(sig_of[lo + k])
        if len(s_) == scheme.sig_len:
            sigs[j] = np.frombuffer(s_, np.uint8)
        else:
            bad_len[j] = True  # an all-zero record never decodes: rejected like kyber's length check
    rounds = np.array([lo + k for k in idx] or [0], dtype=np.uint64)
    dj = np.array(dev_j, dtype=np.int64)
    d_prevs = d_plen = None
    stride = 0
    if scheme.chained and n:
        lens = np.array([len(prevs[j]) for j in dev_j], dtype=np.uint32)
        stride = max(96, (int(lens.max()) + 3) // 4 * 4)
        pcol = np.zeros((n, stride), dtype=np.uint8)
        for t, j in enumerate(dev_j):
            pcol[t, :len(prevs[j])] = np.frombuffer(prevs[j], np.uint8)
        d_prevs = torch.from_numpy(pcol).to(device)
        d_plen = torch.from_numpy(lens.view(np.int32)).to(device)
    d_rounds = torch.from_numpy(np.ascontiguousarray(rounds[dj] if n else rounds[:1]).view(np.int64)).to(device)
    d_sigs = torch.from_numpy(np.ascontiguousarray(sigs[dj] if n else sigs[:1])).to(device)
    d_verdict = torch.zeros(max(n, 1), dtype=torch.uint8, device=device)
    partials = torch.zeros(lib.dh_partial_bytes(scheme.id), dtype=torch.uint8, device=device)
    failed = None
    v = np.zeros(len(idx), dtype=bool)
    try:
        verify_node_batch(lib, scheme, pk, d_rounds, d_sigs, n, d_verdict, None, partials, world, group,
                          d_prevs=d_prevs, prev_stride=stride, d_prev_lens=d_plen, seed=seed, rank=rank,
                          stage_host=stage_host, exchange=exchange)
        v[dj] = d_verdict.cpu().numpy()[:n].astype(bool)
        if oversize:  # host digest + device pairing check (the scheme path routes long records that way)
            j = np.array(oversize, dtype=np.int64)
            v[j], _ = scheme.verify_beacons(pk, rounds[j], sigs[j], [prevs[i] for i in j], seed=seed,
                                            want_randomness=False)
    except RuntimeError as e:  # joined below, so no rank waits in the verdict gather for this one
        failed = str(e)
    v &= ~bad_len[:len(idx)]
    ok_range[np.array(idx, dtype=np.int64)] = v.astype(np.uint8)
    bits = pack_bits(torch.from_numpy(ok_range).to(_collective_device(group) if xchg else torch.device("cpu")))
    faulty = []
    for r_, b_ in enumerate(gather_verdicts(bits, world, group, failed=failed, exchange=exchange)):
        a, z = shard_range(r_, world, last - first + 1)
        got = np.unpackbits(b_.cpu().numpy())[:z - a]
        faulty += [first + a + int(i) for i in np.flatnonzero(got == 0)]
    return faulty


def recover_shard(scheme, commits, t, n, msgs, partials_per_round, rank, world, group=None):
    """tbls Recover over the node (chain/beacon/chainstore.go:202-207, config 4 sharded as SURVEY.md §8e): the rounds
    are split with shard_range, each rank recovers and verifies its own rounds on its GPU (dh_recover_batch: the
    VerifyPartial batch check, selection, Lagrange interpolation and VerifyRecovered, all on the device), and the
    recovered signatures and status flags are all-gathered, so every rank returns the whole node's (signatures
    (n_rounds, sig_len) uint8, ok (n_rounds,) bool) in round order. Rounds are independent (each has its own partials
    and message): no exchange before the gather. A rank whose recovery fails flags it in the gather (NodeFailure on
    every rank)."""
    import torch
    lo, hi = shard_range(rank, world, len(msgs))
    failed = None
    sl = scheme.sig_len
    sigs = np.zeros((hi - lo, sl), np.uint8)
    ok = np.zeros(hi - lo, bool)
    try:
        if hi > lo:
            sigs, ok = scheme.recover_batch(commits, t, n, msgs[lo:hi], partials_per_round[lo:hi])
    except Exception as e:  # noqa: BLE001 - joined below, so no rank waits in the gather for this one
        failed = "rank %d: Recover: %s" % (rank, e)
    if world == 1:
        if failed:
            raise NodeFailure(failed)
        return sigs, ok
    dev = _collective_device(group)
    rec = np.zeros((hi - lo, sl + 1), np.uint8)
    rec[:, :sl] = sigs
    rec[:, sl] = ok
    flat = torch.from_numpy(rec.reshape(-1)).to(dev)
    parts = gather_verdicts(flat, world, group, failed=failed)  # variable-size byte columns, failure flag included
    out = np.concatenate([p.cpu().numpy().reshape(-1, sl + 1) for p in parts])
    return np.ascontiguousarray(out[:, :sl]), out[:, sl].astype(bool)
