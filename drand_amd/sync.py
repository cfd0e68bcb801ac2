"""Batch caller for chain replay: SyncManager.CheckPastBeacons over libdrandhip.

Mirrors /root/reference/chain/beacon/sync_manager.go:170-235 exactly, except that the per-round
VerifyBeacon loop body becomes one dh_verify_batch per window of rounds:
  * up_to is clamped to the last stored round;
  * rounds 1 .. store_len-1 are visited in order (store_len counts stored beacons, genesis included —
    so, as in the reference, a missing beacon shortens the walk by one);
  * a store Get error makes the round faulty; a verification failure records the beacon's round;
  * the walk stops after round >= up_to; the result is ascending; the callback sees every round first.
The store model is the bbolt "trimmed" layout (/root/reference/chain/boltdb/trimmed.go:87-107,156-193):
key = round, value = signature; for chained schemes Get(r) rebuilds PreviousSig from the stored signature of
round r-1 and fails if that one is missing (the genesis "signature" at round 0 is the genesis seed).
"""
import queue
import threading
import time

import numpy as np

from .chain import Beacon


class NoBeaconStored(KeyError):
    """chain/errors.ErrNoBeaconStored"""


class TrimmedMemStore:
    """In-memory store with the trimmed-bolt Get semantics."""

    def __init__(self, requires_previous):
        self.requires_previous = requires_previous
        self._sigs = {}

    def put(self, round_, sig):
        self._sigs[int(round_)] = bytes(sig)

    def delete(self, round_):
        self._sigs.pop(int(round_), None)

    def len(self):
        return len(self._sigs)

    def last(self):
        if not self._sigs:
            raise NoBeaconStored("empty store")
        return self.get(max(self._sigs))

    def get(self, round_):
        round_ = int(round_)
        sig = self._sigs.get(round_)
        if sig is None:
            raise NoBeaconStored(round_)
        prev = b""
        if self.requires_previous and round_ > 0:
            prev = self._sigs.get(round_ - 1)
            if prev is None:
                raise NoBeaconStored(round_ - 1)
        return Beacon(round_, sig, prev)


def check_past_beacons(store, scheme, pubkey, up_to, cb=None, window=1 << 20, seed=0):
    """Faulty rounds (ascending) among the stored rounds 1 .. min(up_to, last); [] when all verify."""
    last = store.last()
    if last.round < up_to:
        up_to = last.round
    store_len = store.len()
    faulty = []
    pending = []  # (round, beacon) awaiting batch verification, in order

    def flush():
        if not pending:
            return
        rounds = np.array([b.round for _, b in pending], dtype=np.uint64)
        sigs = np.zeros((len(pending), scheme.sig_len), dtype=np.uint8)
        bad_len = np.zeros(len(pending), dtype=bool)
        for k, (_, b) in enumerate(pending):
            if len(b.signature) == scheme.sig_len:
                sigs[k] = np.frombuffer(b.signature, dtype=np.uint8)
            else:
                bad_len[k] = True  # an all-zero record never decodes: rejected like kyber's length check
        prevs = [b.previous_signature for _, b in pending] if scheme.chained else None
        ok, _ = scheme.verify_beacons(pubkey, rounds, sigs, prevs, seed=seed, want_randomness=False)
        for (_, b), v, bl in zip(pending, ok, bad_len):
            if bl or not v:
                faulty.append(b.round)
        pending.clear()

    i = 1
    while i < store_len:
        if cb is not None:
            cb(i, up_to)
        try:
            b = store.get(i)
        except NoBeaconStored:
            flush()  # keep the faulty list ascending
            faulty.append(i)
            if i >= up_to:
                break
            i += 1
            continue
        pending.append((i, b))
        if len(pending) >= window:
            flush()
        if i >= up_to:
            break
        i += 1
    flush()
    return faulty


class WrongBeaconID(Exception):
    pass


_END = object()


def _packet_queue(packets):
    """A queue.Queue of the packets (ended by _END): the caller's own queue is used as is (a gRPC receive loop
    feeding it, the 500-deep channel of net/client_grpc.go:209-212); any other iterable is drained by a daemon
    reader thread, so the verifier can wait for the next packet with a timeout."""
    if isinstance(packets, queue.Queue):
        return packets
    q = queue.Queue(maxsize=500)

    def reader():
        try:
            for p in packets:
                q.put(p)
        finally:
            q.put(_END)

    threading.Thread(target=reader, daemon=True).start()
    return q


def sync_from_stream(packets, scheme, pubkey, store, up_to, beacon_id="", window=500, seed=0, idle=0.05,
                     max_delay=1.0):
    """tryNode's receive loop (/root/reference/chain/beacon/sync_manager.go:376-445) with verify-ahead windows
    (SURVEY.md §8f row 4). Packets arrive in order; they are verified in batches of up to `window` (the 500-deep
    gRPC buffer, /root/reference/net/client_grpc.go:209), and also as soon as the stream goes quiet for `idle`
    seconds or the oldest waiting packet has waited `max_delay` seconds — a live follow (one beacon per period)
    stores each beacon right after it arrives instead of waiting for 500 more. After verification, packets are
    stored in order until the first one that has the wrong beacon ID or fails verification (the serial loop stops
    at that packet, having stored everything before it). `packets` is an iterable or a queue.Queue of dicts
    {round, signature, previous_signature[, beacon_id]}, a queue ended by sync.END.
    Returns (done, stored rounds): done = the packet of round `up_to` was stored."""
    stored = []
    buf = []

    def drain():
        if not buf:
            return None
        n = len(buf)
        rounds = np.array([int(p["round"]) for p in buf], dtype=np.uint64)
        sigs = np.zeros((n, scheme.sig_len), dtype=np.uint8)
        bad_len = np.zeros(n, dtype=bool)
        for k, p in enumerate(buf):
            if len(p["signature"]) == scheme.sig_len:
                sigs[k] = np.frombuffer(bytes(p["signature"]), np.uint8)
            else:
                bad_len[k] = True
        prevs = [bytes(p.get("previous_signature", b"")) for p in buf] if scheme.chained else None
        ok, _ = scheme.verify_beacons(pubkey, rounds, sigs, prevs, seed=seed, want_randomness=False)
        for k, p in enumerate(buf):
            if bad_len[k] or not ok[k]:
                return False
            store.put(int(p["round"]), bytes(p["signature"]))
            stored.append(int(p["round"]))
            if int(p["round"]) == up_to:
                return True
        buf.clear()
        return None

    q = _packet_queue(packets)
    first_at = 0.0
    while True:
        timeout = None
        if buf:
            timeout = max(0.0, min(idle, first_at + max_delay - time.monotonic()))
        try:
            p = q.get(timeout=timeout)
        except queue.Empty:  # the stream went quiet (or the oldest packet waited long enough): verify now
            r = drain()
            if r is not None:
                return (r, stored)
            continue
        if p is _END:
            break
        bid = p.get("beacon_id")
        if bid is not None and bid != beacon_id:
            r = drain()  # packets before the mismatch were received first and are processed first
            return (bool(r), stored)
        if not buf:
            first_at = time.monotonic()
        buf.append(p)
        if len(buf) >= window:
            r = drain()
            if r is not None:
                return (r, stored)
    r = drain()
    return (bool(r), stored)


END = _END
