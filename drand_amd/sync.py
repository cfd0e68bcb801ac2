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


class BeaconAlreadyStored(Exception):
    """chain/beacon.ErrBeaconAlreadyStored (/root/reference/chain/beacon/store.go:52-53)."""


class PutError(Exception):
    """Any other error of the chain store's Put (store.go:55-77, 99-124)."""


class ChainStore:
    """The Put checks of the beacon chain store stack that tryNode writes through (s.store,
    /root/reference/chain/beacon/chainstore.go:45-60: callbackStore -> appendStore -> schemeStore ->
    discrepancyStore -> the trimmed bolt store). `store` is the underlying trimmed store (TrimmedMemStore or a
    writable equivalent); both decorators start from its Last() beacon (newAppendStore / NewSchemeStore).
      appendStore.Put (store.go:55-77): same round as the last one -> ErrBeaconAlreadyStored if signature and
        previous signature are equal, an error if either differs; any round other than last+1 -> error.
      schemeStore.Put (store.go:99-124): chained (DefaultSchemeID) -> the previous signature must equal the last
        stored signature; other schemes -> the previous signature is dropped (b.PreviousSig = nil, on the same
        beacon object, so appendStore's `last` keeps no previous signature either).
    The discrepancy and callback stores only log and notify."""

    def __init__(self, store, scheme):
        from .scheme import DEFAULT_SCHEME
        self.store = store
        self._chained_name = scheme.name == DEFAULT_SCHEME
        last = store.last()
        self._append_last = Beacon(last.round, bytes(last.signature), bytes(last.previous_signature or b""))
        self._scheme_last = self._append_last

    def last(self):
        return self.store.last()

    def len(self):
        return self.store.len()

    def get(self, round_):
        return self.store.get(round_)

    def put(self, beacon):
        rnd, sig = int(beacon.round), bytes(beacon.signature)
        prev = bytes(beacon.previous_signature or b"")  # Go: bytes.Equal(nil, []byte{}) is true
        a = self._append_last
        if rnd == a.round:
            if a.signature == sig:
                if a.previous_signature == prev:
                    raise BeaconAlreadyStored("beacon value already stored round %d" % rnd)
                raise PutError("tried to store a duplicate beacon for round %d but the previous signature was "
                               "different" % rnd)
            raise PutError("tried to store a duplicate beacon for round %d but the signature was different" % rnd)
        if rnd != a.round + 1:
            raise PutError("invalid round inserted: last %d, new %d" % (a.round, rnd))
        if self._chained_name:
            if self._scheme_last.signature != prev:
                raise PutError("invalid previous signature for %d" % rnd)
        else:
            prev = b""
        self.store.put(rnd, sig)
        b = Beacon(rnd, sig, prev)
        self._scheme_last = b
        self._append_last = b


_END = object()


def _packet_queue(packets):
    """(queue.Queue of the packets ended by _END, stop function). The caller's own queue is used as is (a gRPC
    receive loop feeding it, the 500-deep channel of net/client_grpc.go:209-212); any other iterable is drained by a
    daemon reader thread, so the verifier can wait for the next packet with a timeout. stop() ends the reader and
    closes the iterator (tryNode's deferred cancel of the peer context, sync_manager.go:335-336): a sync that
    returns early leaves no thread blocked on a full queue and no stream open."""
    if isinstance(packets, queue.Queue):
        return packets, lambda: None
    q = queue.Queue(maxsize=500)
    halt = threading.Event()
    it = iter(packets)

    def reader():
        try:
            for p in it:
                while not halt.is_set():
                    try:
                        q.put(p, timeout=0.05)
                        break
                    except queue.Full:
                        continue
                if halt.is_set():
                    break
        finally:
            for name in ("close", "cancel"):
                fn = getattr(it, name, None) or getattr(packets, name, None)
                if callable(fn):
                    try:
                        fn()
                    except Exception:  # noqa: BLE001 - best effort, the peer is being dropped
                        pass
                    break
            try:
                q.put_nowait(_END)
            except queue.Full:
                pass

    th = threading.Thread(target=reader, daemon=True)
    th.start()

    def stop():
        halt.set()
        th.join(timeout=1.0)

    return q, stop


def sync_from_stream(packets, scheme, pubkey, store, up_to, beacon_id="", window=500, seed=0, idle=0.05,
                     max_delay=1.0, resync=False):
    """tryNode's receive loop (/root/reference/chain/beacon/sync_manager.go:376-445) with verify-ahead windows
    (SURVEY.md §8f row 4). Packets arrive in order; they are verified in batches of up to `window` (the 500-deep
    gRPC buffer, /root/reference/net/client_grpc.go:209), and also as soon as the stream goes quiet for `idle`
    seconds or the oldest waiting packet has waited `max_delay` seconds — a live follow (one beacon per period)
    stores each beacon right after it arrives instead of waiting for 500 more. After verification the packets are
    handled in order exactly as the serial loop handles them: a wrong beacon ID or a failed VerifyBeacon stops the
    peer; then Put — through the chain store's checks (ChainStore: appendStore + schemeStore) unless `resync`
    (from > 0: the insecure store, a plain write, sync_manager.go:410-416). ErrBeaconAlreadyStored ends the peer
    with done = (round == up_to); any other Put error ends it with done = False (:417-425). `store` is a
    ChainStore or a trimmed store (wrapped in a ChainStore here; its Last() must exist, as in tryNode :338-342).
    `packets` is an iterable or a queue.Queue of dicts {round, signature, previous_signature[, beacon_id]}, a queue
    ended by sync.END. Returns (done, stored rounds): done = the packet of round `up_to` was stored."""
    stored = []
    buf = []
    if not resync and not isinstance(store, ChainStore):
        try:
            store = ChainStore(store, scheme)
        except NoBeaconStored:
            return (False, stored)  # tryNode: "unable to fetch from store"

    def put(p):
        if resync:
            store.put(int(p["round"]), bytes(p["signature"]))
            return None
        try:
            store.put(Beacon(int(p["round"]), bytes(p["signature"]), bytes(p.get("previous_signature") or b"")))
        except BeaconAlreadyStored:
            return int(p["round"]) == up_to
        except PutError:
            return False
        return None

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
        prevs = [bytes(p.get("previous_signature") or b"") for p in buf] if scheme.chained else None
        ok, _ = scheme.verify_beacons(pubkey, rounds, sigs, prevs, seed=seed, want_randomness=False)
        for k, p in enumerate(buf):
            if bad_len[k] or not ok[k]:
                return False
            r = put(p)
            if r is not None:
                return r
            stored.append(int(p["round"]))
            if int(p["round"]) == up_to:
                return True
        buf.clear()
        return None

    q, stop = _packet_queue(packets)
    try:
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
    finally:
        stop()


END = _END
