"""Host mirror of drand's crypto.Scheme over libdrandhip (the gfx950 verification engine).

Mirrors /root/reference/crypto/schemes.go:
  Scheme (fields Name / sig & key group sizes)           schemes.go:46-67
  Scheme.VerifyBeacon(beacon, pubkey) -> error (raise)    schemes.go:70-72
  Scheme.DigestBeacon                                     schemes.go:106-114 (chained), 147-151, 187-191
  SchemeFromName / ListSchemes / GetSchemeByIDWithDefault schemes.go:206-235
  GetSchemeFromEnv (SCHEME_ID)                            schemes.go:239-243
plus the batch entry point the reference lacks (Scheme.verify_beacons) and the RFC 9380 quicknet
scheme "bls-unchained-g1-rfc9380", which this snapshot of the reference does not have.

Errors follow the Go shape: VerifyBeacon raises SchemeError for an invalid beacon (Go returns a
non-nil error); batch calls return per-round booleans. Device failures raise DeviceError, never fall
back to a CPU path.
"""
import ctypes
import os
from dataclasses import dataclass

import numpy as np

from . import _lib

DEFAULT_SCHEME = "pedersen-bls-chained"        # DefaultSchemeID
UNCHAINED_SCHEME = "pedersen-bls-unchained"    # UnchainedSchemeID
SHORT_SIG_SCHEME = "bls-unchained-on-g1"       # ShortSigSchemeID
SIGS_ON_G1_SCHEME = "bls-unchained-g1-rfc9380"  # quicknet (RFC 9380 G1 DST); absent from the reference snapshot

_IDS = {DEFAULT_SCHEME: 0, UNCHAINED_SCHEME: 1, SHORT_SIG_SCHEME: 2, SIGS_ON_G1_SCHEME: 3}


class SchemeError(ValueError):
    """A verification / decoding failure (the Go API's non-nil error)."""


class DeviceError(RuntimeError):
    """libdrandhip reported a device / runtime failure."""


class DeviceBusy(DeviceError):
    """DH_EBUSY: every library worker is held by unfinished node batches (dh_batch_begin without dh_batch_finish)
    for longer than DRANDHIP_LEASE_TIMEOUT_MS. Nothing was verified; the call may be retried once the node batches
    have been finished (a thread that holds them must finish them first, or it waits on itself)."""


def _check(rc):
    if rc >= 0:
        return rc
    msg = _lib.last_error()
    if rc in (_lib.DH_EINVAL, _lib.DH_EKEY, _lib.DH_ERECOVER):
        raise SchemeError(msg)
    if rc == _lib.DH_EBUSY:
        raise DeviceBusy("libdrandhip error %d (busy): %s" % (rc, msg))
    raise DeviceError("libdrandhip error %d: %s" % (rc, msg))


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


@dataclass(frozen=True)
class Scheme:
    name: str
    id: int
    sig_len: int   # SigGroup point length (compressed)
    key_len: int   # KeyGroup point length
    chained: bool

    # ---- reference-shaped single-beacon API
    def digest_beacon(self, round_, previous_signature=b""):
        """crypto.Scheme.DigestBeacon: SHA-256(prev || round_be64) (chained) or SHA-256(round_be64)."""
        out = np.zeros(32, dtype=np.uint8)
        rounds = np.array([round_], dtype=np.uint64)
        prev = np.frombuffer(bytes(previous_signature), dtype=np.uint8).copy() if self.chained else None
        plen = np.array([len(previous_signature)], dtype=np.uint32) if self.chained else None
        _check(_lib.load().dh_digest_batch(self.id, _ptr(rounds), _ptr(prev) if prev is not None and len(prev) else None,
                                           max(1, len(previous_signature)), _ptr(plen), 1, _ptr(out)))
        return out.tobytes()

    def verify_beacon(self, beacon, pubkey):
        """crypto.Scheme.VerifyBeacon: raises SchemeError if the beacon does not verify."""
        prev = bytes(beacon.previous_signature or b"") if self.chained else b""
        rc = _lib.load().dh_verify_beacon(self.id, bytes(pubkey), len(pubkey), int(beacon.round),
                                          bytes(beacon.signature), len(beacon.signature), prev, len(prev))
        if _check(rc) != 1:
            raise SchemeError("bls: invalid signature")

    # ---- batch API (new): one call for many rounds sharing the group key
    def verify_beacons(self, pubkey, rounds, signatures, previous_signatures=None, seed=0, want_randomness=True,
                       previous_lengths=None):
        """Verify n rounds at once.

        rounds: (n,) uint64; signatures: (n, sig_len) uint8; previous_signatures (chained only): (n, L) uint8 (row i
        holds previous_lengths[i] bytes, default L) or a list of bytes of any lengths (the reference hashes whatever
        is stored, crypto/schemes.go:106-114). Returns (verdicts (n,) bool, randomness (n, 32) uint8 or None)."""
        rounds = np.ascontiguousarray(rounds, dtype=np.uint64)
        sigs = np.ascontiguousarray(signatures, dtype=np.uint8)
        n = len(rounds)
        if sigs.shape != (n, self.sig_len):
            raise SchemeError("signatures must be (%d, %d)" % (n, self.sig_len))
        if self.chained and previous_signatures is not None and not isinstance(previous_signatures, np.ndarray):
            items = [bytes(p or b"") for p in previous_signatures]
            if len(items) != n:
                raise SchemeError("previous_signatures must have one entry per round")
            big = np.array([len(p) > PREV_SLOT_MAX for p in items], dtype=bool)
            if big.any():
                return self._verify_with_oversize(pubkey, rounds, sigs, items, big, seed, want_randomness)
            previous_signatures = items
        prev = plen = None
        pstride = 0
        if self.chained and previous_signatures is not None:
            prev, plen, pstride = _pack_prevs(previous_signatures, n)
            if previous_lengths is not None:
                plen = np.ascontiguousarray(previous_lengths, dtype=np.uint32)
                if plen.shape != (n,) or (n and int(plen.max()) > pstride):
                    raise SchemeError("previous_lengths must give one length <= the row width per round")
        verdict = np.zeros(n, dtype=np.uint8)
        rand = np.zeros((n, 32), dtype=np.uint8) if want_randomness else None
        _check(_lib.load().dh_verify_batch(self.id, bytes(pubkey), len(pubkey), _ptr(rounds), _ptr(sigs), self.sig_len,
                                           _ptr(prev), pstride, _ptr(plen), n, _ptr(verdict), _ptr(rand), int(seed)))
        return verdict.astype(bool), rand

    def _verify_with_oversize(self, pubkey, rounds, sigs, items, big, seed, want_randomness):
        """Rounds whose previous signature exceeds PREV_SLOT_MAX bytes (a corrupted store, never a real chain):
        VerifyBeacon = VerifyRecovered(pk, DigestBeacon(b), sig) (crypto/schemes.go:70-72), with the digest hashed
        on the host (dh_digest_batch) and the pairing check on the device; the rest go through the batch path."""
        n = len(rounds)
        verdict = np.zeros(n, dtype=bool)
        rand = np.zeros((n, 32), dtype=np.uint8) if want_randomness else None
        small = np.flatnonzero(~big)
        if len(small):
            v, r = self.verify_beacons(pubkey, rounds[small], sigs[small], [items[i] for i in small], seed, want_randomness)
            verdict[small] = v
            if want_randomness:
                rand[small] = r
        large = np.flatnonzero(big)
        msgs = [self.digest_beacon(int(rounds[i]), items[i]) for i in large]
        verdict[large] = self.verify_recovered_batch(pubkey, msgs, sigs[large], seed=seed)
        if want_randomness:
            rand[large] = self.randomness(sigs[large])
        return verdict, rand

    # ---- threshold BLS (kyber sign/tbls as used at chain/beacon/chainstore.go:202,207)
    def verify_recovered(self, pubkey, msg, sig):
        """ThresholdScheme.VerifyRecovered(public, msg, sig) (chain/beacon/chainstore.go:207): raises SchemeError
        if sig is not a valid signature of the 32-byte msg under pubkey."""
        if len(msg) != 32:
            raise SchemeError("messages must be 32-byte digests")
        rc = _lib.load().dh_verify_recovered(self.id, bytes(pubkey), len(pubkey), bytes(msg), bytes(sig), len(sig))
        if _check(rc) != 1:
            raise SchemeError("bls: invalid signature")

    def verify_recovered_batch(self, pubkey, msgs, signatures, seed=0):
        """VerifyRecovered for n (32-byte msg, signature) pairs in one batch: (n,) bool verdicts."""
        n = len(msgs)
        m = np.frombuffer(b"".join(bytes(x) for x in msgs), dtype=np.uint8).copy() if n else np.zeros(0, np.uint8)
        if len(m) != 32 * n:
            raise SchemeError("messages must be 32-byte digests")
        sigs = np.ascontiguousarray(signatures, dtype=np.uint8)
        if sigs.shape != (n, self.sig_len):
            raise SchemeError("signatures must be (%d, %d)" % (n, self.sig_len))
        verdict = np.zeros(n, dtype=np.uint8)
        _check(_lib.load().dh_verify_recovered_batch(self.id, bytes(pubkey), len(pubkey), _ptr(m), _ptr(sigs),
                                                     self.sig_len, n, _ptr(verdict), int(seed)))
        return verdict.astype(bool)

    def index_of(self, partial):
        """ThresholdScheme.IndexOf (chain/beacon/node.go:133): the 2-byte big-endian share index."""
        partial = bytes(partial)
        if len(partial) < 2:
            raise SchemeError("invalid partial signature")
        return int.from_bytes(partial[:2], "big")

    def _pack_partials(self, commits, t, msgs, partials_per_round):
        commits = b"".join(bytes(c) for c in commits)
        if len(commits) != t * self.key_len:
            raise SchemeError("need t commitments of %d bytes" % self.key_len)
        n_rounds = len(msgs)
        m = np.frombuffer(b"".join(bytes(x) for x in msgs), dtype=np.uint8).copy() if n_rounds else np.zeros(0, np.uint8)
        if len(m) != 32 * n_rounds:
            raise SchemeError("messages must be 32-byte digests")
        rec = 2 + self.sig_len
        off = np.zeros(n_rounds + 1, dtype=np.uint32)
        blobs = []
        for j, parts in enumerate(partials_per_round):
            for p in parts:
                p = bytes(p)
                if len(p) != rec:
                    raise SchemeError("partial signature must be %d bytes" % rec)
                blobs.append(p)
            off[j + 1] = len(blobs)
        raw = np.frombuffer(b"".join(blobs), dtype=np.uint8).copy() if blobs else np.zeros(rec, np.uint8)
        return commits, m, raw, off, len(blobs)

    def verify_partials_batch(self, commits, t, n, msgs, partials_per_round):
        """Batch VerifyPartial (chain/beacon/node.go:150): per round, each (index || sig) partial checked against
        PubPoly.Eval(index) for that round's 32-byte message. Returns a list (per round) of bool arrays."""
        commits, m, raw, off, npart = self._pack_partials(commits, t, msgs, partials_per_round)
        ok = np.zeros(max(npart, 1), dtype=np.uint8)
        _check(_lib.load().dh_verify_partials_batch(self.id, commits, int(t), int(n), _ptr(m), _ptr(raw), _ptr(off),
                                                    len(msgs), _ptr(ok)))
        return [ok[off[j]:off[j + 1]].astype(bool) for j in range(len(msgs))]

    def verify_partial(self, commits, t, n, msg, partial):
        """ThresholdScheme.VerifyPartial(pubPoly, msg, partial): raises SchemeError when invalid."""
        if not self.verify_partials_batch(commits, t, n, [msg], [[partial]])[0][0]:
            raise SchemeError("bls: invalid partial signature")

    def recover_batch(self, commits, t, n, msgs, partials_per_round):
        """Batch tbls Recover. commits: t compressed key-group points (PubPoly commits, index 0 = group key);
        msgs: per-round 32-byte messages (DigestBeacon); partials_per_round: per round a list of
        (2-byte BE share index || signature) records, in arrival order.
        Returns (signatures (n_rounds, sig_len) uint8, ok (n_rounds,) bool) where ok[j] is False when
        fewer than t valid partials were given (Go: "not enough good public shares")."""
        commits, m, raw, off, _ = self._pack_partials(commits, t, msgs, partials_per_round)
        n_rounds = len(msgs)
        sigs = np.zeros((n_rounds, self.sig_len), dtype=np.uint8)
        ok = np.zeros(n_rounds, dtype=np.uint8)
        _check(_lib.load().dh_recover_batch(self.id, commits, int(t), int(n), _ptr(m), _ptr(raw), _ptr(off), n_rounds,
                                            _ptr(sigs), _ptr(ok)))
        return sigs, ok.astype(bool)

    def recover_batch_packed(self, commits, t, n, msgs, raw, offsets):
        """recover_batch over caller-packed columns: msgs (n_rounds, 32) uint8, raw (n_partials, 2 + sig_len) uint8
        records (2-byte BE index || signature), offsets (n_rounds + 1,) uint32 into raw."""
        commits = b"".join(bytes(c) for c in commits)
        if len(commits) != t * self.key_len:
            raise SchemeError("need t commitments of %d bytes" % self.key_len)
        msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
        raw = np.ascontiguousarray(raw, dtype=np.uint8)
        off = np.ascontiguousarray(offsets, dtype=np.uint32)
        n_rounds = len(msgs)
        if msgs.shape != (n_rounds, 32) or off.shape != (n_rounds + 1,) or raw.ndim != 2 or raw.shape[1] != 2 + self.sig_len:
            raise SchemeError("bad packed Recover columns")
        sigs = np.zeros((n_rounds, self.sig_len), dtype=np.uint8)
        ok = np.zeros(n_rounds, dtype=np.uint8)
        _check(_lib.load().dh_recover_batch(self.id, commits, int(t), int(n), _ptr(msgs), _ptr(raw), _ptr(off), n_rounds,
                                            _ptr(sigs), _ptr(ok)))
        return sigs, ok.astype(bool)

    def recover(self, commits, msg, partials, t, n):
        """ThresholdScheme.Recover(pubPoly, msg, sigs, t, n): the recovered signature, or SchemeError."""
        sigs, ok = self.recover_batch(commits, t, n, [msg], [partials])
        if not ok[0]:
            raise SchemeError("not enough good public shares")
        return sigs[0].tobytes()

    def randomness(self, signatures):
        sigs = np.ascontiguousarray(signatures, dtype=np.uint8)
        out = np.zeros((len(sigs), 32), dtype=np.uint8)
        _check(_lib.load().dh_randomness_batch(self.id, _ptr(sigs), self.sig_len, len(sigs), _ptr(out)))
        return out

    # ---- synthetic-chain utilities (tests / bench): device signer
    def sign_beacons(self, secret32, rounds, previous_signatures=None, previous_lengths=None):
        rounds = np.ascontiguousarray(rounds, dtype=np.uint64)
        n = len(rounds)
        prev = plen = None
        pstride = 0
        if self.chained and previous_signatures is not None:
            prev, plen, pstride = _pack_prevs(previous_signatures, n)
            if previous_lengths is not None:
                plen = np.ascontiguousarray(previous_lengths, dtype=np.uint32)
        out = np.zeros((n, self.sig_len), dtype=np.uint8)
        _check(_lib.load().dh_sign_batch(self.id, bytes(secret32), _ptr(rounds), _ptr(prev), n if prev is None else n,
                                         _ptr(plen) if plen is not None else None, pstride, _ptr(out)))
        return out

    def public_key(self, secret32):
        out = np.zeros(self.key_len, dtype=np.uint8)
        _check(_lib.load().dh_public_key(self.id, bytes(secret32), _ptr(out)))
        return out.tobytes()

    def __str__(self):
        return self.name


# Previous signatures up to this many bytes travel in one fixed-stride slot array (a stored signature is 96 B);
# longer records only come from corrupted stores and are verified one digest at a time (_verify_with_oversize).
PREV_SLOT_MAX = 4096


class ThresholdScheme:
    """kyber sign.ThresholdScheme over libdrandhip, one call per method — the exact shapes of the cgo type in
    INTEGRATION.md §2 (gpuThresholdScheme), which the reference's constructors install as Scheme.ThresholdScheme
    (crypto/schemes.go:101,142,182). Semantics follow kyber v1.1.18 sign/tbls:
      IndexOf(sig)                          2-byte big-endian prefix (SigShare.Index); error on < 2 bytes
      VerifyPartial(pubPoly, msg, sig)      Verify(PubPoly.Eval(i).V, msg, sig[2:]) for ANY index i: the call passes
                                            n_nodes = i + 1 so the device evaluates the polynomial at exactly x = i + 1
      VerifyRecovered(pk, msg, sig)         bls.Verify (chain/beacon/chainstore.go:207)
      Recover(pubPoly, msg, sigs, t, n)     first t valid partials in arrival order (wrong-length records skipped, as
                                            kyber's Verify of sig[2:] rejects them), Lagrange at 0; n_nodes =
                                            max(n, largest index + 1), so a valid partial of any index counts (kyber)
    Messages are 32-byte beacon digests on the device; `commits` are the PubPoly's compressed commitments."""

    def __init__(self, scheme):
        self.scheme = scheme

    def index_of(self, sig):
        sig = bytes(sig)
        if len(sig) < 2:
            raise SchemeError("unexpected EOF")  # binary.Read of the uint16 index
        return int.from_bytes(sig[:2], "big")

    def verify_partial(self, commits, msg, sig):
        i = self.index_of(sig)
        s = self.scheme
        if len(sig) != 2 + s.sig_len:
            raise SchemeError("bls: invalid signature")
        if not s.verify_partials_batch(commits, len(commits), i + 1, [msg], [[sig]])[0][0]:
            raise SchemeError("bls: invalid signature")

    def verify_recovered(self, pubkey, msg, sig):
        self.scheme.verify_recovered(pubkey, msg, sig)

    def recover(self, commits, msg, sigs, t, n):
        s = self.scheme
        if len(commits) != t:
            raise SchemeError("the device Recover takes the PubPoly's t commitments")
        recs = [bytes(x) for x in sigs if len(x) == 2 + s.sig_len]
        n_nodes = max([n] + [int.from_bytes(x[:2], "big") + 1 for x in recs])
        out, ok = s.recover_batch(commits, t, n_nodes, [msg], [recs])
        if not ok[0]:
            raise SchemeError("share: not enough good public shares to reconstruct secret commitment")
        return out[0].tobytes()


def _pack_prevs(previous_signatures, n):
    """-> (prevs u8[n, stride], lengths u32[n], stride): any lengths up to the stride; the device hashes exactly
    lengths[i] bytes of row i."""
    if isinstance(previous_signatures, np.ndarray) and previous_signatures.ndim == 2:
        prev = np.ascontiguousarray(previous_signatures, dtype=np.uint8)
        if len(prev) != n:
            raise SchemeError("previous_signatures must have one row per round")
        width = prev.shape[1]
        plen = np.full(n, width, dtype=np.uint32)
        if width == 0:
            return np.zeros((n, 4), np.uint8), plen, 4
        return prev, plen, width
    items = [bytes(p or b"") for p in previous_signatures]
    if len(items) != n:
        raise SchemeError("previous_signatures must have one entry per round")
    longest = max((len(p) for p in items), default=0)
    stride = max(96, (longest + 3) // 4 * 4)
    prev = np.zeros((n, stride), dtype=np.uint8)
    plen = np.zeros(n, dtype=np.uint32)
    for i, p in enumerate(items):
        prev[i, :len(p)] = np.frombuffer(p, dtype=np.uint8)
        plen[i] = len(p)
    return prev, plen, stride


_SCHEMES = {
    DEFAULT_SCHEME: Scheme(DEFAULT_SCHEME, 0, 96, 48, True),
    UNCHAINED_SCHEME: Scheme(UNCHAINED_SCHEME, 1, 96, 48, False),
    SHORT_SIG_SCHEME: Scheme(SHORT_SIG_SCHEME, 2, 48, 96, False),
    SIGS_ON_G1_SCHEME: Scheme(SIGS_ON_G1_SCHEME, 3, 48, 96, False),
}


def hash_to_curve(group, messages, dst):
    """RFC 9380 hash_to_curve on the device: group 1 (G1) or 2 (G2), a list of byte strings, one DST. Returns the
    compressed points (list of bytes)."""
    msgs = [bytes(m) for m in messages]
    off = np.zeros(len(msgs) + 1, dtype=np.uint32)
    off[1:] = np.cumsum([len(m) for m in msgs])
    blob = np.frombuffer(b"".join(msgs) or b"\0", dtype=np.uint8).copy()
    size = 48 if group == 1 else 96
    out = np.zeros((len(msgs), size), dtype=np.uint8)
    _check(_lib.load().dh_hash_to_curve(int(group), _ptr(blob), _ptr(off), len(msgs), bytes(dst), len(dst), _ptr(out)))
    return [r.tobytes() for r in out]


def scheme_from_name(name):
    """crypto.SchemeFromName; raises SchemeError("invalid scheme name '...'")."""
    try:
        return _SCHEMES[name]
    except KeyError:
        raise SchemeError("invalid scheme name '%s'" % name) from None


def list_schemes():
    return list(_SCHEMES)


def get_scheme_by_id_with_default(id_):
    return scheme_from_name(id_ or DEFAULT_SCHEME)


def get_scheme_from_env():
    return get_scheme_by_id_with_default(os.environ.get("SCHEME_ID", ""))
