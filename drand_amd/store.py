"""Chain readers for batch replay: bbolt beacon stores and hexjson beacon records,
ingested into the columnar arrays dh_verify_batch takes.

* A minimal read-only bbolt (go.etcd.io/bbolt, file format v2) reader: meta pages 0/1 (the valid one with the
  larger txid), branch / leaf pages, nested and inline buckets, overflow pages.
* BoltTrimmedStore — the trimmed layout (/root/reference/chain/boltdb/trimmed.go:87-107,156-193): bucket
  "beacons", key = round as 8-byte big-endian (chain.RoundToBytes, /root/reference/chain/store.go:82-87),
  value = raw signature; for chained schemes Get(r) takes PreviousSig from the stored signature of r-1.
* BoltUntrimmedStore — the legacy layout (/root/reference/chain/boltdb/store.go:143-168): value = the hexjson
  encoding of chain.Beacon {"PreviousSig","Round","Signature"} (/root/reference/chain/beacon.go:14-39).
Both expose get / len / last like drand_amd.sync.TrimmedMemStore, so check_past_beacons runs over a real
store file, plus columns(first, last) for bulk ingestion.
* hexjson records: client.RandomData {"round","randomness","signature","previous_signature"}
  (/root/reference/client/random.go:5-25) and BeaconPacket-shaped JSON, one object per line or a JSON list.
"""
import json
import struct

import numpy as np

from .chain import Beacon
from .sync import NoBeaconStored

BEACON_BUCKET = b"beacons"  # /root/reference/chain/boltdb/store.go:31
_MAGIC = 0xED0CDAED
_BRANCH, _LEAF, _META = 0x01, 0x02, 0x04
_BUCKET_LEAF = 0x01


class BoltError(ValueError):
    pass


def _fnv64a(b):
    h = 0xcbf29ce484222325
    for x in b:
        h ^= x
        h = (h * 0x100000001b3) & 0xffffffffffffffff
    return h


class BoltFile:
    """Read-only view of a bbolt database file."""

    def __init__(self, path_or_bytes):
        self.data = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else open(path_or_bytes, "rb").read()
        metas = []
        for pg in (0, 1):
            m = self._meta(pg * self._guess_page_size())
            if m:
                metas.append(m)
        if not metas:
            raise BoltError("no valid bbolt meta page")
        self.meta = max(metas, key=lambda m: m["txid"])
        self.page_size = self.meta["page_size"]

    def _guess_page_size(self):
        return struct.unpack_from("<I", self.data, 24)[0] if len(self.data) >= 28 else 4096

    def _meta(self, off):
        if off + 80 > len(self.data):
            return None
        _, flags, _, _ = struct.unpack_from("<QHHI", self.data, off)
        magic, version, psz, _ = struct.unpack_from("<IIII", self.data, off + 16)
        root, _seq, freelist, pgid, txid, cks = struct.unpack_from("<QQQQQQ", self.data, off + 32)
        if not flags & _META or magic != _MAGIC or version != 2:
            return None
        if _fnv64a(self.data[off + 16:off + 72]) != cks:
            return None
        return {"page_size": psz, "root": root, "txid": txid, "pgid": pgid}

    def _page(self, pgid):
        off = pgid * self.page_size
        if off + 16 > len(self.data):
            raise BoltError("page %d beyond end of file" % pgid)
        return self.data, off

    def _walk(self, buf, off):
        """Yield (key, value, flags) of the leaf elements under the page at buf[off:], in key order."""
        _, flags, count, _ = struct.unpack_from("<QHHI", buf, off)
        base = off + 16
        if flags & _LEAF:
            for i in range(count):
                e = base + 16 * i
                fl, pos, ks, vs = struct.unpack_from("<IIII", buf, e)
                k = bytes(buf[e + pos:e + pos + ks])
                v = bytes(buf[e + pos + ks:e + pos + ks + vs])
                yield k, v, fl
        elif flags & _BRANCH:
            for i in range(count):
                e = base + 16 * i
                _pos, _ks, child = struct.unpack_from("<IIQ", buf, e)
                cbuf, coff = self._page(child)
                yield from self._walk(cbuf, coff)
        else:
            raise BoltError("unexpected page flags 0x%x" % flags)

    def _bucket_items(self, root, inline=None):
        if root == 0:  # inline bucket: the page follows the 16-byte bucket header in the value
            return self._walk(inline, 16)
        buf, off = self._page(root)
        return self._walk(buf, off)

    def bucket(self, name):
        """{key: value} of a top-level bucket (sub-buckets are skipped)."""
        for k, v, fl in self._bucket_items(self.meta["root"]):
            if k == name and fl & _BUCKET_LEAF:
                root, _seq = struct.unpack_from("<QQ", v, 0)
                return {bk: bv for bk, bv, bfl in self._bucket_items(root, v) if not bfl & _BUCKET_LEAF}
        raise BoltError("bucket %r not found" % name)


class _BoltStoreBase:
    def __init__(self, path, requires_previous):
        self.requires_previous = bool(requires_previous)
        self._kv = BoltFile(path).bucket(BEACON_BUCKET)
        self._rounds = sorted(struct.unpack(">Q", k)[0] for k in self._kv if len(k) == 8)

    def len(self):
        return len(self._kv)

    def rounds(self):
        return list(self._rounds)

    def last(self):
        if not self._rounds:
            raise NoBeaconStored("empty store")
        return self.get(self._rounds[-1])


class BoltTrimmedStore(_BoltStoreBase):
    """trimmedStore read path (/root/reference/chain/boltdb/trimmed.go:156-193)."""

    def _sig(self, r):
        v = self._kv.get(struct.pack(">Q", r))
        if v is None:
            raise NoBeaconStored(r)
        return v

    def get(self, round_):
        round_ = int(round_)
        sig = self._sig(round_)
        prev = b""
        if self.requires_previous and round_ > 0:
            prev = self._sig(round_ - 1)
        return Beacon(round_, sig, prev)

    def columns(self, first, last, sig_len):
        """Rounds first..last as (rounds u64[n], sigs u8[n, sig_len], prevs list | None, missing rounds).
        Rounds whose record is missing (or whose previous record is missing, chained) are left out of the
        columns and returned in `missing`, which is what CheckPastBeacons reports as faulty for them. A stored
        signature of the wrong length is zero-filled, never cut to a prefix: kilic's UnmarshalBinary rejects
        any wrong-length point and an all-zero record never decodes, so the round is rejected as in Go."""
        rounds, sigs, prevs, missing = [], [], [], []
        for r in range(int(first), int(last) + 1):
            try:
                b = self.get(r)
            except NoBeaconStored:
                missing.append(r)
                continue
            rounds.append(r)
            s = np.zeros(sig_len, np.uint8)
            if len(b.signature) == sig_len:
                s[:] = np.frombuffer(b.signature, np.uint8)
            sigs.append(s)
            prevs.append(b.previous_signature)
        sig_arr = np.array(sigs, dtype=np.uint8).reshape(-1, sig_len)
        return (np.array(rounds, dtype=np.uint64), sig_arr, prevs if self.requires_previous else None, missing)


class BoltUntrimmedStore(_BoltStoreBase):
    """BoltStore read path (/root/reference/chain/boltdb/store.go): hexjson-encoded chain.Beacon values."""

    def get(self, round_):
        v = self._kv.get(struct.pack(">Q", int(round_)))
        if v is None:
            raise NoBeaconStored(round_)
        return beacon_from_hexjson(v)


def _hexbytes(x):
    return bytes.fromhex(x) if x else b""


def beacon_from_hexjson(text):
    """chain.Beacon.Unmarshal (/root/reference/chain/beacon.go:36-39): hexjson with Go field names."""
    d = json.loads(text)
    return Beacon(int(d.get("Round", 0)), _hexbytes(d.get("Signature")), _hexbytes(d.get("PreviousSig")))


def read_random_data(text):
    """client.RandomData records (/root/reference/client/random.go:5-10), as a JSON list or one object per
    line -> list of dicts {round, randomness, signature, previous_signature} with bytes values. BeaconPacket
    JSON field names (round, signature, previous_signature) read the same way."""
    text = text.strip()
    objs = json.loads(text) if text.startswith("[") else [json.loads(l) for l in text.splitlines() if l.strip()]
    out = []
    for o in objs:
        out.append({"round": int(o.get("round", 0)), "randomness": _hexbytes(o.get("randomness")),
                    "signature": _hexbytes(o.get("signature")),
                    "previous_signature": _hexbytes(o.get("previous_signature"))})
    return out


def random_data_columns(records, sig_len):
    """RandomData records -> (rounds u64[n], sigs u8[n, sig_len], prevs list, randomness list). A signature
    of the wrong length is zero-filled (an all-zero record never decodes, so it is rejected like kyber's
    length check)."""
    n = len(records)
    rounds = np.array([r["round"] for r in records], dtype=np.uint64)
    sigs = np.zeros((n, sig_len), dtype=np.uint8)
    for i, r in enumerate(records):
        if len(r["signature"]) == sig_len:
            sigs[i] = np.frombuffer(r["signature"], np.uint8)
    return rounds, sigs, [r["previous_signature"] for r in records], [r["randomness"] for r in records]
