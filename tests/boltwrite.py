"""Test helper: write a minimal bbolt (format v2) file with one top-level bucket, so that store readers can be
tested on chains whose keys are known (the reference's own fixtures tests/golden/boltdb/*.db come from an
unknown key). Layout: pages 0/1 meta, 2 freelist (empty), 3 root leaf holding the bucket entry, then the
bucket's leaf pages (and one branch page when more than one leaf is needed)."""
import struct

PAGE = 4096


def _fnv64a(b):
    h = 0xcbf29ce484222325
    for x in b:
        h ^= x
        h = (h * 0x100000001b3) & 0xffffffffffffffff
    return h


def _leaf(pgid, items, flags_of=lambda k: 0):
    n = len(items)
    hdr = struct.pack("<QHHI", pgid, 0x02, n, 0)
    elems, data = b"", b""
    data_off = 16 * n
    for i, (k, v) in enumerate(items):
        pos = data_off + len(data) - 16 * i
        elems += struct.pack("<IIII", flags_of(k), pos, len(k), len(v))
        data += k + v
    body = hdr + elems + data
    assert len(body) <= PAGE, "leaf overflow"
    return body.ljust(PAGE, b"\0")


def _branch(pgid, children):
    n = len(children)
    hdr = struct.pack("<QHHI", pgid, 0x01, n, 0)
    elems, data = b"", b""
    for i, (k, child) in enumerate(children):
        pos = 16 * n + len(data) - 16 * i
        elems += struct.pack("<IIQ", pos, len(k), child)
        data += k
    return (hdr + elems + data).ljust(PAGE, b"\0")


def _meta(pgid, root, freelist, hw, txid):
    m = struct.pack("<IIII", 0xED0CDAED, 2, PAGE, 0) + struct.pack("<QQQQQ", root, 0, freelist, hw, txid)
    return (struct.pack("<QHHI", pgid, 0x04, 0, 0) + m + struct.pack("<Q", _fnv64a(m))).ljust(PAGE, b"\0")


def write_bolt(path, bucket, kv):
    items = sorted(kv.items())
    leaves, cur, size = [], [], 16
    for k, v in items:
        need = 16 + len(k) + len(v)
        if cur and size + need > PAGE:
            leaves.append(cur)
            cur, size = [], 16
        cur.append((k, v))
        size += need
    leaves.append(cur)
    pages = {}
    first_leaf = 4 if len(leaves) == 1 else 5
    for i, lv in enumerate(leaves):
        pages[first_leaf + i] = _leaf(first_leaf + i, lv)
    broot = 4
    if len(leaves) > 1:
        pages[4] = _branch(4, [(lv[0][0], first_leaf + i) for i, lv in enumerate(leaves)])
    pages[3] = _leaf(3, [(bucket, struct.pack("<QQ", broot, 0))], flags_of=lambda k: 0x01)
    pages[2] = struct.pack("<QHHI", 2, 0x10, 0, 0).ljust(PAGE, b"\0")
    hw = max(pages) + 1
    pages[0] = _meta(0, 3, 2, hw, 2)
    pages[1] = _meta(1, 3, 2, hw, 1)
    with open(path, "wb") as f:
        for p in range(hw):
            f.write(pages[p])
