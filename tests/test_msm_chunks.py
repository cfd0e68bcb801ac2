"""Index model of the MSM bucket pass's chunking (drand_amd/csrc/k_msm.hip k_msm_bucket28 + k_msm_bucket_fix28).

The sorted list (bucket by bucket) is cut into chunks of L entries, one lane each; a key cut by chunk boundaries
leaves a tail partial in the lane where it starts and head partials (kind 2: the key covers the chunk, kind 1: it ends
there) in the lanes after it, and k_msm_bucket_fix28 adds them up (the library's scheme, in_wave=False). in_wave=True
models a variant that resolved such keys inside the 64-lane wave through LDS and left only keys running past the
wave's last lane to the fix-up: correct (this model), but measured slower on the device (G1 MSM 4.86 -> 5.36 ms, G2
18.2 -> 22.3 ms at 1M rounds, profiles/r03m: the tail walk serialised every wave's end and the G2 pass spilled), so
it was not kept. The model replays the control flow with integers standing in for points and checks that every
nonempty bucket is written once, with the sum of its entries, for bucket sizes from one entry per bucket to buckets
spanning several waves. CPU only.
"""
import numpy as np
import pytest

NO_KEY = -1
BLOCK = 256
WAVE = 64


def bucket_pass(off, lst, L, in_wave=True):
    nkeys = len(off) - 1
    total = off[nkeys]
    nch = (total + L - 1) // L
    nthreads = ((nch + BLOCK - 1) // BLOCK) * BLOCK if nch else 0
    buckets = {}
    writes = {}
    part = {}
    meta = {}

    def write(key, v):
        buckets[key] = v
        writes[key] = writes.get(key, 0) + 1

    for b0 in range(0, nthreads, BLOCK):
        sh_head = [None] * BLOCK
        sh_kind = [0] * BLOCK
        tails = {}  # thread -> (key, acc)
        for tid in range(BLOCK):
            t = b0 + tid
            s = t * L
            if s >= total:
                continue
            e = min(s + L, total)
            key = int(np.searchsorted(off, s, side="right")) - 1  # last key with off[key] <= s
            kend = off[key + 1]
            starts_before = off[key] < s
            first = True
            acc = 0
            for j in range(s, e):
                acc += lst[j]
                ends = j + 1 == kend
                if ends or j + 1 == e:
                    if first and starts_before:
                        sh_head[tid] = acc
                        sh_kind[tid] = 1 if ends else 2
                    elif ends:
                        write(key, acc)
                    else:
                        part[2 * t + 1] = acc
                        tails[tid] = (key, acc)
                    if first and starts_before and not in_wave:
                        part[2 * t] = acc
                    first = False
                    if ends and j + 1 < e:
                        key += 1
                        while off[key + 1] <= j + 1:
                            key += 1
                        kend = off[key + 1]
                        acc = 0
        if not in_wave:
            for tid in range(BLOCK):
                t = b0 + tid
                if t * L < total:
                    meta[2 * t] = sh_kind[tid]
                    meta[2 * t + 1] = tails[tid][0] if tid in tails else NO_KEY
            continue
        # after the barrier, per wave
        for tid in range(BLOCK):
            t = b0 + tid
            lane, wb = tid % WAVE, tid - tid % WAVE
            k2 = [sh_kind[wb + v] == 2 for v in range(WAVE)]
            if sh_kind[tid] and all(k2[:lane]):
                part[2 * t] = sh_head[tid]
            tail_key = NO_KEY
            if tid in tails:
                tail_key, acc = tails[tid]
                closed = False
                u = lane + 1
                while u < WAVE:
                    assert sh_kind[wb + u] in (1, 2), "a tail is always followed by a head"
                    acc += sh_head[wb + u]
                    if sh_kind[wb + u] == 1:
                        closed = True
                        break
                    u += 1
                if closed:
                    write(tail_key, acc)
                    tail_key = NO_KEY
                else:
                    part[2 * t + 1] = acc
            if t * L < total:
                meta[2 * t] = sh_kind[tid]
                meta[2 * t + 1] = tail_key
    # k_msm_bucket_fix28
    fix_threads = 0
    for t in range(nch):
        key = meta[2 * t + 1]
        if key == NO_KEY:
            continue
        fix_threads += 1
        acc = part[2 * t + 1]
        u = (t | (WAVE - 1)) + 1 if in_wave else t + 1
        while u < nch:
            acc += part[2 * u]
            if meta[2 * u] == 1:
                break
            u += 1
        write(key, acc)
    return buckets, writes, fix_threads, nch


@pytest.mark.parametrize("in_wave", [False, True])
@pytest.mark.parametrize("mean,L,nkeys", [(1, 8, 5000), (8, 8, 4000), (8, 4, 4000), (64, 8, 600), (64, 32, 3000),
                                          (0.3, 8, 20000), (700, 4, 40), (3000, 8, 20)])
def test_every_bucket_written_once_with_its_sum(mean, L, nkeys, in_wave):
    rng = np.random.default_rng(int(mean * 10) + L + nkeys)
    counts = rng.poisson(mean, nkeys)
    counts[rng.integers(0, nkeys, max(1, nkeys // 50))] = 0  # empty keys
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    lst = rng.integers(1, 1 << 40, int(off[-1])).tolist()
    buckets, writes, fix_threads, nch = bucket_pass(off, lst, L, in_wave)
    for k in range(nkeys):
        if counts[k]:
            assert writes.get(k) == 1, "key %d written %s times" % (k, writes.get(k))
            assert buckets[k] == sum(lst[off[k]:off[k + 1]])
        else:
            assert k not in writes
    if in_wave:  # only keys running past a wave's last lane reach the fix-up pass: at most one per wave
        assert fix_threads <= (nch + WAVE - 1) // WAVE


def test_empty_list():
    buckets, writes, fix_threads, nch = bucket_pass(np.zeros(5, np.int64), [], 8)
    assert not buckets and fix_threads == 0 and nch == 0
