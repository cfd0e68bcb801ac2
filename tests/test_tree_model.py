"""Models (CPU, test infrastructure) of the bisection-from-scaled-points kernels in drand_amd/csrc/k_msm.hip:
  * naf_masks: the non-adjacent form of a scalar part k < 2^63 as two 64-bit digit masks taken from 3k (with the
    device's 64-bit wraparound and the carry into bit 64): sum (pos_i - neg_i) 2^i == k, no two adjacent nonzero
    digits, at most 64 positions;
  * the level sums: k_gsum28 (one lane per (set, group, chunk of up to L entries)) then k_rowsum28 passes (fan-in 16)
    cover every entry of every group exactly once and write row r to outA (r < ngroups) or outB, for the chunk lengths
    gsum_chunk picks, groups of any size and a short last group."""
import random

M64 = (1 << 64) - 1


def naf_masks(k):
    """k_msm.hip naf_masks, in 64-bit unsigned arithmetic"""
    k2 = (k << 1) & M64
    lo = (k + k2) & M64
    c = 1 if lo < k2 else 0
    pos = ((lo & ~k & M64) >> 1) | (c << 63)
    neg = ((~lo & M64) & k) >> 1
    return pos, neg


def test_naf_masks():
    rng = random.Random(5)
    cases = [0, 1, 2, 3, 5, 7, (1 << 31) - 1, (1 << 62) + 1, (1 << 63) - 1, 0x5555555555555555 >> 1,
             0x2AAAAAAAAAAAAAAA] + [rng.getrandbits(63) for _ in range(20000)] + [rng.getrandbits(31) for _ in range(5000)]
    for k in cases:
        pos, neg = naf_masks(k)
        assert pos & neg == 0
        assert sum(((pos >> i) & 1) * (1 << i) - ((neg >> i) & 1) * (1 << i) for i in range(64)) == k, k
        nz = pos | neg
        assert nz & (nz >> 1) == 0, k  # non-adjacent
        if k < (1 << 31):
            assert nz < (1 << 32)  # a 31-bit G2 part needs digit positions 0..31 only


def gsum_chunk(m, gsize):
    L = 2 * m // 262144
    return max(1, min(32, L, gsize))


def level_sums(m, gsize, entries):
    """k_gsum28 + k_rowsum28 over symbolic values: each 'point' is the multiset of (set, entry) it sums"""
    ngroups = (m + gsize - 1) // gsize
    L = gsum_chunk(m, gsize)
    cnt = (gsize + L - 1) // L
    rows = 2 * ngroups
    per_set = ngroups * cnt
    tmp = []
    for t in range(2 * per_set):
        s, r = divmod(t, per_set)
        g, c = divmod(r, cnt)
        g0, gend = g * gsize, min(m, g * gsize + gsize)
        a = g0 + c * L
        b = min(gend, a + L)
        tmp.append([(s, entries[e]) for e in range(a, b)] if a < b else [])
    outA, outB = [None] * ngroups, [None] * ngroups
    while True:
        fan = 16
        cnt_out = (cnt + fan - 1) // fan
        nxt = []
        for t in range(rows * cnt_out):
            r, j = divmod(t, cnt_out)
            a, b = r * cnt + j * fan, r * cnt + min(cnt, (j + 1) * fan)
            acc = sum((tmp[k] for k in range(a, b)), [])
            if cnt_out > 1:
                nxt.append(acc)
            elif r < ngroups:
                outA[r] = acc
            else:
                outB[r - ngroups] = acc
        if cnt_out == 1:
            return outA, outB
        cnt, tmp = cnt_out, nxt


def test_level_sums_cover_each_entry_once():
    rng = random.Random(9)
    for m, gsize in [(1, 2), (7, 2), (64, 64), (65, 64), (1000, 4), (1000, 1000), (40000, 40000), (300000, 1024),
                     (300001, 256), (131072, 131072), (5000, 3)]:
        entries = rng.sample(range(10 * m + 10), m)
        outA, outB = level_sums(m, gsize, entries)
        for g in range(len(outA)):
            want = entries[g * gsize:(g + 1) * gsize]
            assert sorted(outA[g]) == sorted((0, e) for e in want), (m, gsize, g)
            assert sorted(outB[g]) == sorted((1, e) for e in want), (m, gsize, g)


def wnaf4_nibbles(k):
    """fr.hpp fr_wnaf4: 256 nibbles (v in 1..4 = +(2v - 1), 9..12 = -(2(v - 8) - 1)), little-endian positions"""
    out = []
    for _ in range(256):
        v = 0
        if k & 1:
            d = k & 15
            if d >= 8:
                d -= 16
            k -= d
            v = (d + 1) // 2 if d > 0 else 8 + (1 - d) // 2
        k >>= 1
        out.append(v)
    assert k == 0
    return out


def test_wnaf4_digits():
    """The Lagrange coefficients' width-4 NAF as k_lagrange decodes it: digit (v & 7) selects table entry
    (v & 7) - 1 of {P, 3P, 5P, 7P}, bit 8 the sign; sum d_b 2^b == lambda, odd digits in [-7, 7], >= 3 zeros after
    each nonzero digit, for lambda < r."""
    R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
    rng = random.Random(11)
    for lam in [1, 7, 8, 15, 16, 255, R - 1, R - 2, (1 << 254) + 3] + [rng.randrange(R) for _ in range(3000)]:
        nib = wnaf4_nibbles(lam)
        total, last = 0, -10
        for b, v in enumerate(nib):
            if not v:
                continue
            assert v in (1, 2, 3, 4, 9, 10, 11, 12)
            mag = 2 * (v & 7) - 1
            total += (-mag if v & 8 else mag) << b
            assert b - last >= 4
            last = b
        assert total == lam
