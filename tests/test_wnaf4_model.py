"""Model (CPU, test infrastructure) of the width-4 NAF recoding of the tbls Lagrange coefficients (drand_amd/csrc/fr.hpp
fr_wnaf4, written by k_select_lagrange and decoded by k_recover.hip lagrange_wnaf28)."""
import random


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


def reg4_nibbles(w):
    """fr.hpp fr_reg4: 64 odd nonzero signed 4-bit window digits of 0 < w < r (an even w recoded as r - w, negated)"""
    R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
    flip = w % 2 == 0
    k = R - w if flip else w
    out = []
    for i in range(64):
        if i < 63:
            d = (k & 31) - 16
            k = (k - d) >> 4
        else:
            d = k
        if flip:
            d = -d
        out.append(((abs(d) - 1) // 2) | (8 if d < 0 else 0))
    return out


def test_reg4_digits():
    """The regular recoding k_lagrange's divergent waves use: every digit odd and nonzero with |d| <= 15 (table P .. 15P),
    sum d_i 16^i == lambda mod r (== lambda, or -(r - lambda) for an even lambda), for lambda < r."""
    R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
    rng = random.Random(12)
    for lam in [1, 2, 3, 15, 16, 17, 255, 256, R - 1, R - 2, (1 << 254) + 3, (1 << 254)] + \
            [rng.randrange(1, R) for _ in range(3000)]:
        nib = reg4_nibbles(lam)
        total = 0
        for i, v in enumerate(nib):
            mag = 2 * (v & 7) + 1
            assert 1 <= mag <= 15
            total += (-mag if v & 8 else mag) * 16 ** i
        assert total % R == lam, lam


def test_short_signed_wnaf4_of_first_subset():
    """k_lambda (k_recover.hip) recodes the shorter of lambda and r - lambda (fr.hpp fr_short) and negates the digits of
    the latter: the sum is lambda mod r, and for the first t signers (lambda_k = +-C(t, k) mod r, x = 1 .. t) every
    coefficient's width-4 NAF ends below bit 32, so k_lagrange's chain skips the doublings above it."""
    from math import comb
    R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
    t = 33
    for k in range(1, t + 1):
        num = den = 1
        for m in range(1, t + 1):
            if m != k:
                num = num * m % R
                den = den * (m - k) % R
        lam = num * pow(den, R - 2, R) % R
        assert lam in (comb(t, k), R - comb(t, k))
        flip = R - lam < lam
        nib = wnaf4_nibbles(R - lam if flip else lam)
        if flip:
            nib = [v ^ 8 if v else 0 for v in nib]
        total = sum((-(2 * (v & 7) - 1) if v & 8 else 2 * (v & 7) - 1) << b for b, v in enumerate(nib) if v)
        assert total % R == lam
        assert max(b for b, v in enumerate(nib) if v) < 32
