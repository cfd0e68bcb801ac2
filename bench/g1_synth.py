"""Synthetic G1 signature corruptions for the quicknet / g1-legacy workloads (SURVEY.md §8d Cfg5 classes applied to
G1 signatures) — bench / test data only.

  (i)   sigma_k <- sigma_k + g1        a valid subgroup point, the wrong signature
  (ii)  one random bit of sigma_k flipped
  (iii) an on-curve point outside the subgroup
Plain-integer Fp arithmetic with the ZCash compressed encoding (48-byte big-endian x, flags in byte 0: 0x80
compressed, 0x40 infinity, 0x20 y lexicographically largest). Independent of oracle/ (which is reserved for checking
results) and of the library (whose kernels are what the workload measures).
"""
P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
HALF = (P - 1) // 2
G1 = (0x17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb,
      0x08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1)


def _sqrt(a):
    r = pow(a, (P + 1) // 4, P)
    return r if r * r % P == a % P else None


def compress(pt):
    x, y = pt
    b = bytearray(x.to_bytes(48, "big"))
    b[0] |= 0x80 | (0x20 if y > HALF else 0)
    return bytes(b)


def decompress(b):
    """Compressed G1 point -> affine (x, y) (no subgroup check); ValueError when not on E1."""
    if len(b) != 48 or not b[0] & 0x80 or b[0] & 0x40:
        raise ValueError("not a compressed finite G1 point")
    x = int.from_bytes(bytes([b[0] & 0x1f]) + b[1:], "big")
    if x >= P:
        raise ValueError("x >= p")
    y = _sqrt((x * x * x + 4) % P)
    if y is None:
        raise ValueError("not on E1")
    if (y > HALF) != bool(b[0] & 0x20):
        y = P - y
    return (x, y)


def add(p, q):
    """Affine addition of finite points with distinct x."""
    lam = (q[1] - p[1]) * pow(q[0] - p[0], P - 2, P) % P
    x3 = (lam * lam - p[0] - q[0]) % P
    return (x3, (lam * (p[0] - x3) - p[1]) % P)


def plus_generator(sig):
    """class (i): the compressed encoding of sigma + g1."""
    return compress(add(decompress(sig), G1))


def off_subgroup(rng):
    """class (iii): a random point of E1(Fp), compressed. The G1 cofactor is ~2^126, so a random point lies in the
    order-r subgroup with probability ~2^-126 (the verifier's subgroup check is what rejects it)."""
    while True:
        x = rng.randrange(P)
        y = _sqrt((x * x * x + 4) % P)
        if y is not None:
            return compress((x, y))


def flip_bit(sig, rng):
    """class (ii): one random bit flipped."""
    b = bytearray(sig)
    k = rng.randrange(len(b) * 8)
    b[k // 8] ^= 1 << (k % 8)
    return bytes(b)


def corrupt(sigs, bad, rng):
    """The three classes round-robin over rows `bad` of a (n, 48) uint8 array, in place (as chainsynth.corrupt)."""
    import numpy as np
    for k, i in enumerate(bad):
        c = k % 3
        if c == 0:
            sigs[i] = np.frombuffer(plus_generator(sigs[i].tobytes()), np.uint8)
        elif c == 1:
            sigs[i] = np.frombuffer(flip_bit(sigs[i].tobytes(), rng), np.uint8)
        else:
            sigs[i] = np.frombuffer(off_subgroup(rng), np.uint8)
