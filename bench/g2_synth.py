"""Synthetic G2 signature corruptions for the chained-replay workload — bench / test data only.

The three corruption classes of Cfg5 need a little G2 arithmetic on compressed points:
  (i)   sigma_k <- sigma_k + g2        a valid subgroup point, the wrong signature
  (ii)  one random bit of sigma_k flipped
  (iii) an on-curve point outside the subgroup
Plain-integer Fp / Fp2 arithmetic with the ZCash compressed encoding (x.c1 || x.c0, flags in byte 0: 0x80
compressed, 0x40 infinity, 0x20 y lexicographically largest). Independent of oracle/ (which is reserved for
checking results) and of the library (whose kernels are what the workload measures).
"""
P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
HALF = (P - 1) // 2
B2 = (4, 4)  # E2: y^2 = x^3 + 4(1 + i)
G2 = ((0x024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8,
       0x13e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e),
      (0x0ce5d527727d6e118cc9cdc6da2e351aadfd9baa8cbdd3a76d429a695160d12c923ac9cc3baca289e193548608b82801,
       0x0606c4a02ea734cc32acd2b02bc28b99cb3e287e85a763af267492ab572e99ab3f370d275cec1da1aaa9075ff05f79be))


def _add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def _sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def _mul(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def _inv(a):
    n = pow((a[0] * a[0] + a[1] * a[1]) % P, P - 2, P)
    return (a[0] * n % P, -a[1] * n % P)


def _sqrt_fp(a):
    r = pow(a, (P + 1) // 4, P)
    return r if r * r % P == a % P else None


def _sqrt(a):
    """Some square root in Fp2 (complex method, p = 3 mod 4), or None."""
    a0, a1 = a[0] % P, a[1] % P
    if a1 == 0:
        s = _sqrt_fp(a0)
        if s is not None:
            return (s, 0)
        s = _sqrt_fp(-a0 % P)
        return (0, s) if s is not None else None
    s = _sqrt_fp((a0 * a0 + a1 * a1) % P)
    if s is None:
        return None
    inv2 = (P + 1) // 2
    d = (a0 + s) * inv2 % P
    x0 = _sqrt_fp(d)
    if x0 is None:
        x0 = _sqrt_fp((a0 - s) * inv2 % P)
        if x0 is None:
            return None
    x = (x0, a1 * pow(2 * x0, P - 2, P) % P)
    return x if _mul(x, x) == (a0, a1) else None


def _rhs(x):
    return _add(_mul(_mul(x, x), x), B2)


def _largest(y):
    return y[1] > HALF or (y[1] == 0 and y[0] > HALF)


def compress(pt):
    (x0, x1), y = pt
    b = bytearray(x1.to_bytes(48, "big") + x0.to_bytes(48, "big"))
    b[0] |= 0x80 | (0x20 if _largest(y) else 0)
    return bytes(b)


def decompress(b):
    """Compressed G2 point -> affine (x, y) (no subgroup check); ValueError when not on E2."""
    if len(b) != 96 or not b[0] & 0x80 or b[0] & 0x40:
        raise ValueError("not a compressed finite G2 point")
    x1 = int.from_bytes(bytes([b[0] & 0x1f]) + b[1:48], "big")
    x0 = int.from_bytes(b[48:], "big")
    if x0 >= P or x1 >= P:
        raise ValueError("coordinate >= p")
    x = (x0, x1)
    y = _sqrt(_rhs(x))
    if y is None:
        raise ValueError("not on E2")
    if _largest(y) != bool(b[0] & 0x20):
        y = ((-y[0]) % P, (-y[1]) % P)
    return (x, y)


def add(p, q):
    """Affine addition of distinct finite points with distinct x."""
    lam = _mul(_sub(q[1], p[1]), _inv(_sub(q[0], p[0])))
    x3 = _sub(_sub(_mul(lam, lam), p[0]), q[0])
    return (x3, _sub(_mul(lam, _sub(p[0], x3)), p[1]))


def plus_generator(sig):
    """class (i): the compressed encoding of sigma + g2 (a subgroup point that is not the signature)."""
    return compress(add(decompress(sig), G2))


def off_subgroup(rng):
    """class (iii): a random point of E2(Fp2), compressed. E2 has cofactor h2 ~ 2^509, so a random point lies in
    the order-r subgroup with probability ~2^-509 (the verifier's subgroup check is what rejects it)."""
    while True:
        x = (rng.randrange(P), rng.randrange(P))
        y = _sqrt(_rhs(x))
        if y is not None:
            return compress((x, y))


def flip_bit(sig, rng):
    """class (ii): one random bit flipped (usually off the curve or over p; sometimes another valid point)."""
    b = bytearray(sig)
    k = rng.randrange(len(b) * 8)
    b[k // 8] ^= 1 << (k % 8)
    return bytes(b)
