"""CPU: the integer model of the 28-bit lazily reduced G1 subgroup test (fp28.hpp) against the oracle's r * P == O
on points in G1, random curve points, h-torsion points and G1 + torsion sums; and of the 28-bit 11-isogeny (h2c.hpp
iso11_jac) against the oracle's affine map (bls_py.iso_map_g1) on random Jacobian inputs, extreme ones included. The model asserts every bound the
kernel's formulas rely on (product outputs < 2p, limb sums in [0, 2^392)), so a bound violation fails here."""
import random

import bls_py as B
import fp28_model as M

R = M.r
H1 = 0x396c8c005555e1568c00aaab0000aaab  # G1 cofactor (u - 1)^2 / 3


def _curve_point(rng):
    while True:
        x = rng.randrange(M.p)
        y = B.fsqrt((x ** 3 + 4) % M.p)
        if y is not None:
            return (x, y)


def _cases():
    rng = random.Random(7)
    g = B.G1_GEN
    out = [B.ec_mul(B.FP, g, rng.randrange(1, R)) for _ in range(2)]
    out += [_curve_point(rng) for _ in range(2)]
    q = B.ec_mul(B.FP, _curve_point(rng), R)  # h-torsion
    out.append(q)
    out.append(B.ec_mul(B.FP, q, H1 // 3))     # order 3
    out.append(B.ec_add(B.FP, B.ec_mul(B.FP, g, rng.randrange(1, R)), q))
    return [p for p in out if p is not None]


def test_fp28_subgroup_model_matches_oracle():
    for pt in _cases():
        want = B.ec_mul(B.FP, pt, R) is None
        assert M.insub(pt[0], pt[1], M.BETA) == want


def test_fp28_isogeny_model_matches_oracle():
    rng = random.Random(11)
    p, Rm = M.p, M.R % M.p
    mont32 = lambda v: v * Rm % p
    norm = lambda v: v * pow(Rm, -1, p) % p
    cases = [(rng.randrange(p), rng.randrange(p), rng.randrange(1, p)) for _ in range(6)]
    cases += [(p - 1, p - 1, p - 1), (1, 1, 1), (p - 1, 0, 1)]
    for x, y, z in cases:  # affine (x, y) as the Jacobian (x z^2, y z^3, z)
        X, Y, Z = mont32(x * z * z % p), mont32(y * z ** 3 % p), mont32(z)
        Xo, Yo, Zo = M.iso11(X, Y, Z, B.ISO11_XNUM, B.ISO11_XDEN, B.ISO11_YNUM, B.ISO11_YDEN)
        want = B.iso_map_g1((x, y))
        if want is None:
            assert Zo == 0
            continue
        zi = pow(norm(Zo), -1, p)
        assert (norm(Xo) * zi * zi % p, norm(Yo) * zi ** 3 % p) == want
