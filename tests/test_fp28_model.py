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


def test_msm28_bucket_runs_match_oracle():
    """k_msm_bucket28's runs (fast formulas + one zero test of Z per run, exact recomputation when poisoned) on the
    model: random runs of G1 points and their negatives (affine and Jacobian inputs) give the oracle's sums, and the
    exceptional runs — a point added to itself, a point and its negative, a run summing to the identity — are the
    ones flagged poisoned. Every product / sum bound is asserted along the way."""
    rng = random.Random(13)
    g = B.G1_GEN
    pts = [B.ec_mul(B.FP, g, rng.randrange(1, R)) for _ in range(6)]
    enc = lambda P: (M.from_fp(P[0]), M.from_fp(P[1]))  # noqa: E731

    def jac(P):  # a random Jacobian representative (Z != 1), as the hash points arrive
        z = rng.randrange(2, M.p)
        X, Y, Z = P[0] * z * z % M.p, P[1] * z ** 3 % M.p, z
        return (M.from_fp(X), M.from_fp(Y), M.from_fp(Z))

    def oracle_sum(run):
        acc = None
        for P, neg in run:
            acc = B.ec_add(B.FP, acc, (P[0], (-P[1]) % M.p) if neg else P)
        return acc

    runs = [[(pts[k % 6], rng.random() < 0.5) for k in rng.sample(range(60), 9)] for _ in range(4)]
    exceptional = [[(pts[0], False), (pts[0], False)], [(pts[1], False), (pts[1], True), (pts[2], False)],
                   [(pts[3], False), (pts[3], True)],
                   [(pts[4], False), (pts[5], False), (B.ec_add(B.FP, pts[4], pts[5]), True)]]
    for run in runs + exceptional:
        for affine in (True, False):
            got, pois = M.bucket_run([(enc(P) if affine else jac(P), neg) for P, neg in run], affine)
            assert M.to_affine(got) == oracle_sum(run)
            if run in exceptional:
                assert pois
    # the poison persists: once Z = 0 mod p, more fast additions keep it
    acc = M.madd_fast(M.madd_fast(M.inf(), *enc(pts[0])), *enc(pts[0]))
    for P in pts[1:]:
        assert M.poisoned(acc)
        acc = M.madd_fast(acc, *enc(P))
        acc = M.jadd_fast(acc, (*jac(P), False))
        acc = M.jadd_fast((*jac(P), False), acc)
        acc = M.dbl(acc)
    assert M.poisoned(acc)
