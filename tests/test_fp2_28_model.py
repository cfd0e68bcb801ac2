"""CPU: the integer model of the lazily reduced 28-bit Fp2 / G2 arithmetic (tests/fp2_28_model.py, mirroring
drand_amd/csrc/fp2_28.hpp) against the oracle's affine G2 arithmetic (oracle/bls_py.py): Karatsuba products and
complex squarings, the partial reduction f28_red at its extremes, doubling / mixed / Jacobian additions over long
chains, the MSM bucket runs with their exceptional cases (fast formulas poison Z, exact recomputation), and the psi
subgroup test on subgroup points, random curve points and subgroup + torsion sums. Every product input and sum is
bound-checked by the model, so a formula whose bounds do not hold fails here."""
import random

import bls_py as B
import fp28_model as M1
import fp2_28_model as M

P = M.p


def rng_f2(rng):
    return (rng.randrange(P), rng.randrange(P))


def g2_point(rng, subgroup=True):
    if subgroup:
        return B.ec_mul(B.FP2, B.G2_GEN, rng.randrange(1, M1.r))
    while True:
        x = rng_f2(rng)
        y = B.f2sqrt(B.f2add(B.f2mul(B.f2mul(x, x), x), B.B2))
        if y is not None:
            return (x, y)


def enc(pt):
    return (M.from_f2(pt[0]), M.from_f2(pt[1]))


def jac(pt, rng):
    z = rng_f2(rng)
    z2 = B.f2mul(z, z)
    return (M.from_f2(B.f2mul(pt[0], z2)), M.from_f2(B.f2mul(pt[1], B.f2mul(z2, z))), M.from_f2(z), False)


def test_fp2_products_and_reduction():
    rng = random.Random(3)
    for _ in range(200):
        a, b = rng_f2(rng), rng_f2(rng)
        # inputs anywhere inside the bounds the formulas feed them (multiples of p added)
        A = (M.from_f2(a)[0] + rng.randrange(0, 2) * P, M.from_f2(a)[1] + rng.randrange(0, 4) * P)
        Bb = (M.from_f2(b)[0] + rng.randrange(0, 2) * P, M.from_f2(b)[1] + rng.randrange(0, 4) * P)
        assert M.to_f2(M.m2(A, Bb)) == B.f2mul(a, b)
        assert M.to_f2(M.s2(A, 6)) == B.f2mul(a, a)
    for v in (0, 1, P - 1, P, 2 * P - 1, 2 ** 392 - 1, 2519 * P, rng.randrange(2 ** 392)):
        assert M.red(v) % P == v % P


def test_g2_point_formulas_match_oracle():
    rng = random.Random(5)
    pts = [g2_point(rng) for _ in range(4)] + [g2_point(rng, False) for _ in range(2)]
    for pt in pts:
        q = g2_point(rng)
        # doubling chains, mixed and Jacobian additions, the bounds carried through many steps
        acc = (*enc(pt)[:2], M.ONE2, False)
        ref = pt
        for k in range(40):
            acc = M.dbl(acc)
            ref = B.ec_dbl(B.FP2, ref)
            if k % 3 == 0:
                acc = M.madd_fast(acc, *enc(q))
                ref = B.ec_add(B.FP2, ref, q)
            if k % 5 == 0:
                acc = M.jadd(acc, jac(q, rng))
                ref = B.ec_add(B.FP2, ref, q)
            if k % 7 == 0:
                acc = M.jadd_fast(jac(pt, rng), acc)
                ref = B.ec_add(B.FP2, ref, pt)
        assert M.to_affine(acc) == ref


def bucket_run(run, affine, rng):
    """k_msm_bucket28 for G2 on the model: fast formulas, Z tested once, exact recomputation when poisoned"""
    def pts():
        for pt, neg in run:
            if affine:
                x, y = enc(pt)
                yield (x, M.neg2(y) if neg else y)
            else:
                X, Y, Z, _ = jac(pt, rng)
                yield (X, M.neg2(Y) if neg else Y, Z, False)
    acc = M.inf()
    for q in pts():
        acc = M.madd_fast(acc, *q) if affine else M.jadd_fast(acc, q)
    if not M.poisoned(acc):
        return acc, False
    acc = M.inf()
    for q in pts():
        acc = M.madd(acc, *q) if affine else M.jadd(acc, q)
    return acc, True


def test_g2_msm_bucket_runs():
    rng = random.Random(9)
    p = [g2_point(rng) for _ in range(5)]

    def osum(run):
        acc = None
        for pt, neg in run:
            acc = B.ec_add(B.FP2, acc, B.ec_neg(B.FP2, pt) if neg else pt)
        return acc

    normal = [[(p[k % 5], rng.random() < 0.5) for k in rng.sample(range(30), 7)] for _ in range(3)]
    exceptional = [[(p[0], False), (p[0], False)], [(p[1], False), (p[1], True), (p[2], False)],
                   [(p[3], False), (p[4], False), (B.ec_add(B.FP2, p[3], p[4]), True)]]
    for run in normal + exceptional:
        for affine in (True, False):
            got, pois = bucket_run(run, affine, rng)
            assert M.to_affine(got) == osum(run)
            assert pois == (run in exceptional) or run in normal and not pois


def test_g2_subgroup_test_model():
    """fp2_28.hpp g2_in_subgroup28: psi(P) == -[|u|] P on the lazy form, against r P == O"""
    rng = random.Random(11)
    cases = [g2_point(rng) for _ in range(2)] + [g2_point(rng, False) for _ in range(2)]
    tors = B.ec_mul(B.FP2, g2_point(rng, False), M1.r)  # an h2-torsion point
    cases.append(B.ec_add(B.FP2, g2_point(rng), tors))
    for pt in cases:
        want = B.ec_mul(B.FP2, pt, M1.r) is None
        assert M.in_subgroup(pt) == want


def test_g2_cofactor_clearing_model():
    """fp2_28.hpp g2_clear28 (RFC 9380 G.3 on the lazy form) equals [h_eff] P for random E2 points (off G2)"""
    rng = random.Random(17)
    for _ in range(2):
        pt = g2_point(rng, False)
        got = M.to_affine(M.clear(jac(pt, rng)))
        assert got == B.ec_mul(B.FP2, pt, B.H_EFF_G2)


def test_g2_psi_split_scalars():
    """The G2 MSM's four-part scalars (k_scalars parts = 4, k_msm_prep28<c28_g2> images): with psi = [z] on G2,
    a P + b psi(P) + c psi^2(P) + d psi^3(P) = [a + b z + c z^2 + d z^3] P for signatures (in G2), and after the
    group check's cofactor clearing the same holds for the uncleared hash points ([h] commutes with psi). The images
    are formed as the prep kernel forms them (psi affine with conj and PSI_X / PSI_Y, psi^2 with the Fp constants,
    psi^3 = psi(psi^2)), and 31-bit parts give distinct scalars (|value| < r / 2)."""
    rng = random.Random(23)
    z = -M1.U  # the BLS parameter (negative)
    r = M1.r
    bound = (2 ** 31 - 1) * (1 + abs(z) + z * z + abs(z) ** 3)
    assert 2 * bound < r

    def images(pt):
        P0 = (*enc(pt), M.ONE2, False)
        P1 = M.psi_jac(P0)
        P2 = M.psi2_jac(P0)
        P3 = M.psi_jac(P2)
        return [M.to_affine(Q) for Q in (P0, P1, P2, P3)]

    for subgroup in (True, False):
        for _ in range(2):
            pt = g2_point(rng, subgroup)
            parts = [rng.randrange(2 ** 31) for _ in range(4)]
            acc = None
            for k, im in enumerate(images(pt)):
                acc = B.ec_add(B.FP2, acc, B.ec_mul(B.FP2, im, parts[k]))
            s = sum(parts[k] * z ** k for k in range(4))
            if subgroup:
                assert acc == B.ec_mul(B.FP2, pt, s % r)
            else:
                assert B.ec_mul(B.FP2, acc, B.H_EFF_G2) == B.ec_mul(B.FP2, B.ec_mul(B.FP2, pt, B.H_EFF_G2), s % r)


def test_unnormalised_product_operands():
    """fp28.hpp f28_add_nc / f28_sub_nc feed fp_mul28.hpp products with unnormalised limbs: every limb of the
    redundant K p form keeps a + K p - b >= 0 limb by limb for normalised a, b (b's top limb below K p's), and a
    product column (14 limb products of an add_nc and a sub_nc operand + 14 quotient-digit products + the carry-in)
    stays below 2^64."""
    mask = (1 << 28) - 1
    max_sub = 0
    for K in M.KP_AVAILABLE:
        kp = [((K * P) >> (28 * i)) & mask for i in range(14)]
        kp[13] = (K * P) >> (28 * 13)
        red = [kp[0] + (1 << 28)] + [kp[i] + (1 << 28) - 1 for i in range(1, 13)] + [kp[13] - 1]
        assert sum(v << (28 * i) for i, v in enumerate(red)) == K * P
        for i in range(14):
            lo = red[i] - (mask if i < 13 else kp[13] - 1)  # a_i = 0, b_i at its largest
            assert lo >= 0, (K, i)
            max_sub = max(max_sub, mask + red[i])
    max_add = 2 * mask
    column = 14 * max_add * max_sub + 14 * mask * mask + (1 << 36)
    assert max_sub < 2 ** 29.6 and column < 2 ** 63


def test_coz_odd_multiples_table():
    """k_wnaf_table_g2's co-Z chain on the model (fp2_28_model.coz_table, every product and sum bound-checked): entry j
    is (2j + 1) P for subgroup points, and 1 / Z_{j-1} = d_j / Z_j walks the last entry's inverse back over the table."""
    rng = random.Random(21)
    inv2 = lambda a: B.f2inv(a)  # noqa: E731
    for _ in range(6):
        pt = g2_point(rng)
        px, py = enc(pt)
        for ne in (4, 8):
            entries, ds = M.coz_table(px, py, ne)
            for j, (X, Y, Z) in enumerate(entries):
                assert M.to_affine((X, Y, Z, False)) == B.ec_mul(B.FP2, pt, 2 * j + 1), (ne, j)
            zi = inv2(M.to_f2(entries[-1][2]))
            for j in range(ne - 1, 0, -1):
                assert B.f2mul(zi, M.to_f2(entries[j][2])) == (1, 0)
                zi = B.f2mul(zi, M.to_f2(ds[j - 1]))
