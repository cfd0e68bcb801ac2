"""Integer model of the lazily reduced 28-bit Fp2 / G2 arithmetic (drand_amd/csrc/fp2_28.hpp), for
tests/test_fp2_28_model.py. Test infrastructure only.

Every Fp element is the integer the device holds (14 normalised 28-bit limbs, Montgomery radix R' = 2^392): mont()
and lin() come from fp28_model (they assert the < 2p product bound and the [0, 2^392) sum range); red() is
f28_red, the cheap partial reduction (top three limbs as a double, q = floor(top * 2^308 / p * (1 - 2^-40)),
a - q p) and asserts its < 2p output. The Fp2 product is Karatsuba, the squaring the complex method, each
component's bound (in units of p) is what the device formulas rely on: point coordinates X, Y < 3 (reduced after
every formula) and Z < 12, affine inputs < 3. The point formulas follow fp2_28.hpp line by line.
"""
import fp28_model as M

p = M.p
RP = M.RP
mont, lin, lin3 = M.mont, M.lin, M.lin3
ONE = M.ONE
C308 = float(2 ** 308) / float(p) * (1.0 - 2.0 ** -40)


def red(a):
    assert 0 <= a < RP
    l13, l12, l11 = (a >> (28 * 13)) & 0xFFFFFFF, (a >> (28 * 12)) & 0xFFFFFFF, (a >> (28 * 11)) & 0xFFFFFFF
    hi = (float(l13) * 268435456.0 + float(l12)) * 268435456.0 + float(l11)  # the device's fma order
    q = int(hi * C308)
    r = a - q * p
    assert 0 <= r < 2 * p, r / p
    return r


# ---- Fp2: pairs (c0, c1)
def add2(a, b):
    return (lin(0, a[0], 1, b[0], 1), lin(0, a[1], 1, b[1], 1))


def lin2(K0, K1, a, ca, b, cb):
    return (lin(K0, a[0], ca, b[0], cb), lin(K1, a[1], ca, b[1], cb))


def lin32(K0, K1, a, ca, b, cb, c, cc):
    return (lin3(K0, a[0], ca, b[0], cb, c[0], cc), lin3(K1, a[1], ca, b[1], cb, c[1], cc))


def scale2(a, c):
    return (lin(0, a[0], c, a[0], 0), lin(0, a[1], c, a[1], 0))


def red2(a):
    return (red(a[0]), red(a[1]))


def m2(a, b):
    """Karatsuba: (a0 b0 - a1 b1 + 2p, (a0 + a1)(b0 + b1) - a0 b0 - a1 b1 + 4p): components < (4, 6)"""
    t0 = mont(a[0], b[0])
    t1 = mont(a[1], b[1])
    t2 = mont(lin(0, a[0], 1, a[1], 1), lin(0, b[0], 1, b[1], 1))
    return (lin(2, t0, 1, t1, -1), lin3(4, t2, 1, t0, -1, t1, -1))


KP_AVAILABLE = (2, 3, 4, 6, 7, 8, 9, 12, 16, 18, 21, 24, 26, 32, 48)  # fp28.hpp DH_KP constants


def kp_above(K):
    """fp28.hpp kp_above: the smallest K' > K with a K' p constant"""
    return min(k for k in KP_AVAILABLE if k > K)


def sub_nc(K, a, b):
    """fp28.hpp f28_sub_nc<K>: a + K p - b limb by limb with K p in a redundant form; every limb stays >= 0 when b's
    top limb is below K p's (the value is the integer a + K p - b)"""
    assert (b >> (28 * 13)) < ((K * p) >> (28 * 13)), "f28_sub_nc: b's top limb reaches K p's"
    return lin(K, a, 1, b, -1)


def s2(a, K):
    """complex squaring ((a0 + a1)(a0 - a1 + K' p), 2 a0 a1), K >= a1's bound: components < (2, 4). Modelled in
    the NC form (f2_sqr<K, true>: both product operands unnormalised, f28_add_nc / f28_sub_nc with K' = kp_above(K)),
    whose product bound is the larger one; the plain form (K' = K, carries propagated) is bounded by it."""
    assert a[1] < K * p, "f2_sqr<K>: a1 above K p"
    t0 = mont(lin(0, a[0], 1, a[1], 1), sub_nc(kp_above(K), a[0], a[1]))
    t1 = mont(a[0], a[1])
    return (t0, lin(0, t1, 2, t1, 0))


def neg2(a, K=3):
    return (lin(K, a[0], -1, a[0], 0), lin(K, a[1], -1, a[1], 0))


def zero2(a):
    return M.zero(a[0]) and M.zero(a[1])


ONE2 = (ONE, 0)
ZERO2 = (0, 0)


def from_f2(x):
    """a normal Fp2 element (c0, c1) -> the device's 28-bit form (c R' mod p, < 2p), as f28_from_fp per component"""
    return (M.from_fp(x[0]), M.from_fp(x[1]))


def to_f2(a):
    f = lambda v: v * pow(RP, -1, p) % p  # noqa: E731
    return (f(a[0]), f(a[1]))


# ---- G2 Jacobian points (X, Y, Z, inf): X, Y < 3, Z < 12 per component
def inf():
    return (ONE2, ONE2, ZERO2, True)


def dbl(P):
    X, Y, Z, fl = P
    A = s2(X, 3)
    B = s2(Y, 3)
    C = s2(B, 4)
    T = s2(add2(X, B), 7)
    D = lin32(8, 16, T, 2, A, -2, C, -2)          # (12, 24)
    E = scale2(A, 3)                              # (6, 12)
    F = s2(E, 12)
    X3 = red2(lin2(24, 48, F, 1, D, -2))          # (26, 52) -> < 2
    m = m2(E, lin2(3, 3, D, 1, X3, -1))           # E < 12, D - X3 + 3p < 27
    Y3 = red2(lin2(16, 32, m, 1, C, -8))          # (20, 38) -> < 2
    Z3 = scale2(m2(Y, Z), 2)                      # (8, 12)
    return (X3, Y3, Z3, fl)


def madd_core(P, qx, qy, exact):
    X, Y, Z, fl = P
    if fl:
        return (qx, qy, ONE2, False)
    z1z1 = s2(Z, 12)
    u2 = m2(qx, z1z1)
    s2_ = m2(m2(qy, Z), z1z1)
    h = lin2(3, 3, u2, 1, X, -1)                  # (7, 9)
    rr = lin2(3, 3, s2_, 1, Y, -1)                # (7, 9)
    if exact and zero2(h):
        return dbl(P) if zero2(rr) else inf()
    hh = s2(h, 9)
    i = scale2(hh, 4)                             # (8, 16)
    j = m2(h, i)
    r2 = scale2(rr, 2)                            # (14, 18)
    v = m2(X, i)
    X3 = red2(lin32(12, 18, s2(r2, 18), 1, j, -1, v, -2))   # (14, 22) -> < 2
    m = m2(r2, lin2(3, 3, v, 1, X3, -1))          # r2 < 18, v - X3 + 3p < 9
    Y3 = red2(lin2(8, 12, m, 1, m2(Y, j), -2))    # (12, 18) -> < 2
    Z3 = lin32(4, 8, s2(add2(Z, h), 21), 1, z1z1, -1, hh, -1)  # Z + h < 21 -> (6, 12)
    return (X3, Y3, Z3, False)


def add_core(P, Q, exact):
    X1, Y1, Z1, f1 = P
    X2, Y2, Z2, f2 = Q
    if f1:
        return Q
    if f2:
        return P
    z1z1 = s2(Z1, 12)
    z2z2 = s2(Z2, 12)
    u1 = m2(X1, z2z2)
    u2 = m2(X2, z1z1)
    s1 = m2(m2(Y1, Z2), z2z2)
    s2_ = m2(m2(Y2, Z1), z1z1)
    h = lin2(4, 6, u2, 1, u1, -1)                 # (8, 12)
    rr = lin2(4, 6, s2_, 1, s1, -1)               # (8, 12)
    if exact and zero2(h):
        return dbl(P) if zero2(rr) else inf()
    i = s2(scale2(h, 2), 24)                      # 2h < 24
    j = m2(h, i)
    r2 = scale2(rr, 2)                            # (16, 24)
    v = m2(u1, i)
    X3 = red2(lin32(12, 18, s2(r2, 24), 1, j, -1, v, -2))   # (14, 22) -> < 2
    m = m2(r2, lin2(3, 3, v, 1, X3, -1))          # r2 < 24, < 9
    Y3 = red2(lin2(8, 12, m, 1, m2(s1, j), -2))   # (12, 18) -> < 2
    zz = lin32(4, 8, s2(add2(Z1, Z2), 24), 1, z1z1, -1, z2z2, -1)  # Z1 + Z2 < 24 -> (6, 12)
    Z3 = m2(zz, h)                                # (4, 6)
    return (X3, Y3, Z3, False)


def madd(P, qx, qy):
    return madd_core(P, qx, qy, True)


def madd_fast(P, qx, qy):
    return madd_core(P, qx, qy, False)


def jadd(P, Q):
    return add_core(P, Q, True)


def jadd_fast(P, Q):
    return add_core(P, Q, False)


def poisoned(P):
    return (not P[3]) and zero2(P[2])


def to_affine(P):
    import bls_py as B
    X, Y, Z, fl = P
    if fl:
        return None
    x, y, z = to_f2(X), to_f2(Y), to_f2(Z)
    zi = B.f2inv(z)
    zi2 = B.f2mul(zi, zi)
    return (B.f2mul(x, zi2), B.f2mul(y, B.f2mul(zi2, zi)))


# ---- psi and the G2 subgroup test (fp2_28.hpp g2_in_subgroup28): psi(P) == [u] P = -[|u|] P
def _psi_consts():
    import bls_py as B
    xi = (1, 1)
    return B.f2inv(B.f2pow(xi, (p - 1) // 3)), B.f2inv(B.f2pow(xi, (p - 1) // 2))


def conj2(a, K=2):
    return (a[0], lin(K, a[1], -1, a[1], 0))


def in_subgroup(pt):
    cx, cy = _psi_consts()
    x, y = from_f2(pt[0]), from_f2(pt[1])
    acc = (x, y, ONE2, False)
    for b in range(62, -1, -1):
        acc = dbl(acc)
        if (M.U >> b) & 1:
            acc = madd(acc, x, y)
    X, Y, Z, fl = acc
    if fl:
        return False
    px = m2(conj2(x), from_f2(cx))                 # psi(P).x < (4, 6)
    py = m2(conj2(y), from_f2(cy))
    z2 = s2(Z, 12)
    z3 = m2(z2, Z)
    if not zero2(lin2(3, 3, m2(px, z2), 1, X, -1)):  # psi(P).x Z^2 == X
        return False
    return zero2(add2(m2(py, z3), Y))               # psi(P).y Z^3 == -Y


# ---- cofactor clearing [h_eff] P (fp2_28.hpp g2_clear28, RFC 9380 G.3 as h2c.hpp h2c_clear_g2)
def _psi2_consts():
    import bls_py as B
    xi = (1, 1)
    cx = B.f2inv(B.f2pow(xi, (p * p - 1) // 3))
    cy = B.f2inv(B.f2pow(xi, (p * p - 1) // 2))
    assert cx[1] == 0 and cy[1] == 0
    return cx[0], cy[0]


def jneg(P):
    X, Y, Z, fl = P
    return (X, (lin(3, Y[0], -1, Y[0], 0), lin(3, Y[1], -1, Y[1], 0)), Z, fl)


def psi_jac(P):
    cx, cy = _psi_consts()
    X, Y, Z, fl = P
    return (red2(m2(conj2(X), from_f2(cx))), red2(m2(conj2(Y), from_f2(cy))), (Z[0], lin(12, Z[1], -1, Z[1], 0)), fl)


def psi2_jac(P):
    cx, cy = _psi2_consts()
    X, Y, Z, fl = P
    fx, fy = M.from_fp(cx), M.from_fp(cy)
    return ((mont(X[0], fx), mont(X[1], fx)), (mont(Y[0], fy), mont(Y[1], fy)), Z, fl)


def mul_uabs(P):
    acc = P
    for b in range(62, -1, -1):
        acc = dbl(acc)
        if (M.U >> b) & 1:
            acc = jadd(acc, P)
    return acc


def clear(P):
    t1 = jneg(mul_uabs(P))
    t2 = psi_jac(P)
    t3 = psi2_jac(dbl(P))
    t3 = jadd(t3, jneg(t2))
    t2 = jadd(t1, t2)
    t2 = jneg(mul_uabs(t2))
    t3 = jadd(t3, t2)
    t3 = jadd(t3, jneg(t1))
    return jadd(t3, jneg(P))


def coz_table(px, py, ne):
    """k_recover.hip k_wnaf_table_g2 on the model: the odd multiples P, 3P, ..., (2 ne - 1) P of an affine P by DBLU and
    ZADDU co-Z steps, line by line as on the device. Returns the entries as Jacobian triples (entry 0 affine, Z = 1)
    and the factors d_j (Z_j = Z_{j-1} d_j), so the walk back from 1 / Z_last can be checked too."""
    B = red2(s2(py, 2))
    S = red2(scale2(red2(m2(px, B)), 4))
    Mv = scale2(red2(s2(px, 2)), 3)                                        # < 6
    tx = red2(lin2(4, 4, s2(Mv, 6), 1, S, -2))
    e8 = red2(scale2(red2(s2(B, 2)), 8))
    ty = red2(lin2(2, 2, m2(Mv, lin2(2, 2, S, 1, tx, -1)), 1, e8, -1))
    zl = red2(scale2(py, 2))
    rx, ry = S, e8
    entries, ds = [(px, py, ONE2)], []
    for _ in range(1, ne):
        d = lin2(2, 2, tx, 1, rx, -1)                                      # < 4
        C = red2(s2(d, 4))
        w1, w2 = red2(m2(tx, C)), red2(m2(rx, C))
        ee = lin2(2, 2, ty, 1, ry, -1)                                     # < 4
        a1 = red2(m2(ty, lin2(2, 2, w1, 1, w2, -1)))
        rx = red2(lin32(4, 4, s2(ee, 4), 1, w1, -1, w2, -1))
        ry = red2(lin2(2, 2, m2(ee, lin2(2, 2, w1, 1, rx, -1)), 1, a1, -1))
        tx, ty = w1, a1
        zl = red2(m2(zl, d))
        ds.append(red2(d))
        entries.append((rx, ry, zl))
    return entries, ds
