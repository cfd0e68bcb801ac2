#!/usr/bin/env python3
"""Generate csrc/pairing_vm.hpp: the multi-pairing check as a lane-parallel straight-line Fp program.

The per-lane pairing (csrc/pairing.hpp) runs every Fp product of a pairing check one after another on one lane:
~11k products, latency-bound (48 ms per check on MI355X). The tower arithmetic is, however, wide: a Karatsuba
Fp12 product is 54 independent Fp products, a cyclotomic squaring 18, a Miller-loop doubling step 6-9 per level.
This generator traces the SAME algorithms as pairing.hpp (Fp2/Fp6/Fp12 tower over xi = 1 + i, CLN lines on the
M-twist, HHT final exponentiation with Granger-Scott squarings) on symbolic Fp values and emits:

  * phases: each phase is a set of independent Fp products (MUL), linear combinations (LIN: sums of small-integer
    multiples of earlier values), or one inversion (INV);
  * for every op, where its operands live (LDS slots) and where its result goes (slots are reused once a value is
    dead: the whole check fits in a few hundred 48-byte slots).

csrc/k_vm.hip interprets it with one wavefront per check: lane k runs op k of the current phase (one product per
lane), phases are separated by a workgroup barrier. Additions are folded into the operands of the products that
consume them (an operand is a linear combination of up to MAXT earlier values); sums stay symbolic up to MAXT_LIN
terms and are materialised by LIN ops, larger ones as a balanced tree of LIN ops (one phase per level). Slots hold
the VM's own representation (14 x 28-bit limbs, Montgomery radix 2^392: fp_mul28.hpp mont_mul), so the constants
are emitted in it.

The program is validated here by evaluating the scheduled, slot-allocated program in Python (the exact
computation the device does, in the normal rather than Montgomery domain) on points from oracle/bls_py.py:
e(P,Q)e(-P,Q) = 1, bilinearity e(aP,Q)e(-P,aQ) = 1, and e(P,Q)e(P,Q) != 1, e(P,Q) != 1.
"""
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_consts as gc  # noqa: E402

P = gc.P
U_ABS = -gc.U
MAXT = 15        # terms per product operand (two operands share one op record)
MAXT_LIN = 30    # terms per LIN op (the record's words 1..15 and 17..31: two halves, one per lane of a lane pair)
MAXC = 32767     # |coefficient| per term (16-bit signed field of a term word)
LANES = 64
RP = 1 << 392    # the VM's Montgomery radix (k_vm.hip: 14 x 28-bit limbs)


# ----------------------------------------------------------------------------------------- program builder
class Prog:
    def __init__(self):
        self.nodes = []  # dict(kind, ...)
        self.inputs = []
        self.consts = {}  # value -> node

    def _add(self, **kw):
        self.nodes.append(kw)
        return len(self.nodes) - 1

    def inp(self, name):
        n = self._add(kind="in", name=name)
        self.inputs.append(n)
        return n

    def const(self, v):
        v %= P
        if v not in self.consts:
            self.consts[v] = self._add(kind="const", value=v)
        return self.consts[v]

    def mul(self, a, b):
        return self._add(kind="mul", a=a.terms_list(), b=b.terms_list())

    def lin(self, a):
        return self._add(kind="lin", a=a.terms_list())

    def lin_terms(self, items):
        """a LIN op from a (node, coeff) list (a node may repeat)"""
        return self._add(kind="lin", a=list(items))

    def inv(self, a):
        return self._add(kind="inv", a=a.terms_list())


PROG = None


class L:
    """Linear combination of program nodes with small integer coefficients (an Fp value)."""
    __slots__ = ("t",)

    def __init__(self, t=None):
        self.t = {k: v for k, v in (t or {}).items() if v % P}

    @staticmethod
    def node(n):
        return L({n: 1})

    @staticmethod
    def zero():
        return L()

    @staticmethod
    def const(v):
        return L.node(PROG.const(v)) if v % P else L()

    def terms_list(self):
        return sorted(self.t.items())

    def _ok(self, limit):
        return len(self.t) <= limit and all(abs(c) <= MAXC for c in self.t.values())

    def _norm(self):
        """a product operand: at most MAXT terms, else one LIN op"""
        if self._ok(MAXT):
            return self
        return L.node(PROG.lin(self._split()))

    def _split(self):
        """at most MAXT_LIN terms of |c| <= MAXC; larger sums become a balanced tree of LIN ops (every chunk of a
        level is independent, so a level costs one phase)"""
        items = []
        for k, c in sorted(self.t.items()):
            while abs(c) > MAXC:  # never met by the tower code; kept for completeness
                sgn = 1 if c > 0 else -1
                items.append((k, sgn * MAXC))
                c -= sgn * MAXC
            items.append((k, c))
        merged = {}
        for k, c in items:  # a split coefficient keeps separate terms for the same node
            merged.setdefault(k, []).append(c)
        items = [(k, c) for k, cs in sorted(merged.items()) for c in cs]
        while len(items) > MAXT_LIN:
            nxt = []
            for i in range(0, len(items), MAXT_LIN):
                chunk = items[i:i + MAXT_LIN]
                if len(chunk) == 1:
                    nxt.append(chunk[0])
                else:
                    nxt.append((PROG.lin_terms(chunk), 1))
            items = nxt
        if len({k for k, _ in items}) != len(items):
            return L.node(PROG.lin_terms(items))
        return L(dict(items))

    def single(self):
        assert len(self.t) == 1 and list(self.t.values())[0] == 1
        return list(self.t)[0]

    def __add__(self, o):
        t = dict(self.t)
        for k, v in o.t.items():
            t[k] = t.get(k, 0) + v
        r = L(t)
        return r if r._ok(MAXT_LIN) else L.node(PROG.lin(r._split()))

    def __sub__(self, o):
        return self + (-o)

    def __neg__(self):
        return L({k: -v for k, v in self.t.items()})

    def dbl(self):
        return (self + self)

    def __mul__(self, o):
        if not self.t or not o.t:
            return L()
        return L.node(PROG.mul(self._norm(), o._norm()))

    def mat(self):
        """a value held in one slot (for outputs / loop-carried state)"""
        if len(self.t) == 1 and list(self.t.values())[0] == 1:
            return self
        if not self.t:
            return self
        return L.node(PROG.lin(self._split()))

    def inv(self):
        return L.node(PROG.inv(self._norm()))


# ----------------------------------------------------------------------------------------- tower (pairing.hpp)
class F2:
    def __init__(self, a, b):
        self.a, self.b = a, b

    @staticmethod
    def zero():
        return F2(L(), L())

    @staticmethod
    def const(c):
        return F2(L.const(c[0]), L.const(c[1]))

    def __add__(s, o):
        return F2(s.a + o.a, s.b + o.b)

    def __sub__(s, o):
        return F2(s.a - o.a, s.b - o.b)

    def __neg__(s):
        return F2(-s.a, -s.b)

    def dbl(s):
        return s + s

    def __mul__(s, o):
        t0, t1 = s.a * o.a, s.b * o.b
        t2 = (s.a + s.b) * (o.a + o.b)
        return F2(t0 - t1, t2 - t0 - t1)

    def sqr(s):
        # fp2_sqr: (a + b)(a - b), 2ab
        return F2((s.a + s.b) * (s.a - s.b), (s.a * s.b).dbl())

    def mul_fp(s, x):
        return F2(s.a * x, s.b * x)

    def mul_xi(s):
        return F2(s.a - s.b, s.a + s.b)

    def conj(s):
        return F2(s.a, -s.b)

    def mat(s):
        return F2(s.a.mat(), s.b.mat())

    def inv(s):
        t = (s.a * s.a + s.b * s.b).inv()
        return F2(s.a * t, -(s.b * t))


class F6:
    def __init__(self, c0, c1, c2):
        self.c0, self.c1, self.c2 = c0, c1, c2

    @staticmethod
    def zero():
        return F6(F2.zero(), F2.zero(), F2.zero())

    def __add__(s, o):
        return F6(s.c0 + o.c0, s.c1 + o.c1, s.c2 + o.c2)

    def __sub__(s, o):
        return F6(s.c0 - o.c0, s.c1 - o.c1, s.c2 - o.c2)

    def __neg__(s):
        return F6(-s.c0, -s.c1, -s.c2)

    def __mul__(a, b):
        t0, t1, t2 = a.c0 * b.c0, a.c1 * b.c1, a.c2 * b.c2
        u0 = ((a.c1 + a.c2) * (b.c1 + b.c2) - t1 - t2).mul_xi() + t0
        u1 = (a.c0 + a.c1) * (b.c0 + b.c1) - t0 - t1 + t2.mul_xi()
        u2 = (a.c0 + a.c2) * (b.c0 + b.c2) - t0 - t2 + t1
        return F6(u0, u1, u2)

    def mul_01(a, b0, b1):
        t0, t1 = a.c0 * b0, a.c1 * b1
        u0 = (a.c2 * b1).mul_xi() + t0
        u1 = (a.c0 + a.c1) * (b0 + b1) - t0 - t1
        u2 = a.c2 * b0 + t1
        return F6(u0, u1, u2)

    def mul_1(a, b1):
        return F6((a.c2 * b1).mul_xi(), a.c0 * b1, a.c1 * b1)

    def mul_v(a):
        return F6(a.c2.mul_xi(), a.c0, a.c1)

    def inv(a):
        c0 = a.c0.sqr() - (a.c1 * a.c2).mul_xi()
        c1 = a.c2.sqr().mul_xi() - a.c0 * a.c1
        c2 = a.c1.sqr() - a.c0 * a.c2
        t = ((a.c2 * c1 + a.c1 * c2).mul_xi() + a.c0 * c0).mat()
        t = t.inv()
        return F6(c0 * t, c1 * t, c2 * t)

    def frob(a, k):
        c0, c1, c2 = a.c0, a.c1, a.c2
        if k & 1:
            c0, c1, c2 = c0.conj(), c1.conj(), c2.conj()
        c1 = c1 * F2.const(FROB6_C1[k - 1])
        c2 = c2 * F2.const(FROB6_C2[k - 1])
        return F6(c0, c1, c2)

    def mat(s):
        return F6(s.c0.mat(), s.c1.mat(), s.c2.mat())


class F12:
    def __init__(self, c0, c1):
        self.c0, self.c1 = c0, c1

    @staticmethod
    def one():
        return F12(F6(F2(L.const(1), L()), F2.zero(), F2.zero()), F6.zero())

    def __mul__(a, b):
        t0, t1 = a.c0 * b.c0, a.c1 * b.c1
        s = (a.c0 + a.c1) * (b.c0 + b.c1) - t0 - t1
        return F12(t0 + t1.mul_v(), s)

    def sqr(a):
        ab = a.c0 * a.c1
        t = (a.c0 + a.c1) * (a.c0 + a.c1.mul_v())
        return F12(t - ab - ab.mul_v(), ab + ab)

    def conj(a):
        return F12(a.c0, -a.c1)

    def inv(a):
        t = a.c0 * a.c0 - (a.c1 * a.c1).mul_v()
        t = t.mat().inv()
        return F12(a.c0 * t, -(a.c1 * t))

    def frob(a, k):
        c0, c1 = a.c0.frob(k), a.c1.frob(k)
        w = F2.const(FROB12_C[k - 1])
        return F12(c0, F6(c1.c0 * w, c1.c1 * w, c1.c2 * w))

    def mul_line(f, a, b, c):
        t0 = f.c0.mul_01(a, b)
        t1 = f.c1.mul_1(c)
        s = (f.c0 + f.c1).mul_01(a, b + c) - t0 - t1
        return F12(t0 + t1.mul_v(), s)

    def cyc_sqr(a):
        def fp4_sqr(x, y):
            t0, t1 = x.sqr(), y.sqr()
            return t1.mul_xi() + t0, (x + y).sqr() - t0 - t1
        t0, t1 = fp4_sqr(a.c0.c0, a.c1.c1)
        t2, t3 = fp4_sqr(a.c1.c0, a.c0.c2)
        t4, t5 = fp4_sqr(a.c0.c1, a.c1.c2)
        r00 = (t0 - a.c0.c0).dbl() + t0
        r11 = (t1 + a.c1.c1).dbl() + t1
        t5x = t5.mul_xi()
        r10 = (t5x + a.c1.c0).dbl() + t5x
        r02 = (t4 - a.c0.c2).dbl() + t4
        r01 = (t2 - a.c0.c1).dbl() + t2
        r12 = (t3 + a.c1.c2).dbl() + t3
        return F12(F6(r00, r01, r02), F6(r10, r11, r12))

    def mat(s):
        return F12(s.c0.mat(), s.c1.mat())

    def coords(s):
        out = []
        for c6 in (s.c0, s.c1):
            for c2 in (c6.c0, c6.c1, c6.c2):
                out += [c2.a, c2.b]
        return out


def ml_dbl(T):
    X, Y, Z = T
    t0, t1 = X.sqr(), Y.sqr()
    t2 = t1.sqr()
    t3 = ((t1 + X).sqr() - t0 - t2).dbl()
    t4 = t0.dbl() + t0
    t6 = X + t4
    t5 = t4.sqr()
    zz = Z.sqr()
    nx = t5 - t3 - t3
    nz = (Z + Y).sqr() - t1 - zz
    ny = (t3 - nx) * t4 - t2.dbl().dbl().dbl()
    c1 = -((t4 * zz).dbl())
    c2 = t6.sqr() - t0 - t5 - t1.dbl().dbl()
    c0 = (nz * zz).dbl()
    return (nx.mat(), ny.mat(), nz.mat()), (c0, c1, c2)


def ml_add(T, Q):
    X, Y, Z = T
    qx, qy = Q
    zz, yy = Z.sqr(), qy.sqr()
    t0 = zz * qx
    t1 = ((qy + Z).sqr() - yy - zz) * zz
    t2 = t0 - X
    t3 = t2.sqr()
    t4 = t3.dbl().dbl()
    t5 = t4 * t2
    t6 = t1 - Y - Y
    t9 = t6 * qx
    t7 = t4 * X
    nx = t6.sqr() - t5 - t7 - t7
    nz = (Z + t2).sqr() - zz - t3
    t10 = qy + nz
    t8 = (t7 - nx) * t6
    ny = t8 - (Y * t5).dbl()
    t10 = t10.sqr() - yy - nz.sqr()
    t9 = t9.dbl() - t10
    t10 = nz.dbl()
    t1 = (-t6).dbl()
    return (nx.mat(), ny.mat(), nz.mat()), (t10, t1, t9)


def miller_loop(Ps, Qs):
    """Ps: affine (x, y), or Jacobian (X, Y, Z): then every line is scaled by Z^3, an Fp factor the final
    exponentiation removes (c2 Z^3, c1 X Z, c0 Y for c2, c1 x, c0 y), so a check needs no inversion for its G1 side."""
    ev = []
    for P in Ps:
        if len(P) == 3:
            X, Y, Z = P
            ev.append((X * Z, Y, (Z * Z) * Z))
        else:
            ev.append((P[0], P[1], None))

    def line(f, k, c0, c1, c2):
        px, py, z3 = ev[k]
        return f.mul_line(c2 if z3 is None else c2.mul_fp(z3), c1.mul_fp(px), c0.mul_fp(py))

    f = F12.one()
    T = [(Q[0], Q[1], F2(L.const(1), L())) for Q in Qs]
    started = False
    for b in range(62, -1, -1):
        if started:
            f = f.sqr()
        started = True
        for k in range(len(Ps)):
            T[k], (c0, c1, c2) = ml_dbl(T[k])
            f = line(f, k, c0, c1, c2)
        if (U_ABS >> b) & 1:
            for k in range(len(Ps)):
                T[k], (c0, c1, c2) = ml_add(T[k], Qs[k])
                f = line(f, k, c0, c1, c2)
        f = f.mat()
    return f.conj()


# The state of a cyclotomic squaring run is materialised (LIN ops) every CYC_MAT squarings and before each
# multiplication: in between, the next squaring's product operands take the unmaterialised linear combinations
# (up to MAXT terms; L._norm adds a LIN op where one would exceed it). Every squaring materialised: 746 phases for
# the final exponentiation; every third: 546 (the 2-pair check 1162 -> 950 with the critical-path schedule).
CYC_MAT = 3


def cyc_exp_u(a):
    acc = a
    it = 0
    for b in range(62, -1, -1):
        acc = acc.cyc_sqr()
        it += 1
        if it % CYC_MAT == 0 or (U_ABS >> b) & 1:
            acc = acc.mat()
        if (U_ABS >> b) & 1:
            acc = (acc * a).mat()
    return acc.mat().conj()


def final_exp(f):
    t0 = (f.conj() * f.inv()).mat()
    t0 = (t0 * t0.frob(2)).mat()
    a = (cyc_exp_u(t0) * t0.conj()).mat()
    b = (cyc_exp_u(a) * a.conj()).mat()
    c = cyc_exp_u(b).mat()
    d = (cyc_exp_u(c) * b.conj()).mat()
    e = (cyc_exp_u(d) * (t0.cyc_sqr() * t0)).mat()
    e = (e * d.frob(1)).mat()
    e = (e * c.frob(2)).mat()
    return (e * b.frob(3)).mat()


# constants (normal form, as pairs (c0, c1))
XI = (1, 1)
FROB6_C1 = [gc.f2pow(XI, (P ** k - 1) // 3) for k in (1, 2, 3)]
FROB6_C2 = [gc.f2pow(XI, 2 * (P ** k - 1) // 3) for k in (1, 2, 3)]
FROB12_C = [gc.f2pow(XI, (P ** k - 1) // 6) for k in (1, 2, 3)]


# ----------------------------------------------------------------------------------------- G2 cofactor clearing
# [h_eff] Q by the endomorphism method of RFC 9380 Appendix G.3, the same steps as fp2_28.hpp g2_clear28 (the group
# check of G2-signature schemes clears the RLC sum of the uncleared hash points): in the program its ~128 doublings
# run as ~3 product phases each on the lanes instead of on one lane (k_vm_prep_groups<fp2>, 3.9 ms per check).
# Jacobian formulas without exceptional-case tests: an exceptional case leaves Z = 0, which every later step keeps,
# so the program also outputs Z and a zero Z sends the check to the exact one-lane path (k_vm.hip k_vm_pairing_c).
PSI_X = gc.f2inv(gc.f2pow(XI, (P - 1) // 3))
PSI_Y = gc.f2inv(gc.f2pow(XI, (P - 1) // 2))
PSI2_X = gc.f2mul(gc.f2pow(PSI_X, P), PSI_X)
PSI2_Y = gc.f2mul(gc.f2pow(PSI_Y, P), PSI_Y)
assert PSI2_X[1] == 0 and PSI2_Y[1] == 0


def g2_dbl(T):
    """dbl-2009-l (a = 0)"""
    X, Y, Z = T
    A, B = X.sqr(), Y.sqr()
    C = B.sqr()
    D = ((X + B).sqr() - A - C).dbl()
    E = A.dbl() + A
    X3 = E.sqr() - D.dbl()
    Y3 = E * (D - X3) - C.dbl().dbl().dbl()
    Z3 = (Y * Z).dbl()
    return (X3, Y3, Z3)


def g2_add(T1, T2):
    """add-2007-bl, both Jacobian"""
    X1, Y1, Z1 = T1
    X2, Y2, Z2 = T2
    z1z1, z2z2 = Z1.sqr(), Z2.sqr()
    u1, u2 = X1 * z2z2, X2 * z1z1
    s1, s2 = Y1 * (Z2 * z2z2), Y2 * (Z1 * z1z1)
    h = u2 - u1
    i = h.dbl().sqr()
    j = h * i
    r = (s2 - s1).dbl()
    v = u1 * i
    X3 = r.sqr() - j - v.dbl()
    Y3 = r * (v - X3) - (s1 * j).dbl()
    Z3 = ((Z1 + Z2).sqr() - z1z1 - z2z2) * h
    return (X3, Y3, Z3)


def g2_neg(T):
    return (T[0], -T[1], T[2])


def g2_psi(T):
    return (T[0].conj() * F2.const(PSI_X), T[1].conj() * F2.const(PSI_Y), T[2].conj())


def g2_psi2(T):
    return (T[0].mul_fp(L.const(PSI2_X[0])), T[1].mul_fp(L.const(PSI2_Y[0])), T[2])


def g2_mul_uabs(T):
    """[|u|] T: the doubling runs between |u|'s set bits (fp2_28.hpp uabs_run)"""
    acc = T
    for r, k in enumerate((1, 2, 3, 9, 32, 16)):
        for _ in range(k):
            acc = g2_dbl(acc)
        if r < 5:
            acc = g2_add(acc, T)
    return acc


def g2_clear(p):
    t1 = g2_neg(g2_mul_uabs(p))
    t3 = g2_add(g2_psi2(g2_dbl(p)), g2_neg(g2_psi(p)))
    t2 = g2_neg(g2_mul_uabs(g2_add(t1, g2_psi(p))))
    return g2_add(g2_add(g2_add(t3, t2), g2_neg(t1)), g2_neg(p))


def _fp12_input(prefix):
    c = [L.node(PROG.inp("%s%d" % (prefix, i))) for i in range(12)]
    return F12(F6(F2(c[0], c[1]), F2(c[2], c[3]), F2(c[4], c[5])), F6(F2(c[6], c[7]), F2(c[8], c[9]), F2(c[10], c[11])))


def build_tag(tag):
    """Programs: NP1 / NP2 = the full check of 1 / 2 pairs; ML1 = the Miller loop of one pair (f out, for
    multi-pairings of many pairs run one workgroup per pair); MUL12 = f * g; FE = final exponentiation."""
    global PROG
    if tag == "NP2C":
        return build_np2c()
    if tag.startswith("NP") and tag.endswith("J"):
        return build(int(tag[2:-1]), jac=True)
    if tag.startswith("NP"):
        return build(int(tag[2:]))
    PROG = Prog()
    if tag == "ML1":
        px, py = L.node(PROG.inp("P0.x")), L.node(PROG.inp("P0.y"))
        qx = F2(L.node(PROG.inp("Q0.x0")), L.node(PROG.inp("Q0.x1")))
        qy = F2(L.node(PROG.inp("Q0.y0")), L.node(PROG.inp("Q0.y1")))
        r = miller_loop([(px, py)], [(qx, qy)])
    elif tag == "MUL12":
        r = _fp12_input("F") * _fp12_input("G")
    elif tag == "FE":
        r = final_exp(_fp12_input("F"))
    else:
        raise ValueError(tag)
    outs = []
    for c in r.coords():
        m = c.mat()
        if not m.t:
            raise RuntimeError("zero output coordinate")
        outs.append(m.single())
    prog = PROG
    PROG = None
    return prog, outs


def build(np_, jac=False):
    """NP1 / NP2: np_ pairs with affine P; NP1J / NP2J (jac): P Jacobian (P%d.x, .y, .z), for the G1-signature checks,
    whose G1 sides are RLC sums and hash points in Jacobian form (no inversion before the program)."""
    global PROG
    PROG = Prog()
    Ps, Qs = [], []
    for k in range(np_):
        P = tuple(L.node(PROG.inp("P%d.%s" % (k, c))) for c in ("xyz" if jac else "xy"))
        qx = F2(L.node(PROG.inp("Q%d.x0" % k)), L.node(PROG.inp("Q%d.x1" % k)))
        qy = F2(L.node(PROG.inp("Q%d.y0" % k)), L.node(PROG.inp("Q%d.y1" % k)))
        Ps.append(P)
        Qs.append((qx, qy))
    r = final_exp(miller_loop(Ps, Qs))
    outs = []
    for c in r.coords():
        m = c.mat()
        if not m.t:  # an identically zero coordinate cannot happen for a generic input
            raise RuntimeError("zero output coordinate")
        outs.append(m.single())
    prog = PROG
    PROG = None
    return prog, outs


def build_np2c():
    """The group check of a G2-signature scheme, e(P0, [h_eff] B) e(P1, Q1) == 1, with the RLC hash sum B entering
    uncleared and Jacobian (B.x0 .. B.z1): cofactor clearing, affine form (one inversion), 2-pair Miller loop, final
    exponentiation. Outputs: the 12 coordinates of the result, then Z of [h_eff] B (c0, c1)."""
    global PROG
    PROG = Prog()
    p0 = (L.node(PROG.inp("P0.x")), L.node(PROG.inp("P0.y")))
    b = tuple(F2(L.node(PROG.inp("B.%s0" % c)), L.node(PROG.inp("B.%s1" % c))) for c in "xyz")
    p1 = (L.node(PROG.inp("P1.x")), L.node(PROG.inp("P1.y")))
    q1 = (F2(L.node(PROG.inp("Q1.x0")), L.node(PROG.inp("Q1.x1"))), F2(L.node(PROG.inp("Q1.y0")), L.node(PROG.inp("Q1.y1"))))
    X, Y, Z = g2_clear(b)
    Z = Z.mat()
    zi = Z.inv()
    zi2 = zi.sqr()
    q0 = ((X * zi2).mat(), (Y * (zi2 * zi)).mat())
    r = final_exp(miller_loop([p0, p1], [q0, q1]))
    outs = []
    for c in r.coords() + [Z.a, Z.b]:
        m = c.mat()
        if not m.t:
            raise RuntimeError("zero output coordinate")
        outs.append(m.single())
    prog = PROG
    PROG = None
    return prog, outs


# ----------------------------------------------------------------------------------------- scheduling
def deps(n):
    k = n["kind"]
    if k in ("in", "const"):
        return []
    out = [s for s, _ in n["a"]]
    if k == "mul":
        out += [s for s, _ in n["b"]]
    return out


def schedule(prog, outs):
    """Critical-path list scheduling into phases of one kind (MUL: <= LANES products, LIN: <= LANES, INV: one op).
    Each step runs the kind whose ready set holds the op with the longest path to an output (its height), filled by
    height. The r02-r04 ASAP order ran every ready LIN op right after each product phase, so a chain that needed only
    products (the G2 cofactor clearing of NP2C beside the other pair's Miller loop) paid a LIN phase after each of its
    product phases: NP2C 1790 -> 1572 phases, ML1 410 -> 337, NP2 1162 -> 1150 (before CYC_MAT)."""
    nodes = prog.nodes
    # dead-code elimination from the outputs
    live = set(outs)
    for i in range(len(nodes) - 1, -1, -1):
        if i in live:
            live.update(deps(nodes[i]))
    done = {i for i, n in enumerate(nodes) if n["kind"] in ("in", "const") and i in live}
    pending = [i for i, n in enumerate(nodes) if n["kind"] not in ("in", "const") and i in live]
    users = {}
    for i in pending:
        for d in set(deps(nodes[i])):
            users.setdefault(d, []).append(i)
    height = {}
    for i in sorted(pending, reverse=True):  # users come after their operands in node order
        height[i] = 1 + max((height[u] for u in users.get(i, [])), default=0)
    ndeps = {i: len(set(d for d in deps(nodes[i]) if d not in done)) for i in pending}
    ready = {"mul": [], "lin": [], "inv": []}
    for i in pending:
        if ndeps[i] == 0:
            ready[nodes[i]["kind"]].append(i)
    phases = []
    remaining = len(pending)
    while remaining:
        best = None
        for kind in ("mul", "lin", "inv"):
            if ready[kind]:
                m = max(height[i] for i in ready[kind])
                if best is None or m > best[0]:
                    best = (m, kind)
        if best is None:
            raise RuntimeError("scheduling deadlock")
        kind = best[1]
        ready[kind].sort(key=lambda i: (-height[i], i))
        cap = 1 if kind == "inv" else LANES
        batch, ready[kind] = ready[kind][:cap], ready[kind][cap:]
        phases.append((kind, batch))
        for i in batch:
            done.add(i)
            remaining -= 1
        for i in batch:
            for u in set(users.get(i, [])):
                ndeps[u] -= 1
                if ndeps[u] == 0:
                    ready[nodes[u]["kind"]].append(u)
    return phases, live


def allocate(prog, outs, phases, live):
    """Slots: a value occupies a slot from its producing phase to its last reading phase (outputs to the end)."""
    nodes = prog.nodes
    prod = {}
    for pi, (_, batch) in enumerate(phases):
        for i in batch:
            prod[i] = pi
    last = {}
    for pi, (_, batch) in enumerate(phases):
        for i in batch:
            for d in deps(nodes[i]):
                last[d] = max(last.get(d, -1), pi)
    end = len(phases)
    for o in outs:
        last[o] = end
    slot = {}
    free = []
    nslots = 0
    # inputs and constants first (phase -1)
    pre = [i for i, n in enumerate(nodes) if n["kind"] in ("in", "const") and i in live]
    for i in pre:
        slot[i] = nslots
        nslots += 1
    frees_after = {}
    for i in pre:
        frees_after.setdefault(last.get(i, -1), []).append(slot[i])
    for s in frees_after.pop(-1, []):
        free.append(s)
    for pi, (_, batch) in enumerate(phases):
        for i in batch:
            if free:
                free.sort()
                s = free.pop(0)
            else:
                s = nslots
                nslots += 1
            slot[i] = s
            frees_after.setdefault(last.get(i, pi), []).append(s)
        # values whose last read is this phase become free for later phases
        for s in frees_after.pop(pi, []):
            free.append(s)
    return slot, nslots


# ----------------------------------------------------------------------------------------- reference evaluation
def evaluate(prog, outs, phases, slot, nslots, inputs):
    """Run the scheduled program exactly as the device does (slots, phases), normal-domain ints."""
    nodes = prog.nodes
    S = [None] * nslots
    for i, n in enumerate(nodes):
        if i in slot and n["kind"] == "in":
            S[slot[i]] = inputs[n["name"]] % P
        elif i in slot and n["kind"] == "const":
            S[slot[i]] = n["value"]

    def lin(terms):
        return sum(c * S[slot[s]] for s, c in terms) % P

    for kind, batch in phases:
        res = []
        for i in batch:
            n = nodes[i]
            if kind == "mul":
                res.append(lin(n["a"]) * lin(n["b"]) % P)
            elif kind == "lin":
                res.append(lin(n["a"]))
            else:
                res.append(pow(lin(n["a"]), P - 2, P))
        for i, v in zip(batch, res):  # all reads of a phase happen before its writes
            S[slot[i]] = v
    return [S[slot[o]] for o in outs]


def _bls_points():
    sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
    import bls_py as B
    return B


def validate_split(progs):
    """ML1 / MUL12 / FE composed must give the NP2 check: e(G1,G2) e(-G1,G2) = 1 and e(aP,Q) e(-P,aQ) = 1."""
    B = _bls_points()
    one = [1] + [0] * 11
    run = {}
    for tag, prog, outs, phases, slot, nslots in progs:
        run[tag] = (lambda p=prog, o=outs, ph=phases, sl=slot, ns=nslots: (lambda inp: evaluate(p, o, ph, sl, ns, inp)))()

    def ml(Pt, Qt):
        return run["ML1"]({"P0.x": Pt[0], "P0.y": Pt[1], "Q0.x0": Qt[0][0], "Q0.x1": Qt[0][1],
                           "Q0.y0": Qt[1][0], "Q0.y1": Qt[1][1]})

    def mul(f, g):
        d = {"F%d" % i: f[i] for i in range(12)}
        d.update({"G%d" % i: g[i] for i in range(12)})
        return run["MUL12"](d)

    def fe(f):
        return run["FE"]({"F%d" % i: f[i] for i in range(12)})

    G1, G2 = B.G1_GEN, B.G2_GEN
    a = random.Random(2).randrange(2, 1 << 64)
    Pa, Qa = B.ec_mul(B.FP, G1, a), B.ec_mul(B.FP2, G2, a)
    negG1 = B.ec_neg(B.FP, G1)
    assert fe(mul(ml(G1, G2), ml(negG1, G2))) == one
    assert fe(mul(mul(ml(Pa, G2), ml(negG1, Qa)), ml(G1, G2))) != one
    assert fe(mul(mul(ml(Pa, G2), ml(negG1, Qa)), mul(ml(G1, G2), ml(negG1, G2)))) == one


def validate_np2c(prog, outs, phases, slot, nslots):
    """e(pk, [h_eff] B) e(-G1, [sk][h_eff] B) = 1 for an uncleared B given in Jacobian form with a random Z, != 1
    for a wrong signature sum; the Z output is that of [h_eff] B (nonzero)."""
    B = _bls_points()
    rng = random.Random(3)
    h = B.iso_map_g2(B.sswu_g2((rng.randrange(P), rng.randrange(P))))
    assert B.g2_on_curve(h)
    hh = B.ec_mul(B.FP2, h, B.H_EFF_G2)
    sk = rng.randrange(2, B.R)
    pk = B.ec_mul(B.FP, B.G1_GEN, sk)
    sig = B.ec_mul(B.FP2, hh, sk)
    ng1 = B.ec_neg(B.FP, B.G1_GEN)
    z = (rng.randrange(1, P), rng.randrange(P))
    z2 = B.f2mul(z, z)
    jx, jy = B.f2mul(h[0], z2), B.f2mul(h[1], B.f2mul(z2, z))

    def run(q1):
        inp = {"P0.x": pk[0], "P0.y": pk[1], "B.x0": jx[0], "B.x1": jx[1], "B.y0": jy[0], "B.y1": jy[1],
               "B.z0": z[0], "B.z1": z[1], "P1.x": ng1[0], "P1.y": ng1[1],
               "Q1.x0": q1[0][0], "Q1.x1": q1[0][1], "Q1.y0": q1[1][0], "Q1.y1": q1[1][1]}
        return evaluate(prog, outs, phases, slot, nslots, inp)

    one = [1] + [0] * 11
    res = run(sig)
    assert res[:12] == one, "NP2C: e(pk, [h]B) e(-G1, sk [h]B) != 1"
    assert res[12:] != [0, 0]
    assert run(B.ec_add(B.FP2, sig, B.G2_GEN))[:12] != one, "NP2C accepted a wrong signature sum"


def validate(np_, prog, outs, phases, slot, nslots):
    if np_ == "NP2C":
        return validate_np2c(prog, outs, phases, slot, nslots)
    jac = False
    if isinstance(np_, str):
        if not np_.startswith("NP"):
            return  # checked in validate_split
        jac = np_.endswith("J")
        np_ = int(np_[2:].rstrip("J"))
    B = _bls_points()
    rng = random.Random(1)
    one = [1] + [0] * 11

    def run(pairs):
        inp = {}
        for k, (Pt, Qt) in enumerate(pairs):
            if jac:  # the same point with a random Z: X = x Z^2, Y = y Z^3
                z = rng.randrange(1, P)
                inp["P%d.x" % k], inp["P%d.y" % k], inp["P%d.z" % k] = Pt[0] * z * z % P, Pt[1] * z * z * z % P, z
                inp["Q%d.x0" % k], inp["Q%d.x1" % k] = Qt[0]
                inp["Q%d.y0" % k], inp["Q%d.y1" % k] = Qt[1]
                continue
            inp["P%d.x" % k], inp["P%d.y" % k] = Pt[0], Pt[1]
            inp["Q%d.x0" % k], inp["Q%d.x1" % k] = Qt[0]
            inp["Q%d.y0" % k], inp["Q%d.y1" % k] = Qt[1]
        return evaluate(prog, outs, phases, slot, nslots, inp)

    G1, G2 = B.G1_GEN, B.G2_GEN
    a = rng.randrange(2, 1 << 64)
    Pa = B.ec_mul(B.FP, G1, a)
    Qa = B.ec_mul(B.FP2, G2, a)
    negG1 = B.ec_neg(B.FP, G1)
    if np_ == 2:
        assert run([(G1, G2), (negG1, G2)]) == one, "e(P,Q) e(-P,Q) != 1"
        assert run([(Pa, G2), (negG1, Qa)]) == one, "bilinearity"
        assert run([(G1, G2), (G1, G2)]) != one
        assert run([(Pa, G2), (negG1, G2)]) != one
    else:
        assert run([(G1, G2)]) != one
        # e(P, Q)^r = 1 is not directly testable here; bilinearity via two single pairings:
        x, y = run([(Pa, G2)]), run([(G1, Qa)])
        assert x == y, "bilinearity (single)"


# ----------------------------------------------------------------------------------------- emission
REC = 32  # words per op record: header, MAXT A terms, half header, MAXT B terms (LIN: its terms in the two halves)


def c_fp28(v):
    """an Fp constant in the VM's representation: v R' mod p as 14 x 28-bit limbs"""
    m = v * RP % P
    return "{" + ", ".join("0x%07xu" % ((m >> (28 * i)) & 0xfffffff) for i in range(14)) + "}"


def emit(progs):
    """progs: list of (np, prog, outs, phases, slot, nslots).

    Layout read by k_vm.hip: PHASES[2 * ph] = kind | cnt << 8, PHASES[2 * ph + 1] = index of the phase's first op;
    op k of phase ph is the REC-word record OPS[REC * (first + k) ...] in two 16-word halves: word 0 = dst slot |
    na << 16 | nb << 24, words 1..na = the first half's terms; word 16 = nb << 16, words 17..16+nb = the second half's
    terms. A product's halves are its operands A and B, a LIN op's the first MAXT of its terms and the rest; a term =
    slot | (coeff & 0xffff) << 16. k_vm.hip runs a phase of at most 32 ops on lane pairs, each lane reading one half
    (its count at bits 16..23 of the half's first word), and a wider phase one op per lane over both halves.
    Constants are emitted in the VM's representation (c_fp28)."""
    assert 2 * (1 + MAXT) == REC and MAXT_LIN == 2 * MAXT
    lines = ["// generated by drand_amd/tools/gen_pairing_vm.py — do not edit",
             "// Lane-parallel multi-pairing check programs (see the generator's docstring).",
             "#pragma once", "#include <stdint.h>", "", "namespace dh {", "namespace vm {", ""]
    lines.append("constexpr int MAXT = %d, MAXT_LIN = %d, MAXC = %d, REC = %d;" % (MAXT, MAXT_LIN, MAXC, REC))
    lines.append("// values in slots: v R' mod p (R' = 2^392) as 14 x 28-bit limbs, v < 2p (k_vm.hip)")
    lines.append("__device__ __constant__ uint32_t ONE28[14] = %s;  // R' mod p" % c_fp28(1))
    lines.append("__device__ __constant__ uint32_t RP3_28[14] = %s;  // R'^3 mod p (raw limbs)" % (
        "{" + ", ".join("0x%07xu" % ((pow(RP, 3, P) >> (28 * i)) & 0xfffffff) for i in range(14)) + "}"))
    lines.append("enum : uint32_t { PH_MUL = 0, PH_LIN = 1, PH_INV = 2 };")
    lines.append("")
    for np_, prog, outs, phases, slot, nslots in progs:
        nodes = prog.nodes
        ph_words, op_words = [], []
        nops = 0
        for kind, batch in phases:
            ph_words += [{"mul": 0, "lin": 1, "inv": 2}[kind] | (len(batch) << 8), nops]
            for i in batch:
                n = nodes[i]
                a = n["a"]
                b = n.get("b", [])
                assert len(a) <= (MAXT_LIN if kind == "lin" else MAXT) and len(b) <= MAXT
                if kind == "lin":
                    a, b = a[:MAXT], a[MAXT:]
                rec = [0] * REC
                rec[0] = slot[i] | (len(a) << 16) | (len(b) << 24)
                rec[1 + MAXT] = len(b) << 16
                for k, (s_, c) in enumerate(a):
                    rec[1 + k] = slot[s_] | ((c & 0xffff) << 16)
                for k, (s_, c) in enumerate(b):
                    rec[2 + MAXT + k] = slot[s_] | ((c & 0xffff) << 16)
                op_words += rec
                nops += 1
        op_words += [0] * (REC // 2)  # pad: k_vm.hip's record loads read a full record from a pair lane's half
        ins = [slot[i] for i in prog.inputs]
        consts = [(slot[n], v) for v, n in prog.consts.items() if n in slot]
        tag = np_ if isinstance(np_, str) else "NP%d" % np_
        lines.append("// %s: %d phases (%d MUL, %d LIN, %d INV), %d ops, %d slots" % (
            tag, len(phases), sum(k == "mul" for k, _ in phases), sum(k == "lin" for k, _ in phases),
            sum(k == "inv" for k, _ in phases), nops, nslots))
        lines.append("constexpr int %s_NPHASES = %d, %s_NSLOTS = %d, %s_NCONST = %d;" % (
            tag, len(phases), tag, nslots, tag, len(consts)))
        lines.append("__device__ __constant__ uint32_t %s_INPUT_SLOT[%d] = {%s};" % (tag, len(ins), ", ".join(map(str, ins))))
        lines.append("__device__ __constant__ uint32_t %s_OUTPUT_SLOT[%d] = {%s};" % (
            tag, len(outs), ", ".join(str(slot[o]) for o in outs)))
        lines.append("__device__ __constant__ uint32_t %s_CONST_SLOT[%d] = {%s};" % (
            tag, len(consts), ", ".join(str(s) for s, _ in consts)))
        lines.append("__device__ __constant__ uint32_t %s_CONST_VAL[%d][14] = {%s};" % (
            tag, len(consts), ", ".join(c_fp28(v) for _, v in consts)))
        lines.append("__device__ const uint32_t %s_PHASES[%d] = {%s};" % (tag, len(ph_words), ", ".join(map(str, ph_words))))
        lines.append("__device__ const uint32_t __attribute__((aligned(16))) %s_OPS[%d] = {%s};" % (
            tag, len(op_words), ", ".join("0x%x" % w for w in op_words)))
        lines.append("")
    lines += ["}  // namespace vm", "}  // namespace dh", ""]
    return "\n".join(lines)


TAGS = ("NP1", "NP2", "ML1", "MUL12", "FE", "NP2C", "NP1J", "NP2J")


def build_all():
    progs = []
    for tag in TAGS:
        prog, outs = build_tag(tag)
        phases, live = schedule(prog, outs)
        slot, nslots = allocate(prog, outs, phases, live)
        validate(tag, prog, outs, phases, slot, nslots)
        progs.append((tag, prog, outs, phases, slot, nslots))
    validate_split(progs)
    return progs


def main():
    progs = build_all()
    for tag, prog, outs, phases, slot, nslots in progs:
        nm = sum(k == "mul" for k, _ in phases)
        print("%s: %d nodes, %d phases (%d MUL), %d slots, %d products" % (
            tag, len(prog.nodes), len(phases), nm, nslots, sum(len(b) for k, b in phases if k == "mul")))
    out = os.path.join(HERE, "..", "csrc", "pairing_vm.hpp")
    open(out, "w").write(emit(progs))


if __name__ == "__main__":
    main()
