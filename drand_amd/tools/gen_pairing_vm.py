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
MAXT_LIN = 31    # terms per LIN op (the record's words 1..31)
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
    f = F12.one()
    T = [(Q[0], Q[1], F2(L.const(1), L())) for Q in Qs]
    started = False
    for b in range(62, -1, -1):
        if started:
            f = f.sqr()
        started = True
        for k in range(len(Ps)):
            T[k], (c0, c1, c2) = ml_dbl(T[k])
            f = f.mul_line(c2, c1.mul_fp(Ps[k][0]), c0.mul_fp(Ps[k][1]))
        if (U_ABS >> b) & 1:
            for k in range(len(Ps)):
                T[k], (c0, c1, c2) = ml_add(T[k], Qs[k])
                f = f.mul_line(c2, c1.mul_fp(Ps[k][0]), c0.mul_fp(Ps[k][1]))
        f = f.mat()
    return f.conj()


def cyc_exp_u(a):
    acc = a
    for b in range(62, -1, -1):
        acc = acc.cyc_sqr().mat()
        if (U_ABS >> b) & 1:
            acc = (acc * a).mat()
    return acc.conj()


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


def _fp12_input(prefix):
    c = [L.node(PROG.inp("%s%d" % (prefix, i))) for i in range(12)]
    return F12(F6(F2(c[0], c[1]), F2(c[2], c[3]), F2(c[4], c[5])), F6(F2(c[6], c[7]), F2(c[8], c[9]), F2(c[10], c[11])))


def build_tag(tag):
    """Programs: NP1 / NP2 = the full check of 1 / 2 pairs; ML1 = the Miller loop of one pair (f out, for
    multi-pairings of many pairs run one workgroup per pair); MUL12 = f * g; FE = final exponentiation."""
    global PROG
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


def build(np_):
    global PROG
    PROG = Prog()
    Ps, Qs = [], []
    for k in range(np_):
        px, py = L.node(PROG.inp("P%d.x" % k)), L.node(PROG.inp("P%d.y" % k))
        qx = F2(L.node(PROG.inp("Q%d.x0" % k)), L.node(PROG.inp("Q%d.x1" % k)))
        qy = F2(L.node(PROG.inp("Q%d.y0" % k)), L.node(PROG.inp("Q%d.y1" % k)))
        Ps.append((px, py))
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
    """Greedy ASAP list scheduling into phases: MUL phase (<= LANES products), then LIN sub-phases, then INV."""
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
        for d in deps(nodes[i]):
            users.setdefault(d, []).append(i)
    ndeps = {i: len(set(d for d in deps(nodes[i]) if d not in done)) for i in pending}
    ready = {"mul": [], "lin": [], "inv": []}
    for i in pending:
        if ndeps[i] == 0:
            ready[nodes[i]["kind"]].append(i)
    phases = []
    remaining = len(pending)

    def finish(batch):
        nonlocal remaining
        for i in batch:
            done.add(i)
            remaining -= 1
        for i in batch:
            for u in set(users.get(i, [])):
                ndeps[u] -= len([d for d in set(deps(nodes[u])) if d == i])
                if ndeps[u] == 0:
                    ready[nodes[u]["kind"]].append(u)

    while remaining:
        progressed = False
        for kind, cap in (("mul", LANES), ("lin", LANES), ("inv", 1)):
            while ready[kind]:
                ready[kind].sort()
                batch, ready[kind] = ready[kind][:cap], ready[kind][cap:]
                phases.append((kind, batch))
                finish(batch)
                progressed = True
                if kind == "mul":
                    break  # re-offer LIN / INV work between product phases
        if not progressed:
            raise RuntimeError("scheduling deadlock")
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


def validate(np_, prog, outs, phases, slot, nslots):
    if isinstance(np_, str):
        if not np_.startswith("NP"):
            return  # checked in validate_split
        np_ = int(np_[2:])
    B = _bls_points()
    rng = random.Random(1)
    one = [1] + [0] * 11

    def run(pairs):
        inp = {}
        for k, (Pt, Qt) in enumerate(pairs):
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
REC = 32  # words per op record: header, MAXT A terms, MAXT B terms (fixed positions), padding; LIN: MAXT_LIN A terms


def c_fp28(v):
    """an Fp constant in the VM's representation: v R' mod p as 14 x 28-bit limbs"""
    m = v * RP % P
    return "{" + ", ".join("0x%07xu" % ((m >> (28 * i)) & 0xfffffff) for i in range(14)) + "}"


def emit(progs):
    """progs: list of (np, prog, outs, phases, slot, nslots).

    Layout read by k_vm.hip: PHASES[2 * ph] = kind | cnt << 8, PHASES[2 * ph + 1] = index of the phase's first op;
    op k of phase ph is the REC-word record OPS[REC * (first + k) ...]: word 0 = dst slot | na << 16 | nb << 24,
    words 1..MAXT = A terms, words 1+MAXT..2*MAXT = B terms (a LIN op: words 1..MAXT_LIN = A terms), a term =
    slot | (coeff & 0xffff) << 16. Constants are emitted in the VM's representation (c_fp28)."""
    assert 1 + 2 * MAXT <= REC and 1 + MAXT_LIN <= REC
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
                rec = [0] * REC
                rec[0] = slot[i] | (len(a) << 16) | (len(b) << 24)
                for k, (s_, c) in enumerate(a):
                    rec[1 + k] = slot[s_] | ((c & 0xffff) << 16)
                for k, (s_, c) in enumerate(b):
                    rec[1 + MAXT + k] = slot[s_] | ((c & 0xffff) << 16)
                op_words += rec
                nops += 1
        ins = [slot[i] for i in prog.inputs]
        consts = [(slot[n], v) for v, n in prog.consts.items() if n in slot]
        tag = np_ if isinstance(np_, str) else "NP%d" % np_
        lines.append("// %s: %d phases (%d MUL, %d LIN, %d INV), %d ops, %d slots" % (
            tag, len(phases), sum(k == "mul" for k, _ in phases), sum(k == "lin" for k, _ in phases),
            sum(k == "inv" for k, _ in phases), nops, nslots))
        lines.append("constexpr int %s_NPHASES = %d, %s_NSLOTS = %d, %s_NCONST = %d;" % (
            tag, len(phases), tag, nslots, tag, len(consts)))
        lines.append("__device__ __constant__ uint32_t %s_INPUT_SLOT[%d] = {%s};" % (tag, len(ins), ", ".join(map(str, ins))))
        lines.append("__device__ __constant__ uint32_t %s_OUTPUT_SLOT[12] = {%s};" % (tag, ", ".join(str(slot[o]) for o in outs)))
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


TAGS = ("NP1", "NP2", "ML1", "MUL12", "FE")


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
