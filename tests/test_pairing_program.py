"""CPU: the lane-parallel pairing program (drand_amd/csrc/pairing_vm.hpp, run by k_vm.hip) is regenerated from
drand_amd/tools/gen_pairing_vm.py, its scheduled / slot-allocated form is evaluated in Python exactly as the
device runs it (phase by phase, LDS slots reused), and it is checked on oracle points: e(P,Q)e(-P,Q) = 1,
bilinearity, and non-degenerate products != 1. The committed header must equal the regenerated one."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "drand_amd", "tools"))


def test_pairing_program_valid_and_committed():
    import gen_pairing_vm as g
    progs = g.build_all()  # validates NP1 / NP2 on oracle points and ML1 x MUL12 x FE composed
    for tag, prog, outs, phases, slot, nslots in progs:
        # invariants the device interpreter relies on
        assert nslots <= 400
        for kind, batch in phases:
            assert len(batch) <= (1 if kind == "inv" else g.LANES)
            written = {slot[i] for i in batch}
            read = {slot[s] for i in batch for s, _ in prog.nodes[i]["a"] + prog.nodes[i].get("b", [])}
            assert not (written & read), "a phase reads a slot it writes"
            for i in batch:
                n = prog.nodes[i]
                assert len(n["a"]) <= g.MAXT and len(n.get("b", [])) <= g.MAXT
                assert all(abs(c) <= g.MAXC for _, c in n["a"] + n.get("b", []))
    text = g.emit(progs)
    with open(os.path.join(ROOT, "drand_amd", "csrc", "pairing_vm.hpp")) as f:
        assert f.read() == text, "csrc/pairing_vm.hpp is stale: rerun drand_amd/tools/gen_pairing_vm.py"


def _vm_finish_model(terms, K):
    """Python restatement of k_vm.hip vm_acc_term + vm_finish (same limb arithmetic, IEEE doubles)."""
    P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
    pl = [(P >> (32 * i)) & 0xffffffff for i in range(12)]
    pos, neg = [0] * 12, [0] * 12
    for v, c in terms:
        vl = [(v >> (32 * i)) & 0xffffffff for i in range(12)]
        for i in range(12):
            pos[i] += vl[i] * max(c, 0)
            neg[i] += vl[i] * max(-c, 0)
    kp = K * P
    kpl = [(kp >> (32 * i)) & 0xffffffff for i in range(13)]
    v, carry = [0] * 13, 0
    for i in range(12):
        t = pos[i] - neg[i] + kpl[i] + carry
        v[i] = t & 0xffffffff
        carry = t >> 32
    v[12] = kpl[12] + carry
    d = (float(v[12]) * 4294967296.0 + float(v[11])) * 4294967296.0 + float(v[10])
    qd = d * 5.336752789664505e-19
    q = int(qd) if qd > 0 else 0
    q = q - 1 if q > 0 else 0
    V = sum(x << (32 * i) for i, x in enumerate(v)) - q * P
    assert 0 <= V < 3 * P, "quotient estimate out of range"
    for _ in range(2):
        if V >= P:
            V -= P
    return V


def test_lazy_linear_combination_model():
    import random
    import gen_pairing_vm as g
    P = g.P
    rng = random.Random(5)
    K = g.MAXT * g.MAXC
    for trial in range(3000):
        n = rng.randint(1, g.MAXT)
        terms = []
        for _ in range(n):
            v = rng.choice([0, 1, P - 1, P - 2, rng.randrange(P), rng.randrange(1 << 64)])
            c = rng.choice([g.MAXC, -g.MAXC, 1, -1, rng.randint(-g.MAXC, g.MAXC)])
            terms.append((v, c))
        assert _vm_finish_model(terms, K) == sum(v * c for v, c in terms) % P
