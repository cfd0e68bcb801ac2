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
                assert len(n["a"]) <= (g.MAXT_LIN if kind == "lin" else g.MAXT) and len(n.get("b", [])) <= g.MAXT
                assert all(abs(c) <= g.MAXC for _, c in n["a"] + n.get("b", []))
    text = g.emit(progs)
    with open(os.path.join(ROOT, "drand_amd", "csrc", "pairing_vm.hpp")) as f:
        assert f.read() == text, "csrc/pairing_vm.hpp is stale: rerun drand_amd/tools/gen_pairing_vm.py"
    # k_vm.hip stages one 16-bit descriptor (kind | count << 8) per phase and finds a phase's first op record as the
    # running sum of the counts: the emitted records must follow phase order and the descriptors fit 16 bits
    import re
    for tag in g.TAGS:
        m = re.search(r"%s_PHASES\[\d*\]\s*=\s*\{([^}]*)\}" % tag, text)
        v = [int(x.strip().rstrip("u"), 0) for x in m.group(1).split(",") if x.strip()]
        desc, first = v[0::2], v[1::2]
        assert first[0] == 0 and all(first[i + 1] == first[i] + (desc[i] >> 8) for i in range(len(desc) - 1)), tag
        assert max(desc) < 1 << 16, tag


def _vm_finish_model(terms):
    """Python restatement of k_vm.hip vm_lin + vm_finish: terms (v, c) with v < 2p held as 14 x 28-bit limbs,
    signed 64-bit per-limb sums, one signed carry pass, q = floor(top * 2^364 / p - 2^-10) in IEEE doubles, V - q p
    in the same radix. Returns the limbs' value, which must be in [0, 2p)."""
    import math
    P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
    M = (1 << 28) - 1
    pl = [(P >> (28 * i)) & M for i in range(14)]
    acc = [0] * 14
    for v, c in terms:
        for j in range(14):
            acc[j] += c * ((v >> (28 * j)) & M)
    limbs, c = [0] * 14, 0
    for j in range(14):
        t = acc[j] + c
        limbs[j], c = t & M, t >> 28
    top = float(c) * 268435456.0 + float(limbs[13])
    q = math.floor(top * float.fromhex("0x1.3b06ba5e7993dp-17") - 2.0 ** -10)
    c2 = 0
    for j in range(14):
        t = limbs[j] - q * pl[j] + c2
        limbs[j], c2 = t & M, t >> 28
    assert c + c2 == 0, "the reduced value left 14 limbs"
    return sum(x << (28 * j) for j, x in enumerate(limbs))


def test_lazy_linear_combination_model():
    import random
    import gen_pairing_vm as g
    P = g.P
    rng = random.Random(5)
    for trial in range(3000):
        n = rng.randint(1, g.MAXT_LIN)
        terms = []
        for _ in range(n):
            v = rng.choice([0, 1, P - 1, P, 2 * P - 1, rng.randrange(2 * P)])
            c = rng.choice([g.MAXC, -g.MAXC, 1, -1, rng.randint(-g.MAXC, g.MAXC)])
            terms.append((v, c))
        r = _vm_finish_model(terms)
        assert 0 <= r < 2 * P and r % P == sum(v * c for v, c in terms) % P
