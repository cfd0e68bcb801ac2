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
    progs = []
    for np_ in (1, 2):
        prog, outs = g.build(np_)
        phases, live = g.schedule(prog, outs)
        slot, nslots = g.allocate(prog, outs, phases, live)
        g.validate(np_, prog, outs, phases, slot, nslots)
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
        progs.append((np_, prog, outs, phases, slot, nslots))
    text = g.emit(progs)
    with open(os.path.join(ROOT, "drand_amd", "csrc", "pairing_vm.hpp")) as f:
        assert f.read() == text, "csrc/pairing_vm.hpp is stale: rerun drand_amd/tools/gen_pairing_vm.py"
