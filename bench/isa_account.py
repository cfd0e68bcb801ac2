#!/usr/bin/env python3
"""Instruction-level accounting of a per-round kernel (VERDICT r05 Next #3: where does k_prep_sig<fp>'s time go?).

Static part, from the gfx950 code object of the built library (drand_amd/csrc/k_prep.o): the instruction mix of the
out-of-line field-product bodies and of the kernel's loop bodies (the hot loops are the inlined Jacobian doublings of
the subgroup test's two [|u|] runs), classified as
  MAD64  v_mad_u64_u32                       (one partial product of the 28-bit schoolbook / Montgomery columns)
  V64    v_lshrrev_b64 / v_lshl_add_u64 ...  (the column carries)
  MUL32  v_mul_lo_u32                        (the Montgomery quotient digits)
  VALU   every other vector instruction       (masks, the limb-wise sums of the point formulas, moves, selects)
  SALU / SMEM / scratch / branches / s_nop / s_waitcnt.
Dynamic part, from the PMC passes of bench/pmc_isa.sh (one 262,144-round single-stream batch): SQ_INSTS_VALU_INT64,
SQ_INSTS_VALU_INT32, SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, SQ_WAVE_CYCLES, GRBM_GUI_ACTIVE per kernel.

The cycle model it checks (MI355X_MICROARCH.md: a wave64 VALU instruction issues over 2 cycles on a SIMD-32; the
measured v_mad_u64_u32 peak, 37.15 T/s = 1024 SIMDs x 2.27 GHz x 16 lanes per cycle, makes the MAD a 4-cycle
issue): issue cycles per wave = 4 INT64 + 2 (VALU - INT64), against the wave's share of the SIMD's cycles.

    python bench/isa_account.py [--obj drand_amd/csrc/k_prep.o] [--pmc gpurun_out/pmc_isa_X --busy gpurun_out/pmc_isabusy_X]
        [--kernel k_prep_sig<fp>] [--rounds 262144] [--launch-ms 22.386 --launch-rounds 1048576]
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "drand_amd", "tools"))
sys.path.insert(0, os.path.join(ROOT, "bench"))
from check_fp_abi import LLVM, device_elf  # noqa: E402

BODIES = ("dh_fp28_mul_vec", "dh_fp28_sqr_vec", "dh_fp_mul_vec", "dh_fp_sqr_vec")
MANGLED = {"k_prep_sig<fp>": "_ZN2dh10k_prep_sigINS_2fpEEEvPKhmmPhPjS4_",
           "k_prep_msg_g1": "_ZN2dh13k_prep_msg_g1EPKmPKhmPKjS3_miiPhPj",
           "k_sub_sig_g2": "_ZN2dh12k_sub_sig_g2EmPhPj",
           "k_sswu_g2": "_ZN2dh9k_sswu_g2EPKjmPj"}


def klass(ins):
    op = ins.split()[0]
    if op.startswith("v_mad_u64_u32"):
        return "MAD64"
    if op.startswith(("v_mul_lo_u32", "v_mul_hi_u32")):
        return "MUL32"
    if op.startswith(("v_lshrrev_b64", "v_lshlrev_b64", "v_ashrrev_i64", "v_lshl_add_u64", "v_add_u64", "v_sub_u64",
                      "v_mov_b64")):
        return "V64"
    if op.startswith("v_"):
        return "VALU"
    if op.startswith(("scratch_", "buffer_")):
        return "SCRATCH"
    if op.startswith(("global_", "flat_")):
        return "VMEM"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith("s_waitcnt"):
        return "WAITCNT"
    if op.startswith("s_nop"):
        return "NOP"
    if op.startswith(("s_load", "s_buffer_load")):
        return "SMEM"
    if op.startswith("s_swappc"):
        return "CALL"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_getpc")):
        return "BRANCH"
    if op.startswith("s_"):
        return "SALU"
    return "OTHER"


def disassemble(obj):
    with tempfile.TemporaryDirectory() as tmp:
        elf = device_elf(obj, tmp)
        return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", elf],
                              capture_output=True, text=True, check=True).stdout


def function(dis, name):
    m = re.search(r"^[0-9a-f]+ <%s>:\n(.*?)(?=^[0-9a-f]+ <|\Z)" % re.escape(name), dis, re.M | re.S)
    out = []
    if not m:
        return out
    for line in m.group(1).splitlines():
        mm = re.match(r"\s*(\S.*?)\s*//\s*([0-9A-F]+):", line)
        if mm:
            out.append((int(mm.group(2), 16), mm.group(1)))
    return out


def mix(instrs):
    c = collections.Counter(klass(i) for _, i in instrs)
    return {k: c[k] for k in sorted(c)}


def loops(instrs):
    """innermost backward-branch loops: (start, end, mix)"""
    addr = {a: i for i, (a, _) in enumerate(instrs)}
    found = []
    for i, (a, ins) in enumerate(instrs):
        if not ins.startswith(("s_cbranch", "s_branch")):
            continue
        tok = ins.split()
        try:
            off = int(tok[1])
        except (IndexError, ValueError):
            continue
        if off >= 32768:
            off -= 65536
        tgt = a + 4 + 4 * off
        if tgt < a and tgt in addr:
            found.append((addr[tgt], i))
    inner = [(s, e) for s, e in found if not any(s < s2 and e2 < e for s2, e2 in found if (s2, e2) != (s, e))]
    return [(instrs[s][0], instrs[e][0], mix(instrs[s:e + 1])) for s, e in sorted(set(inner))]


def model_cycles(m):
    """issue cycles of one wave's pass through m (SIMD-32: 2 cycles per wave64 VALU instruction, 4 for the MAD)"""
    v = m.get("VALU", 0) + m.get("V64", 0) + m.get("MUL32", 0)
    return 4 * m.get("MAD64", 0) + 2 * v


def pmc(dirs, kernel):
    import pmc_summary as ps
    tot = collections.defaultdict(float)
    for d in dirs:
        if not d:
            continue
        agg, cnt = ps.load(d)
        for k, v in agg.items():
            if k == kernel:
                ndisp = max([cnt[(k, c)] for c in v if not c.startswith("_")] or [1])
                for c, x in v.items():  # per dispatch
                    tot[c] = max(tot[c], x / ndisp) if c.startswith("_") else x / ndisp
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--obj", default=os.path.join(ROOT, "drand_amd", "csrc", "k_prep.o"))
    ap.add_argument("--kernel", default="k_prep_sig<fp>")
    ap.add_argument("--pmc", default="")
    ap.add_argument("--busy", default="")
    ap.add_argument("--rounds", type=int, default=262144)
    ap.add_argument("--launch-ms", type=float, default=0.0, help="measured launch time (HIP events / rocprofv3)")
    ap.add_argument("--launch-rounds", type=int, default=1 << 20)
    ap.add_argument("--clock-ghz", type=float, default=0.0, help="effective clock (default: from GRBM_GUI_ACTIVE)")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    dis = disassemble(a.obj)
    rep = {"bodies": {}, "kernel": a.kernel}
    for b in BODIES:
        f = function(dis, b)
        if f:
            m = mix(f)
            rep["bodies"][b] = {"instructions": len(f), "mix": m, "model_issue_cycles": model_cycles(m),
                                "mad_share_of_issue_cycles": round(4 * m.get("MAD64", 0) / model_cycles(m), 3)}
    k = function(dis, MANGLED.get(a.kernel, a.kernel))
    if k:
        rep["kernel_static"] = {"instructions": len(k), "mix": mix(k)}
        rep["inner_loops"] = [{"range": "%x..%x" % (s, e), "mix": m, "model_issue_cycles": model_cycles(m),
                               "mad_share_of_issue_cycles": round(4 * m.get("MAD64", 0) / max(1, model_cycles(m)), 3)}
                              for s, e, m in loops(k)]
    if a.pmc:
        c = pmc([a.pmc, a.busy], a.kernel)
        waves = c.get("SQ_WAVES", 0) or (a.rounds / 64)
        per_wave = {x: c[x] / waves for x in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_INT32",
                                              "SQ_INSTS_SALU", "SQ_INSTS_VALU_CVT") if x in c}
        rep["dynamic_per_wave"] = {k2: round(v, 1) for k2, v in per_wave.items()}
        i64 = per_wave.get("SQ_INSTS_VALU_INT64", 0)
        valu = per_wave.get("SQ_INSTS_VALU", 0)
        cyc = 4 * i64 + 2 * (valu - i64)
        rep["model_issue_cycles_per_wave"] = round(cyc)
        rep["int64_share_of_model_cycles"] = round(4 * i64 / cyc, 3) if cyc else None
        if "SQ_WAVE_CYCLES" in c and "SQ_ACTIVE_INST_VALU" in c:
            rep["valu_active_frac_of_wave_cycles"] = round(c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"], 4)
            rep["wave_cycles_per_wave"] = round(4 * c["SQ_WAVE_CYCLES"] / waves)  # quad-cycles
        if c.get("GRBM_GUI_ACTIVE") and c.get("_dur_ns"):
            rep["effective_clock_ghz"] = round(c["GRBM_GUI_ACTIVE"] / 8 / c["_dur_ns"], 3)
        clk = a.clock_ghz or rep.get("effective_clock_ghz") or 2.0
        if a.launch_ms:
            simds = 1024
            waves_launch = a.launch_rounds / 64
            avail = a.launch_ms * 1e-3 * clk * 1e9 * simds  # SIMD-cycles in the launch
            need = cyc * waves_launch
            rep["launch"] = {"ms": a.launch_ms, "rounds": a.launch_rounds, "clock_ghz": clk,
                             "simd_cycles_available": round(avail), "model_issue_cycles": round(need),
                             "issue_share_of_launch": round(need / avail, 3)}
    txt = json.dumps(rep, indent=1)
    print(txt)
    if a.json:
        open(a.json, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
