#!/usr/bin/env python3
"""Build-time guard for the field-product call convention of fp.hpp (DH_FP_CALL / DH_FP_CALL_CLOBBERS) and fp28.hpp
(DH_FP28_CALL_CLOBBERS).

The kernels enter dh_fp_mul_vec / dh_fp_sqr_vec through an inline-asm s_swappc_b64 whose clobber list
names exactly the registers the two bodies may touch. The bodies are ordinary compiled functions, so this
script disassembles every gfx950 code object it is given and fails (exit 1) if a body
  * mentions a VGPR outside its declared set (v0-v39, v48-v53) or an SGPR outside s0-s17, s30-s31 (plus vcc /
    exec reads), ranged operands (v[4:5]) included,
  * touches the stack (scratch_* / buffer_* instructions, s32 / s33), or calls anything,
  * writes s[30:31] (the return address) or does not return with s_setpc_b64 s[30:31],
  * writes M0, or writes EXEC other than restoring it after an s_and_saveexec (SCC and VCC are clobbered).

    python check_fp_abi.py csrc/k_prep.o csrc/k_msm.o ...
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
FUNCS = ("dh_fp_mul_vec", "dh_fp_sqr_vec", "dh_fp28_mul_vec", "dh_fp28_sqr_vec")
# fp.hpp DH_FP_CALL_CLOBBERS (+ the v0-v23 operands) and fp28.hpp DH_FP28_CALL_CLOBBERS (+ the v0-v31 operands)
ALLOWED_V = {"dh_fp_mul_vec": set(range(0, 40)) | set(range(48, 54)),
             "dh_fp_sqr_vec": set(range(0, 40)) | set(range(48, 54)),
             "dh_fp28_mul_vec": set(range(0, 40)) | set(range(48, 54)),
             "dh_fp28_sqr_vec": set(range(0, 40)) | set(range(48, 54))}
ALLOWED_S = set(range(0, 18)) | {30, 31}
# ranged operands (v[4:5]) end in "]", after which \b never matches: only the single-register form takes \b
REG = re.compile(r"\b([vs])(?:\[(\d+):(\d+)\]|(\d+)\b)")


def device_elf(obj, tmp):
    """The gfx950 code object of a host object built by `hipcc -c` (offload bundle in .hip_fatbin)."""
    fat = os.path.join(tmp, os.path.basename(obj) + ".fatbin")
    subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", ".hip_fatbin=" + fat, obj, os.devnull])
    out = os.path.join(tmp, os.path.basename(obj) + ".gfx950.elf")
    subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--type=o", "--input=" + fat,
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + out, "--unbundle"])
    return out


def bodies(elf):
    dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", elf],
                         capture_output=True, text=True, check=True).stdout
    cur, out = None, {}
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\w+)>:", line)
        if m:
            cur = m.group(1) if m.group(1) in FUNCS else None
            if cur:
                out[cur] = []
            continue
        if cur and line.strip():
            out[cur].append(line.split("//")[0].strip())
    for ins in out.values():  # alignment padding after the return
        while ins and ins[-1].split()[0] in ("s_nop", "s_code_end"):
            ins.pop()
    return out


def check_body(name, insns):
    errs = []
    if not insns or insns[-1] != "s_setpc_b64 s[30:31]":
        errs.append("%s does not end with s_setpc_b64 s[30:31]" % name)
    exec_saved = False
    for k, ins in enumerate(insns):
        op = ins.split()[0]
        if op.startswith(("scratch_", "buffer_", "s_swappc", "s_call", "s_setpc")) and k != len(insns) - 1:
            errs.append("%s: forbidden instruction '%s'" % (name, ins))
        if "m0" in ins.split():
            errs.append("%s: M0 touched in '%s'" % (name, ins))
        if op in ("s_and_saveexec_b64", "s_or_saveexec_b64"):
            exec_saved = True
        elif re.match(r"^s_\w+ exec,", ins):
            # EXEC may only be restored (s_or_b64 exec, exec, s[..] / s_mov_b64 exec, s[..]) after a save
            if not exec_saved or op not in ("s_or_b64", "s_mov_b64"):
                errs.append("%s: EXEC written in '%s'" % (name, ins))
            exec_saved = False
        for m in REG.finditer(ins):
            kind = m.group(1)
            lo = int(m.group(2) if m.group(2) is not None else m.group(4))
            hi = int(m.group(3)) if m.group(3) is not None else lo
            allowed = ALLOWED_V[name] if kind == "v" else ALLOWED_S
            for r in range(lo, hi + 1):
                if r not in allowed:
                    errs.append("%s: %s%d outside the declared clobbers in '%s'" % (name, kind, r, ins))
                if kind == "s" and r in (30, 31) and k != len(insns) - 1:
                    errs.append("%s: return address s[30:31] touched in '%s'" % (name, ins))
    return errs


def main(objs):
    errs, seen = [], 0
    with tempfile.TemporaryDirectory() as tmp:
        for obj in objs:
            b = bodies(device_elf(obj, tmp))
            for name, insns in b.items():
                seen += 1
                errs += ["%s: %s" % (obj, e) for e in check_body(name, insns)]
    if errs:
        print("\n".join(errs[:40]), file=sys.stderr)
        print("check_fp_abi: %d violation(s): update DH_FP_CALL_CLOBBERS in fp.hpp and ALLOWED_* here together"
              % len(errs), file=sys.stderr)
        return 1
    print("check_fp_abi: %d field-product bodies in %d code objects within the declared clobbers" % (seen, len(objs)))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
