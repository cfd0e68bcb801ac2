#!/usr/bin/env python3
"""Per-kernel resources of the gfx950 code objects (VGPR / AGPR / SGPR counts, scratch bytes per lane, LDS), from the
AMDGPU metadata notes: python3 drand_amd/tools/kernel_resources.py drand_amd/csrc/k_msm.o [name-filter]"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from check_fp_abi import LLVM, device_elf  # noqa: E402


def resources(obj):
    with tempfile.TemporaryDirectory() as tmp:
        elf = device_elf(obj, tmp)
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", elf], capture_output=True, text=True,
                               check=True).stdout
    out, cur = [], None
    for line in notes.splitlines():
        m = re.match(r"\s+- (\.\w+):\s+(.*)$", line) or re.match(r"\s+(\.\w+):\s+(.*)$", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2).strip()
        if k == ".agpr_count":
            cur = {"agpr": v}
            out.append(cur)
        elif cur is not None:
            cur[k] = v
    return out


if __name__ == "__main__":
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    for r in resources(sys.argv[1]):
        name = r.get(".name", "?")
        if flt in name:
            print("%-70s vgpr %4s agpr %4s sgpr %4s scratch %5s lds %6s" % (
                name[:70], r.get(".vgpr_count"), r.get("agpr"), r.get(".sgpr_count"),
                r.get(".private_segment_fixed_size"), r.get(".group_segment_fixed_size")))
