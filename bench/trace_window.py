#!/usr/bin/env python3
"""Kernel timeline windows from a rocprofv3 kernel-trace database: the dispatches following the k-th occurrence of a
kernel (start offsets and durations in ms), for reading one call's critical path.
    python bench/trace_window.py gpurun_out/prof_x/run_results.db --kernel k_prep_sig --at 5,60 --count 14"""
import argparse
import glob
import os
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--kernel", default="k_prep_sig")
    ap.add_argument("--at", default="5")
    ap.add_argument("--count", type=int, default=14)
    a = ap.parse_args()
    path = a.path
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
    db = sqlite3.connect(path)
    rows = list(db.execute("select name, start, end from kernels order by start"))
    idx = [i for i, r in enumerate(rows) if re.search(a.kernel, r[0])]
    for k in (int(x) for x in a.at.split(",")):
        if k >= len(idx):
            continue
        t0 = rows[idx[k]][1]
        for name, s, e in rows[idx[k]:idx[k] + a.count]:
            print("%-58s start %8.3f  end %8.3f  dur %7.3f ms" % (re.sub(r"\(.*", "", name)[:58], (s - t0) / 1e6,
                                                                  (e - t0) / 1e6, (e - s) / 1e6))
        print("---")


if __name__ == "__main__":
    main()
