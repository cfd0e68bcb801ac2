#!/usr/bin/env python3
"""Occupancy of the GPU over a rocprofv3 kernel trace (rocpd .db or *_kernel_trace.csv): over the window between the
first and last dispatch of a chosen kernel (the timed region's per-round kernels), the fraction of time at least one
kernel runs, the time-averaged number of kernels in flight, the idle gaps, and each kernel's summed duration — what
separates "the chip is full" from "the batches wait on each other" when more batches are put in flight.
    python bench/trace_busy.py gpurun_out/prof_r05g_3 [--anchor k_prep_sig] [--skip-frac 0.1]"""
import argparse
import collections
import csv
import glob
import json
import os
import sqlite3


def load(path):
    if os.path.isdir(path):
        c = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        path = c[0] if c else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
    if path.endswith(".csv"):
        rows = csv.DictReader(open(path))
        ev = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    else:
        db = sqlite3.connect(path)
        ev = [(n, int(s), int(s) + int(d)) for n, s, d in db.execute("select name, start, duration from kernels")]
    ev.sort(key=lambda e: e[1])
    return ev


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--anchor", default="k_prep_sig", help="kernel-name substring whose dispatches bound the window")
    ap.add_argument("--skip-frac", type=float, default=0.1, help="drop this fraction of the window at each end")
    a = ap.parse_args()
    ev = load(a.trace)
    anch = [e for e in ev if a.anchor in e[0]]
    t0, t1 = anch[0][1], anch[-1][2]
    span = t1 - t0
    w0, w1 = t0 + int(a.skip_frac * span), t1 - int(a.skip_frac * span)
    win = [(n, max(s, w0), min(e, w1)) for n, s, e in ev if e > w0 and s < w1]
    # sweep: busy time, concurrency-weighted time, gaps
    pts = sorted([(s, 1) for _, s, _ in win] + [(e, -1) for _, _, e in win])
    busy = conc = 0
    level, last = 0, w0
    gaps = []
    gap_start = w0
    for t, d in pts:
        if level > 0:
            busy += t - last
            conc += level * (t - last)
        elif t > last:
            gaps.append(t - gap_start)
        last = t
        level += d
        if level == 0:
            gap_start = t
    if last < w1:
        gaps.append(w1 - last)
    per = collections.defaultdict(lambda: [0, 0])
    for n, s, e in win:
        k = n.split("(")[0].replace("void ", "")
        per[k][0] += 1
        per[k][1] += e - s
    W = w1 - w0
    out = {
        "window_ms": W / 1e6,
        "busy_frac": busy / W,
        "mean_kernels_in_flight": conc / W,
        "idle_gaps": len(gaps),
        "idle_ms": sum(gaps) / 1e6,
        "largest_gaps_us": [g / 1e3 for g in sorted(gaps)[-5:]],
        "kernel_ms": {k: {"calls": c, "sum_ms": round(d / 1e6, 3)} for k, (c, d) in sorted(per.items(), key=lambda x: -x[1][1])[:25]},
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
