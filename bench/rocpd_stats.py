#!/usr/bin/env python3
"""Per-kernel stats (ns) from a rocprofv3 kernel trace (rocpd .db or *_kernel_trace.csv), in the column layout of
rocprofv3 --stats. With --last N, also one row per kernel over its last N dispatches: bench.py times its roofline
on the single-stream batches it runs after the timed region, so those are the launches its HIP events measure.
    python bench/rocpd_stats.py gpurun_out/prof_r01c [--last 2] > profiles/rocprof_kernel_stats_r01c.csv"""
import argparse
import collections
import csv
import glob
import os
import sqlite3
import statistics
import sys


def dispatches(path):
    if os.path.isdir(path):
        c = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        if c:
            path = c[0]
        else:
            path = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
    if path.endswith(".csv"):
        rows = list(csv.DictReader(open(path)))
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        return [(r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in rows]
    db = sqlite3.connect(path)
    return [(n, int(d)) for n, d in db.execute("select name, duration from kernels order by start")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--last", type=int, default=0)
    a = ap.parse_args()
    d = collections.defaultdict(list)
    for name, dur in dispatches(a.path):
        d[name].append(dur)
    tot = sum(sum(v) for v in d.values())
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])

    def row(name, v):
        w.writerow([name, len(v), sum(v), sum(v) / len(v), round(100.0 * sum(v) / tot, 2), min(v), max(v),
                    statistics.pstdev(v) if len(v) > 1 else 0.0])

    for name, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        row(name, v)
    if a.last:
        for name, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
            if len(v) > a.last:
                row("%s [last %d dispatches]" % (name, a.last), v[-a.last:])


if __name__ == "__main__":
    main()
