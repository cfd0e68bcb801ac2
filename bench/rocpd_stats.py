#!/usr/bin/env python3
"""Per-kernel stats (ns) from a rocprofv3 kernel trace (rocpd .db or *_kernel_trace.csv), in the column layout of
rocprofv3 --stats. With --last N, also one row per kernel over its last N dispatches: bench.py times its roofline
on the single-stream batches it runs after the timed region, so those are the launches its HIP events measure.
    python bench/rocpd_stats.py gpurun_out/prof_r01c [--last 2] [--grid 1048576] > profiles/rocprof_kernel_stats_r01c.csv
Since r06 bench.py times one-beacon calls after its single-stream batches, so the headline kernel's last dispatches
are those small calls' unless --grid keeps the [last N] rows to the 1M-round launches."""
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
        return [(r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0))
                for r in rows]
    db = sqlite3.connect(path)
    return [(n, int(d), int(g)) for n, d, g in db.execute("select name, duration, grid_x from kernels order by start")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--grid", type=int, default=0, help="the [last N] rows count only dispatches of this grid size (in "
                    "threads), e.g. 1048576: the bench's 1M single-stream batches, not the one-beacon calls it times after them")
    a = ap.parse_args()
    d = collections.defaultdict(list)
    dg = collections.defaultdict(list)
    for name, dur, grid in dispatches(a.path):
        d[name].append(dur)
        if not a.grid or grid == a.grid:
            dg[name].append(dur)
    tot = sum(sum(v) for v in d.values())
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])

    def row(name, v):
        w.writerow([name, len(v), sum(v), sum(v) / len(v), round(100.0 * sum(v) / tot, 2), min(v), max(v),
                    statistics.pstdev(v) if len(v) > 1 else 0.0])

    for name, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        row(name, v)
    if a.last:
        tag = " of grid %d" % a.grid if a.grid else ""
        for name, v in sorted(dg.items(), key=lambda kv: -sum(kv[1])):
            if len(v) > a.last:
                row("%s [last %d dispatches%s]" % (name, a.last, tag), v[-a.last:])


if __name__ == "__main__":
    main()
