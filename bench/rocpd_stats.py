#!/usr/bin/env python3
"""Per-kernel stats (ns) from a rocprofv3 rocpd database, in the column layout of rocprofv3 --stats csv.
    python bench/rocpd_stats.py gpurun_out/prof_r01b/run_results.db > profiles/rocprof_kernel_stats_r01b.csv"""
import collections
import csv
import sqlite3
import statistics
import sys

db = sqlite3.connect(sys.argv[1])
d = collections.defaultdict(list)
for name, dur in db.execute("select name, duration from kernels"):
    d[name].append(int(dur))
tot = sum(sum(v) for v in d.values())
w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
for name, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    w.writerow([name, len(v), sum(v), sum(v) / len(v), round(100.0 * sum(v) / tot, 2), min(v), max(v),
                statistics.pstdev(v) if len(v) > 1 else 0.0])
