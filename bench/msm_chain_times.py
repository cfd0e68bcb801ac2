#!/usr/bin/env python3
"""Durations of the MSM kernel chain that follows each dispatch of a given kernel and grid size on the same stream,
from a rocprofv3 kernel trace (rocpd .db): every kernel up to and including the window Horner (k_msm_windows28).
The minimum over the dispatches is the single-stream batches' time (bench.py runs its roofline batches and its
single calls one at a time); the median mixes in the batches that ran 8 in flight.
    python bench/msm_chain_times.py gpurun_out/prof_<tag>/run_results.db "k_msm_bucket_fix28<dh::c28_g1>" 262144"""
import collections
import sqlite3
import statistics
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    first, grid = sys.argv[2], int(sys.argv[3])
    rows = list(db.execute("select name, start, end, grid_x, stream_id from kernels order by start"))
    short = lambda n: n.split("(")[0].replace("void ", "").replace("dh::", "")  # noqa: E731
    acc = collections.defaultdict(list)
    for i, r in enumerate(rows):
        if first in r[0] and r[3] == grid:
            seq = [x for x in rows[i:] if x[4] == r[4]][:14]
            for x in seq:
                acc[short(x[0])].append((x[2] - x[1]) / 1e6)
                if "windows" in x[0]:
                    break
    for k, v in acc.items():
        print(f"{k[:50]:50s} n {len(v):3d} median {statistics.median(v):7.3f} min {min(v):7.3f}")


if __name__ == "__main__":
    main()
