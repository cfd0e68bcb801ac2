#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE, SQ_*) of one bench.py run into a per-kernel json.

    python bench/pmc_summary.py --rounds 262144 --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write \
        --sq gpurun_out/pmc_sq --out profiles/pmc_r01.json

Corrections follow /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half of the bytes of wide streaming reads, so it is doubled. Per-kernel values
are summed over launches and divided by the rounds one launch processes, so bench.py can report the traffic
of a launch at any batch size (hbm_bytes_per_round x rounds). The dominant kernels' traffic is scratch (register
spill) traffic, not input: their algorithmic input is ~60-100 B per round.
"""
import argparse
import collections
import csv
import json
import os
import glob
import re
import sqlite3


def rows(d):
    """(kernel name, counter, value, scratch bytes/lane, vgprs) from a rocprofv3 output dir: csv or rocpd sqlite."""
    csvs = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if csvs:
        for r in csv.DictReader(open(csvs[0])):
            yield r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"]), int(r["Scratch_Size"]), int(r["VGPR_Count"])
        return
    db = sqlite3.connect(glob.glob(os.path.join(d, "*.db"))[0])
    for r in db.execute("select kernel_name, counter_name, value, scratch_size, vgpr_count from counters_collection"):
        yield r[0], r[1], float(r[2]), int(r[3] or 0), int(r[4] or 0)


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for name, cname, val, scratch, vgpr in rows(d):
        m = re.match(r"(?:void )?dh::(k_\w+)(<dh::(fp2?)(?:, (true|false))?>)?", name)
        if not m:
            continue
        key = m.group(1) + ("<%s>" % m.group(3) if m.group(3) else "")
        agg[key][cname] += val
        agg[key]["_scratch_per_lane"] = scratch
        agg[key]["_vgpr"] = vgpr
        n[(key, cname)] += 1
    return agg, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--sq", default=None)
    ap.add_argument("--out", required=True)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    f, _ = load(a.fetch)
    w, _ = load(a.write)
    sq = load(a.sq)[0] if a.sq else {}
    out = {"_meta": {"rounds_per_launch": a.rounds, "units": "bytes per round; FETCH_SIZE KiB x1024 x2 (gfx950 "
                     "half-count correction), WRITE_SIZE KiB x1024", "note": a.note}}
    for k in sorted(set(f) | set(w)):
        fb = f.get(k, {}).get("FETCH_SIZE", 0.0) * 1024 * 2
        wb = w.get(k, {}).get("WRITE_SIZE", 0.0) * 1024
        e = {"fetch_bytes_per_round": round(fb / a.rounds, 2), "write_bytes_per_round": round(wb / a.rounds, 2),
             "hbm_bytes_per_round": round((fb + wb) / a.rounds, 2),
             "scratch_bytes_per_lane": int(f.get(k, {}).get("_scratch_per_lane", 0)),
             "vgprs": int(f.get(k, {}).get("_vgpr", 0))}
        if k in sq:
            s = sq[k]
            e["valu_insts_per_round"] = round(s.get("SQ_INSTS_VALU", 0) * 64 / a.rounds, 1)  # per lane = per round
            e["salu_insts_per_wave"] = round(s.get("SQ_INSTS_SALU", 0) / max(1.0, s.get("SQ_WAVES", 1)), 1)
            e["flat_insts_per_round"] = round(s.get("SQ_INSTS_FLAT", 0) * 64 / a.rounds, 1)
        out[k] = e
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({k: v.get("hbm_bytes_per_round") for k, v in out.items() if k != "_meta"}))


if __name__ == "__main__":
    main()
