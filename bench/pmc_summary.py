#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE, SQ_*) of one bench.py run into a per-kernel json.

    python bench/pmc_summary.py --rounds 262144 --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write \
        --sq gpurun_out/pmc_sq --busy gpurun_out/pmc_busy --out profiles/pmc_r02.json

Units follow /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are in KiB and
count the L2's memory-side requests, Infinity-Cache hits included, so they bound fabric traffic, not HBM bytes.
On gfx950 FETCH_SIZE reads exactly half the bytes of a WIDE COALESCED STREAMING read; that correction is not
applied blanket: each kernel reports the raw value and the doubled one, and which applies depends on its access
pattern (the per-round prep kernels read 16-B-per-lane records: doubled; the MSM bucket pass gathers scattered
points: raw). Per-kernel values are summed over launches and divided by the rounds one launch processes, so
bench.py can report the traffic of a launch at any batch size (x rounds).
Counters are averaged per dispatch (a kernel that also runs while the bench signs its chain, as the G2 hash kernels
do, is not double counted). The VALU-busy pass: SQ_ACTIVE_INST_VALU (quad-cycles in which a wave issued VALU work, summed over waves) over
SQ_WAVE_CYCLES (quad-cycles of wave lifetime, summed over waves) = VALU-active share of a wave's life;
SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES = issue stalls (dependency / pipe), SQ_WAIT_ANY / SQ_WAVE_CYCLES = parked on
s_waitcnt (memory); GRBM_GUI_ACTIVE / 8 XCDs / duration = effective clock.
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
    """(kernel name, counter, value, scratch bytes/lane, vgprs, duration ns) from a rocprofv3 output dir: csv or
    rocpd sqlite."""
    csvs = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if csvs:
        for r in csv.DictReader(open(csvs[0])):
            dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) if "End_Timestamp" in r else 0
            yield (r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"]), int(r["Scratch_Size"]),
                   int(r["VGPR_Count"]), dur)
        return
    db = sqlite3.connect(glob.glob(os.path.join(d, "*.db"))[0])
    for r in db.execute("select kernel_name, counter_name, value, scratch_size, vgpr_count from counters_collection"):
        yield r[0], r[1], float(r[2]), int(r[3] or 0), int(r[4] or 0), 0


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    seen = set()
    for name, cname, val, scratch, vgpr, dur in rows(d):
        m = re.match(r"(?:void )?dh::(k_\w+)(?:<dh::(fp2?)(?:, (true|false))?>|<(true|false)>)?", name)
        if not m:
            continue
        targs = [x for x in (m.group(2), m.group(3), m.group(4)) if x]
        key = m.group(1) + ("<%s>" % ", ".join(targs) if targs else "")
        agg[key][cname] += val
        agg[key]["_scratch_per_lane"] = scratch
        agg[key]["_vgpr"] = vgpr
        if (key, name, dur) not in seen and cname == "GRBM_GUI_ACTIVE":  # one duration per dispatch
            seen.add((key, name, dur))
            agg[key]["_dur_ns"] += dur
        n[(key, cname)] += 1
    return agg, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--sq", default=None)
    ap.add_argument("--busy", default=None)
    ap.add_argument("--out", required=True)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    f, fn = load(a.fetch)
    w, wn = load(a.write)
    sq, sqn = load(a.sq) if a.sq else ({}, {})
    busy = load(a.busy)[0] if a.busy else {}
    out = {"_meta": {"rounds_per_launch": a.rounds, "units": "bytes per round; FETCH_SIZE KiB x1024 (raw, and x2 "
                     "for streaming-read kernels), WRITE_SIZE KiB x1024", "note": a.note}}
    nd = {}  # dispatches per kernel: the same kernel may run more than once (e.g. the G2 hash kernels also sign)
    for agg, cnt in ((f, fn), (w, wn)):
        for (k, c), v in cnt.items():
            nd[k] = max(nd.get(k, 1), v)
    for k in sorted(set(f) | set(w)):
        d = float(nd.get(k, 1))
        fr = f.get(k, {}).get("FETCH_SIZE", 0.0) * 1024 / d
        wb = w.get(k, {}).get("WRITE_SIZE", 0.0) * 1024 / d
        streaming = k.startswith("k_prep") or k.startswith("k_h2f") or k.startswith("k_sswu") or k.startswith("k_add_iso")
        fb = fr * 2 if streaming else fr
        e = {"fetch_bytes_per_round_raw": round(fr / a.rounds, 2), "fetch_correction": "x2" if streaming else "none",
             "fetch_bytes_per_round": round(fb / a.rounds, 2), "write_bytes_per_round": round(wb / a.rounds, 2),
             "hbm_bytes_per_round": round((fb + wb) / a.rounds, 2),
             "scratch_bytes_per_lane": int(f.get(k, {}).get("_scratch_per_lane", 0)),
             "vgprs": int(f.get(k, {}).get("_vgpr", 0))}
        if k in sq:
            s = sq[k]
            ds = float(max(1, sqn.get((k, "SQ_INSTS_VALU"), 1)))
            e["dispatches"] = int(ds)
            e["valu_insts_per_round"] = round(s.get("SQ_INSTS_VALU", 0) * 64 / a.rounds / ds, 1)  # per lane = per round
            e["salu_insts_per_wave"] = round(s.get("SQ_INSTS_SALU", 0) / max(1.0, s.get("SQ_WAVES", 1)), 1)
            e["flat_insts_per_round"] = round(s.get("SQ_INSTS_FLAT", 0) * 64 / a.rounds / ds, 1)
        if k in busy:
            b = busy[k]
            wc = max(1.0, b.get("SQ_WAVE_CYCLES", 0))
            e["valu_active_frac_of_wave_cycles"] = round(b.get("SQ_ACTIVE_INST_VALU", 0) / wc, 3)
            e["issue_stall_frac"] = round(b.get("SQ_WAIT_INST_ANY", 0) / wc, 3)
            e["waitcnt_frac"] = round(b.get("SQ_WAIT_ANY", 0) / wc, 3)
            if b.get("_dur_ns"):
                e["effective_clock_ghz"] = round(b.get("GRBM_GUI_ACTIVE", 0) / 8 / b["_dur_ns"], 3)
        out[k] = e
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({k: v.get("hbm_bytes_per_round") for k, v in out.items() if k != "_meta"}))


if __name__ == "__main__":
    main()
