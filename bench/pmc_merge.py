#!/usr/bin/env python3
"""Merge the PMC summaries of the two scheme families (bench/pmc_summary.py outputs) into the one file bench.py reads
for its traffic field, and point bench/workmodel.json at it.

    python bench/pmc_merge.py profiles/pmc_<tag>.json profiles/pmc_<tag>_g2.json bench/pmc_<tag>.json

Kernels both schemes run keep the quicknet entry under their name and the G2 one as '<name> [g2]';
k_prep_sig<fp2> / k_prep_msg<fp2> (the bench's stage names for the G2 passes) are the sums of their kernels."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    g1_path, g2_path, out_path = sys.argv[1:4]
    g1, g2 = json.load(open(g1_path)), json.load(open(g2_path))
    out = {"_meta": {"g1": g1.get("_meta"), "g2": g2.get("_meta"),
                     "_doc": "bench/pmc.sh passes (one 262,144-round single-stream batch per scheme) summarised by "
                             "bench/pmc_summary.py (%s, %s) and merged by bench/pmc_merge.py" % (g1_path, g2_path)}}
    for k, v in g1.items():
        if not k.startswith("_"):
            out[k] = v
    for k, v in g2.items():
        if not k.startswith("_"):
            out[k + " [g2]" if k in out else k] = v

    def stage(keys):
        return {"hbm_bytes_per_round": round(sum(g2[k]["hbm_bytes_per_round"] for k in keys), 1), "sum_of": keys}

    out["k_prep_sig<fp2>"] = stage(["k_dec_sig_g2", "k_sub_sig_g2"])
    out["k_prep_msg<fp2>"] = stage(["k_h2f_g2", "k_sswu_g2", "k_add_iso_g2"])
    with open(out_path, "w") as f:
        json.dump(out, f, indent=1)
    wm_path = os.path.join(HERE, "workmodel.json")
    wm = json.load(open(wm_path))
    wm["pmc_file"] = os.path.relpath(out_path, os.path.dirname(HERE))
    with open(wm_path, "w") as f:
        json.dump(wm, f, indent=2)
        f.write("\n")
    print(out_path, "k_prep_sig<fp>", out.get("k_prep_sig<fp>", {}).get("hbm_bytes_per_round"),
          "k_prep_sig<fp2>", out["k_prep_sig<fp2>"]["hbm_bytes_per_round"])


if __name__ == "__main__":
    main()
