#!/usr/bin/env python3
"""Write the executed-work credits of bench/workmodel.json from a bench/count_products.py result.

    python bench/update_workmodel.py profiles/count_products_r03x.json

Every kernel's credit (kernel_units_M_per_round) becomes the field products it was COUNTED executing per round on
the device (the counting build, DH_COUNT_PRODUCTS), at the bench's 1,048,576-round batch for the per-round kernels
and the MSM, and at the recover run's shape for tbls; executed_M_per_beacon = prep_sig + prep_msg + MSM. The SURVEY's
canonical per-algorithm model (W_M_per_beacon, W_*_terms_M) is kept as is, for reference: it prices algorithms the
library does not execute as written (an Fp2 exponentiation per sqrt_ratio, cofactor clearing per round)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    src = sys.argv[1]
    counts = json.load(open(src))["per_round"]
    wm_path = os.path.join(HERE, "workmodel.json")
    wm = json.load(open(wm_path))

    def pick(prefix, n):
        key = "%s/%d" % (prefix, n)
        return counts[key]

    q = pick("bls-unchained-g1-rfc9380", 1048576)
    u = pick("pedersen-bls-unchained", 1048576)
    rec = next(v for k, v in counts.items() if k.startswith("tbls-recover-n64-t33/"))
    rec_r = next((v for k, v in counts.items() if k.startswith("tbls-recover-n64-t33-random/")), None)
    units = {
        "k_prep_sig<fp>": q["k_prep_sig<fp>"],
        "k_prep_msg<fp>": q["k_prep_msg<fp>"],
        "k_prep_sig<fp2>": u["k_prep_sig<fp2>"],
        "k_prep_msg<fp2>": u["k_prep_msg<fp2>"],
        "msm_level0": q["msm_level0"] + q.get("k_msm_prep28<fp>", 0.0),
        "msm_level0<fp2>": u["msm_level0"] + u.get("k_msm_prep28<fp2>", 0.0),
        "k_lagrange_t33": rec["k_lagrange"],
    }
    if rec_r is not None:  # random signer subsets: every round its own basis, the regular-window chains
        units["k_lagrange_t33_random"] = rec_r["k_lagrange"]
        units["k_wnaf_table_t33_random"] = rec_r.get("k_wnaf_table", 0.0)
    units["k_wnaf_table_t33"] = rec.get("k_wnaf_table", 0.0)
    wm["kernel_units_M_per_round"] = {k: round(v, 1) for k, v in units.items()}
    wm["executed_M_per_beacon"] = {
        "g1_sig": round(units["k_prep_sig<fp>"] + units["k_prep_msg<fp>"] + units["msm_level0"], 1),
        "g2_sig": round(units["k_prep_sig<fp2>"] + units["k_prep_msg<fp2>"] + units["msm_level0<fp2>"], 1),
    }
    wm["counts_source"] = os.path.relpath(src, os.path.dirname(HERE))
    wm["_doc_credit"] = ("kernel_units_M_per_round and executed_M_per_beacon are COUNTED executed field products per "
                         "round (bench/count_products.py on the counting build, 1,048,576-round batches; tbls at the "
                         "n = 64, t = 33 recover shape), one M = one Fp product or squaring = 300 mul32; the MSM's "
                         "count includes its point conversion (k_msm_prep28: lazy form, affine hash points, "
                         "endomorphism images), poison tests, bucket reduction and window Horner")
    wm.pop("_doc_k_lagrange", None)
    with open(wm_path, "w") as f:
        json.dump(wm, f, indent=2)
        f.write("\n")
    print(json.dumps(wm["kernel_units_M_per_round"]), json.dumps(wm["executed_M_per_beacon"]))


if __name__ == "__main__":
    main()
