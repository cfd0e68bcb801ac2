"""Child process for tests/test_gpu_parity.py::test_one_lane_pairing_path: verifies the golden negative sets
with DRANDHIP_LANE_PAIRING=1 (the one-lane tower pairing of k_check.hip instead of the lane-parallel program)
and prints the verdict lists as JSON."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drand_amd import scheme_from_name  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
out = {}
# Recover first in a fresh process (no earlier verify call has sized the key buffers)
rc = json.load(open(os.path.join(GOLD, "recover.json")))["pedersen-bls-unchained"]
s = scheme_from_name("pedersen-bls-unchained")
sigs, ok = s.recover_batch([bytes.fromhex(x) for x in rc["commits"]], rc["t"], rc["n"],
                           [bytes.fromhex(x["msg"]) for x in rc["cases"]],
                           [[bytes.fromhex(p) for p in x["partials"]] for x in rc["cases"]])
out["recover"] = [sigs[k].tobytes().hex() if ok[k] else None for k in range(len(rc["cases"]))]
neg = json.load(open(os.path.join(GOLD, "negatives.json")))
for name in ("bls-unchained-g1-rfc9380", "pedersen-bls-chained"):
    c = neg[name]
    s = scheme_from_name(name)
    sigs = np.array([np.frombuffer(bytes.fromhex(x["sig"]), np.uint8) for x in c["cases"]])
    prevs = [bytes.fromhex(x["prev"]) for x in c["cases"]] if s.chained else None
    v, _ = s.verify_beacons(bytes.fromhex(c["pk"]), [x["round"] for x in c["cases"]], sigs, prevs, seed=3)
    out[name] = [bool(x) for x in v]
print(json.dumps(out))
