"""Child process for tests/test_gpu_parity.py::test_fixed_bisection_ladder: with DRANDHIP_BISECT set by the parent
(a fixed ladder of group sizes instead of the expected-cost choice), verifies a quicknet batch with 0.5% corrupted
rounds and prints the rejected indices and the expected set as JSON."""
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drand_amd import scheme_from_name  # noqa: E402

s = scheme_from_name("bls-unchained-g1-rfc9380")
sk = hashlib.sha256(b"ladder").digest()
n = 40000
rounds = np.arange(3, n + 3, dtype=np.uint64)
sigs = s.sign_beacons(sk, rounds)
pk = s.public_key(sk)
bad = np.sort(np.random.default_rng(4242).choice(n, size=n // 200, replace=False))
for k, i in enumerate(bad):
    if k % 2 == 0:
        sigs[i] = sigs[(i + 3) % n]
    else:
        sigs[i, 0] ^= 0x20
v, _ = s.verify_beacons(pk, rounds, sigs, seed=21)
print(json.dumps({"rejected": np.flatnonzero(~v).tolist(), "expected": bad.tolist()}))
