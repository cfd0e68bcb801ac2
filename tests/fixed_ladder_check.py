"""Child process for tests/test_gpu_parity.py::test_fixed_bisection_ladder: with DRANDHIP_BISECT set by the parent
(a fixed ladder of group sizes instead of the expected-cost choice) and DRANDHIP_SKIP_LEVEL0, verifies a quicknet batch with 0.5% corrupted rounds twice, then a G2 (pedersen-bls-unchained) batch with one forged round through the device entry point, and prints
the rejected indices, the expected sets and the G2 batch statistics as JSON."""
import hashlib
import json
import os
import sys

import numpy as np

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drand_amd import scheme_from_name  # noqa: E402

# torch carries its own HIP runtime: bring it up before the library's runtime has created its streams
torch.zeros(1, device="cuda")

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
out = {"rejected": np.flatnonzero(~v).tolist(), "expected": bad.tolist()}
# the same batch again: the worker's first bisection saw dense faults (0.5%), so this call skips level 0 and starts
# at the ladder's first size (unless DRANDHIP_SKIP_LEVEL0=0)
v2, _ = s.verify_beacons(pk, rounds, sigs, seed=22)
out["rejected_again"] = np.flatnonzero(~v2).tolist()

# G2: one forged round; every bisection level of the ladder must fail exactly one group (its group)
import ctypes  # noqa: E402
from drand_amd import _lib  # noqa: E402
lib = _lib.load()
g2 = scheme_from_name("pedersen-bls-unchained")
m = 3000
r2 = np.arange(1, m + 1, dtype=np.uint64)
s2 = g2.sign_beacons(sk, r2)
s2[1234] = s2[1235]
pk2 = g2.public_key(sk)
dev = torch.device("cuda", 0)
d_r, d_s = torch.from_numpy(r2.view(np.int64)).to(dev), torch.from_numpy(s2).to(dev)
d_v = torch.zeros(m, dtype=torch.uint8, device=dev)
stats = (ctypes.c_uint64 * 4)()
rc = lib.dh_verify_batch_device(g2.id, pk2, len(pk2), ctypes.c_void_p(d_r.data_ptr()), ctypes.c_void_p(d_s.data_ptr()),
                                g2.sig_len, None, 0, None, m, ctypes.c_void_p(d_v.data_ptr()), None, 7, None, stats)
assert rc == 0, _lib.last_error()
torch.cuda.synchronize()
out["g2_rejected"] = np.flatnonzero(d_v.cpu().numpy() == 0).tolist()
out["g2_stats"] = list(stats)
print(json.dumps(out))
