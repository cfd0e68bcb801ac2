"""Child process of test_gpu_pack.test_packed_checks (DRANDHIP_VM_PACK, DRANDHIP_BISECT and DRANDHIP_NP2C are read once
per process): faulty batches of a G1 and a G2 scheme whose bisection runs every group check and leaf launch of two or
more checks through the two-checks-per-wave kernels (DRANDHIP_VM_PACK=2), with a fixed ladder that gives odd and even
check counts per launch and undecodable rounds among the leaves (the packed kernels' one-check fallback). Prints one
JSON line per scheme: the rejected rounds, the corrupted ones and the bisection stats."""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from drand_amd import _lib, scheme_from_name
    lib = _lib.load()
    assert lib.dh_init(1) == 0, _lib.last_error()
    n = 3000
    rng = np.random.default_rng(7)
    for name in ("bls-unchained-g1-rfc9380", "pedersen-bls-unchained"):
        s = scheme_from_name(name)
        sk = hashlib.sha256(b"vmpack" + name.encode()).digest()
        rounds = np.arange(1, n + 1, dtype=np.uint64)
        sigs = s.sign_beacons(sk, rounds)
        pk = s.public_key(sk)
        bad = sorted(set(int(x) for x in rng.choice(n - 1, 45, replace=False)))
        for k, i in enumerate(bad):
            if k % 3 == 0:
                sigs[i] = sigs[i + 1]        # a valid point, the wrong round: fails its pairing check
            elif k % 3 == 1:
                sigs[i, 7] ^= 0x10           # x off the curve (or off the subgroup): rejected at decode
            else:
                sigs[i, 0] ^= 0x20           # the sign flag: the negated point, fails its pairing check
        v, _ = s.verify_beacons(pk, rounds, sigs, seed=11)
        stats = s.last_stats if hasattr(s, "last_stats") else None
        print(json.dumps({"scheme": name, "rejected": np.flatnonzero(~v).tolist(), "expected": bad, "stats": stats}),
              flush=True)


if __name__ == "__main__":
    main()
