"""VM phase profile: run with DRANDHIP_LIB pointing at a library whose k_vm.hip was built with -DDH_VM_PROF; the
first workgroup of every k_vm_pairing launch prints the wall-clock ticks (100 MHz) spent per phase kind."""
import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drand_amd import _lib, scheme_from_name  # noqa: E402

lib = _lib.load()
assert lib.dh_init(1) == 0
for name in ("bls-unchained-g1-rfc9380", "pedersen-bls-unchained"):
    s = scheme_from_name(name)
    sk = hashlib.sha256(b"vmprof").digest()
    rounds = np.arange(1, 4097, dtype=np.uint64)
    sigs = s.sign_beacons(sk, rounds)
    pk = s.public_key(sk)
    for rep in range(2):
        v, _ = s.verify_beacons(pk, rounds, sigs, seed=rep + 1)
        assert v.all()
    print(name, "ok", flush=True)
