"""Child process of test_gpu_paths.test_single_call_split (DRANDHIP_SPLIT is read once per process): one host-buffer
call and one device-buffer call (inputs produced on a torch stream, handed over as hip_stream) over 60 000 quicknet
rounds, each split by the library into chunks on several internal streams. Prints one JSON line."""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from drand_amd import _lib, scheme_from_name
    lib = _lib.load()
    assert lib.dh_init(1) == 0, _lib.last_error()
    s = scheme_from_name("bls-unchained-g1-rfc9380")
    sk = hashlib.sha256(b"split").digest()
    n = 60000
    rounds = np.arange(1, n + 1, dtype=np.uint64)
    sigs = s.sign_beacons(sk, rounds)
    pk = s.public_key(sk)
    bad = [5, 5999, 6000, 17777, 59999]
    for k, i in enumerate(bad):
        if k % 2:
            sigs[i, 0] ^= 0x20
        else:
            sigs[i] = sigs[(i + 1) % n]
    v, rand = s.verify_beacons(pk, rounds, sigs, seed=0)
    rand_ok = all(rand[i].tobytes() == hashlib.sha256(sigs[i].tobytes()).digest() for i in (0, 5999, 6000, n - 1))
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(st):  # inputs produced on the caller's stream
        d_r = torch.from_numpy(rounds.view(np.int64)).to(dev, non_blocking=True)
        d_s = torch.from_numpy(sigs).to(dev, non_blocking=True)
        d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
    stats = (ctypes.c_uint64 * 4)()
    rc = lib.dh_verify_batch_device(s.id, pk, len(pk), ctypes.c_void_p(d_r.data_ptr()), ctypes.c_void_p(d_s.data_ptr()),
                                    s.sig_len, None, 0, None, n, ctypes.c_void_p(d_v.data_ptr()), None, 3,
                                    ctypes.c_void_p(st.cuda_stream), stats)
    assert rc == 0, _lib.last_error()
    dv = d_v.cpu().numpy()
    print(json.dumps({"rejected": np.flatnonzero(~v).tolist(), "device_rejected": np.flatnonzero(dv == 0).tolist(),
                      "expected": bad, "rand_ok": rand_ok, "stats": list(stats)}))


if __name__ == "__main__":
    main()
