#!/usr/bin/env python3
"""One-call throughput sweep (the drop-in callers' shape: ONE dh_verify_batch_device at a time): for each
(chunk rounds, workers) of the library's internal split, time K single calls over 1M quicknet rounds in HBM.

    python bench/split_sweep.py [--rounds 1048576] [--calls 4] [--grid 65536x8,131072x8,...]
Prints one JSON line per setting and a final line with the best."""
import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=1 << 20)
    ap.add_argument("--calls", type=int, default=4)
    ap.add_argument("--scheme", default="bls-unchained-g1-rfc9380")
    ap.add_argument("--grid", default="0x1,262144x3,262144x2,131072x3,131072x2,196608x3,524288x2")
    args = ap.parse_args()
    import torch
    from drand_amd import _lib, scheme_from_name
    torch.zeros(1, device="cuda")
    lib = _lib.load()
    assert lib.dh_init(1) == 0
    s = scheme_from_name(args.scheme)
    n = args.rounds
    sk = hashlib.sha256(b"sweep").digest()
    rounds = np.arange(1, n + 1, dtype=np.uint64)
    sigs = s.sign_beacons(sk, rounds)
    pk = s.public_key(sk)
    dev = torch.device("cuda", 0)
    d_r = torch.from_numpy(rounds.view(np.int64)).to(dev)
    d_s = torch.from_numpy(sigs).to(dev)
    d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    def call():
        rc = lib.dh_verify_batch_device(s.id, pk, len(pk), ctypes.c_void_p(d_r.data_ptr()), ctypes.c_void_p(d_s.data_ptr()),
                                        s.sig_len, None, 0, None, n, ctypes.c_void_p(d_v.data_ptr()), None, 0, None, None)
        assert rc == 0, _lib.last_error()

    best = None
    for item in args.grid.split(","):
        chunk, workers = (int(x) for x in item.split("x"))
        lib.dh_set_split(chunk, workers)
        call()
        call()  # warm every worker of this setting
        t0 = time.perf_counter()
        for _ in range(args.calls):
            call()
        dt = (time.perf_counter() - t0) / args.calls
        ok = bool(d_v.cpu().numpy().all())
        row = {"chunk": chunk, "workers": workers, "ms_per_call": round(dt * 1000, 2), "beacons_per_s": round(n / dt, 1),
               "verdicts_ok": ok}
        print(json.dumps(row), flush=True)
        if ok and (best is None or dt < best[0]):
            best = (dt, row)
    print(json.dumps({"best": best[1]}), flush=True)


if __name__ == "__main__":
    main()
