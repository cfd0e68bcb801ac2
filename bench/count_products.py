#!/usr/bin/env python3
"""Field products each kernel EXECUTES per round, counted on the device (the basis of bench/workmodel.json).

Loads the counting build of the library (make -C drand_amd count -> libdrandhip_count.so: every Fp / 28-bit product
or squaring a lane executes bumps a device counter, read back after each profiled launch, fp_mul28.hpp
DH_COUNT_PRODUCTS) and runs one clean single-stream batch per scheme; products / rounds per stage. The counts are
executed work (the code path as built: 2-exponentiation Fp2 sqrt_ratio, cofactor clearing once per group,
endomorphism-split MSM ...), not the SURVEY's canonical per-algorithm model.

    DRANDHIP_LIB=drand_amd/libdrandhip_count.so python bench/count_products.py [--rounds 131072] [--out f.json]
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
R_ORDER = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001


def secret(tag):
    return (int.from_bytes(hashlib.sha256(tag).digest(), "big") % R_ORDER).to_bytes(32, "big")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, nargs="+", default=[131072])
    ap.add_argument("--recover-rounds", type=int, default=2048)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    os.environ.setdefault("DRANDHIP_LIB", os.path.join(ROOT, "drand_amd", "libdrandhip_count.so"))
    import torch
    from drand_amd import _lib, scheme_from_name
    lib = _lib.load()
    assert "count" in _lib.LIB_PATH, "needs the counting build (DRANDHIP_LIB=.../libdrandhip_count.so)"
    assert lib.dh_init(1) == 0, _lib.last_error()
    torch.zeros(1, device="cuda")
    dev = torch.device("cuda", 0)

    def prof():
        buf = ctypes.create_string_buffer(1 << 16)
        lib.dh_profile_read(buf, len(buf))
        return json.loads(buf.value.decode())

    out = {"_doc": __doc__.strip().splitlines()[0], "per_round": {}}
    for name in ("bls-unchained-g1-rfc9380", "pedersen-bls-unchained", "pedersen-bls-chained"):
        s = scheme_from_name(name)
        sk = secret(b"count-" + name.encode())
        pk = s.public_key(sk)
        for n in args.rounds:
            rounds = np.arange(1, n + 1, dtype=np.uint64)
            prevs = None
            if s.chained:
                prevs = np.random.default_rng(1).integers(0, 256, (n, 96), dtype=np.uint8)
                sigs = s.sign_beacons(sk, rounds, prevs)
            else:
                sigs = s.sign_beacons(sk, rounds)
            d_r = torch.from_numpy(rounds.view(np.int64)).to(dev)
            d_s = torch.from_numpy(sigs).to(dev)
            d_p = torch.from_numpy(prevs).to(dev) if prevs is not None else None
            d_v = torch.zeros(n, dtype=torch.uint8, device=dev)
            d_rand = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
            torch.cuda.synchronize()
            lib.dh_profile(1)
            rc = lib.dh_verify_batch_device(s.id, pk, len(pk), ctypes.c_void_p(d_r.data_ptr()),
                                            ctypes.c_void_p(d_s.data_ptr()), s.sig_len,
                                            ctypes.c_void_p(d_p.data_ptr()) if d_p is not None else None,
                                            96 if d_p is not None else 0, None, n, ctypes.c_void_p(d_v.data_ptr()),
                                            ctypes.c_void_p(d_rand.data_ptr()), 7, None, None)
            assert rc == 0, _lib.last_error()
            torch.cuda.synchronize()
            p = prof()
            lib.dh_profile(0)
            assert bool(d_v.all()), "clean batch rejected rounds"
            key = "%s/%d" % (name, n)
            out["per_round"][key] = {k: round(v["products"] / n, 2) for k, v in p.items()}
            out["per_round"][key]["_per_batch"] = {k: v["products"] for k, v in p.items()}
            print(key, out["per_round"][key], flush=True)
    # tbls Recover at the BASELINE shape n = 64, t = 33 (products per recovered round)
    s = scheme_from_name("pedersen-bls-unchained")
    n_nodes, t, nr = 64, 33, args.recover_rounds
    coeffs = [int.from_bytes(hashlib.sha256(b"count-poly-%d" % j).digest(), "big") % R_ORDER for j in range(t)]
    commits = [s.public_key(c.to_bytes(32, "big")) for c in coeffs]
    rounds = np.arange(1, nr + 1, dtype=np.uint64)
    shares = []
    for i in range(n_nodes):
        x, acc = i + 1, 0
        for c in reversed(coeffs):
            acc = (acc * x + c) % R_ORDER
        shares.append(s.sign_beacons(acc.to_bytes(32, "big"), rounds))
    msgs = [s.digest_beacon(int(r)) for r in rounds]
    rng = np.random.default_rng(5)
    # "first": signers 0 .. t-1 every round (configs[3]'s default); "random": a random t-subset per round (its variant:
    # every round its own Lagrange basis, the regular-window chains)
    for mode in ("first", "random"):
        ids = [list(range(t)) if mode == "first" else list(rng.permutation(n_nodes)[:t]) for _ in range(nr)]
        parts = [[int(i).to_bytes(2, "big") + shares[i][j].tobytes() for i in ids[j]] for j in range(nr)]
        lib.dh_profile(1)
        sigs, ok = s.recover_batch(commits, t, n_nodes, msgs, parts)
        p = prof()
        lib.dh_profile(0)
        assert ok.all()
        key = "tbls-recover-n64-t33%s/%d" % ("" if mode == "first" else "-random", nr)
        out["per_round"][key] = {k: round(v["products"] / nr, 2) for k, v in p.items()}
        print(key, out["per_round"][key], flush=True)
    line = json.dumps(out)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    print(line)


if __name__ == "__main__":
    main()
