"""Generate the committed golden fixtures under tests/golden/ — run in the build container.

    python tests/golden/make_golden.py

Inputs and expected outputs come from the CPU oracle (oracle/liboracle.so, itself pinned by the
reference's known-answer tests /root/reference/crypto/schemes_test.go:81-130 and
/root/reference/crypto/curve_test.go:10-31, see tests/test_oracle.py) and from the pure-Python model
(oracle/bls_py.py) for hand-built invalid encodings. Synthetic chains follow the reference's mock
generator pattern (/root/reference/client/test/result/mock/result.go:84-127): one secret, chained
prev <- sig, genesis seed 32 bytes for round 1.

Output: tests/golden/chains.json (per scheme: sk, pk, rounds, sigs, prevs, expected verdicts,
randomness) and tests/golden/negatives.json (per scheme: malformed / wrong signatures with the
oracle's verdicts). Only data is written; nothing here ships with the product.
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import bls_py  # noqa: E402
import oracle_ctypes as orc  # noqa: E402

R = bls_py.R
P = bls_py.P
SCHEMES = ["pedersen-bls-chained", "pedersen-bls-unchained", "bls-unchained-on-g1", "bls-unchained-g1-rfc9380"]
GENESIS_SEED = hashlib.sha256(b"drandhip-genesis").digest()


def secret(scheme):
    """sk = SHA-256("drandhip-sk-" || scheme) mod r, as 32 big-endian bytes."""
    k = int.from_bytes(hashlib.sha256(b"drandhip-sk-" + scheme.encode()).digest(), "big") % R
    return k.to_bytes(32, "big")


def chain(scheme, n, start=1):
    sk = secret(scheme)
    pk = orc.public_key(scheme, sk)
    chained = scheme == "pedersen-bls-chained"
    rounds, sigs, prevs = [], [], []
    prev = GENESIS_SEED if start == 1 else b""
    for r in range(start, start + n):
        p = prev if chained else b""
        msg = orc.digest_beacon(scheme, r, p)
        s = orc.sign(scheme, sk, msg)
        rounds.append(r)
        sigs.append(s)
        prevs.append(p)
        prev = s
    return sk, pk, rounds, sigs, prevs


def non_subgroup_g1(rng):
    while True:
        x = rng.randrange(P)
        y = bls_py.fsqrt(x * x * x + 4)
        if y is None:
            continue
        pt = (x, y)
        if bls_py.ec_mul(bls_py.FP, pt, R) is not None:
            return bls_py.g1_compress(pt)


def non_subgroup_g2(rng):
    while True:
        x = (rng.randrange(P), rng.randrange(P))
        y = bls_py.f2sqrt(bls_py.f2add(bls_py.f2mul(bls_py.f2sqr(x), x), bls_py.B2))
        if y is None:
            continue
        pt = (x, y)
        if bls_py.ec_mul(bls_py.FP2, pt, R) is not None:
            return bls_py.g2_compress(pt)


def negatives(scheme, sk, pk, rng):
    """(name, round, sig, prev) cases; expected verdicts come from the oracle."""
    g2sig = scheme in ("pedersen-bls-chained", "pedersen-bls-unchained")
    slen = 96 if g2sig else 48
    chained = scheme == "pedersen-bls-chained"
    prev = hashlib.sha256(b"prev").digest() * 3 if chained else b""  # 96 bytes
    r = 4242
    good = orc.sign(scheme, sk, orc.digest_beacon(scheme, r, prev))
    cases = [("valid", r, good, prev), ("wrong_round", r + 1, good, prev)]
    flip = bytearray(good)
    flip[slen // 2] ^= 0x10
    cases.append(("bit_flip", r, bytes(flip), prev))
    flip = bytearray(good)
    flip[0] ^= 0x20  # sign bit: the negated point
    cases.append(("sign_flag_flip", r, bytes(flip), prev))
    noc = bytearray(good)
    noc[0] &= 0x7F
    cases.append(("no_compression_flag", r, bytes(noc), prev))
    inf = bytes([0xC0]) + bytes(slen - 1)
    cases.append(("infinity", r, inf, prev))
    badinf = bytes([0xC0]) + bytes(slen - 2) + b"\x01"
    cases.append(("bad_infinity", r, badinf, prev))
    big = bytearray(P.to_bytes(48, "big"))
    big[0] |= 0x80
    cases.append(("x_eq_p", r, bytes(big) + (bytes(48) if g2sig else b""), prev))
    cases.append(("all_ff", r, b"\xff" * slen, prev))
    nsg = non_subgroup_g2(rng) if g2sig else non_subgroup_g1(rng)
    cases.append(("non_subgroup", r, nsg, prev))
    other = orc.sign(scheme, sk, orc.digest_beacon(scheme, r + 7, prev))
    cases.append(("other_rounds_sig", r, other, prev))
    if chained:
        cases.append(("wrong_prev", r, good, hashlib.sha256(b"other").digest() * 3))
        cases.append(("empty_prev", r, good, b""))
    out = []
    for name, rr, s, p in cases:
        v = orc.verify_beacon(scheme, pk, rr, s, p)
        out.append({"name": name, "round": rr, "sig": s.hex(), "prev": p.hex(), "valid": bool(v)})
    assert out[0]["valid"], scheme
    return out


def recover_fixture(scheme, t, n, rounds, rng):
    """Dealer polynomial -> commits, shares; per round a list of partials in arrival order, some invalid,
    expected outputs from the oracle's restatement of kyber tbls.Recover + share.RecoverCommit."""
    coeffs = [int.from_bytes(hashlib.sha256(b"tbls-%s-%d" % (scheme.encode(), j)).digest(), "big") % R for j in range(t)]
    commits = [orc.public_key(scheme, c.to_bytes(32, "big")) for c in coeffs]

    def share(i):  # f(i + 1)
        x, acc = i + 1, 0
        for c in reversed(coeffs):
            acc = (acc * x + c) % R
        return acc.to_bytes(32, "big")

    cases = []
    for k, r in enumerate(rounds):
        msg = orc.digest_beacon(scheme, r, b"")
        ids = rng.sample(range(n), t + 2)
        parts = [i.to_bytes(2, "big") + orc.sign(scheme, share(i), msg) for i in ids]
        if k % 4 == 1:   # an invalid partial first: skipped, the t valid ones after it are used
            bad = bytearray(parts[0]); bad[5] ^= 1; parts[0] = bytes(bad)
        if k % 4 == 2:   # duplicate of an index and an out-of-range index
            parts.insert(1, parts[0])
            parts.insert(2, (n + 3).to_bytes(2, "big") + parts[3][2:])
        if k % 4 == 3:   # too few valid partials -> error
            parts = parts[: t - 1]
        got = orc.recover(scheme, commits, t, n, msg, parts)
        if got is not None:
            assert got == orc.sign(scheme, coeffs[0].to_bytes(32, "big"), msg)
        cases.append({"round": r, "msg": msg.hex(), "partials": [p.hex() for p in parts],
                      "expected": got.hex() if got else None})
    return {"t": t, "n": n, "commits": [c.hex() for c in commits], "group_key": commits[0].hex(), "cases": cases}


def main():
    rng = random.Random(20250117)
    chains, negs = {}, {}
    for scheme in SCHEMES:
        sk, pk, rounds, sigs, prevs = chain(scheme, 24)
        verdicts = [orc.verify_beacon(scheme, pk, r, s, p) for r, s, p in zip(rounds, sigs, prevs)]
        assert all(verdicts), scheme
        chains[scheme] = {
            "sk": sk.hex(), "pk": pk.hex(), "rounds": rounds, "sigs": [s.hex() for s in sigs],
            "prevs": [p.hex() for p in prevs], "valid": [bool(v) for v in verdicts],
            "randomness": [hashlib.sha256(s).hexdigest() for s in sigs],
        }
        negs[scheme] = {"pk": pk.hex(), "cases": negatives(scheme, sk, pk, rng)}
        print(scheme, "ok", [c["name"] for c in negs[scheme]["cases"] if c["valid"]])
    # corrupted chained mini-chain: stored sig of round 10 replaced by round 9's -> rounds 10 and 11 faulty
    # (chained replay uses the stored previous signature, /root/reference/chain/boltdb/trimmed.go:183,
    # faulty-count rule /root/reference/core/drand_test.go:1105-1111)
    c = chains["pedersen-bls-chained"]
    sigs = [bytes.fromhex(s) for s in c["sigs"]]
    stored = list(sigs)
    stored[9] = sigs[8]
    prevs = [GENESIS_SEED] + stored[:-1]
    pk = bytes.fromhex(c["pk"])
    verdicts = [orc.verify_beacon("pedersen-bls-chained", pk, r, s, p) for r, s, p in zip(c["rounds"], stored, prevs)]
    faulty = [r for r, v in zip(c["rounds"], verdicts) if not v]
    assert faulty == [10, 11], faulty
    replay = {"pk": c["pk"], "rounds": c["rounds"], "stored_sigs": [s.hex() for s in stored],
              "genesis_seed": GENESIS_SEED.hex(), "faulty": faulty}
    rec = {s_: recover_fixture(s_, 5, 9, list(range(100, 108)), rng)
           for s_ in ("pedersen-bls-unchained", "bls-unchained-g1-rfc9380")}
    with open(os.path.join(HERE, "recover.json"), "w") as f:
        json.dump(rec, f, indent=1)
    with open(os.path.join(HERE, "chains.json"), "w") as f:
        json.dump(chains, f, indent=1)
    with open(os.path.join(HERE, "negatives.json"), "w") as f:
        json.dump(negs, f, indent=1)
    with open(os.path.join(HERE, "replay.json"), "w") as f:
        json.dump(replay, f, indent=1)
    print("wrote fixtures")


if __name__ == "__main__":
    main()
