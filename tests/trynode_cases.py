"""tryNode + chain-store Put cases (test infrastructure, shared by the CPU and GPU tests).

The reference loop (/root/reference/chain/beacon/sync_manager.go:376-445) verifies each streamed beacon, then
Puts it through the chain store (chainstore.go:45-60: appendStore over schemeStore, store.go:55-77,99-124).
`serial_trynode` restates that loop and the two Put checks one packet at a time on the CPU oracle; the product
(drand_amd.sync.sync_from_stream over drand_amd.sync.ChainStore) must give the same (done, stored rounds) on every
case built by `cases`. Signatures are made with the oracle's signer, so any previous-signature linkage can be
forged validly.
"""
import hashlib

R_ORDER = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
GENESIS = hashlib.sha256(b"drandhip-genesis").digest()


def secret(name):
    return (int.from_bytes(hashlib.sha256(b"trynode-" + name.encode()).digest(), "big") % R_ORDER).to_bytes(32, "big")


def sign(oracle, name, sk, rnd, prev):
    return oracle.sign(name, sk, oracle.digest_beacon(name, rnd, prev if name == "pedersen-bls-chained" else b""))


def build_chain(oracle, name, n):
    """rounds 0..n: round 0 = the genesis seed record, round k signed over the stored signature of k-1 (chained)."""
    sk = secret(name)
    sig = {0: GENESIS}
    for r in range(1, n + 1):
        sig[r] = sign(oracle, name, sk, r, sig[r - 1])
    return sk, sig


def packet(name, sig, r, prev=None, **kw):
    chained = name == "pedersen-bls-chained"
    p = {"round": r, "signature": sig[r], "previous_signature": (sig[r - 1] if chained else b"") if prev is None else prev}
    p.update(kw)
    return p


def cases(oracle, name):
    """(label, base rounds stored (0..base), packets, up_to, resync) for one scheme. The chain has 12 rounds."""
    sk, sig = build_chain(oracle, name, 12)
    chained = name == "pedersen-bls-chained"
    P = lambda r, **kw: packet(name, sig, r, **kw)  # noqa: E731
    out = [("clean", 5, [P(r) for r in range(6, 11)], 10, False)]
    if chained:
        wrong = hashlib.sha256(b"another fork").digest() * 3
        forged7 = {"round": 7, "signature": sign(oracle, name, sk, 7, wrong), "previous_signature": wrong}
        out.append(("mislinked previous signature", 5, [P(6), forged7, P(8)], 10, False))
        other6 = {"round": 6, "signature": sign(oracle, name, sk, 6, wrong), "previous_signature": wrong}
        out.append(("duplicate round with another signature", 5, [P(6), other6, P(7)], 10, False))
    else:
        out.append(("duplicate of the last round carrying a previous signature", 5,
                    [P(5, prev=b"\x01" * 96), P(6)], 10, False))
        out.append(("stored beacon has its previous signature dropped", 5,
                    [P(6, prev=b"\x02" * 96), P(6, prev=b"\x02" * 96), P(7)], 10, False))
        other6 = {"round": 6, "signature": sign(oracle, name, secret("other key"), 6, b""), "previous_signature": b""}
        out.append(("duplicate round with an invalid signature", 5, [P(6), other6, P(7)], 10, False))
    out += [
        ("out-of-order round", 5, [P(6), P(8), P(9)], 10, False),
        ("duplicate of the last stored round, not up_to", 5, [P(5), P(6)], 10, False),
        ("duplicate of the last stored round at up_to", 5, [P(5), P(6)], 5, False),
        ("duplicate inside the stream", 5, [P(6), P(6), P(7)], 10, False),
        ("duplicate inside the stream at up_to", 5, [P(6), P(7), P(7), P(8)], 7, False),
        ("invalid signature", 5, [P(6), dict(P(7), signature=sig[9]), P(8)], 10, False),
        ("wrong beacon id", 5, [P(6), P(7, beacon_id="other"), P(8)], 10, False),
        ("resync: insecure store, no Put checks", 9, [P(3), P(4), P(12)], 12, True),
    ]
    return sig, out


def base_items(sig, base):
    return [(r, sig[r]) for r in range(0, base + 1)]


def serial_trynode(oracle, name, pk, items, packets, up_to, resync, beacon_id=""):
    """sync_manager.go:376-445 one packet at a time, with appendStore / schemeStore Put (store.go:55-124) over a
    trimmed store given as (round, signature) items. Returns (done, stored rounds, final store dict)."""
    chained = name == "pedersen-bls-chained"
    store = dict(items)
    last_round = max(store)
    last = {"round": last_round, "sig": store[last_round],
            "prev": store.get(last_round - 1, b"") if chained and last_round > 0 else b""}
    scheme_last_sig = last["sig"]
    stored = []
    for p in packets:
        if p.get("beacon_id") is not None and p["beacon_id"] != beacon_id:
            return False, stored, store
        rnd, s, prev = int(p["round"]), bytes(p["signature"]), bytes(p.get("previous_signature") or b"")
        if not oracle.verify_beacon(name, pk, rnd, s, prev if chained else b""):
            return False, stored, store
        if resync:
            store[rnd] = s
        else:
            if rnd == last["round"]:
                if last["sig"] == s and last["prev"] == prev:
                    return rnd == up_to, stored, store  # ErrBeaconAlreadyStored
                return False, stored, store
            if rnd != last["round"] + 1:
                return False, stored, store
            if chained:
                if scheme_last_sig != prev:
                    return False, stored, store
            else:
                prev = b""
            store[rnd] = s
            last = {"round": rnd, "sig": s, "prev": prev}
            scheme_last_sig = s
        stored.append(rnd)
        if rnd == up_to:
            return True, stored, store
    return False, stored, store
