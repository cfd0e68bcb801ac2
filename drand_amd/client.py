"""Client-side range verification over libdrandhip.

Mirrors verifyingClient (/root/reference/client/verify.go:95-199): `verify` checks one RandomData result
(optionally walking the chain from the point of trust in strict mode) and sets its randomness to
SHA-256(signature); the walk of getTrustedPreviousSignature (:109-168) is batched: every round between the
point of trust and the target is fetched, then the whole run is verified in one dh_verify_batch call instead of
one VerifyBeacon per round. Outcomes are the serial walk's: the first failing round (in round order) decides the
error, a fetch error only counts if every earlier round verified, and the point of trust advances only on
success.

One reference detail is kept as is: on the slow path (no usable point of trust) the walk starts from
trustRound = 1 with trustPrevSig = the genesis seed (:119-127), so round 2 is checked against the genesis seed.
"""
import numpy as np

from .chain import randomness_from_signature


class ClientError(Exception):
    pass


class BatchVerifyingClient:
    """`get_signature(round) -> bytes` plays the indirect client's Get; `info` is a chain.Info."""

    def __init__(self, info, scheme, get_signature=None, strict=False, seed=0):
        self.info = info
        self.scheme = scheme
        self.get_signature = get_signature
        self.strict = strict
        self.seed = seed
        self.point_of_trust = None  # (round, signature)

    def _verify_run(self, rounds, sigs, prevs):
        arr = np.zeros((len(sigs), self.scheme.sig_len), dtype=np.uint8)
        bad_len = np.zeros(len(sigs), dtype=bool)
        for i, s in enumerate(sigs):
            if len(s) == self.scheme.sig_len:
                arr[i] = np.frombuffer(bytes(s), np.uint8)
            else:
                bad_len[i] = True
        ok, _ = self.scheme.verify_beacons(self.info.public_key, np.array(rounds, dtype=np.uint64), arr,
                                           list(prevs) if self.scheme.chained else None, seed=self.seed,
                                           want_randomness=False)
        return np.asarray(ok, dtype=bool) & ~bad_len

    def trusted_previous_signature(self, round_):
        """getTrustedPreviousSignature (/root/reference/client/verify.go:109-168), batched."""
        if round_ == 1:
            return bytes(self.info.genesis_seed)
        pot = self.point_of_trust
        if pot is None or pot[0] > round_:
            trust_round, trust_prev = 1, self.trusted_previous_signature(1)
        else:
            trust_round, trust_prev = pot
        initial = trust_round
        rounds, sigs, fetch_err = [], [], None
        for r in range(trust_round + 1, round_):
            try:
                sigs.append(bytes(self.get_signature(r)))
            except Exception as e:  # noqa: BLE001 - any fetch failure ends the walk there
                fetch_err = ClientError("could not get round %d: %s" % (r, e))
                break
            rounds.append(r)
        if rounds:
            ok = self._verify_run(rounds, sigs, [trust_prev] + sigs[:-1])
            bad = np.flatnonzero(~ok)
            if len(bad):
                raise ClientError("verifying beacon: round %d" % rounds[bad[0]])
        if fetch_err is not None:
            raise fetch_err
        if rounds:
            trust_round, trust_prev = rounds[-1], sigs[-1]
        if trust_round == round_ - 1 and trust_round > initial:
            self.point_of_trust = (trust_round, trust_prev)
        if trust_round != round_ - 1:
            raise ClientError("unexpected trust round %d" % trust_round)
        return trust_prev

    def verify(self, record):
        """verifyingClient.verify (/root/reference/client/verify.go:171-199) for one RandomData dict
        {round, signature, previous_signature, randomness}; sets record["randomness"] on success."""
        self.verify_many([record], raise_first=True)

    def verify_many(self, records, raise_first=False):
        """verify() over many results; non-strict results are checked in ONE batch. Returns a list of
        None (valid) or ClientError per record."""
        errs = [None] * len(records)
        prevs = []
        for i, r in enumerate(records):
            ps = r.get("previous_signature", b"")
            if self.strict:
                try:
                    ps = self.trusted_previous_signature(int(r["round"]))
                except ClientError as e:
                    errs[i] = e
            prevs.append(ps)
        live = [i for i in range(len(records)) if errs[i] is None]
        if live:
            ok = self._verify_run([int(records[i]["round"]) for i in live], [records[i]["signature"] for i in live],
                                  [prevs[i] for i in live])
            for i, v in zip(live, ok):
                if v:
                    records[i]["randomness"] = randomness_from_signature(records[i]["signature"])
                else:
                    errs[i] = ClientError("verification of round %d failed" % int(records[i]["round"]))
        if raise_first:
            for e in errs:
                if e is not None:
                    raise e
        return errs


def marshal_random_data(rec):
    """encoding/json of client.RandomData (/root/reference/client/random.go:5-10): fields round, randomness,
    signature, previous_signature in that order, []byte as standard base64, zero values omitted (omitempty)."""
    import base64
    import json
    out = {}
    if int(rec.get("round", 0)):
        out["round"] = int(rec["round"])
    for key in ("randomness", "signature", "previous_signature"):
        v = bytes(rec.get(key) or b"")
        if v:
            out[key] = base64.b64encode(v).decode()
    return json.dumps(out, separators=(",", ":")).encode()


def relay_s3_sync(client, get_record, upload, begin, end, window=4096, log=None):
    """relay-s3 `sync` (/root/reference/cmd/relay-s3/main.go:182-195) with the per-round verify batched: rounds
    begin..end are fetched window by window (get_record(round) -> RandomData dict or raises, the verifying client's
    Get), every fetched window is verified in ONE batch (BatchVerifyingClient.verify_many: the same verdicts and
    randomness as verifyingClient.verify per round), and each verified round is uploaded as upload(key, body) with
    key "public/<round>" and body the JSON of client.RandomData. As in the reference, a failed fetch, verification or
    upload is logged and skipped (the loop goes on). Returns the uploaded rounds in order."""
    uploaded = []

    def note(*a):
        if log is not None:
            log(*a)

    for lo in range(int(begin), int(end) + 1, window):
        recs = []
        for rnd in range(lo, min(int(end), lo + window - 1) + 1):
            try:
                recs.append(dict(get_record(rnd)))
            except Exception as e:  # noqa: BLE001 - the reference logs and continues
                note("failed to get randomness", rnd, e)
        if not recs:
            continue
        errs = client.verify_many(recs)
        for rec, err in zip(recs, errs):
            if err is not None:
                note("failed to get randomness", rec.get("round"), err)
                continue
            try:
                upload("public/%d" % int(rec["round"]), marshal_random_data(rec))
            except Exception as e:  # noqa: BLE001
                note("failed to upload randomness", e)
                continue
            uploaded.append(int(rec["round"]))
    return uploaded
