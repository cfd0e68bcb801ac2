"""chain.Beacon mirror (/root/reference/chain/beacon.go:15-44) and RandomnessFromSignature
(/root/reference/crypto/schemes.go:249-252)."""
import hashlib
from dataclasses import dataclass


def randomness_from_signature(sig):
    """SHA-256 of the compressed signature (host helper; the batch path computes it on the device)."""
    return hashlib.sha256(bytes(sig)).digest()


@dataclass
class Beacon:
    round: int
    signature: bytes
    previous_signature: bytes = b""

    def get_round(self):
        return self.round

    def get_signature(self):
        return self.signature

    def get_previous_signature(self):
        return self.previous_signature

    def randomness(self):
        return randomness_from_signature(self.signature)


DEFAULT_BEACON_ID = "default"


def is_default_beacon_id(beacon_id):
    """common.IsDefaultBeaconID (/root/reference/common/beacon.go:27-29)."""
    return beacon_id in ("", DEFAULT_BEACON_ID)


@dataclass
class Info:
    """chain.Info (/root/reference/chain/info.go:19-26): what a client needs to verify a chain.

    The public key is kept as its compressed bytes; it is decoded (and subgroup-checked) by libdrandhip the
    first time a batch is verified against it (a bad key makes every verify call fail with DH_EKEY)."""
    public_key: bytes
    period: int  # seconds
    scheme: str
    genesis_time: int
    genesis_seed: bytes  # JSON "groupHash"
    id: str = ""

    def hash(self):
        """Info.Hash (/root/reference/chain/info.go:48-67): SHA-256(period_u32BE || genesis_i64BE || pk ||
        genesis seed [|| ID unless default])."""
        h = hashlib.sha256()
        h.update(int(self.period).to_bytes(4, "big"))
        h.update(int(self.genesis_time).to_bytes(8, "big", signed=True))
        h.update(bytes(self.public_key))
        h.update(bytes(self.genesis_seed))
        if not is_default_beacon_id(self.id):
            h.update(self.id.encode())
        return h.digest()

    def hash_string(self):
        return self.hash().hex()

    def to_json(self):
        """Info.ToJSON (/root/reference/chain/convert.go:73-76 via ToProto :36-56): ChainInfoPacket with
        hexjson byte fields."""
        import json
        return json.dumps({"public_key": bytes(self.public_key).hex(), "period": int(self.period),
                           "genesis_time": int(self.genesis_time), "hash": self.hash().hex(),
                           "groupHash": bytes(self.genesis_seed).hex(), "schemeID": self.scheme,
                           "metadata": {"beaconID": self.id}})


def info_from_json(text):
    """InfoFromJSON (/root/reference/chain/convert.go:58-70 -> InfoFromProto :15-34). Unknown scheme IDs are
    rejected; an empty schemeID means the default scheme (GetSchemeByIDWithDefault). Like the reference, the
    packet's own "hash" field is not trusted or checked here: callers compare Info.hash() with the chain hash
    they were configured with (client/client.go)."""
    import json
    from .scheme import get_scheme_by_id_with_default
    d = json.loads(text)
    sch = get_scheme_by_id_with_default(d.get("schemeID", ""))
    info = Info(public_key=bytes.fromhex(d.get("public_key", "")), period=int(d.get("period", 0)),
                scheme=sch.name, genesis_time=int(d.get("genesis_time", 0)),
                genesis_seed=bytes.fromhex(d.get("groupHash", "")),
                id=(d.get("metadata") or {}).get("beaconID", ""))
    if len(info.public_key) != sch.key_len:
        raise ValueError("invalid chain info: public key is %d bytes, scheme %s wants %d"
                         % (len(info.public_key), sch.name, sch.key_len))
    return info
