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
