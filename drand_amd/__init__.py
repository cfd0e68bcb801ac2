"""drand_amd — MI355X-native (gfx950) batch verification of drand beacons over BLS12-381.

The product is libdrandhip.so (hand-written HIP behind the C ABI in include/drandhip.h). This package
is the host-side mirror of the reference's crypto.Scheme surface (/root/reference/crypto/schemes.go)
over that ABI; see drand_amd.scheme.
"""
from .scheme import (  # noqa: F401
    Scheme,
    SchemeError,
    DeviceError,
    DeviceBusy,
    scheme_from_name,
    list_schemes,
    DEFAULT_SCHEME,
    UNCHAINED_SCHEME,
    SHORT_SIG_SCHEME,
    SIGS_ON_G1_SCHEME,
    hash_to_curve,
)
from .chain import Beacon, randomness_from_signature  # noqa: F401
