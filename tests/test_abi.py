"""CPU: the C-ABI library loads and exports every symbol include/drandhip.h declares; host-only entry
points (no device work) behave like the reference's crypto package."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "drand_amd", "libdrandhip.so")


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "drandhip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(dh_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ["dh_init", "dh_verify_batch", "dh_verify_batch_device", "dh_verify_beacon", "dh_recover_batch",
              "dh_randomness_batch", "dh_scheme_from_name", "dh_last_error_string"]:
        assert s in syms


@pytest.mark.skipif(not os.path.exists(LIB), reason="libdrandhip.so not built")
def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    for s in declared_symbols():
        assert hasattr(lib, s), s
    from drand_amd import _lib
    assert set(_lib.SIGNATURES) == set(declared_symbols())


@pytest.mark.skipif(not os.path.exists(LIB), reason="libdrandhip.so not built")
def test_scheme_registry_host_only():
    from drand_amd import _lib, scheme_from_name, list_schemes, SchemeError
    lib = _lib.load()
    for i, name in enumerate(["pedersen-bls-chained", "pedersen-bls-unchained", "bls-unchained-on-g1",
                              "bls-unchained-g1-rfc9380"]):
        assert lib.dh_scheme_from_name(name.encode()) == i
        s = scheme_from_name(name)
        assert s.id == i and lib.dh_sig_len(i) == s.sig_len and lib.dh_key_len(i) == s.key_len
    assert lib.dh_scheme_from_name(b"nope") == _lib.DH_EINVAL
    assert "invalid scheme name 'nope'" in _lib.last_error()
    assert lib.dh_sig_len(7) == _lib.DH_EINVAL
    assert len(list_schemes()) == 4
    with pytest.raises(SchemeError, match="invalid scheme name"):
        scheme_from_name("bogus")


@pytest.mark.skipif(not os.path.exists(LIB), reason="libdrandhip.so not built")
def test_digest_beacon_host_matches_oracle(oracle):
    """crypto.Scheme.DigestBeacon (schemes.go:106-114,147-151,187-191) through the C ABI (host SHA-256)."""
    from drand_amd import scheme_from_name
    rng = np.random.default_rng(1)
    for name in ["pedersen-bls-chained", "pedersen-bls-unchained", "bls-unchained-on-g1", "bls-unchained-g1-rfc9380"]:
        s = scheme_from_name(name)
        for rnd in [0, 1, 2634945, 2 ** 63 + 5]:
            for plen in [0, 32, 96]:
                prev = rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
                want = oracle.digest_beacon(name, rnd, prev if s.chained else b"")
                assert s.digest_beacon(rnd, prev if s.chained else b"") == want
