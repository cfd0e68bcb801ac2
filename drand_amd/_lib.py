"""ctypes binding of libdrandhip.so (the product library).

The library is built in-tree by `make -C drand_amd` (or __graft_entry__.build()). There is no CPU
fallback: if the library or the GPU is missing, calls raise. The CPU oracle under oracle/ is test
infrastructure and is never imported here.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DRANDHIP_LIB") or os.path.join(HERE, "libdrandhip.so")

DH_OK = 0
DH_EINVAL = -1
DH_EDEVICE = -2
DH_ENOMEM = -3
DH_EKEY = -4
DH_ERECOVER = -5
DH_EBUSY = -6
DH_EABANDONED = -7
DH_NODE_CHECKED = 2

# every symbol declared in include/drandhip.h, with (restype, argtypes)
_c = ctypes
_P = _c.c_void_p
SIGNATURES = {
    "dh_init": (_c.c_int, [_c.c_uint32]),
    "dh_shutdown": (None, []),
    "dh_scheme_from_name": (_c.c_int, [_c.c_char_p]),
    "dh_sig_len": (_c.c_int, [_c.c_int]),
    "dh_key_len": (_c.c_int, [_c.c_int]),
    "dh_verify_batch": (_c.c_int, [_c.c_int, _c.c_char_p, _c.c_size_t, _P, _P, _c.c_size_t, _P, _c.c_size_t, _P,
                                   _c.c_size_t, _P, _P, _c.c_uint64]),
    "dh_verify_batch_device": (_c.c_int, [_c.c_int, _c.c_char_p, _c.c_size_t, _P, _P, _c.c_size_t, _P, _c.c_size_t,
                                          _P, _c.c_size_t, _P, _P, _c.c_uint64, _P, _P]),
    "dh_verify_beacon": (_c.c_int, [_c.c_int, _c.c_char_p, _c.c_size_t, _c.c_uint64, _c.c_char_p, _c.c_size_t,
                                    _c.c_char_p, _c.c_size_t]),
    "dh_verify_recovered": (_c.c_int, [_c.c_int, _c.c_char_p, _c.c_size_t, _c.c_char_p, _c.c_char_p, _c.c_size_t]),
    "dh_verify_recovered_batch": (_c.c_int, [_c.c_int, _c.c_char_p, _c.c_size_t, _P, _P, _c.c_size_t, _c.c_size_t, _P,
                                             _c.c_uint64]),
    "dh_digest_batch": (_c.c_int, [_c.c_int, _P, _P, _c.c_size_t, _P, _c.c_size_t, _P]),
    "dh_randomness_batch": (_c.c_int, [_c.c_int, _P, _c.c_size_t, _c.c_size_t, _P]),
    "dh_recover_batch": (_c.c_int, [_c.c_int, _c.c_char_p, _c.c_int, _c.c_int, _P, _P, _P, _c.c_size_t, _P, _P]),
    "dh_verify_partials_batch": (_c.c_int, [_c.c_int, _c.c_char_p, _c.c_int, _c.c_int, _P, _P, _P, _c.c_size_t, _P]),
    "dh_sign_batch": (_c.c_int, [_c.c_int, _c.c_char_p, _P, _P, _c.c_size_t, _P, _c.c_size_t, _P]),
    "dh_public_key": (_c.c_int, [_c.c_int, _c.c_char_p, _P]),
    "dh_partial_bytes": (_c.c_int, [_c.c_int]),
    "dh_set_split": (_c.c_int, [_c.c_uint64, _c.c_int]),
    "dh_hash_to_curve": (_c.c_int, [_c.c_int, _P, _P, _c.c_size_t, _c.c_char_p, _c.c_size_t, _P]),
    "dh_batch_begin": (_c.c_int, [_c.c_int, _c.c_char_p, _c.c_size_t, _P, _P, _c.c_size_t, _P, _c.c_size_t, _P,
                                  _c.c_size_t, _P, _P, _c.c_uint64, _P, _c.POINTER(_P), _P]),
    "dh_batch_check": (_c.c_int, [_P, _P, _c.c_size_t, _P]),
    "dh_batch_stream": (_P, [_P]),
    "dh_check_partials": (_c.c_int, [_c.c_int, _c.c_char_p, _c.c_size_t, _P, _c.c_size_t, _c.POINTER(_c.c_int)]),
    "dh_batch_finish": (_c.c_int, [_P, _c.c_int, _P]),
    "dh_profile": (_c.c_int, [_c.c_int]),
    "dh_profile_read": (_c.c_int, [_c.c_char_p, _c.c_size_t]),
    "dh_last_error_string": (_c.c_char_p, []),
    "dh_version": (_c.c_char_p, []),
}

_lib = None


class LibraryMissing(RuntimeError):
    pass


def load():
    """Load libdrandhip.so (no build, no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LibraryMissing(
            "libdrandhip.so not found at %s: build it with `make -C drand_amd` or __graft_entry__.build()" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error():
    return (load().dh_last_error_string() or b"").decode()
