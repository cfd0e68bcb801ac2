"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; never by the
product package. Builds liboracle.so on first use if it is missing and gcc is present.
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

SCHEME_IDS = {
    "pedersen-bls-chained": 0,
    "pedersen-bls-unchained": 1,
    "bls-unchained-on-g1": 2,
    "bls-unchained-g1-rfc9380": 3,
}
SIG_LEN = {0: 96, 1: 96, 2: 48, 3: 48}
KEY_LEN = {0: 48, 1: 48, 2: 96, 3: 96}

_lib = None


def build():
    src = os.path.join(HERE, "bls_oracle.c")
    if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE])


def lib(fast_subgroup=False):
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(LIB_PATH)
        c = ctypes
        _lib.or_verify.argtypes = [c.c_int, c.c_char_p, c.c_size_t, c.c_char_p, c.c_size_t, c.c_char_p, c.c_size_t]
        _lib.or_verify_beacon.argtypes = [c.c_int, c.c_char_p, c.c_size_t, c.c_uint64, c.c_char_p, c.c_size_t,
                                          c.c_char_p, c.c_size_t]
        _lib.or_sign.argtypes = [c.c_int, c.c_char_p, c.c_char_p, c.c_size_t, c.c_char_p]
        _lib.or_public_key.argtypes = [c.c_int, c.c_char_p, c.c_char_p]
        _lib.or_hash_to_curve.argtypes = [c.c_int, c.c_char_p, c.c_size_t, c.c_char_p, c.c_size_t, c.c_char_p]
        _lib.or_decode.argtypes = [c.c_int, c.c_char_p]
        _lib.or_expand_message_xmd.argtypes = [c.c_char_p, c.c_size_t, c.c_char_p, c.c_size_t, c.c_char_p, c.c_size_t]
        _lib.or_sha256.argtypes = [c.c_char_p, c.c_char_p, c.c_size_t]
        _lib.or_digest_beacon.argtypes = [c.c_char_p, c.c_int, c.c_uint64, c.c_char_p, c.c_size_t]
        _lib.or_verify_batch.argtypes = [c.c_int, c.c_char_p, c.c_size_t, c.c_void_p, c.c_void_p, c.c_size_t,
                                         c.c_void_p, c.c_size_t, c.c_void_p, c.c_size_t, c.c_int, c.c_void_p,
                                         c.c_void_p]
        _lib.or_recover.argtypes = [c.c_int, c.c_char_p, c.c_int, c.c_int, c.c_char_p, c.c_size_t, c.c_char_p,
                                    c.c_int, c.c_char_p]
        _lib.or_pubpoly_eval.argtypes = [c.c_int, c.c_char_p, c.c_int, c.c_int, c.c_char_p]
        _lib.or_init.argtypes = [c.c_int]
    _lib.or_init(1 if fast_subgroup else 0)
    return _lib


def sid(scheme):
    return SCHEME_IDS[scheme] if isinstance(scheme, str) else int(scheme)


def verify(scheme, pk, msg, sig):
    return bool(lib().or_verify(sid(scheme), pk, len(pk), msg, len(msg), sig, len(sig)))


def verify_beacon(scheme, pk, round_, sig, prev=b""):
    return bool(lib().or_verify_beacon(sid(scheme), pk, len(pk), round_, sig, len(sig), prev, len(prev)))


def digest_beacon(scheme, round_, prev=b""):
    out = ctypes.create_string_buffer(32)
    lib().or_digest_beacon(out, sid(scheme), round_, prev, len(prev))
    return out.raw


def sign(scheme, sk32, msg):
    s = sid(scheme)
    out = ctypes.create_string_buffer(SIG_LEN[s])
    lib().or_sign(s, sk32, msg, len(msg), out)
    return out.raw


def public_key(scheme, sk32):
    s = sid(scheme)
    out = ctypes.create_string_buffer(KEY_LEN[s])
    lib().or_public_key(s, sk32, out)
    return out.raw


def hash_to_curve(g2, msg, dst):
    out = ctypes.create_string_buffer(96 if g2 else 48)
    lib().or_hash_to_curve(1 if g2 else 0, msg, len(msg), dst, len(dst), out)
    return out.raw


def decode(g2, b):
    return lib().or_decode(1 if g2 else 0, b)


def expand_message_xmd(msg, dst, n):
    out = ctypes.create_string_buffer(n)
    lib().or_expand_message_xmd(out, n, msg, len(msg), dst, len(dst))
    return out.raw


def sha256(b):
    out = ctypes.create_string_buffer(32)
    lib().or_sha256(out, b, len(b))
    return out.raw


def verify_batch(scheme, pk, rounds, sigs, prevs=None, nthreads=1, want_rand=True, fast_subgroup=False):
    """rounds: uint64 numpy array; sigs: (n, siglen) uint8; prevs: (n, plen) uint8 or None."""
    import numpy as np
    s = sid(scheme)
    lib(fast_subgroup)
    n = len(rounds)
    rounds = np.ascontiguousarray(rounds, dtype=np.uint64)
    sigs = np.ascontiguousarray(sigs, dtype=np.uint8)
    verdict = np.zeros(n, dtype=np.uint8)
    rand = np.zeros((n, 32), dtype=np.uint8) if want_rand else None
    pv = None
    pstride = 0
    if prevs is not None:
        prevs = np.ascontiguousarray(prevs, dtype=np.uint8)
        pv = prevs.ctypes.data
        pstride = prevs.shape[1]
    lib().or_verify_batch(s, pk, len(pk), rounds.ctypes.data, sigs.ctypes.data, sigs.shape[1], pv, pstride, None, n,
                          nthreads, verdict.ctypes.data, rand.ctypes.data if rand is not None else None)
    lib(False)
    return verdict, rand


def recover(scheme, commits, t, n, msg, partials):
    s = sid(scheme)
    out = ctypes.create_string_buffer(SIG_LEN[s])
    blob = b"".join(partials)
    rc = lib().or_recover(s, b"".join(commits), t, n, msg, len(msg), blob, len(partials), out)
    return out.raw if rc > 0 else None


def pubpoly_eval(scheme, commits, index):
    s = sid(scheme)
    out = ctypes.create_string_buffer(KEY_LEN[s])
    rc = lib().or_pubpoly_eval(s, b"".join(commits), len(commits), index, out)
    return out.raw if rc > 0 else None
