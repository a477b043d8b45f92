"""Independent ECDSA cross-check through OpenSSL libcrypto (ctypes) — test
infrastructure only.

OpenSSL is a second, independent implementation of the same ECDSA-over-
secp256k1 verification equation that ecdsa.Verify evaluates (Go 1.13,
steps 2-10), so it pins the oracle's math on well-formed items (r, s in
[1, N-1], uncompressed on-curve key).  It is NOT an oracle for the Go parsing
and panic semantics (it accepts compressed keys, has no base-36 text), which is
why only well-formed items are routed here.
"""
from __future__ import annotations

import ctypes
import ctypes.util
from typing import Optional

NID_secp256k1 = 714
_lib = None


def available() -> bool:
    try:
        _load()
        return True
    except OSError:
        return False


def _load():
    global _lib
    if _lib is not None:
        return _lib
    name = ctypes.util.find_library("crypto") or "libcrypto.so.3"
    L = ctypes.CDLL(name)
    L.EC_KEY_new_by_curve_name.restype = ctypes.c_void_p
    L.EC_KEY_new_by_curve_name.argtypes = [ctypes.c_int]
    L.EC_KEY_free.argtypes = [ctypes.c_void_p]
    L.o2i_ECPublicKey.restype = ctypes.c_void_p
    L.o2i_ECPublicKey.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_char_p), ctypes.c_long]
    L.BN_bin2bn.restype = ctypes.c_void_p
    L.BN_bin2bn.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p]
    L.ECDSA_SIG_new.restype = ctypes.c_void_p
    L.ECDSA_SIG_set0.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.ECDSA_SIG_free.argtypes = [ctypes.c_void_p]
    L.ECDSA_do_verify.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    L.ECDSA_do_verify.restype = ctypes.c_int
    _lib = L
    return L


def verify(pub65: bytes, digest: bytes, r: int, s: int) -> Optional[bool]:
    """ECDSA_do_verify on secp256k1; None if OpenSSL rejects the key encoding."""
    L = _load()
    key = ctypes.c_void_p(L.EC_KEY_new_by_curve_name(NID_secp256k1))
    buf = ctypes.c_char_p(bytes(pub65))
    res = L.o2i_ECPublicKey(ctypes.byref(key), ctypes.byref(buf), len(pub65))
    if not res:
        L.EC_KEY_free(key)
        return None
    sig = L.ECDSA_SIG_new()
    rb = L.BN_bin2bn(r.to_bytes(32, "big"), 32, None)
    sb = L.BN_bin2bn(s.to_bytes(32, "big"), 32, None)
    L.ECDSA_SIG_set0(sig, rb, sb)
    rv = L.ECDSA_do_verify(bytes(digest), len(digest), sig, key)
    L.ECDSA_SIG_free(sig)
    L.EC_KEY_free(key)
    if rv < 0:
        return None
    return rv == 1
