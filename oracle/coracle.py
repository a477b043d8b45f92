"""CPU ORACLE (ctypes wrapper of oracle/oracle.c) — test infrastructure only.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker; never by the product path.  See oracle/oracle.c for the reference
call sites it restates.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


class _Batch(ctypes.Structure):
    # Mirrors bv_batch (include/babbleverify.h).
    _fields_ = [
        ("n_msgs", ctypes.c_uint64),
        ("msg_bytes", ctypes.c_void_p),
        ("msg_off", ctypes.c_void_p),
        ("n_keys", ctypes.c_uint32),
        ("key_bytes", ctypes.c_void_p),
        ("key_off", ctypes.c_void_p),
        ("n_items", ctypes.c_uint64),
        ("item_msg", ctypes.c_void_p),
        ("item_key", ctypes.c_void_p),
        ("r_be", ctypes.c_void_p),
        ("s_be", ctypes.c_void_p),
        ("pre", ctypes.c_void_p),
    ]


def default_threads() -> int:
    """Host threads the oracle may use: this process's CPU affinity, capped at
    16 (the GPU box's CPU share per GPU)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_sha256.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_item_status.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint8,
                                         ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_item_status.restype = ctypes.c_int
        L.oracle_verify_batch.argtypes = [ctypes.POINTER(_Batch), ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_int]
        L.oracle_unmarshal.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_scalar_base_mult.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_init.argtypes = []
        L.port_verify_batch.argtypes = [ctypes.POINTER(_Batch), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.port_verify_batch.restype = ctypes.c_int
        _lib = L
    return _lib


def sha256(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    buf = ctypes.create_string_buffer(bytes(data), len(data) + 1)
    lib().oracle_sha256(buf, len(data), out)
    return out.raw


def item_status(pub: bytes, digest: bytes, pre: int, r_be: bytes, s_be: bytes) -> int:
    pb = ctypes.create_string_buffer(bytes(pub), len(pub) + 1)
    return lib().oracle_item_status(pb, len(pub), bytes(digest), pre, bytes(r_be), bytes(s_be))


def scalar_base_mult(k: int):
    out = ctypes.create_string_buffer(64)
    ok = lib().oracle_scalar_base_mult(k.to_bytes(32, "big"), out)
    if not ok:
        return None
    return int.from_bytes(out.raw[:32], "big"), int.from_bytes(out.raw[32:], "big")


def _cbatch(arrs: dict, keep: list) -> _Batch:
    def ptr(a):
        a = np.ascontiguousarray(a)
        keep.append(a)
        return a.ctypes.data if a.size else 0

    b = _Batch()
    b.n_msgs = len(arrs["msg_off"]) - 1
    b.msg_bytes = ptr(arrs["msg_bytes"])
    b.msg_off = ptr(arrs["msg_off"].astype(np.uint64))
    b.n_keys = len(arrs["key_off"]) - 1
    b.key_bytes = ptr(arrs["key_bytes"])
    b.key_off = ptr(arrs["key_off"].astype(np.uint64))
    b.n_items = len(arrs["item_msg"])
    b.item_msg = ptr(arrs["item_msg"].astype(np.uint32))
    b.item_key = ptr(arrs["item_key"].astype(np.uint32))
    b.r_be = ptr(arrs["r_be"])
    b.s_be = ptr(arrs["s_be"])
    b.pre = ptr(arrs["pre"]) if arrs.get("pre") is not None else 0
    return b


OSSL_SKIP = 0xFE
_ossl = None


def ossl_lib():
    global _ossl
    if _ossl is None:
        path = os.path.join(_HERE, "_build", "libosslref.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.ossl_verify_batch.argtypes = [ctypes.POINTER(_Batch), ctypes.c_void_p, ctypes.c_int]
        L.ossl_verify_batch.restype = ctypes.c_int
        _ossl = L
    return _ossl


def ossl_verify_batch(arrs: dict, n_threads: int = 0) -> np.ndarray:
    """OpenSSL libcrypto over a packed batch (oracle/openssl_ref.c): per item
    SHA-256 + SEC1 decode + ECDSA_do_verify; 1 / 0 for well-formed items,
    OSSL_SKIP for items OpenSSL is no oracle for."""
    keep: list = []
    b = _cbatch(arrs, keep)
    st = np.zeros(max(b.n_items, 1), np.uint8)
    ossl_lib().ossl_verify_batch(ctypes.byref(b), st.ctypes.data, n_threads or default_threads())
    return st[: b.n_items]


def verify_batch(arrs: dict, n_threads: int = 0):
    """Run the oracle over a packed batch (dict of numpy arrays, see
    babble_amd.batch.pack layout).  Returns (msg_hash[n_msgs,32], status[n], bits)."""
    L = lib()
    if n_threads <= 0:
        n_threads = default_threads()
    b = _Batch()
    n_msgs = len(arrs["msg_off"]) - 1
    n_items = len(arrs["item_msg"])
    keep = []

    def ptr(a):
        a = np.ascontiguousarray(a)
        keep.append(a)
        return a.ctypes.data if a.size else 0

    b.n_msgs = n_msgs
    b.msg_bytes = ptr(arrs["msg_bytes"])
    b.msg_off = ptr(arrs["msg_off"].astype(np.uint64))
    b.n_keys = len(arrs["key_off"]) - 1
    b.key_bytes = ptr(arrs["key_bytes"])
    b.key_off = ptr(arrs["key_off"].astype(np.uint64))
    b.n_items = n_items
    b.item_msg = ptr(arrs["item_msg"].astype(np.uint32))
    b.item_key = ptr(arrs["item_key"].astype(np.uint32))
    b.r_be = ptr(arrs["r_be"])
    b.s_be = ptr(arrs["s_be"])
    b.pre = ptr(arrs["pre"]) if arrs.get("pre") is not None else 0
    h = np.zeros((max(n_msgs, 1), 32), np.uint8)
    st = np.zeros(max(n_items, 1), np.uint8)
    bits = np.zeros(max((n_items + 63) // 64, 1), np.uint64)
    L.oracle_verify_batch(ctypes.byref(b), h.ctypes.data, st.ctypes.data, bits.ctypes.data, n_threads)
    return h[:n_msgs], st[:n_items], bits[: (n_items + 63) // 64]


def port_verify_batch(arrs: dict, n_threads: int = 0) -> np.ndarray:
    """The btcec-algorithm CPU port (oracle.c: GLV + NAF ScalarMult, byte-table
    ScalarBaseMult, mixed additions) over a packed batch: statuses.  Timed as
    bench.py's cpu_baseline "port" leg; checked against the oracle in tests."""
    keep: list = []
    b = _cbatch(arrs, keep)
    h = np.zeros((max(b.n_msgs, 1), 32), np.uint8)
    st = np.zeros(max(b.n_items, 1), np.uint8)
    lib().port_verify_batch(ctypes.byref(b), h.ctypes.data, st.ctypes.data, n_threads or default_threads())
    return st[: b.n_items]


class Prepared:
    """A packed batch converted once for repeated timed calls (bench.py's CPU
    legs): the ctypes struct, the kept arrays and the output buffers, so a
    timed call is the C call alone."""

    def __init__(self, arrs: dict):
        self._keep: list = []
        self.b = _cbatch(arrs, self._keep)
        self.h = np.zeros((max(self.b.n_msgs, 1), 32), np.uint8)
        self.st = np.zeros(max(self.b.n_items, 1), np.uint8)
        lib()
        ossl_lib()

    def port(self, n_threads: int) -> np.ndarray:
        lib().port_verify_batch(ctypes.byref(self.b), self.h.ctypes.data, self.st.ctypes.data, n_threads)
        return self.st[: self.b.n_items]

    def oracle(self, n_threads: int) -> np.ndarray:
        lib().oracle_verify_batch(ctypes.byref(self.b), self.h.ctypes.data, self.st.ctypes.data, None, n_threads)
        return self.st[: self.b.n_items]

    def openssl(self, n_threads: int) -> np.ndarray:
        ossl_lib().ossl_verify_batch(ctypes.byref(self.b), self.st.ctypes.data, n_threads)
        return self.st[: self.b.n_items]
