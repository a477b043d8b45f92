"""ctypes wrapper of tests/emu/_build/libbvemu.so (host build of the device
per-unit code; test infrastructure only)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "_build", "libbvemu.so")
_lib = None


class _Batch(ctypes.Structure):
    _fields_ = [
        ("n_msgs", ctypes.c_uint64), ("msg_bytes", ctypes.c_void_p), ("msg_off", ctypes.c_void_p),
        ("n_keys", ctypes.c_uint32), ("key_bytes", ctypes.c_void_p), ("key_off", ctypes.c_void_p),
        ("n_items", ctypes.c_uint64), ("item_msg", ctypes.c_void_p), ("item_key", ctypes.c_void_p),
        ("r_be", ctypes.c_void_p), ("s_be", ctypes.c_void_p), ("pre", ctypes.c_void_p),
    ]


def lib():
    global _lib
    if _lib is None:
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
        L = ctypes.CDLL(LIB)
        L.emu_verify_batch.argtypes = [ctypes.POINTER(_Batch), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_int, ctypes.c_int]
        L.emu_verify_batch.restype = ctypes.c_int
        for f in ("emu_fe_mul", "emu_fe_add", "emu_fe_sub", "emu_sc_mont"):
            getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        for f in ("emu_fe_sqr", "emu_fe_inv", "emu_sc_inverse", "emu_fe_inv_var", "emu_sc_inverse_var"):
            getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        _lib = L
    return _lib


def _limbs(x: int) -> np.ndarray:
    return np.array([(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)], np.uint32)


def _int(a: np.ndarray) -> int:
    return sum(int(a[i]) << (32 * i) for i in range(8))


def binop(name: str, a: int, b: int) -> int:
    out = np.zeros(8, np.uint32)
    x, y = _limbs(a), _limbs(b)  # keep the buffers alive across the call
    getattr(lib(), name)(x.ctypes.data, y.ctypes.data, out.ctypes.data)
    return _int(out)


def unop(name: str, a: int) -> int:
    out = np.zeros(8, np.uint32)
    x = _limbs(a)
    getattr(lib(), name)(x.ctypes.data, out.ctypes.data)
    return _int(out)


def verify_batch(arrs: dict, n_threads: int = 0, force_mode: int = -1):
    L = lib()
    n_threads = n_threads or min(16, len(os.sched_getaffinity(0)))
    keep = []

    def ptr(a, dt):
        a = np.ascontiguousarray(a, dtype=dt)
        keep.append(a)
        return a.ctypes.data if a.size else 0

    b = _Batch()
    n_msgs = len(arrs["msg_off"]) - 1
    n_items = len(arrs["item_msg"])
    b.n_msgs = n_msgs
    b.msg_bytes = ptr(arrs["msg_bytes"], np.uint8)
    b.msg_off = ptr(arrs["msg_off"], np.uint64)
    b.n_keys = len(arrs["key_off"]) - 1
    b.key_bytes = ptr(arrs["key_bytes"], np.uint8)
    b.key_off = ptr(arrs["key_off"], np.uint64)
    b.n_items = n_items
    b.item_msg = ptr(arrs["item_msg"], np.uint32)
    b.item_key = ptr(arrs["item_key"], np.uint32)
    b.r_be = ptr(arrs["r_be"], np.uint8)
    b.s_be = ptr(arrs["s_be"], np.uint8)
    b.pre = ptr(arrs["pre"], np.uint8) if arrs.get("pre") is not None else 0
    h = np.zeros((max(n_msgs, 1), 32), np.uint8)
    st = np.zeros(max(n_items, 1), np.uint8)
    bits = np.zeros(max((n_items + 63) // 64, 1), np.uint64)
    mode = L.emu_verify_batch(ctypes.byref(b), h.ctypes.data, st.ctypes.data, bits.ctypes.data, n_threads,
                              force_mode)
    return h[:n_msgs], st[:n_items], bits[: (n_items + 63) // 64], mode


def dump_batch(path: str, arrs: dict) -> None:
    """Write a batch in emu_main.cpp's "BVB1" format (sanitizer driver input)."""
    n_msgs = len(arrs["msg_off"]) - 1
    n_keys = len(arrs["key_off"]) - 1
    n_items = len(arrs["item_msg"])
    pre = arrs.get("pre")
    msg = np.ascontiguousarray(arrs["msg_bytes"], np.uint8)
    key = np.ascontiguousarray(arrs["key_bytes"], np.uint8)
    with open(path, "wb") as f:
        f.write(b"BVB1")
        f.write(np.array([n_msgs, n_keys, n_items, msg.size, key.size, pre is not None], np.uint64).tobytes())
        f.write(np.ascontiguousarray(arrs["msg_off"], np.uint64).tobytes())
        f.write(msg.tobytes())
        f.write(np.ascontiguousarray(arrs["key_off"], np.uint64).tobytes())
        f.write(key.tobytes())
        f.write(np.ascontiguousarray(arrs["item_msg"], np.uint32).tobytes())
        f.write(np.ascontiguousarray(arrs["item_key"], np.uint32).tobytes())
        f.write(np.ascontiguousarray(arrs["r_be"], np.uint8).tobytes())
        f.write(np.ascontiguousarray(arrs["s_be"], np.uint8).tobytes())
        if pre is not None:
            f.write(np.ascontiguousarray(pre, np.uint8).tobytes())


def ev_bodies(eb):
    """emu_ev_bodies over an events.EventWireBatch: (bodies: list[bytes],
    digests[n, 32]) built by the device's own per-event code on the host."""
    L = lib()
    L.emu_ev_bodies.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    L.emu_ev_bodies.restype = ctypes.c_uint64
    keep: list = []
    cb = eb.c_struct(keep)
    n = eb.n_events
    cap = 1024 * n + 4 * int(eb.tx_bytes.size) + int(eb.itx_json.size) + int(eb.bsig_json.size) + 4096
    bodies = np.zeros(cap, np.uint8)
    offs = np.zeros(n + 1, np.uint64)
    dig = np.zeros((max(n, 1), 32), np.uint8)
    total = L.emu_ev_bodies(ctypes.byref(cb), bodies.ctypes.data, cap, offs.ctypes.data, dig.ctypes.data)
    assert total == offs[n]
    return [bodies[offs[i]:offs[i + 1]].tobytes() for i in range(n)], dig[:n]


def ev_body_hash(eb) -> np.ndarray:
    """emu_ev_body_hash: the device's streaming serialise-and-hash
    (k_ev_body_hash) on the host: digests[n, 32]."""
    L = lib()
    L.emu_ev_body_hash.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.emu_ev_body_hash.restype = None
    keep: list = []
    cb = eb.c_struct(keep)
    dig = np.zeros((max(eb.n_events, 1), 32), np.uint8)
    L.emu_ev_body_hash(ctypes.byref(cb), dig.ctypes.data)
    return dig[: eb.n_events]


def host_dag_hash(eb, threads: int = 1, portable: bool = False) -> np.ndarray:
    """The product's host DAG hasher (babble_amd/csrc/hostdag.cpp, linked
    into the emulator library): digests[n, 32] of an events.EventWireBatch."""
    L = lib()
    L.emu_host_dag_hash.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    L.emu_host_dag_hash.restype = None
    keep: list = []
    cb = eb.c_struct(keep)
    dig = np.zeros((max(eb.n_events, 1), 32), np.uint8)
    L.emu_host_dag_hash(ctypes.byref(cb), dig.ctypes.data, threads, 1 if portable else 0)
    return dig[: eb.n_events]


def host_sha256(msg: bytes, portable: bool = False) -> bytes:
    """The product's host SHA-256 (babble_amd/csrc/hostsha.cpp)."""
    L = lib()
    L.emu_host_sha256.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
    L.emu_host_sha256.restype = None
    out = ctypes.create_string_buffer(32)
    L.emu_host_sha256(msg, len(msg), out, 1 if portable else 0)
    return out.raw


def host_sha_accelerated() -> bool:
    return bool(lib().emu_host_sha_accelerated())
