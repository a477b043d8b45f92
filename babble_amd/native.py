"""ctypes binding of libbabbleverify.so (include/babbleverify.h).

The product path: every verify goes through this library's gfx950 kernels.
If the library or a gfx950 device is missing the calls raise — there is no
CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libbabbleverify.so")

BV_OK = 0
BV_E_ARGS = -1
BV_E_NODEVICE = -2
BV_E_OOM = -3
BV_E_LAUNCH = -4
BV_E_COMM = -5

REJECT, ACCEPT, REJECT_ERR, REF_PANIC = 0, 1, 2, 3
SC_OK, SC_NIL, SC_NONPOS, SC_GE_N = 0, 1, 2, 3
PRE_PARTS_BAD = 0x80
F_DEFAULT = 0
ABI_VERSION = 6
ARENA_SLOTS = 32
F_KEY_CACHE = 1
F_K8 = 2

# Every symbol include/babbleverify.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "bv_abi_version", "bv_create", "bv_destroy", "bv_last_error", "bv_verify_batch",
    "bv_verify_batch_device", "bv_sha256_batch", "bv_get_timing", "bv_decode_signature",
    "bv_hex_decode", "bv_group_create", "bv_group_destroy", "bv_group_last_error", "bv_group_verify_batch",
    "bv_group_get_timing", "bv_plan_shards", "bv_sync", "bv_peer_set_hash", "bv_verify_events",
    "bv_last_stream", "bv_host_alloc", "bv_host_free", "bv_merge_shard_bits", "bv_plan_group",
    "bv_kc_register", "bv_arena_create", "bv_arena_destroy", "bv_arena_reserve",
)


class BvBatch(ctypes.Structure):
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


class BvResult(ctypes.Structure):
    _fields_ = [
        ("msg_hash", ctypes.c_void_p),
        ("status", ctypes.c_void_p),
        ("accept_bits", ctypes.c_void_p),
    ]


class BvTiming(ctypes.Structure):
    _fields_ = [
        ("ms_total", ctypes.c_float),
        ("ms_sha256", ctypes.c_float),
        ("ms_keyprep", ctypes.c_float),
        ("ms_scalar", ctypes.c_float),
        ("ms_verify_g", ctypes.c_float),
        ("ms_verify", ctypes.c_float),
        ("ms_h2d", ctypes.c_float),
        ("ms_d2h", ctypes.c_float),
        ("ms_host", ctypes.c_float),
        ("ms_host_prep", ctypes.c_float),
        ("ms_host_out", ctypes.c_float),
        ("key_path", ctypes.c_uint32),
        ("kc_hits", ctypes.c_uint32),
        ("kc_builds", ctypes.c_uint32),
        ("kc_keys", ctypes.c_uint32),
    ]


class BvError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"babbleverify error {code}: {msg}")
        self.code = code


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise BvError(BV_E_NODEVICE, f"{LIB_PATH} not built; run __graft_entry__.build()")
    # One HIP runtime per process: PyTorch-ROCm bundles its own
    # libamdhip64.so (soname libamdhip64.so.7).  Loading torch first makes
    # the dynamic loader resolve our NEEDED libamdhip64.so.7 to that same
    # runtime, so torch tensors (HBM plumbing, RCCL collectives) and our
    # kernels share one device context.  Without torch the library binds to
    # /opt/rocm's runtime (the cgo / plain C use).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.c_void_p
    L.bv_abi_version.restype = ctypes.c_int
    L.bv_create.argtypes = [ctypes.POINTER(P), ctypes.c_int, ctypes.c_uint32]
    L.bv_create.restype = ctypes.c_int
    L.bv_destroy.argtypes = [P]
    L.bv_last_error.argtypes = [P]
    L.bv_last_error.restype = ctypes.c_char_p
    L.bv_verify_batch.argtypes = [P, ctypes.POINTER(BvBatch), ctypes.POINTER(BvResult)]
    L.bv_verify_batch.restype = ctypes.c_int
    L.bv_verify_batch_device.argtypes = [P, ctypes.POINTER(BvBatch), ctypes.POINTER(BvResult), P, ctypes.c_int]
    L.bv_verify_batch_device.restype = ctypes.c_int
    L.bv_sha256_batch.argtypes = [P, ctypes.c_uint64, P, P, P]
    L.bv_sha256_batch.restype = ctypes.c_int
    L.bv_get_timing.argtypes = [P, ctypes.POINTER(BvTiming)]
    L.bv_get_timing.restype = ctypes.c_int
    L.bv_decode_signature.argtypes = [ctypes.c_char_p, ctypes.c_size_t, P, P]
    L.bv_decode_signature.restype = ctypes.c_uint8
    L.bv_hex_decode.argtypes = [ctypes.c_char_p, ctypes.c_size_t, P]
    L.bv_hex_decode.restype = ctypes.c_int64
    L.bv_group_create.argtypes = [ctypes.POINTER(P), ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_uint32]
    L.bv_group_create.restype = ctypes.c_int
    L.bv_group_destroy.argtypes = [P]
    L.bv_group_last_error.argtypes = [P]
    L.bv_group_last_error.restype = ctypes.c_char_p
    L.bv_group_verify_batch.argtypes = [P, ctypes.POINTER(BvBatch), ctypes.POINTER(BvResult)]
    L.bv_group_verify_batch.restype = ctypes.c_int
    L.bv_group_get_timing.argtypes = [P, ctypes.c_int, ctypes.POINTER(BvTiming)]
    L.bv_group_get_timing.restype = ctypes.c_int
    L.bv_verify_events.argtypes = [P, P, ctypes.POINTER(BvResult)]
    L.bv_verify_events.restype = ctypes.c_int
    L.bv_peer_set_hash.argtypes = [P, ctypes.c_uint32, P, P, P]
    L.bv_peer_set_hash.restype = ctypes.c_int
    L.bv_sync.argtypes = [P]
    L.bv_sync.restype = ctypes.c_int
    L.bv_plan_shards.argtypes = [ctypes.POINTER(BvBatch), ctypes.c_int, P]
    L.bv_plan_shards.restype = ctypes.c_int
    L.bv_last_stream.argtypes = [P]
    L.bv_last_stream.restype = P
    L.bv_host_alloc.argtypes = [ctypes.c_size_t, ctypes.POINTER(P)]
    L.bv_host_alloc.restype = ctypes.c_int
    L.bv_host_free.argtypes = [P]
    L.bv_host_free.restype = None
    L.bv_merge_shard_bits.argtypes = [P, ctypes.c_uint64, ctypes.c_int, P, P]
    L.bv_merge_shard_bits.restype = ctypes.c_int
    L.bv_plan_group.argtypes = [ctypes.POINTER(BvBatch), ctypes.c_int, P, P, P]
    L.bv_plan_group.restype = ctypes.c_int
    L.bv_kc_register.argtypes = [P, ctypes.c_uint32, P, P]
    L.bv_kc_register.restype = ctypes.c_int
    L.bv_arena_create.argtypes = [ctypes.POINTER(P)]
    L.bv_arena_create.restype = ctypes.c_int
    L.bv_arena_destroy.argtypes = [P]
    L.bv_arena_destroy.restype = None
    L.bv_arena_reserve.argtypes = [P, ctypes.c_uint32, ctypes.c_size_t, ctypes.c_size_t, ctypes.POINTER(P),
                                   ctypes.POINTER(ctypes.c_size_t)]
    L.bv_arena_reserve.restype = ctypes.c_int
    if L.bv_abi_version() != ABI_VERSION:
        raise BvError(BV_E_ARGS, "ABI version mismatch")
    _lib = L
    return L


def decode_signature(sig: bytes):
    """bv_decode_signature: keys.DecodeSignature + pre-class -> (pre, r_be, s_be)."""
    if isinstance(sig, str):
        sig = sig.encode("utf-8")
    r = ctypes.create_string_buffer(32)
    s = ctypes.create_string_buffer(32)
    pre = lib().bv_decode_signature(sig, len(sig), r, s)
    return pre, r.raw, s.raw


class ReferencePanic(Exception):
    """The Go reference would panic on this input (unrecovered in Babble)."""


def hex_decode(s) -> bytes:
    """bv_hex_decode: common.DecodeFromString semantics (partial prefix kept)."""
    if isinstance(s, str):
        s = s.encode("utf-8")
    out = ctypes.create_string_buffer(max(len(s) // 2, 1))
    n = lib().bv_hex_decode(s, len(s), out)
    if n < 0:
        raise ReferencePanic("slice bounds out of range in DecodeFromString")
    return out.raw[:n]
