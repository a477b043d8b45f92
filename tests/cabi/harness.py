"""ctypes front of tests/cabi/libshimharness.so — the cgo shim's call
sequence replayed in C through the C ABI.  Test
and bench infrastructure only (tests/test_cabi.py, bench.py `shim_path`)."""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libshimharness.so")
P = ctypes.c_void_p


class ShimWire(ctypes.Structure):
    """shim_wire (shim_harness.c): a SyncResponse after ReadWireBatch."""
    _fields_ = [("n_events", ctypes.c_uint64), ("rep_bytes", P), ("rep_off", P), ("creator_id", P), ("index", P),
                ("timestamp", P), ("parent_kind", P), ("parent_event", P), ("parent_hash", P), ("tx_start", P),
                ("tx_off", P), ("tx_bytes", P), ("tx_list_nil", P), ("tx_nil", P), ("itx_off", P), ("bsig_off", P),
                ("itx_json", P), ("bsig_json", P), ("sig_off", P), ("sig_text", P)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        from babble_amd import native

        native.lib()  # libbabbleverify.so first (torch's HIP runtime), so the harness binds to the same copy
        L = ctypes.CDLL(LIB_PATH)
        L.shim_open.argtypes = [ctypes.c_int, ctypes.c_uint32]
        L.shim_close.restype = None
        L.shim_last_error.restype = ctypes.c_char_p
        L.shim_set_peers.argtypes = [ctypes.c_uint32, P, P]
        L.shim_sync.argtypes = [ctypes.POINTER(ShimWire), P, P, ctypes.POINTER(ctypes.c_double)]
        B = ctypes.c_char_p
        L.shim_verify_event.argtypes = [B, ctypes.c_size_t, B, ctypes.c_size_t, B, ctypes.c_size_t, P, P,
                                        ctypes.POINTER(ctypes.c_double)]
        L.shim_last_phases.argtypes = [P]
        L.shim_last_phases.restype = None
        L.shim_encode_signatures.argtypes = [ctypes.c_uint64, P, P, P, P]
        _lib = L
    return _lib


def _ptr(a, keep):
    if a is None:
        return None
    a = np.ascontiguousarray(a)
    keep.append(a)
    return a.ctypes.data if a.size else None


def encode_signatures(r_be: np.ndarray, s_be: np.ndarray):
    """keys.EncodeSignature of every (r, s): (text bytes, offsets)."""
    n = len(r_be)
    text = np.zeros(max(1, 101 * n), np.uint8)
    off = np.zeros(n + 1, np.uint64)
    r = np.ascontiguousarray(r_be, np.uint8)
    s = np.ascontiguousarray(s_be, np.uint8)
    lib().shim_encode_signatures(n, r.ctypes.data, s.ctypes.data, text.ctypes.data, off.ctypes.data)
    return text[:int(off[-1])].copy(), off


def signature_text(text: np.ndarray, off: np.ndarray, i: int) -> bytes:
    return text[int(off[i]):int(off[i + 1])].tobytes()


class Shim:
    """The shim's process state: one context (the key cache on, as
    verifier() creates it) and its pool of arena-backed batch builders."""

    def __init__(self, device: int = 0, flags: int = 1):
        self.L = lib()
        rc = self.L.shim_open(device, flags)
        if rc != 0:
            raise RuntimeError(f"shim_open: {rc}")

    def close(self):
        self.L.shim_close()

    def set_peers(self, keys):
        kb = np.frombuffer(b"".join(keys), np.uint8).copy()
        ko = np.zeros(len(keys) + 1, np.uint64)
        ko[1:] = np.cumsum([len(k) for k in keys])
        rc = self.L.shim_set_peers(len(keys), kb.ctypes.data if kb.size else None, ko.ctypes.data)
        if rc != 0:
            raise RuntimeError(self.L.shim_last_error().decode())

    def wire(self, w, sig=None) -> tuple:
        """(ShimWire, keep) from an events.EventWireBatch: creator ids index
        its key table (the repertoire); HASH parents as 32-byte values."""
        keep: list = []
        n = w.n_events
        kind = np.ascontiguousarray(w.parent_kind, np.uint8).reshape(n, 2)
        ref = np.ascontiguousarray(w.parent_ref, np.uint64).reshape(n, 2)
        ph = np.zeros((n, 2, 32), np.uint8)
        hashes = np.asarray(w.parent_hashes, np.uint8).reshape(-1, 32)
        for j in range(2):
            m = kind[:, j] == 1
            if m.any():
                ph[m, j] = hashes[ref[m, j].astype(np.int64)]
        text, off = sig if sig is not None else encode_signatures(w.r_be, w.s_be)
        sw = ShimWire()
        sw.n_events = n
        sw.rep_bytes, sw.rep_off = _ptr(w.key_bytes, keep), _ptr(np.asarray(w.key_off, np.uint64), keep)
        sw.creator_id = _ptr(np.asarray(w.creator, np.uint32), keep)
        sw.index, sw.timestamp = _ptr(np.asarray(w.index, np.int64), keep), _ptr(np.asarray(w.timestamp, np.int64),
                                                                                    keep)
        sw.parent_kind, sw.parent_event, sw.parent_hash = _ptr(kind, keep), _ptr(ref, keep), _ptr(ph, keep)
        sw.tx_start, sw.tx_off = _ptr(np.asarray(w.tx_start, np.uint64), keep), _ptr(np.asarray(w.tx_off, np.uint64),
                                                                                     keep)
        sw.tx_bytes, sw.tx_list_nil, sw.tx_nil = _ptr(w.tx_bytes, keep), _ptr(w.tx_list_nil, keep), _ptr(w.tx_nil, keep)
        sw.itx_off = _ptr(None if w.itx_off is None else np.asarray(w.itx_off, np.uint64), keep)
        sw.bsig_off = _ptr(None if w.bsig_off is None else np.asarray(w.bsig_off, np.uint64), keep)
        sw.itx_json, sw.bsig_json = _ptr(w.itx_json, keep), _ptr(w.bsig_json, keep)
        sw.sig_off, sw.sig_text = _ptr(off, keep), _ptr(text, keep)
        return sw, keep

    def sync(self, sw: ShimWire):
        """VerifySync: (digests [n, 32], statuses [n], wall ms)."""
        n = sw.n_events
        dig = np.zeros((n, 32), np.uint8)
        st = np.zeros(n, np.uint8)
        ms = ctypes.c_double()
        rc = self.L.shim_sync(ctypes.byref(sw), dig.ctypes.data, st.ctypes.data, ctypes.byref(ms))
        if rc != 0:
            raise RuntimeError(self.L.shim_last_error().decode())
        return dig, st, ms.value

    def phases(self) -> dict:
        """The last sync's wall ms split: build (the fill), lib
        (bv_verify_events), out (the copy-out)."""
        v = (ctypes.c_double * 3)()
        self.L.shim_last_phases(v)
        return {"build": v[0], "lib": v[1], "out": v[2]}

    def verify_event(self, body: bytes, key: bytes, sig: bytes):
        """VerifyEvents([ev]): (digest, status, wall ms)."""
        dig = ctypes.create_string_buffer(32)
        st = ctypes.c_uint8()
        ms = ctypes.c_double()
        rc = self.L.shim_verify_event(body, len(body), key, len(key), sig, len(sig), dig, ctypes.byref(st),
                                      ctypes.byref(ms))
        if rc != 0:
            raise RuntimeError(self.L.shim_last_error().decode())
        return dig.raw, st.value, ms.value
