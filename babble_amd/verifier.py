"""Verifier: the Python handle on one bv_ctx (one gfx950 device).

    v = Verifier(device=0)
    res = v.verify(packed_batch)          # host buffers (bv_verify_batch)
    res.status, res.accept_bits, res.msg_hash

    dev = v.to_device(packed_batch)       # inputs resident in HBM (torch
    v.verify_device(dev)                  # tensors as plumbing), then
                                          # bv_verify_batch_device
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import native
from .batch import PackedBatch


@dataclass
class VerifyResult:
    msg_hash: np.ndarray     # [n_msgs, 32] u8
    status: np.ndarray       # [n_items] u8
    accept_bits: np.ndarray  # [ceil(n_items/64)] u64


def _p(a: np.ndarray) -> int:
    return a.ctypes.data if a is not None and a.size else 0


class DeviceBatch:
    """Device-resident copy of a PackedBatch plus its result buffers."""

    def __init__(self, packed: PackedBatch, device: int):
        import torch

        dev = torch.device("cuda", device)

        def t(a, dtype, pad=0):
            a = np.ascontiguousarray(a)
            out = torch.zeros(max(a.size + pad, 1), dtype=dtype, device=dev)
            if a.size:
                out[: a.size].copy_(torch.from_numpy(a.view(np.uint8) if dtype == torch.uint8 else a).to(dev))
            return out

        self.n_msgs, self.n_keys, self.n_items = packed.n_msgs, packed.n_keys, packed.n_items
        self.msg_bytes = t(packed.msg_bytes, torch.uint8, pad=64)
        self.msg_off = t(packed.msg_off.astype(np.int64), torch.int64)
        self.key_bytes = t(packed.key_bytes, torch.uint8, pad=64)
        self.key_off = t(packed.key_off.astype(np.int64), torch.int64)
        self.item_msg = t(packed.item_msg.astype(np.int32), torch.int32)
        self.item_key = t(packed.item_key.astype(np.int32), torch.int32)
        self.r_be = t(packed.r_be.reshape(-1), torch.uint8)
        self.s_be = t(packed.s_be.reshape(-1), torch.uint8)
        self.pre = t(packed.pre, torch.uint8) if packed.pre is not None else None
        self.msg_hash = torch.zeros(max(self.n_msgs, 1) * 32, dtype=torch.uint8, device=dev)
        self.status = torch.zeros(max(self.n_items, 1), dtype=torch.uint8, device=dev)
        self.accept_bits = torch.zeros(max((self.n_items + 63) // 64, 1), dtype=torch.int64, device=dev)
        b = native.BvBatch()
        b.n_msgs = self.n_msgs
        b.msg_bytes = self.msg_bytes.data_ptr()
        b.msg_off = self.msg_off.data_ptr()
        b.n_keys = self.n_keys
        b.key_bytes = self.key_bytes.data_ptr()
        b.key_off = self.key_off.data_ptr()
        b.n_items = self.n_items
        b.item_msg = self.item_msg.data_ptr()
        b.item_key = self.item_key.data_ptr()
        b.r_be = self.r_be.data_ptr()
        b.s_be = self.s_be.data_ptr()
        b.pre = self.pre.data_ptr() if self.pre is not None else 0
        self.cbatch = b
        # the copies above run on torch's stream; the library may run on its
        # own non-blocking stream, so they must be complete before any call
        torch.cuda.current_stream(dev).synchronize()
        self._pending = None
        r = native.BvResult()
        r.msg_hash = self.msg_hash.data_ptr()
        r.status = self.status.data_ptr()
        r.accept_bits = self.accept_bits.data_ptr()
        self.cresult = r

    def result(self) -> VerifyResult:
        # .cpu() runs on torch's current stream: ordered after a verify that
        # was enqueued on it; an async verify on the library's own stream is
        # waited for explicitly
        if self._pending is not None:
            self._pending.sync()
            self._pending = None
        return VerifyResult(
            self.msg_hash.cpu().numpy()[: self.n_msgs * 32].reshape(self.n_msgs, 32),
            self.status.cpu().numpy()[: self.n_items],
            self.accept_bits.cpu().numpy().view(np.uint64)[: (self.n_items + 63) // 64],
        )


class Verifier:
    def __init__(self, device: int = 0, flags: int = native.F_DEFAULT):
        self._L = native.lib()
        self.device = device
        ctx = ctypes.c_void_p()
        rc = self._L.bv_create(ctypes.byref(ctx), device, flags)
        if rc != native.BV_OK:
            raise native.BvError(rc, "bv_create failed (no usable gfx950 device?)")
        self._ctx = ctx

    def close(self):
        if self._ctx:
            self._L.bv_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int):
        if rc != native.BV_OK:
            raise native.BvError(rc, self._L.bv_last_error(self._ctx).decode(errors="replace"))

    def verify(self, b: PackedBatch) -> VerifyResult:
        keep: list = []
        cb = _cbatch(b, keep)
        # one allocation for the three result arrays (the library writes
        # every byte of them)
        nm, ni, nw = max(b.n_msgs, 1) * 32, max(b.n_items, 1), max((b.n_items + 63) // 64, 1)
        buf = np.empty(8 * nw + nm + ni, np.uint8)
        bits = buf[: 8 * nw].view(np.uint64)
        h = buf[8 * nw: 8 * nw + nm].reshape(-1, 32)
        st = buf[8 * nw + nm:]
        base = _p(buf)
        res = native.BvResult(base + 8 * nw, base + 8 * nw + nm, base)
        self._check(self._L.bv_verify_batch(self._ctx, ctypes.byref(cb), ctypes.byref(res)))
        return VerifyResult(h[: b.n_msgs], st[: b.n_items], bits[: (b.n_items + 63) // 64])

    def to_device(self, b: PackedBatch) -> DeviceBatch:
        return DeviceBatch(b, self.device)

    def verify_device(self, d: DeviceBatch, stream: Optional[int] = None, sync: bool = True) -> None:
        """bv_verify_batch_device on `stream` (a hipStream_t handle).  The
        default is PyTorch's current stream on this device, so the work is
        ordered after the tensor copies that filled `d` and before any later
        torch op (DeviceBatch.result()'s copies) without extra syncs."""
        if stream is None:
            import torch

            stream = torch.cuda.current_stream(self.device).cuda_stream
        # (handle 0 = torch's legacy default stream: the library then uses its
        # own stream; DeviceBatch synchronised its copies at construction and
        # result() waits for an async call through bv_sync)
        self._check(self._L.bv_verify_batch_device(self._ctx, ctypes.byref(d.cbatch), ctypes.byref(d.cresult),
                                                   stream or 0, 0 if sync else 1))
        d._pending = None if sync else self

    def last_stream(self) -> int:
        """bv_last_stream: the hipStream_t the last call ran on (a NULL-stream
        device call runs on the library's lane for its work slot)."""
        return self._L.bv_last_stream(self._ctx) or 0

    def verify_into(self, b: PackedBatch, res: VerifyResult) -> VerifyResult:
        """bv_verify_batch into caller-owned result arrays (e.g. PinnedArena
        arrays, which the results reach by DMA without a host copy)."""
        keep: list = []
        cb = _cbatch(b, keep)
        r = native.BvResult(_p(res.msg_hash), _p(res.status), _p(res.accept_bits))
        self._check(self._L.bv_verify_batch(self._ctx, ctypes.byref(cb), ctypes.byref(r)))
        return res

    def sync(self) -> None:
        """bv_sync: wait for this ctx's last (async) call."""
        self._check(self._L.bv_sync(self._ctx))

    def sha256(self, msgs: Sequence[bytes]) -> list:
        msgs = [bytes(m) for m in msgs]
        if not msgs:
            return []
        buf = np.frombuffer(b"".join(msgs) or b"\0", np.uint8).copy()
        off = np.zeros(len(msgs) + 1, np.uint64)
        off[1:] = np.cumsum([len(m) for m in msgs], dtype=np.uint64)
        out = np.zeros((len(msgs), 32), np.uint8)
        self._check(self._L.bv_sha256_batch(self._ctx, len(msgs), buf.ctypes.data, off.ctypes.data, out.ctypes.data))
        return [out[i].tobytes() for i in range(len(msgs))]

    def verify_events(self, eb) -> VerifyResult:
        """bv_verify_events over an events.EventWireBatch: the device builds,
        hashes (DAG levels in-batch) and verifies every EventBody."""
        keep: list = []
        cb = eb.c_struct(keep)
        n = eb.n_events
        h = np.zeros((max(n, 1), 32), np.uint8)
        st = np.zeros(max(n, 1), np.uint8)
        bits = np.zeros(max((n + 63) // 64, 1), np.uint64)
        res = native.BvResult(h.ctypes.data, st.ctypes.data, bits.ctypes.data)
        self._check(self._L.bv_verify_events(self._ctx, ctypes.byref(cb), ctypes.byref(res)))
        return VerifyResult(h[:n], st[:n], bits[: (n + 63) // 64])

    def verify_events_into(self, eb, res: VerifyResult) -> VerifyResult:
        """bv_verify_events into caller-owned result arrays (PinnedArena
        arrays are reached by DMA; so are the wire fields of a batch built by
        PinnedArena.wire)."""
        keep: list = []
        cb = eb.c_struct(keep)
        r = native.BvResult(_p(res.msg_hash), _p(res.status), _p(res.accept_bits))
        self._check(self._L.bv_verify_events(self._ctx, ctypes.byref(cb), ctypes.byref(r)))
        return res

    def peer_set_hash(self, pubkeys: Sequence[bytes]) -> bytes:
        """bv_peer_set_hash: PeerSet.Hash over the peers' key bytes (b"" for
        an empty set, as Go's []byte{})."""
        pubkeys = [bytes(k) for k in pubkeys]
        if not pubkeys:
            return b""
        buf = np.frombuffer(b"".join(pubkeys) or b"\0", np.uint8).copy()
        off = np.zeros(len(pubkeys) + 1, np.uint64)
        off[1:] = np.cumsum([len(k) for k in pubkeys], dtype=np.uint64)
        out = np.zeros(32, np.uint8)
        self._check(self._L.bv_peer_set_hash(self._ctx, len(pubkeys), buf.ctypes.data, off.ctypes.data,
                                             out.ctypes.data))
        return out.tobytes()

    def register_keys(self, pubkeys: Sequence[bytes]) -> None:
        """bv_kc_register: the key cache's registered keys (the PeerSet's
        PubKeyBytes) replace the previous set; their tables are built now."""
        pubkeys = [bytes(k) for k in pubkeys]
        buf = np.frombuffer(b"".join(pubkeys) or b"\0", np.uint8).copy()
        off = np.zeros(len(pubkeys) + 1, np.uint64)
        off[1:] = np.cumsum([len(k) for k in pubkeys], dtype=np.uint64)
        self._check(self._L.bv_kc_register(self._ctx, len(pubkeys), buf.ctypes.data, off.ctypes.data))

    def timing(self) -> dict:
        t = native.BvTiming()
        self._check(self._L.bv_get_timing(self._ctx, ctypes.byref(t)))
        return {k: getattr(t, k) for k, _ in native.BvTiming._fields_}


_CB_FIELDS = (("msg_bytes", np.uint8), ("msg_off", np.uint64), ("key_bytes", np.uint8), ("key_off", np.uint64),
              ("item_msg", np.uint32), ("item_key", np.uint32), ("r_be", np.uint8), ("s_be", np.uint8),
              ("pre", np.uint8))


def _cbatch(b: PackedBatch, keep: list) -> "native.BvBatch":
    """The bv_batch of `b` (arrays converted to the C dtypes, contiguous).
    Cached on the batch while its arrays are the same objects and needed no
    conversion: a batch verified again (latency loops, streaming callers)
    skips the pointer look-ups (~25 us of Python per call)."""
    arrays = tuple(getattr(b, f) for f, _ in _CB_FIELDS)
    # identity alone is not enough: an in-place ndarray.resize keeps the
    # object but moves its data, so the cache is keyed on each
    # array's data pointer and shape too
    sig = tuple((a.__array_interface__["data"][0], a.shape) if isinstance(a, np.ndarray) else id(a) for a in arrays)
    cached = getattr(b, "_cb_cache", None)
    if (cached is not None and len(cached[0]) == len(arrays) and all(x is y for x, y in zip(cached[0], arrays))
            and cached[3] == sig):
        keep.append(cached[2])
        return cached[1]
    conv = []

    def c(a, dt):
        a = np.ascontiguousarray(a, dtype=dt)
        conv.append(a)
        return a

    cb = native.BvBatch()
    cb.n_msgs = b.n_msgs
    cb.msg_bytes = _p(c(b.msg_bytes, np.uint8))
    cb.msg_off = _p(c(b.msg_off, np.uint64))
    cb.n_keys = b.n_keys
    cb.key_bytes = _p(c(b.key_bytes, np.uint8))
    cb.key_off = _p(c(b.key_off, np.uint64))
    cb.n_items = b.n_items
    cb.item_msg = _p(c(b.item_msg, np.uint32))
    cb.item_key = _p(c(b.item_key, np.uint32))
    cb.r_be = _p(c(b.r_be, np.uint8))
    cb.s_be = _p(c(b.s_be, np.uint8))
    cb.pre = _p(c(b.pre, np.uint8)) if b.pre is not None else 0
    keep.append(conv)
    # cached only when no array was converted: the pointers are then the
    # caller's own arrays, so later in-place edits of them are seen
    if all(x is y for x, y in zip(conv, (a for a in arrays if a is not None))):
        try:
            b._cb_cache = (arrays, cb, conv, sig)
        except AttributeError:  # (a batch type without a __dict__: no cache)
            pass
    return cb


def plan_shards(b: PackedBatch, n_shards: int) -> np.ndarray:
    """bv_plan_shards: the item bounds bv_group_verify_batch uses (host only)."""
    keep: list = []
    cb = _cbatch(b, keep)
    out = np.zeros(n_shards + 1, np.uint64)
    rc = native.lib().bv_plan_shards(ctypes.byref(cb), n_shards, out.ctypes.data)
    if rc != native.BV_OK:
        raise native.BvError(rc, "bv_plan_shards")
    return out


class Group:
    """bv_group: one verifier over several devices of this process; items
    sharded message-aligned, accept bitmasks all-gathered over RCCL."""

    def __init__(self, devices: Sequence[int], flags: int = native.F_DEFAULT):
        self._L = native.lib()
        self.devices = list(devices)
        arr = (ctypes.c_int * len(self.devices))(*self.devices)
        g = ctypes.c_void_p()
        rc = self._L.bv_group_create(ctypes.byref(g), arr, len(self.devices), flags)
        if rc != native.BV_OK:
            raise native.BvError(rc, "bv_group_create failed")
        self._g = g

    def close(self):
        if self._g:
            self._L.bv_group_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def verify(self, b: PackedBatch) -> VerifyResult:
        keep: list = []
        cb = _cbatch(b, keep)
        h = np.zeros((max(b.n_msgs, 1), 32), np.uint8)
        st = np.zeros(max(b.n_items, 1), np.uint8)
        bits = np.zeros(max((b.n_items + 63) // 64, 1), np.uint64)
        res = native.BvResult(h.ctypes.data, st.ctypes.data, bits.ctypes.data)
        rc = self._L.bv_group_verify_batch(self._g, ctypes.byref(cb), ctypes.byref(res))
        if rc != native.BV_OK:
            raise native.BvError(rc, self._L.bv_group_last_error(self._g).decode(errors="replace"))
        return VerifyResult(h[: b.n_msgs], st[: b.n_items], bits[: (b.n_items + 63) // 64])

    def verify_into(self, b: PackedBatch, res: VerifyResult) -> VerifyResult:
        """bv_group_verify_batch into caller-owned result arrays (PinnedArena
        arrays: a batch built there is DMA'd to every device in place)."""
        keep: list = []
        cb = _cbatch(b, keep)
        r = native.BvResult(_p(res.msg_hash), _p(res.status), _p(res.accept_bits))
        rc = self._L.bv_group_verify_batch(self._g, ctypes.byref(cb), ctypes.byref(r))
        if rc != native.BV_OK:
            raise native.BvError(rc, self._L.bv_group_last_error(self._g).decode(errors="replace"))
        return res

    def timing(self, i: int = 0) -> dict:
        t = native.BvTiming()
        rc = self._L.bv_group_get_timing(self._g, i, ctypes.byref(t))
        if rc != native.BV_OK:
            raise native.BvError(rc, "bv_group_get_timing")
        return {k: getattr(t, k) for k, _ in native.BvTiming._fields_}


def plan_group(b: PackedBatch, n_shards: int):
    """bv_plan_group: (permuted, perm, item_bounds, msg_bounds) — the plan
    bv_group_verify_batch follows (host only)."""
    keep: list = []
    cb = _cbatch(b, keep)
    ib = np.zeros(n_shards + 1, np.uint64)
    mb = np.zeros(n_shards + 1, np.uint64)
    perm = np.zeros(max(b.n_items, 1), np.uint32)
    rc = native.lib().bv_plan_group(ctypes.byref(cb), n_shards, ib.ctypes.data, mb.ctypes.data, perm.ctypes.data)
    if rc < 0:
        raise native.BvError(rc, "bv_plan_group")
    return bool(rc), perm[: b.n_items], ib, mb


def merge_shard_bits(gathered: np.ndarray, words_per_shard: int, bounds) -> np.ndarray:
    """bv_merge_shard_bits: the global bitmask from all-gathered shard words
    (host only; what bv_group_verify_batch does after its all-gather)."""
    g = np.ascontiguousarray(gathered, dtype=np.uint64)
    bd = np.ascontiguousarray(bounds, dtype=np.uint64)
    out = np.zeros(max((int(bd[-1]) + 63) // 64, 1), np.uint64)
    rc = native.lib().bv_merge_shard_bits(_p(g), words_per_shard, len(bd) - 1, bd.ctypes.data, out.ctypes.data)
    if rc != native.BV_OK:
        raise native.BvError(rc, "bv_merge_shard_bits")
    return out[: (int(bd[-1]) + 63) // 64]


class PinnedArena:
    """Arrays in bv_host_alloc memory (page-locked): a batch built here is
    DMA'd by bv_verify_batch without the staging copy (what the cgo shim does
    instead of C.CBytes).  Freed with close()."""

    def __init__(self):
        self._L = native.lib()
        self._blocks = []

    def array(self, shape, dtype) -> np.ndarray:
        dtype = np.dtype(dtype)
        n = int(np.prod(shape)) * dtype.itemsize
        p = ctypes.c_void_p()
        rc = self._L.bv_host_alloc(max(n, 1), ctypes.byref(p))
        if rc != native.BV_OK:
            raise native.BvError(rc, "bv_host_alloc")
        self._blocks.append(p.value)
        buf = (ctypes.c_uint8 * max(n, 1)).from_address(p.value)
        return np.frombuffer(buf, dtype=np.uint8, count=n).view(dtype).reshape(shape)

    def copy(self, a: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(a)
        out = self.array(a.shape, a.dtype)
        out[...] = a
        return out

    def batch(self, b: PackedBatch) -> PackedBatch:
        """The same batch with every array in pinned memory."""
        return PackedBatch(self.copy(b.msg_bytes), self.copy(b.msg_off.astype(np.uint64)), self.copy(b.key_bytes),
                           self.copy(b.key_off.astype(np.uint64)), self.copy(b.item_msg.astype(np.uint32)),
                           self.copy(b.item_key.astype(np.uint32)), self.copy(b.r_be), self.copy(b.s_be),
                           None if b.pre is None else self.copy(b.pre))

    def wire(self, eb):
        """The same events.EventWireBatch with every array in pinned memory
        (in the dtypes the C struct takes, so none is converted again)."""
        import dataclasses

        dt = {"key_off": np.uint64, "creator": np.uint32, "index": np.int64, "timestamp": np.int64,
              "parent_kind": np.uint8, "parent_ref": np.uint64, "tx_start": np.uint64, "tx_off": np.uint64,
              "itx_off": np.uint64, "bsig_off": np.uint64}
        out = {}
        for f in dataclasses.fields(eb):
            a = getattr(eb, f.name)
            out[f.name] = None if a is None else self.copy(np.asarray(a).astype(dt.get(f.name, a.dtype), copy=False))
        return type(eb)(**out)

    def close(self):
        for p in self._blocks:
            self._L.bv_host_free(p)
        self._blocks = []
