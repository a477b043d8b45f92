"""Events from their wire fields (bv_verify_events, include/babbleverify.h):
the device builds each canonical EventBody (event.go:38-45), hashes it —
level by level when a parent is an earlier event of the same batch — and
verifies the creator's signature.  SURVEY §8f rows 1-2.

    b = EventBatchBuilder()
    k = b.add_key(creator_pubkey)
    e0 = b.add_event(k, index=0, timestamp=t, parents=[None, None], transactions=[tx], signature=sig)
    e1 = b.add_event(k, index=1, timestamp=t + 1, parents=[("event", e0), ("hash", h32)], ...)
    res = verifier.verify_events(b.pack())      # msg_hash = Event.Hash(), status per event

Parents follow Hashgraph.ReadWireInfo (hashgraph.go:1540-1595): None -> ""
(wire index < 0), ("hash", 32 bytes) -> "0X" + hex of a hash from the store,
("event", i) -> the hash of event i of this batch (i < the child's index).
InternalTransactions / BlockSignatures are given as their encoding/json
fragments (b"" = nil -> null); the ITX signatures themselves are verified
through bv_verify_batch items (Event.Verify's ITX loop), not here.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple, Union

import numpy as np

from . import native

PARENT_NONE, PARENT_HASH, PARENT_EVENT = 0, 1, 2


class BvEventBatch(ctypes.Structure):
    P = ctypes.c_void_p
    _fields_ = [
        ("n_events", ctypes.c_uint64), ("n_keys", ctypes.c_uint32), ("key_bytes", P), ("key_off", P),
        ("creator", P), ("index", P), ("timestamp", P), ("parent_kind", P), ("parent_ref", P),
        ("n_parent_hashes", ctypes.c_uint64), ("parent_hashes", P), ("tx_start", P), ("tx_off", P),
        ("tx_bytes", P), ("tx_list_nil", P), ("tx_nil", P), ("itx_off", P), ("itx_json", P), ("bsig_off", P),
        ("bsig_json", P), ("r_be", P), ("s_be", P), ("pre", P), ("sig_off", P), ("sig_text", P),
    ]


@dataclass
class EventWireBatch:
    key_bytes: np.ndarray       # u8
    key_off: np.ndarray         # u64 [n_keys + 1]
    creator: np.ndarray         # u32 [n]
    index: np.ndarray           # i64 [n]
    timestamp: np.ndarray       # i64 [n]
    parent_kind: np.ndarray     # u8 [n, 2]
    parent_ref: np.ndarray      # u64 [n, 2]
    parent_hashes: np.ndarray   # u8 [m, 32]
    tx_start: np.ndarray        # u64 [n + 1]
    tx_off: np.ndarray          # u64 [n_tx + 1]
    tx_bytes: np.ndarray        # u8
    tx_list_nil: Optional[np.ndarray]  # u8 [n] or None
    tx_nil: Optional[np.ndarray]       # u8 [n_tx] or None
    itx_off: Optional[np.ndarray]      # u64 [n + 1] or None (all nil)
    itx_json: np.ndarray
    bsig_off: Optional[np.ndarray]
    bsig_json: np.ndarray
    r_be: np.ndarray            # u8 [n, 32]
    s_be: np.ndarray            # u8 [n, 32]
    pre: Optional[np.ndarray]   # u8 [n]
    # or the Event.Signature text (decoded on the device; r_be / s_be / pre
    # are then not sent): u64 [n + 1] offsets and the bytes
    sig_off: Optional[np.ndarray] = None
    sig_text: Optional[np.ndarray] = None

    @property
    def n_events(self) -> int:
        return len(self.creator)

    def c_struct(self, keep: list) -> BvEventBatch:
        def p(a, dt=None):
            if a is None:
                return None
            a = np.ascontiguousarray(a if dt is None else a.astype(dt, copy=False))
            keep.append(a)
            return a.ctypes.data if a.size else None

        b = BvEventBatch()
        b.n_events = self.n_events
        b.n_keys = len(self.key_off) - 1
        b.key_bytes, b.key_off = p(self.key_bytes), p(self.key_off, np.uint64)
        b.creator, b.index, b.timestamp = p(self.creator, np.uint32), p(self.index, np.int64), p(self.timestamp,
                                                                                                 np.int64)
        b.parent_kind, b.parent_ref = p(self.parent_kind, np.uint8), p(self.parent_ref, np.uint64)
        b.n_parent_hashes = len(self.parent_hashes)
        b.parent_hashes = p(self.parent_hashes)
        b.tx_start, b.tx_off, b.tx_bytes = p(self.tx_start, np.uint64), p(self.tx_off, np.uint64), p(self.tx_bytes)
        b.tx_list_nil, b.tx_nil = p(self.tx_list_nil), p(self.tx_nil)
        b.itx_off, b.itx_json = p(self.itx_off, np.uint64), p(self.itx_json)
        b.bsig_off, b.bsig_json = p(self.bsig_off, np.uint64), p(self.bsig_json)
        if self.sig_text is not None:  # the text only (the library decodes it on the device)
            b.sig_off, b.sig_text = p(self.sig_off, np.uint64), p(self.sig_text)
            if not b.sig_text:  # all signatures empty: a valid non-null pointer to zero bytes
                keep.append(np.zeros(1, np.uint8))
                b.sig_text = keep[-1].ctypes.data
        else:
            b.r_be, b.s_be, b.pre = p(self.r_be), p(self.s_be), p(self.pre)
        return b

    def with_signature_text(self, text: np.ndarray, off: np.ndarray) -> "EventWireBatch":
        """The same events carrying their Signature text instead of r / s /
        pre (bv_event_batch sig_text)."""
        import dataclasses

        return dataclasses.replace(self, sig_off=np.asarray(off, np.uint64),
                                   sig_text=np.asarray(text, np.uint8))


Parent = Union[None, Tuple[str, Union[int, bytes]]]


class EventBatchBuilder:
    def __init__(self):
        self._keys: List[bytes] = []
        self._key_idx = {}
        self._ev = []
        self._hashes: List[bytes] = []

    def add_key(self, pub: bytes) -> int:
        pub = bytes(pub)
        k = self._key_idx.get(pub)
        if k is None:
            k = self._key_idx[pub] = len(self._keys)
            self._keys.append(pub)
        return k

    def add_event(self, creator: int, index: int, timestamp: int, parents: Sequence[Parent],
                  transactions: Optional[Sequence[Optional[bytes]]], signature, itx_json: bytes = b"",
                  bsig_json: bytes = b"") -> int:
        """`signature`: the Event.Signature text (decoded as
        keys.DecodeSignature) or a (pre, r_be, s_be) tuple."""
        kinds, refs = [], []
        for p in parents:
            if p is None:
                kinds.append(PARENT_NONE)
                refs.append(0)
            elif p[0] == "hash":
                kinds.append(PARENT_HASH)
                refs.append(len(self._hashes))
                self._hashes.append(bytes(p[1]))
            else:
                kinds.append(PARENT_EVENT)
                refs.append(int(p[1]))
        if isinstance(signature, tuple):
            pre, r, s = signature
        else:
            pre, r, s = native.decode_signature(signature)
        self._ev.append((creator, index, timestamp, kinds, refs,
                         None if transactions is None else [None if t is None else bytes(t) for t in transactions],
                         bytes(itx_json), bytes(bsig_json), pre, r, s))
        return len(self._ev) - 1

    def pack(self) -> EventWireBatch:
        n = len(self._ev)
        key_off = np.zeros(len(self._keys) + 1, np.uint64)
        key_off[1:] = np.cumsum([len(k) for k in self._keys], dtype=np.uint64)
        txs = [t for e in self._ev for t in (e[5] or [])]
        tx_start = np.zeros(n + 1, np.uint64)
        tx_start[1:] = np.cumsum([len(e[5] or []) for e in self._ev], dtype=np.uint64)
        tx_off = np.zeros(len(txs) + 1, np.uint64)
        tx_off[1:] = np.cumsum([len(t or b"") for t in txs], dtype=np.uint64)
        itx = [e[6] for e in self._ev]
        bsg = [e[7] for e in self._ev]

        def frag(xs):
            if not any(xs):
                return None, np.zeros(0, np.uint8)
            off = np.zeros(n + 1, np.uint64)
            off[1:] = np.cumsum([len(x) for x in xs], dtype=np.uint64)
            return off, np.frombuffer(b"".join(xs), np.uint8).copy()

        itx_off, itx_json = frag(itx)
        bsig_off, bsig_json = frag(bsg)
        return EventWireBatch(
            key_bytes=np.frombuffer(b"".join(self._keys), np.uint8).copy(), key_off=key_off,
            creator=np.array([e[0] for e in self._ev], np.uint32),
            index=np.array([e[1] for e in self._ev], np.int64),
            timestamp=np.array([e[2] for e in self._ev], np.int64),
            parent_kind=np.array([e[3] for e in self._ev], np.uint8).reshape(n, 2),
            parent_ref=np.array([e[4] for e in self._ev], np.uint64).reshape(n, 2),
            parent_hashes=np.frombuffer(b"".join(self._hashes), np.uint8).reshape(-1, 32).copy(),
            tx_start=tx_start, tx_off=tx_off, tx_bytes=np.frombuffer(b"".join(t or b"" for t in txs), np.uint8).copy(),
            tx_list_nil=np.array([e[5] is None for e in self._ev], np.uint8)
            if any(e[5] is None for e in self._ev) else None,
            tx_nil=np.array([t is None for t in txs], np.uint8) if any(t is None for t in txs) else None,
            itx_off=itx_off, itx_json=itx_json, bsig_off=bsig_off, bsig_json=bsig_json,
            r_be=np.frombuffer(b"".join(e[9] for e in self._ev), np.uint8).reshape(n, 32).copy(),
            s_be=np.frombuffer(b"".join(e[10] for e in self._ev), np.uint8).reshape(n, 32).copy(),
            pre=np.array([e[8] for e in self._ev], np.uint8))


def wire_bytes(b: EventWireBatch) -> int:
    """Bytes bv_verify_events stages over PCIe for this batch."""
    arrs = [b.key_bytes, b.key_off, b.creator, b.index, b.timestamp, b.parent_kind, b.parent_ref, b.parent_hashes,
            b.tx_start, b.tx_off, b.tx_bytes, b.itx_json, b.bsig_json, b.r_be, b.s_be]
    arrs += [a for a in (b.tx_list_nil, b.tx_nil, b.itx_off, b.bsig_off, b.pre) if a is not None]
    return int(sum(a.nbytes for a in arrs))
