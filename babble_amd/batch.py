"""Packed struct-of-arrays batches for the C ABI (bv_batch).

A batch holds N messages (canonical JSON bodies, hashed once each), K public
keys (raw bytes, validated on the device) and M signature items, each naming
a message and a key and carrying r, s (32-byte big-endian) plus the host
pre-class byte (keys.DecodeSignature result, see include/babbleverify.h).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np

from . import native


@dataclass
class PackedBatch:
    msg_bytes: np.ndarray          # u8
    msg_off: np.ndarray            # u64, n_msgs + 1
    key_bytes: np.ndarray          # u8
    key_off: np.ndarray            # u64, n_keys + 1
    item_msg: np.ndarray           # u32
    item_key: np.ndarray           # u32
    r_be: np.ndarray               # u8 [n, 32]
    s_be: np.ndarray               # u8 [n, 32]
    pre: Optional[np.ndarray]      # u8 [n] or None (all zero)

    @property
    def n_msgs(self) -> int:
        return len(self.msg_off) - 1

    @property
    def n_keys(self) -> int:
        return len(self.key_off) - 1

    @property
    def n_items(self) -> int:
        return len(self.item_msg)

    def as_dict(self) -> Dict[str, np.ndarray]:
        return dict(msg_bytes=self.msg_bytes, msg_off=self.msg_off, key_bytes=self.key_bytes,
                    key_off=self.key_off, item_msg=self.item_msg, item_key=self.item_key,
                    r_be=self.r_be, s_be=self.s_be, pre=self.pre)

    def message(self, m: int) -> bytes:
        return self.msg_bytes[self.msg_off[m]:self.msg_off[m + 1]].tobytes()

    def key(self, k: int) -> bytes:
        return self.key_bytes[self.key_off[k]:self.key_off[k + 1]].tobytes()


class BatchBuilder:
    """Incrementally builds a PackedBatch; keys are de-duplicated by bytes."""

    def __init__(self):
        self._msgs: List[bytes] = []
        self._keys: List[bytes] = []
        self._key_idx: Dict[bytes, int] = {}
        self._item_msg: List[int] = []
        self._item_key: List[int] = []
        self._r: List[bytes] = []
        self._s: List[bytes] = []
        self._pre: List[int] = []

    def add_msg(self, body: bytes) -> int:
        self._msgs.append(bytes(body))
        return len(self._msgs) - 1

    def add_key(self, pub: bytes) -> int:
        pub = bytes(pub)
        k = self._key_idx.get(pub)
        if k is None:
            k = len(self._keys)
            self._keys.append(pub)
            self._key_idx[pub] = k
        return k

    def add_item(self, msg: int, key: int, signature) -> int:
        """signature: the r|s text of EncodeSignature (DecodeSignature semantics)."""
        pre, r, s = native.decode_signature(signature)
        return self.add_item_raw(msg, key, pre, r, s)

    def add_item_raw(self, msg: int, key: int, pre: int, r_be: bytes, s_be: bytes) -> int:
        self._item_msg.append(msg)
        self._item_key.append(key)
        self._pre.append(pre)
        self._r.append(bytes(r_be))
        self._s.append(bytes(s_be))
        return len(self._item_msg) - 1

    def pack(self) -> PackedBatch:
        def cat(chunks):
            off = np.zeros(len(chunks) + 1, np.uint64)
            if chunks:
                off[1:] = np.cumsum([len(c) for c in chunks], dtype=np.uint64)
            buf = np.frombuffer(b"".join(chunks), np.uint8).copy() if chunks else np.zeros(0, np.uint8)
            return buf, off

        mb, mo = cat(self._msgs)
        kb, ko = cat(self._keys)
        n = len(self._item_msg)
        r = np.frombuffer(b"".join(self._r), np.uint8).reshape(n, 32).copy() if n else np.zeros((0, 32), np.uint8)
        s = np.frombuffer(b"".join(self._s), np.uint8).reshape(n, 32).copy() if n else np.zeros((0, 32), np.uint8)
        return PackedBatch(mb, mo, kb, ko, np.array(self._item_msg, np.uint32), np.array(self._item_key, np.uint32),
                           r, s, np.array(self._pre, np.uint8))
