"""Seeded synthetic workloads for the SURVEY §8d configurations (bench and
test input only — not part of the verification path).

  events(...)       C1 (4 creators, 10k), C2 (64 creators, 1M), C3 shards
  adversarial(...)  C4: C2-style batch + the 1 % corruption mix
  blocks(...)       C5: BlockBodies x validators

Generation runs in libbvsynth.so (OpenSSL signing with per-signer nonce
pools; see babble_amd/synth/synth.cpp).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

from .batch import PackedBatch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libbvsynth.so")

N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
P = 2**256 - 2**32 - 977
TS0 = 1_600_000_000
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built; run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        u64, u32, i64, vp = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int64, ctypes.c_void_p
        L.synth_events_capacity.argtypes = [u64, u32, u32]
        L.synth_events_capacity.restype = u64
        L.synth_events.argtypes = [u64, u32, u64, u32, u32, u32, i64, vp, u64, vp, vp, vp, vp, vp]
        L.synth_events.restype = u64
        L.synth_events_fields.argtypes = [u64, u32, u64, u32, u32, u32, i64, vp, u64, vp, vp, vp, vp, vp, vp, vp,
                                          vp, vp, vp]
        L.synth_events_fields.restype = u64
        L.synth_blocks_capacity.argtypes = [u64, u32, u32]
        L.synth_blocks_capacity.restype = u64
        L.synth_blocks.argtypes = [u64, u32, u64, u32, u32, u32, i64, vp, u64, vp, vp, vp, vp, vp, vp, vp]
        L.synth_blocks.restype = u64
        _lib = L
    return _lib


def events(n_events: int, n_creators: int = 64, seed: int = 2, n_tx: int = 1, tx_bytes: int = 64,
           nonce_pool: int = 64, ts0: int = TS0) -> PackedBatch:
    """Signed Events of a round-robin hashgraph; item i = event i."""
    L = lib()
    cap = L.synth_events_capacity(n_events, n_tx, tx_bytes)
    msg = np.zeros(cap + 64, np.uint8)
    off = np.zeros(n_events + 1, np.uint64)
    keys = np.zeros(65 * n_creators, np.uint8)
    item_key = np.zeros(n_events, np.uint32)
    r = np.zeros((n_events, 32), np.uint8)
    s = np.zeros((n_events, 32), np.uint8)
    used = L.synth_events(seed, n_creators, n_events, n_tx, tx_bytes, min(nonce_pool, max(n_events, 1)), ts0,
                          msg.ctypes.data, cap, off.ctypes.data, keys.ctypes.data, item_key.ctypes.data,
                          r.ctypes.data, s.ctypes.data)
    if used == 0 and n_events > 0:
        raise RuntimeError("synth_events failed")
    key_off = np.arange(n_creators + 1, dtype=np.uint64) * 65
    return PackedBatch(msg[:used], off, keys, key_off, np.arange(n_events, dtype=np.uint32), item_key, r, s,
                       np.zeros(n_events, np.uint8))


def event_fields(n_events: int, n_creators: int = 64, seed: int = 2, n_tx: int = 1, tx_bytes: int = 64,
                 nonce_pool: int = 64, ts0: int = TS0, parents: str = "event"):
    """The synth_events hashgraph as (PackedBatch of serialized bodies,
    events.EventWireBatch of the same events' wire fields).  parents="event":
    in-batch parents by event index (the core.sync DAG); "hash": every
    parent by its known hash (a store / bootstrap replay: no in-batch
    dependency)."""
    from .events import PARENT_EVENT, PARENT_HASH, PARENT_NONE, EventWireBatch

    L = lib()
    cap = L.synth_events_capacity(n_events, n_tx, tx_bytes)
    msg = np.zeros(cap + 64, np.uint8)
    off = np.zeros(n_events + 1, np.uint64)
    keys = np.zeros(65 * n_creators, np.uint8)
    item_key = np.zeros(n_events, np.uint32)
    r = np.zeros((n_events, 32), np.uint8)
    s = np.zeros((n_events, 32), np.uint8)
    dig = np.zeros((n_events, 32), np.uint8)
    par = np.zeros((n_events, 2), np.int64)
    idx = np.zeros(n_events, np.int64)
    ts = np.zeros(n_events, np.int64)
    tx = np.zeros(n_events * n_tx * tx_bytes, np.uint8)
    used = L.synth_events_fields(seed, n_creators, n_events, n_tx, tx_bytes, min(nonce_pool, max(n_events, 1)), ts0,
                                 msg.ctypes.data, cap, off.ctypes.data, keys.ctypes.data, item_key.ctypes.data,
                                 r.ctypes.data, s.ctypes.data, dig.ctypes.data, par.ctypes.data, idx.ctypes.data,
                                 ts.ctypes.data, tx.ctypes.data)
    if used == 0 and n_events > 0:
        raise RuntimeError("synth_events failed")
    key_off = np.arange(n_creators + 1, dtype=np.uint64) * 65
    packed = PackedBatch(msg[:used].copy(), off, keys, key_off, np.arange(n_events, dtype=np.uint32), item_key, r, s,
                         np.zeros(n_events, np.uint8))
    kind = np.where(par < 0, PARENT_NONE, PARENT_EVENT if parents == "event" else PARENT_HASH).astype(np.uint8)
    if parents == "event":
        ref = np.where(par < 0, 0, par).astype(np.uint64)
        hashes = np.zeros((0, 32), np.uint8)
    else:
        ref = np.where(par < 0, 0, par).astype(np.uint64)  # parent_hashes[i] = digest of event i
        hashes = dig
    wire = EventWireBatch(
        key_bytes=keys, key_off=key_off, creator=item_key, index=idx, timestamp=ts, parent_kind=kind,
        parent_ref=ref, parent_hashes=hashes, tx_start=np.arange(n_events + 1, dtype=np.uint64) * n_tx,
        tx_off=np.arange(n_events * n_tx + 1, dtype=np.uint64) * tx_bytes, tx_bytes=tx,
        tx_list_nil=np.ones(n_events, np.uint8) if n_tx == 0 else None, tx_nil=None, itx_off=None,
        itx_json=np.zeros(0, np.uint8), bsig_off=None, bsig_json=np.zeros(0, np.uint8), r_be=r.copy(), s_be=s.copy(),
        pre=np.zeros(n_events, np.uint8))
    return packed, wire


def c3_chunk(idx: int, n: int = 1_000_000, n_creators: int = 64):
    """Chunk `idx` of the C3 workload (10^8 events, seed 3, 64
    creators, streamed in chunks): the same 64 creators (seed 3) in every
    chunk, chunk idx's events timestamped after chunk idx-1's (one stream of
    10^8 distinct bodies); about one item in 10^4 (seeded by idx) gets one r
    bit flipped, so the exact accept bitmask is known by construction.
    Returns (batch, sorted indices of the flipped items)."""
    b = events(n, n_creators=n_creators, seed=3, ts0=TS0 + idx * n)
    rng = np.random.default_rng(1000 + idx)
    bad = np.sort(rng.choice(n, max(1, n // 10_000), replace=False))
    b.r_be[bad, int(rng.integers(0, 32))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    return b, bad


def expected_bits(n: int, rejected) -> np.ndarray:
    """Accept bitmask words (LSB-first) with every item accepted except `rejected`."""
    ok = np.ones(n, bool)
    ok[np.asarray(rejected, dtype=np.int64)] = False
    pk = np.packbits(ok, bitorder="little")
    return np.concatenate([pk, np.zeros((-len(pk)) % 8, np.uint8)]).view(np.uint64)[: (n + 63) // 64]


@dataclass
class BlockWorkload:
    batch: PackedBatch
    n_blocks: int
    n_validators: int
    peers_hash: bytes


def blocks(n_blocks: int, n_validators: int = 100, seed: int = 5, n_tx: int = 16, tx_bytes: int = 64,
           nonce_pool: int = 64, ts0: int = TS0) -> BlockWorkload:
    L = lib()
    n_items = n_blocks * n_validators
    cap = L.synth_blocks_capacity(n_blocks, n_tx, tx_bytes)
    msg = np.zeros(cap + 64, np.uint8)
    off = np.zeros(n_blocks + 1, np.uint64)
    keys = np.zeros(65 * n_validators, np.uint8)
    ph = np.zeros(32, np.uint8)
    item_msg = np.zeros(n_items, np.uint32)
    item_key = np.zeros(n_items, np.uint32)
    r = np.zeros((n_items, 32), np.uint8)
    s = np.zeros((n_items, 32), np.uint8)
    used = L.synth_blocks(seed, n_validators, n_blocks, n_tx, tx_bytes, nonce_pool, ts0, msg.ctypes.data, cap,
                          off.ctypes.data, keys.ctypes.data, ph.ctypes.data, item_msg.ctypes.data,
                          item_key.ctypes.data, r.ctypes.data, s.ctypes.data)
    if used == 0 and n_blocks > 0:
        raise RuntimeError("synth_blocks failed")
    key_off = np.arange(n_validators + 1, dtype=np.uint64) * 65
    b = PackedBatch(msg[:used].copy(), off, keys, key_off, item_msg, item_key, r, s, np.zeros(n_items, np.uint8))
    return BlockWorkload(b, n_blocks, n_validators, ph.tobytes())


# ---------------------------------------------------------------------------
# C4 adversarial mix
# ---------------------------------------------------------------------------
def _cls(v: int) -> int:
    if v <= 0:
        return 2  # NONPOS
    if v >= N:
        return 3  # GE_N
    return 0


def _be(v: int) -> bytes:
    return (v % 2**256).to_bytes(32, "big")


def adversarial(n_events: int, seed: int = 4, n_creators: int = 64, scale_per_million=None) -> PackedBatch:
    """C2-style batch with the C4 corruption mix, scaled to n_events.

    Per 10^6 items: 2500 r bit-flips, 2500 s bit-flips, 1000 body mutations,
    1000 high-S (N - s, must ACCEPT), 500 r/s in {0, N, N+1, -x}, 500 string
    format errors (parts != 2 -> REJECT_ERR; empty part / bad char -> nil),
    1000 malformed public keys (empty, 33-byte compressed, prefix 0x06,
    x >= p, off-curve y, valid-but-wrong key).
    """
    b = events(n_events, n_creators=n_creators, seed=seed)
    rng = np.random.default_rng(seed)
    mix = scale_per_million or dict(rflip=2500, sflip=2500, body=1000, highs=1000, range=500, fmt=500, key=1000)
    counts = {k: max(1, int(round(v * n_events / 1_000_000))) for k, v in mix.items()}
    total = sum(counts.values())
    if total > n_events:
        raise ValueError("batch too small for the mix")
    idx = rng.permutation(n_events)[:total]
    groups = {}
    o = 0
    for k, c in counts.items():
        groups[k] = idx[o:o + c]
        o += c
    r, s, pre = b.r_be, b.s_be, b.pre
    msg = b.msg_bytes
    for i in groups["rflip"]:
        bit = int(rng.integers(256))
        v = int.from_bytes(r[i].tobytes(), "big") ^ (1 << bit)
        r[i] = np.frombuffer(_be(v), np.uint8)
        pre[i] = _cls(v) | (_cls(int.from_bytes(s[i].tobytes(), "big")) << 2)
    for i in groups["sflip"]:
        bit = int(rng.integers(256))
        v = int.from_bytes(s[i].tobytes(), "big") ^ (1 << bit)
        s[i] = np.frombuffer(_be(v), np.uint8)
        pre[i] = _cls(int.from_bytes(r[i].tobytes(), "big")) | (_cls(v) << 2)
    for i in groups["body"]:
        # mutate one byte of the Timestamp digits (body stays valid JSON-ish)
        end = int(b.msg_off[i + 1])
        pos = end - 3  # last timestamp digit before "}\n"
        msg[pos] = ord("0") + (msg[pos] - ord("0") + 1) % 10
    for i in groups["highs"]:
        v = N - int.from_bytes(s[i].tobytes(), "big")
        s[i] = np.frombuffer(_be(v), np.uint8)
    specials = [0, N, N + 1, -5]
    for j, i in enumerate(groups["range"]):
        # the host decode leaves the 32-byte value zero when the class is not OK
        v = specials[j % 4]
        if (j // 4) % 2 == 0:
            r[i] = 0
            pre[i] = _cls(v) | (pre[i] & 0x0C)
        else:
            s[i] = 0
            pre[i] = (pre[i] & 0x03) | (_cls(v) << 2)
    for j, i in enumerate(groups["fmt"]):
        kind = j % 4
        if kind in (0, 1):        # 1 or 3 parts -> DecodeSignature error
            pre[i] = 0x80
            r[i] = 0
            s[i] = 0
        elif kind == 2:           # empty r part -> SetString fails -> nil r
            pre[i] = 1 | (pre[i] & 0x0C)
            r[i] = 0
        else:                     # bad char in s -> nil s
            pre[i] = (pre[i] & 0x03) | (1 << 2)
            s[i] = 0
    # malformed keys appended to the key table
    keys = [b.key(k) for k in range(b.n_keys)]
    good = keys[0]
    x = int.from_bytes(good[1:33], "big")
    y = int.from_bytes(good[33:65], "big")
    bad = [
        b"",
        bytes([2 + (y & 1)]) + good[1:33],
        b"\x06" + good[1:],
        b"\x04" + (P + 1).to_bytes(32, "big") + good[33:],   # x >= p
        b"\x04" + good[1:33] + (y ^ 1).to_bytes(32, "big"),  # off-curve y
        keys[1 % len(keys)],  # valid but wrong key -> REJECT
    ]
    base = len(keys)
    keys_all = keys + bad
    key_off = np.zeros(len(keys_all) + 1, np.uint64)
    key_off[1:] = np.cumsum([len(k) for k in keys_all])
    item_key = b.item_key
    for j, i in enumerate(groups["key"]):
        kk = j % len(bad)
        if kk == 5:
            item_key[i] = (item_key[i] + 1) % b.n_keys  # another creator's valid key
        else:
            item_key[i] = base + kk
    b.key_bytes = np.frombuffer(b"".join(keys_all), np.uint8).copy()
    b.key_off = key_off
    return b
