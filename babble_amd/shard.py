"""Multi-GPU sharding of a verify batch.

Items are independent once bodies are serialised, so a batch shards by
contiguous item ranges, one range per rank (one process per GPU).  Ranges are
64-aligned so every rank's accept-bitmask words are whole and the global
bitmask is the plain concatenation of the per-rank bitmasks — one
all-gather (RCCL over xGMI on MI355X; gloo in CPU tests) and no other
data-path collective.  Block workloads shard by block (a block's signatures
stay on one rank) by choosing ranges on message boundaries.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

from .batch import PackedBatch


def shard_bounds(n_items: int, world: int, rank: int, align: int = 64) -> Tuple[int, int]:
    """[lo, hi) of rank's contiguous share; lo and hi are multiples of
    `align` except hi == n_items for the last non-empty shard."""
    words = (n_items + align - 1) // align
    per = (words + world - 1) // world
    lo = min(rank * per * align, n_items)
    hi = min((rank + 1) * per * align, n_items)
    return lo, hi


def slice_batch(b: PackedBatch, lo: int, hi: int) -> PackedBatch:
    """Items [lo, hi) with only the messages they reference (re-indexed);
    the key table is kept whole (it is small and replicated per rank)."""
    item_msg = b.item_msg[lo:hi]
    used, inv = np.unique(item_msg, return_inverse=True)
    lens = (b.msg_off[used + 1] - b.msg_off[used]).astype(np.uint64)
    off = np.zeros(len(used) + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    if len(used) and np.all(np.diff(used) == 1):  # contiguous messages: one slice
        msg = b.msg_bytes[int(b.msg_off[used[0]]):int(b.msg_off[used[-1] + 1])].copy()
    else:
        msg = np.concatenate([b.msg_bytes[int(b.msg_off[m]):int(b.msg_off[m + 1])] for m in used]) \
            if len(used) else np.zeros(0, np.uint8)
    return PackedBatch(msg, off, b.key_bytes, b.key_off, inv.astype(np.uint32), b.item_key[lo:hi].copy(),
                       b.r_be[lo:hi].copy(), b.s_be[lo:hi].copy(),
                       None if b.pre is None else b.pre[lo:hi].copy())


def allgather_bits(local_bits, n_items: int, world: int, rank: int):
    """Concatenate every rank's accept-bitmask words (torch.distributed
    all_gather_into_tensor; the local tensor's device picks the backend
    path).  Returns the global bitmask (ceil(n_items/64) words)."""
    import torch
    import torch.distributed as dist

    per_words = max((shard_bounds(n_items, world, r)[1] - shard_bounds(n_items, world, r)[0] + 63) // 64
                    for r in range(world))
    send = torch.zeros(per_words, dtype=torch.int64, device=local_bits.device)
    send[: local_bits.numel()] = local_bits
    out = torch.empty(per_words * world, dtype=torch.int64, device=local_bits.device)
    dist.all_gather_into_tensor(out, send)
    words = []
    for r in range(world):
        lo, hi = shard_bounds(n_items, world, r)
        words.append(out[r * per_words: r * per_words + (hi - lo + 63) // 64])
    return torch.cat(words)
