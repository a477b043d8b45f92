"""Multi-GPU sharding of a verify batch — the torch.distributed
(one process per GPU) side; the single-process C-ABI group (bv_group_*,
csrc/bv_group.cpp) uses the same plan.

Items are independent once bodies are serialised, so a batch shards by
contiguous item ranges, one range per rank, with one all-gather of the accept
bitmasks (RCCL over xGMI on MI355X; gloo in CPU tests) and no other
data-path collective.  Two plans:

* `shard_bounds`: 64-aligned ranges, so every rank's bitmask words are whole
  and the global bitmask is the plain concatenation (events: one item per
  message);
* `plan_shards`: the C ABI's bv_plan_shards — balanced ranges cut only where
  the message changes, so the items of one message (a BlockBody's 100
  validator signatures, block.go:343 / hashgraph.go:1599-1630) stay on one
  rank and the body is hashed once; bitmasks are then merged by bit shifts
  (`merge_bits`).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

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


def plan_shards(item_msg: np.ndarray, world: int) -> List[int]:
    """bv_plan_shards (csrc/bv_group.cpp): world + 1 bounds; cut c is the
    first index >= n * g / world where item_msg changes."""
    n = len(item_msg)
    bounds = [0]
    for g in range(1, world):
        c = max(bounds[-1], n * g // world)
        while 0 < c < n and item_msg[c] == item_msg[c - 1]:
            c += 1
        bounds.append(min(c, n))
    bounds.append(n)
    return bounds


def plan_group(item_msg: np.ndarray, n_msgs: int, world: int):
    """bv_plan_group (csrc/hostplan.cpp) restated: (permuted, perm,
    item_bounds, msg_bounds).  Items are stably sorted by message when
    item_msg is not non-decreasing; item shards follow plan_shards over that
    order; device d hashes messages [msg_bounds[d], msg_bounds[d+1]) — a
    partition of [0, n_msgs) cut at each shard's first message."""
    im = np.asarray(item_msg, dtype=np.int64)
    n = len(im)
    permuted = bool(n > 1 and np.any(im[1:] < im[:-1]))
    perm = np.argsort(im, kind="stable") if permuted else np.arange(n)
    srt = im[perm]
    bounds = plan_shards(srt, world)
    mb, prev = [], 0
    for d in range(world):
        cut = 0 if d == 0 else (int(srt[bounds[d]]) if bounds[d] < n else n_msgs)
        prev = max(prev, cut)
        mb.append(prev)
    return permuted, perm, bounds, mb + [n_msgs]


def merge_bits(shard_words: Sequence[np.ndarray], bounds: Sequence[int]) -> np.ndarray:
    """Global accept bitmask from per-shard bitmasks whose bit 0 is the
    shard's first item (the host merge after bv_group's all-gather)."""
    n = bounds[-1]
    W = (n + 63) // 64
    out = np.zeros(max(W, 1), np.uint64)
    for d, words in enumerate(shard_words):
        a, cnt = bounds[d], bounds[d + 1] - bounds[d]
        for w in range((cnt + 63) // 64):
            v = int(words[w])
            valid = min(64, cnt - 64 * w)
            if valid < 64:
                v &= (1 << valid) - 1
            bit = a + 64 * w
            q, s = bit // 64, bit % 64
            out[q] |= np.uint64((v << s) & 0xFFFFFFFFFFFFFFFF)
            if s and q + 1 < W:
                out[q + 1] |= np.uint64(v >> (64 - s))
    return out[:W]


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
    path) for 64-aligned `shard_bounds` shards.  Returns the global bitmask
    (ceil(n_items/64) words)."""
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


def allgather_bits_planned(local_bits, bounds: Sequence[int], world: int):
    """The same for message-aligned `plan_shards` bounds: pad every shard's
    words to the largest, ONE all-gather, then merge by bit shifts."""
    import torch
    import torch.distributed as dist

    per_words = max(1, max((bounds[r + 1] - bounds[r] + 63) // 64 for r in range(world)))
    send = torch.zeros(per_words, dtype=torch.int64, device=local_bits.device)
    send[: local_bits.numel()] = local_bits
    out = torch.empty(per_words * world, dtype=torch.int64, device=local_bits.device)
    dist.all_gather_into_tensor(out, send)
    g = out.cpu().numpy().view(np.uint64).reshape(world, per_words)
    return merge_bits([g[r] for r in range(world)], bounds)
