"""Shared test helpers: golden fixture loading and batch construction."""
from __future__ import annotations

import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def load(name: str):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def golden_items_batch():
    """PackedBatch of golden_items.json built from the fixture's pre/r/s
    (one message and one key per item, keys deduplicated by bytes) plus the
    expected statuses."""
    from babble_amd.batch import BatchBuilder

    items = load("golden_items.json")
    bb = BatchBuilder()
    for it in items:
        m = bb.add_msg(bytes.fromhex(it["body"]))
        k = bb.add_key(bytes.fromhex(it["pub"]))
        bb.add_item_raw(m, k, it["pre"], bytes.fromhex(it["r"]), bytes.fromhex(it["s"]))
    return bb.pack(), np.array([it["status"] for it in items], np.uint8), items


def bits_from_status(st: np.ndarray) -> np.ndarray:
    n = len(st)
    out = np.zeros((n + 63) // 64, np.uint64)
    for i in np.flatnonzero(st == 1):
        out[i // 64] |= np.uint64(1) << np.uint64(i % 64)
    return out
