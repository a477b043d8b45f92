"""Diagnose two-in-flight slot ordering: run call sequences and count
status mismatches against the C oracle per key."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from babble_amd import synth  # noqa: E402
from babble_amd.verifier import Verifier  # noqa: E402
from oracle import coracle  # noqa: E402

MIX = dict(rflip=20000, sflip=20000, body=10000, highs=10000, range=8000, fmt=8000, key=12000)
bs = [synth.adversarial(n, seed=63 + i, n_creators=c, scale_per_million=MIX)
      for i, (n, c) in enumerate([(70_000, 8), (9_000, 3), (40_000, 12)])]
want = [coracle.verify_batch(b.as_dict())[1] for b in bs]


def report(tag, j, res):
    bad = np.flatnonzero(res.status != want[j])
    keys = np.bincount(bs[j].item_key[bad], minlength=bs[j].n_keys).tolist() if bad.size else []
    print(f"{tag}: batch {j} mismatches {bad.size} per-key {keys}", flush=True)


def g6(tail, tag, pre=True):
    v = Verifier(device=0)
    ds = [v.to_device(b) for b in bs]
    ss = [torch.cuda.Stream(0), torch.cuda.Stream(0)]
    torch.cuda.synchronize()
    if pre:
        for k in range(6):
            v.verify_device(ds[k % 3], stream=ss[k % 2].cuda_stream, sync=False)
        torch.cuda.synchronize()
        v.sync()
    used = []
    for op, j, si in tail:
        if op == "h":
            report(tag + " host", j, v.verify(bs[j]))
        elif op == "x":
            with torch.cuda.stream(ss[si]):
                a = torch.randn(8192, 8192, device="cuda:0")
                for _ in range(20):
                    a = a @ a
                    a = a / a.norm()
        elif op == "s":
            torch.cuda.synchronize()
            v.sync()
        else:
            v.verify_device(ds[j], stream=ss[si].cuda_stream, sync=False)
            used.append(j)
    torch.cuda.synchronize()
    v.sync()
    for j in dict.fromkeys(used):
        report(tag, j, ds[j].result())
    v.close()


g6([("h", 1, 0), ("d", 1, 0), ("d", 0, 1)], "M")
g6([("h", 2, 0), ("d", 1, 0), ("d", 0, 1)], "N")  # host with 12 keys
g6([("h", 1, 0), ("d", 1, 0), ("d", 2, 1)], "O")  # ds2 (12 keys) on slot0
g6([("h", 1, 0), ("x", 0, 0), ("d", 0, 1)], "P")  # torch work on s0 instead of a call
g6([("h", 1, 0), ("d", 1, 1), ("d", 0, 0)], "Q")  # swapped streams
g6([("h", 1, 0), ("d", 1, 0), ("d", 0, 1)], "R", pre=False)  # fresh ctx
g6([("d", 1, 0), ("d", 1, 0), ("d", 0, 1)], "S", pre=False)  # device call instead of host
