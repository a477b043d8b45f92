"""Mid-size cold batches: per-batch K8 vs K12 key tables (BV_F_K8) at
62.5k / 125k / 250k / 500k C2 events from 64 creators, device-resident, two
batches in flight (as bench.py), variants interleaved; median of 3 rounds."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from babble_amd import native, synth  # noqa: E402
from babble_amd.verifier import Verifier  # noqa: E402

res = {}
for n in (62_500, 125_000, 250_000, 500_000):
    b = synth.events(n, n_creators=64, seed=2)
    for rnd in range(3):
        for name, flags in (("K12-rule", 0), ("K8", native.F_K8)):
            v = Verifier(0, flags=flags)
            ds = [v.to_device(b) for _ in range(2)]
            for k in range(4):
                v.verify_device(ds[k % 2], stream=0, sync=False)
            torch.cuda.synchronize()
            v.sync()
            steps = 30
            t0 = time.perf_counter()
            for k in range(steps):
                v.verify_device(ds[k % 2], stream=0, sync=False)
            v.sync()
            el = time.perf_counter() - t0
            assert np.all(ds[0].result().status == 1)
            kp = v.timing()["key_path"]
            res.setdefault((n, name), []).append((n * steps / el / 1e6, kp))
            v.close()
for (n, name), xs in sorted(res.items()):
    print(f"events {n:7d} {name:8s} key_path {xs[0][1]:2d}  {np.median([x[0] for x in xs]):7.1f} M/s  {[round(x[0], 1) for x in xs]}")
