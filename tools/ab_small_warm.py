"""Warm (key cache) latency of host batches of 256..4096 events through
k_small (one workgroup per item; BV_SMALL_WARM_MAX >= n) against the bulk
pipeline (BV_SMALL_WARM_MAX=256), 4 and 64 registered creators.  Median wall
ms of 20 calls; statuses checked (development tool)."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from babble_amd import native, synth  # noqa: E402
from babble_amd.verifier import Verifier  # noqa: E402

for creators in (4, 64):
    bs = {n: synth.events(n, n_creators=creators, seed=500 + n) for n in (256, 512, 1000, 2000, 4096)}
    for rnd in range(2):
        for mx in ("256", "4096"):
            os.environ["BV_SMALL_WARM_MAX"] = mx
            v = Verifier(0, flags=native.F_KEY_CACHE)
            v.register_keys([bs[256].key(k) for k in range(bs[256].n_keys)])
            for n, b in bs.items():
                v.verify(b)
                ts = []
                for _ in range(20):
                    t0 = time.perf_counter()
                    r = v.verify(b)
                    ts.append((time.perf_counter() - t0) * 1e3)
                assert np.all(r.status == 1)
                t = v.timing()
                print(f"creators {creators:3d} warm_max {mx:>5s} n {n:5d} median {statistics.median(ts):7.3f} ms "
                      f"kernels {t['ms_total']:.3f} key_path {t['key_path']}", flush=True)
            v.close()
