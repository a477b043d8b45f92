"""Small-batch latency: bv_verify_batch from host buffers at
1 / 16 / 64 / 100 / 256 / 1000 events from 4 creators, cold (no key cache)
and warm (creators registered with bv_kc_register), through the small-batch
kernel (default) and the bulk pipeline (BV_SMALL=0).  Median wall ms of 30
calls and the device kernel span of the last call; every result checked."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from babble_amd import native, synth  # noqa: E402
from babble_amd.verifier import Verifier  # noqa: E402

sizes = [int(x) for x in (sys.argv[1:] or ["1", "16", "64", "100", "256", "1000"])]
bs = {n: synth.events(n, n_creators=min(4, n), seed=900 + n) for n in sizes}
for small in ("1", "0"):
    os.environ["BV_SMALL"] = small
    for mode in ("cold", "warm"):
        v = Verifier(0, flags=native.F_KEY_CACHE if mode == "warm" else 0)
        for n, b in bs.items():
            if mode == "warm":
                v.register_keys([b.key(k) for k in range(b.n_keys)])
            v.verify(b)
            ts = []
            for _ in range(30):
                t0 = time.perf_counter()
                r = v.verify(b)
                ts.append((time.perf_counter() - t0) * 1e3)
            assert np.all(r.status == 1), (small, mode, n)
            t = v.timing()
            print(f"small={small} {mode:4s} n={n:5d} median {np.median(ts):.3f} ms  min {min(ts):.3f}  "
                  f"kernels {t['ms_total']:.3f}  key_path {t['key_path']}", flush=True)
        v.close()
