"""Small-batch latency breakdown of bv_verify_batch (development tool):
wall time per call and the library's host / device phases, key cache warm."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from babble_amd import native, synth  # noqa: E402
from babble_amd.verifier import Verifier  # noqa: E402

vc = Verifier(0, flags=native.F_KEY_CACHE)
for n in (1, 100, 1000, 10000):
    b = synth.events(n, n_creators=min(4, n), seed=900 + n)
    vc.verify(b)
    rows = []
    for _ in range(20):
        t0 = time.perf_counter()
        vc.verify(b)
        wall = (time.perf_counter() - t0) * 1e3
        t = vc.timing()
        rows.append([wall, t["ms_host"], t["ms_host_prep"], t["ms_h2d"], t["ms_total"], t["ms_host_out"],
                     t["ms_sha256"], t["ms_verify_g"], t["ms_verify"]])
    m = np.median(np.array(rows), axis=0)
    print(f"n={n:6d} wall {m[0]:.3f} host {m[1]:.3f} prep {m[2]:.3f} h2d {m[3]:.3f} dev_total {m[4]:.3f} "
          f"out {m[5]:.3f} | sha {m[6]:.3f} g {m[7]:.3f} q {m[8]:.3f}", flush=True)
