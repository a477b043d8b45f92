"""Small-batch latency anatomy (development tool): 20 bv_verify_batch calls
of one event (cold: K8 tables; warm: key cache) after a warm-up, for a
rocprofv3 --kernel-trace --memory-copy-trace run; prints each call's wall
time.  tools/lat_timeline.py then lays the kernels and copies of the last
calls on one time axis."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402,F401
import torch  # noqa: E402,F401

from babble_amd import native, synth  # noqa: E402
from babble_amd import verifier as V  # noqa: E402

if len(sys.argv) > 1:  # a library build other than the in-tree one
    native.LIB_PATH = os.path.abspath(sys.argv[1])
    native._lib = None
b = synth.events(1, n_creators=1, seed=901)
for mode, flags in (("cold", native.F_DEFAULT), ("warm", native.F_KEY_CACHE)):
    v = V.Verifier(0, flags=flags)
    for _ in range(5):
        v.verify(b)
    ts = []
    for _ in range(20):
        t0 = time.perf_counter()
        v.verify(b)
        ts.append((time.perf_counter() - t0) * 1e3)
    print(mode, "median ms", round(float(np.median(ts)), 3), flush=True)
    v.close()
