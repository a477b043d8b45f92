"""The SyncResponse DAG call (1000 events, 4 registered creators) repeated
for a kernel + copy trace (development tool): run under rocprofv3
--kernel-trace --memory-copy-trace, then tools/lat_timeline.py lays out the
last call."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from babble_amd import native, synth  # noqa: E402
from babble_amd.verifier import Verifier  # noqa: E402

packed, dag = synth.event_fields(1000, n_creators=4, seed=31, parents="event")
v = Verifier(0, flags=native.F_KEY_CACHE)
v.register_keys([packed.key(k) for k in range(packed.n_keys)])
ts = []
for _ in range(20):
    t0 = time.perf_counter()
    r = v.verify_events(dag)
    ts.append((time.perf_counter() - t0) * 1e3)
assert np.all(r.status == 1)
print("median ms", round(float(np.median(ts)), 3), "last", round(ts[-1], 3), v.timing())
