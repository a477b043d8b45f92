"""bv_verify_events on the bench's bulk events batch (1M C2 events, every
parent a known hash), 5 calls after a warm-up, for a rocprofv3
--kernel-trace --memory-copy-trace run (development tool): prints each
call's wall time; tools/lat_timeline.py lays out the last call."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from babble_amd import synth  # noqa: E402
from babble_amd.verifier import Verifier  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
_, wire = synth.event_fields(n, n_creators=64, seed=2, parents="hash")
v = Verifier(0)
v.verify_events(wire)
for _ in range(5):
    t0 = time.perf_counter()
    res = v.verify_events(wire)
    print("call ms", round((time.perf_counter() - t0) * 1e3, 3), v.timing(), flush=True)
assert np.all(res.status == 1)
v.close()
