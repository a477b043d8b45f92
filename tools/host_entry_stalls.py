"""How often a pageable host-entry call stalls: one
process, one context, 1M C2 events, 2 untimed calls then 60 timed ones;
prints the median call, the calls slower than 1.3x the median and the
verifies/s over all 60.  Run once per variant (env knobs are read at
bv_create)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from babble_amd import synth  # noqa: E402
from babble_amd.verifier import Verifier  # noqa: E402

b = synth.events(1_000_000, n_creators=64, seed=2)
v = Verifier(device=0)
v.verify(b)
v.verify(b)
ts = []
for _ in range(60):
    t0 = time.perf_counter()
    v.verify(b)
    ts.append((time.perf_counter() - t0) * 1e3)
v.close()
med = float(np.median(ts))
slow = [round(t, 1) for t in ts if t > 1.3 * med]
print(f"{os.environ.get('TAG', '')} median {med:.2f} ms  stalls {len(slow)}/60 {slow}  "
      f"mean rate {b.n_items * 60 / (sum(ts) * 1e-3) / 1e6:.1f} M/s", flush=True)
