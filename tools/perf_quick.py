"""Quick device-path timing on a C2-style batch (development tool)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from babble_amd import synth  # noqa: E402
from babble_amd.verifier import Verifier  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
t = time.time()
b = synth.events(n, n_creators=64, seed=2)
print(f"gen {n} events: {time.time() - t:.1f}s", flush=True)
v = Verifier(0)
d = v.to_device(b)
for it in range(4):
    t = time.time()
    v.verify_device(d)
    dt = time.time() - t
    tm = v.timing()
    print(f"iter {it}: wall {dt*1e3:.2f} ms  {n/dt/1e6:.2f} M/s  timing {tm}", flush=True)
res = d.result()
print("status counts", np.bincount(res.status, minlength=4).tolist())
