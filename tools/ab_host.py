"""Same-box A/B of bv_verify_batch (the generic host entry) on the bench's
1M C2 batch built in bv_host_alloc memory (results pinned too), one child
process per variant (development tool).  A variant is colon-separated
KEY=VAL knobs read at bv_create ("base" for none); ROUNDS=n, CALLS=n.

    python tools/ab_host.py base BV_QFIRST=0 "BV_QFIRST=0:BV_EV_D2H=0"
"""
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

specs = sys.argv[1:] or ["base"]
if os.environ.get("AB_CHILD") is None:
    for spec in specs * int(os.environ.get("ROUNDS", "1")):
        env = dict(os.environ, AB_CHILD="1")
        for kv in spec.split(":"):
            if "=" in kv:
                k, v = kv.split("=")
                env[k] = v
        subprocess.run([sys.executable, "-u", os.path.abspath(__file__), spec], env=env, check=True)
    sys.exit(0)

import numpy as np  # noqa: E402

from babble_amd import synth  # noqa: E402
from babble_amd.verifier import PinnedArena, Verifier, VerifyResult  # noqa: E402

n = 1_000_000
batch = synth.events(n, n_creators=64, seed=2, tx_bytes=64)
v = Verifier(0)
arena = PinnedArena()
pb = arena.batch(batch)
res = VerifyResult(arena.array((n, 32), np.uint8), arena.array(n, np.uint8), arena.array((n + 63) // 64, np.uint64))
pageable = os.environ.get("PAGEABLE") == "1"  # the arrays and results in ordinary memory
call = (lambda: v.verify(batch)) if pageable else (lambda: v.verify_into(pb, res))
call()
ts, tm = [], []
for _ in range(int(os.environ.get("CALLS", "7"))):
    t0 = time.perf_counter()
    out = call()
    ts.append((time.perf_counter() - t0) * 1e3)
    tm.append(v.timing())
assert np.all((out if pageable else res).status == 1)
ms = float(np.median(ts))
print(f"host_entry {'pageable' if pageable else 'pinned'} {specs[0]:>28s} median {ms:.3f} ms ({n / ms / 1e3:.1f} M/s)  min {min(ts):.3f}  "
      f"h2d {np.median([t['ms_h2d'] for t in tm]):.3f}  device {np.median([t['ms_total'] for t in tm]):.3f}  "
      f"host_prep {np.median([t['ms_host_prep'] for t in tm]):.3f}", flush=True)
arena.close()
v.close()
