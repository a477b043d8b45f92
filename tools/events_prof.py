"""bv_verify_events on the bench's bulk events batch (1M C2 events, every
parent a known hash), 5 calls after a warm-up (development tool): prints
each call's wall time and timing breakdown.  `pinned` as the second
argument builds the wire batch and results in bv_host_alloc memory (the
bench's events_entry.bulk_pinned).  Run under rocprofv3 --kernel-trace
--memory-copy-trace, tools/lat_timeline.py lays out the last call; with
BV_EV_CHUNK_MB it A/Bs the staging chunk size."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from babble_amd import synth  # noqa: E402
from babble_amd.verifier import PinnedArena, Verifier, VerifyResult  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
pinned = len(sys.argv) > 2 and sys.argv[2] == "pinned"
_, wire = synth.event_fields(n, n_creators=64, seed=2, parents="hash")
v = Verifier(0)
arena = PinnedArena()
if pinned:
    wire = arena.wire(wire)
    res = VerifyResult(arena.array((n, 32), np.uint8), arena.array(n, np.uint8), arena.array((n + 63) // 64, np.uint64))
    call = lambda: v.verify_events_into(wire, res)  # noqa: E731
else:
    call = lambda: v.verify_events(wire)  # noqa: E731
call()
ts = []
for _ in range(7):
    t0 = time.perf_counter()
    res = call()
    ts.append((time.perf_counter() - t0) * 1e3)
assert np.all(res.status == 1)
tm = v.timing()
print("chunk_mb", os.environ.get("BV_EV_CHUNK_MB", "64"), "pinned", pinned, "median call ms", round(float(np.median(ts)), 3),
      {k: round(tm[k], 3) for k in ("ms_h2d", "ms_host_prep", "ms_sha256", "ms_verify")}, flush=True)
v.close()
arena.close()
