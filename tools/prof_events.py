"""Profile bv_verify_events (bulk, 1M events, parents by hash) and a
1000-event sync DAG: host wall times per call; run under rocprofv3
--kernel-trace --stats for the device side."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from babble_amd import native, synth  # noqa: E402
from babble_amd.verifier import Verifier  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
_, wire = synth.event_fields(n, n_creators=64, seed=2, parents="hash")
v = Verifier(0)
for i in range(4):
    t0 = time.perf_counter()
    res = v.verify_events(wire)
    t = v.timing()
    print(f"bulk {n}: {1e3 * (time.perf_counter() - t0):.2f} ms  prep {t['ms_host_prep']:.2f} out {t['ms_host_out']:.2f} h2d {t['ms_h2d']:.2f}  dev_total {t['ms_total']:.2f} "
          f"sha {t['ms_sha256']:.2f} g {t['ms_verify_g']:.2f} q {t['ms_verify']:.2f}", flush=True)
assert np.all(res.status == 1)
_, dag = synth.event_fields(1000, n_creators=4, seed=31, parents="event")
vc = Verifier(0, flags=native.F_KEY_CACHE)
for i in range(6):
    t0 = time.perf_counter()
    res = vc.verify_events(dag)
    print(f"sync dag 1000: {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
assert np.all(res.status == 1)
