"""Single-call cold latency of generic-path batches (many keys, few items per
key) for library variants (development tool):
  python tools/lat_gen.py gpurun_var/a.so gpurun_var/b.so
Median wall ms of 15 bv_verify_batch calls per size, 1000 creators, every
result checked against the expected all-accept."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from babble_amd import native, synth  # noqa: E402

os.environ["BV_TABLE_MIN_ITEMS"] = "100000"
bs = {n: synth.events(n, n_creators=1000, seed=900 + n) for n in (2000, 8000, 32000, 64000)}
for rnd in range(2):
    for lib in sys.argv[1:]:
        native.LIB_PATH = os.path.abspath(lib)
        native._lib = None
        from babble_amd import verifier as V
        v = V.Verifier(0)
        for n, b in bs.items():
            v.verify(b)
            ts = []
            for _ in range(15):
                t0 = time.perf_counter()
                r = v.verify(b)
                ts.append((time.perf_counter() - t0) * 1e3)
            assert np.all(r.status == 1) and v.timing()["key_path"] == 0
            print(rnd, os.path.basename(lib), n, round(statistics.median(ts), 3), flush=True)
        v.close()
