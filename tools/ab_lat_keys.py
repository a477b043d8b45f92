"""Cold latency of mid-small host batches by key count (development tool):
bv_verify_batch on C2 events, n items from k creators, generic per-lane path
(k > BV_LAT_TABLE_KEYS) against per-batch K8 tables (k <= it).  Median wall
ms of 20 calls; every result checked against the expected all-accept."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from babble_amd import synth  # noqa: E402
from babble_amd.verifier import Verifier  # noqa: E402

rows = []
for lat_keys in ("16", "100000", "16", "100000"):
    os.environ["BV_LAT_TABLE_KEYS"] = lat_keys
    v = Verifier(0)
    for k in (32, 64, 128, 256):
        for n in (300, 1000, 2000, 4000):
            b = synth.events(n, n_creators=k, seed=7000 + n + k)
            v.verify(b)
            ts = []
            for _ in range(20):
                t0 = time.perf_counter()
                r = v.verify(b)
                ts.append((time.perf_counter() - t0) * 1e3)
            assert np.all(r.status == 1)
            kp = v.timing()["key_path"]
            rows.append((k, n, lat_keys, statistics.median(ts), kp))
            print(f"keys {k:4d} items {n:5d} lat_table_keys {lat_keys:>6s} median {statistics.median(ts):7.3f} ms "
                  f"key_path {kp}", flush=True)
    v.close()
