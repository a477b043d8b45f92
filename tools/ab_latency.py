"""Same-box A/B of library variants on small-batch latency (development
tool): bv_verify_batch from host buffers at 1 / 1000 events, cold and with
the key cache warm, variants interleaved round-robin."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from babble_amd import native, synth  # noqa: E402
from babble_amd import verifier as V  # noqa: E402

libs = sys.argv[1:]
bs = {n: synth.events(n, n_creators=min(4, n), seed=900 + n) for n in (1, 1000)}
res = {}
for rnd in range(3):
    for lib in libs:
        native.LIB_PATH = os.path.abspath(lib)
        native._lib = None
        for mode, flags in (("cold", native.F_DEFAULT), ("warm", native.F_KEY_CACHE)):
            v = V.Verifier(0, flags=flags)
            for n, b in bs.items():
                v.verify(b)
                ts = []
                for _ in range(30):
                    t0 = time.perf_counter()
                    v.verify(b)
                    ts.append((time.perf_counter() - t0) * 1e3)
                res.setdefault((os.path.basename(lib), mode, n), []).append(float(np.median(ts)))
            v.close()
for k, v in sorted(res.items()):
    print(k, [round(x, 3) for x in v])
