"""Same-box A/B of library variants (development tool): for each .so given,
time bv_verify_batch_device over the same resident 1M-event C2 batch, cold
(per-key tables rebuilt each call) and warm (key cache), interleaving the
variants round-robin so clock drift hits all of them alike."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from babble_amd import native, synth  # noqa: E402

libs = sys.argv[1:]
n = int(os.environ.get("AB_N", "1000000"))
b = synth.events(n, n_creators=64, seed=2)
res = {l: {"cold": [], "warm": [], "sha": []} for l in libs}
from babble_amd import verifier as V  # noqa: E402

for rnd in range(3):
    for l in libs:
        native.LIB_PATH = os.path.abspath(l)  # Verifier binds native.lib() at construction
        native._lib = None
        for mode, flags in (("cold", native.F_DEFAULT), ("warm", native.F_KEY_CACHE)):
            v = V.Verifier(0, flags=flags)
            d = v.to_device(b)
            v.verify_device(d)
            v.verify_device(d)
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                v.verify_device(d)
                ts.append(time.perf_counter() - t0)
            st = d.result().status
            assert np.count_nonzero(st == 1) == n, np.bincount(st)
            res[l][mode].append(min(ts) * 1e3)
            if mode == "cold":
                res[l]["sha"].append(v.timing()["ms_sha256"])
            v.close()
        print(rnd, l, {m: round(res[l][m][-1], 4) for m in res[l]}, flush=True)
for l in libs:
    print(f"{l}: cold {min(res[l]['cold']):.4f} ms  warm {min(res[l]['warm']):.4f} ms  k_sha256 {min(res[l]['sha']):.4f} ms")
