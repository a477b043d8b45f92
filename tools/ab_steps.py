"""Same-box A/B of library builds (development tool), bench-shaped: for each
.so given, the C2 headline step (1M resident events, per-key tables rebuilt,
two batches in flight on the library's lanes) timed over K steps, plus the
per-kernel breakdown of a batch alone on the chip; variants interleaved
round-robin so clock drift hits all alike.  Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from babble_amd import native, synth  # noqa: E402
from babble_amd import verifier as V  # noqa: E402

libs = sys.argv[1:]
steps = int(os.environ.get("AB_STEPS", "30"))
b = synth.events(1_000_000, n_creators=64, seed=2)
out = {l: {"ms_per_step": [], "breakdown": []} for l in libs}
for rnd in range(int(os.environ.get("AB_ROUNDS", "3"))):
    for l in libs:
        native.LIB_PATH = os.path.abspath(l)
        native._lib = None
        v = V.Verifier(0)
        ds = [v.to_device(b) for _ in range(2)]
        for k in range(4):
            v.verify_device(ds[k % 2], stream=0, sync=False)
        v.sync()
        t0 = time.perf_counter()
        for k in range(steps):
            v.verify_device(ds[k % 2], stream=0, sync=False)
        v.sync()
        out[l]["ms_per_step"].append((time.perf_counter() - t0) / steps * 1e3)
        ts = []
        for _ in range(3):
            v.verify_device(ds[0], sync=True)
            ts.append(v.timing())
        out[l]["breakdown"].append({k: float(np.mean([t[k] for t in ts]))
                                    for k in ("ms_sha256", "ms_scalar", "ms_verify_g", "ms_verify", "ms_total")})
        for d in ds:
            assert np.count_nonzero(d.result().status == 1) == b.n_items
        v.close()
        print(rnd, os.path.basename(l), round(out[l]["ms_per_step"][-1], 4), out[l]["breakdown"][-1], flush=True)
print(json.dumps({os.path.basename(l): {"best_ms_per_step": min(r["ms_per_step"]),
                                         "verifies_per_s": 1e6 / (min(r["ms_per_step"]) * 1e-3),
                                         "breakdown_best": min(r["breakdown"], key=lambda x: x["ms_total"])}
                  for l, r in out.items()}))
