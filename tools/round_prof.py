"""Per-item kernel time of device-resident verify launches at 250k vs 1M
items, back to back (development tool): whether a launch of about one round
of waves (250k items: ~3.8 waves per SIMD) is slower per item than a 1M
launch when the chip stays busy, or only after idle gaps (the chunked host
entries)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from babble_amd import synth  # noqa: E402
from babble_amd.verifier import Verifier  # noqa: E402

v = Verifier(0)
for n in (250_000, 1_000_000, 250_000):
    b = synth.events(n, n_creators=64, seed=5)
    d = v.to_device(b)
    for gap in (0.0, 0.005):
        rows = []
        for _ in range(8):
            v.verify_device(d, stream=0, sync=True)
            rows.append(v.timing())
            if gap:
                torch.cuda.synchronize()
                import time

                time.sleep(gap)
        med = {k: round(float(np.median([r[k] for r in rows[2:]])), 3) for k in ("ms_verify_g", "ms_verify", "ms_sha256")}
        print("n", n, "idle gap ms", gap * 1e3, med, "q ns/item", round(med["ms_verify"] * 1e6 / n, 2), flush=True)
v.close()
