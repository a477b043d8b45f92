"""Same-box latency A/B of library builds on the small-batch path: 1 and 100
events from 4 creators, cold (no key cache: k_small's Q doubling chain) and
warm (registered creators: the cooperative XYZZ tree), median wall ms of 30
calls, every result checked; the libraries alternate over 3 rounds.

  python tools/ab_small_lat_libs.py gpurun_var/old.so babble_amd/libbabbleverify.so
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from babble_amd import native, synth  # noqa: E402

bs = {n: synth.events(n, n_creators=min(4, n), seed=900 + n) for n in (1, 100)}
for rnd in range(3):
    for lib in sys.argv[1:]:
        native.LIB_PATH = os.path.abspath(lib)
        native._lib = None
        from babble_amd.verifier import Verifier
        for mode in ("cold", "warm"):
            v = Verifier(0, flags=native.F_KEY_CACHE if mode == "warm" else 0)
            for n, b in bs.items():
                if mode == "warm":
                    v.register_keys([b.key(k) for k in range(b.n_keys)])
                v.verify(b)
                ts = []
                for _ in range(30):
                    t0 = time.perf_counter()
                    r = v.verify(b)
                    ts.append((time.perf_counter() - t0) * 1e3)
                assert np.all(r.status == 1), (lib, mode, n)
                print(f"round {rnd} {os.path.basename(lib):24s} {mode:4s} n={n:4d} median {np.median(ts):.4f} ms",
                      flush=True)
            v.close()
