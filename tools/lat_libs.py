import os, sys, time, statistics
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
import numpy as np
from babble_amd import native, synth
bs = {n: synth.events(n, n_creators=4, seed=900 + n) for n in (50000, 100000)}
for rnd in range(2):
    for lib in sys.argv[1:]:
        native.LIB_PATH = os.path.abspath(lib); native._lib = None
        from babble_amd import verifier as V
        for mode in ("cold", "warm"):
            v = V.Verifier(0, flags=native.F_KEY_CACHE if mode == "warm" else 0)
            for n, b in bs.items():
                if mode == "warm":
                    v.register_keys([b.key(k) for k in range(b.n_keys)])
                v.verify(b)
                ts = []
                for _ in range(15):
                    t0 = time.perf_counter(); r = v.verify(b); ts.append((time.perf_counter() - t0) * 1e3)
                assert np.all(r.status == 1)
                print(rnd, os.path.basename(lib), mode, n, round(statistics.median(ts), 3), flush=True)
            v.close()
