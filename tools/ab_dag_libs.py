"""Same-box A/B of library variants on the in-batch DAG path (development
tool): bv_verify_events over a SyncLimit 1000-event batch and C1's 10k events
(4 creators, parents in the batch), key cache warm; variants interleaved,
median of 15 calls per round, 3 rounds.  python tools/ab_dag_libs.py a.so b.so"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from babble_amd import native, synth  # noqa: E402

dags = {n: synth.event_fields(n, n_creators=4, seed=1, parents="event") for n in (1000, 10_000)}
res = {}
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for lib in sys.argv[1:]:
        native.LIB_PATH = os.path.abspath(lib)
        native._lib = None
        from babble_amd import verifier as V

        for n, (packed, dag) in dags.items():
            v = V.Verifier(0, flags=native.F_KEY_CACHE)
            v.register_keys([packed.key(k) for k in range(packed.n_keys)])
            v.verify_events(dag)
            ts = []
            for _ in range(15):
                t0 = time.perf_counter()
                r = v.verify_events(dag)
                ts.append((time.perf_counter() - t0) * 1e3)
            assert np.all(r.status == 1)
            v.close()
            res.setdefault((lib, n), []).append(float(np.median(ts)))
for (lib, n), xs in sorted(res.items()):
    print(f"{lib:28s} events {n:6d}  {min(xs):7.3f} ms  {[round(x, 3) for x in xs]}")
