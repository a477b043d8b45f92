"""Where a SyncResponse's DAG hashing spends its time (development tool):
runs bv_verify_events over the 1000-event, 4-creator SyncResponse DAG
(bench.py events_entry sync_dag_1000) with diagnostic builds of the library
(-DBV_CHAIN_STAMPS: k_ev_hash_chain stamps s_memrealtime at its phase
boundaries) and prints, per library, the median per-level time of each
phase: B (parent hex splice + barrier), C (schedules + barrier), D (rounds,
wave 0), E (the end-of-level barrier: staging beside D), and the call's
median wall time."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from babble_amd import native, synth  # noqa: E402
from babble_amd import verifier as V  # noqa: E402

_, dag = synth.event_fields(1000, n_creators=4, seed=31, parents="event")
out = {}
for lib in sys.argv[1:]:
    native.LIB_PATH = os.path.abspath(lib)
    native._lib = None
    v = V.Verifier(0, flags=native.F_KEY_CACHE)
    v.verify_events(dag)
    ts = []
    for _ in range(11):
        t0 = time.perf_counter()
        res = v.verify_events(dag)
        ts.append((time.perf_counter() - t0) * 1e3)
    assert np.all(res.status == 1)
    L = ctypes.CDLL(native.LIB_PATH)
    buf = (ctypes.c_uint64 * (5 * 96 + 1))()
    assert L.bv_debug_chain_stamps(buf) == 0
    st = np.frombuffer(buf, np.uint64)
    nl = int(st[-1])
    s = st[: 5 * min(nl, 96)].reshape(-1, 5).astype(np.int64)
    ph = np.diff(s, axis=1) * 10.0 / 1000.0  # 100 MHz ticks -> us
    nxt = (s[1:, 0] - s[:-1, 4]) * 10.0 / 1000.0
    out[os.path.basename(lib)] = {
        "call_ms_median": float(np.median(ts)), "levels_in_launch": nl,
        "us_per_level_median": {"B_splice": float(np.median(ph[:, 0])), "C_sched": float(np.median(ph[:, 1])),
                                "D_rounds": float(np.median(ph[:, 2])), "E_barrier": float(np.median(ph[:, 3])),
                                "between_levels": float(np.median(nxt)) if len(nxt) else None,
                                "total": float(np.median(s[:, 4] - s[:, 0]) * 10.0 / 1000.0)},
        "us_per_level_mean": {k: round(float(np.mean(ph[:, c])), 2) for c, k in enumerate(("B", "C", "D", "E"))},
        "total_p10_p90_max": [round(float(np.percentile(s[:, 4] - s[:, 0], q)) * 0.01, 2) for q in (10, 90, 100)],
        "launch_us": round(float(s[-1, 4] - s[0, 0]) * 0.01, 1)}
    v.close()
    print(os.path.basename(lib), json.dumps(out[os.path.basename(lib)]), flush=True)
