"""The SyncResponse DAG path: a SyncLimit-sized
(config.go:44) 1000-event batch from 4 creators with in-batch parents (333
levels of 3) through bv_verify_events, bodies built and hashed on the host
(hostdag.cpp); cold (per-batch tables) and key cache (creators registered).
Median wall ms over 25 calls; every call's digests and statuses checked.
(Round 4's A/B against the device level chain, k_ev_mid + k_ev_hash_chain,
since removed: profiles/r04_ab_dag.log.)"""
import hashlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from babble_amd import native, synth  # noqa: E402
from babble_amd.verifier import Verifier  # noqa: E402

packed, dag = synth.event_fields(1000, n_creators=4, seed=31, parents="event")
want = np.frombuffer(b"".join(hashlib.sha256(packed.message(i)).digest() for i in range(1000)), np.uint8).reshape(-1, 32)
keys = [dag.key_bytes[int(dag.key_off[k]):int(dag.key_off[k + 1])].tobytes() for k in range(len(dag.key_off) - 1)]
for mode in ("host",):
    for cache in (False, True):
        v = Verifier(0, flags=native.F_KEY_CACHE if cache else 0)
        if cache:
            v.register_keys(keys)
        v.verify_events(dag)
        ts = []
        for _ in range(25):
            t0 = time.perf_counter()
            res = v.verify_events(dag)
            ts.append((time.perf_counter() - t0) * 1e3)
            assert np.array_equal(res.msg_hash, want) and np.all(res.status == 1)
        t = v.timing()
        print(f"{mode:6s} {'key_cache' if cache else 'cold':9s} median {np.median(ts):.3f} ms  min {min(ts):.3f}  "
              f"host_prep {t['ms_host_prep']:.3f}  device {t['ms_total']:.3f}  key_path {t['key_path']}", flush=True)
        v.close()
