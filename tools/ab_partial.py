"""the key cache's partial mode against the per-batch
tables for a 1M-event batch of 20 creators where ONE creator (50k items)
has no table.  Partial mode keeps the 19 cached keys on the KC kernels and
finishes the fresh key's items on the generic per-lane path
(k_verify_deferred); the alternative is the per-batch K12 tables for all 20
keys (a context without the key cache).  Device entry (batch resident) and
host entry (pinned), 5 timed calls each after one untimed; BV_KC_ADMIT is
raised so the fresh key stays fresh.  Every result is checked.
Partial mode is off by default now (the result of this A/B): the first
variant turns it on with BV_KC_PARTIAL=1, the second shows the default."""
import os
import sys
import time

os.environ.setdefault("BV_KC_ADMIT", "1000")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from babble_amd import native, synth  # noqa: E402
from babble_amd.verifier import PinnedArena, Verifier, VerifyResult  # noqa: E402

def run(v, b, label):
    d = v.to_device(b)
    v.verify_device(d, sync=True)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        v.verify_device(d, sync=True)
        ts.append((time.perf_counter() - t0) * 1e3)
    assert np.all(d.result().status == 1)
    t = v.timing()
    out = f"{label:34s} device entry {np.median(ts):7.3f} ms (key_path {t['key_path']}, kc_hits {t['kc_hits']})"
    if b.n_items >= 1_000_000:
        arena = PinnedArena()
        try:
            pb = arena.batch(b)
            res = VerifyResult(arena.array((b.n_msgs, 32), np.uint8), arena.array(b.n_items, np.uint8),
                               arena.array((b.n_items + 63) // 64, np.uint64))
            v.verify_into(pb, res)
            th = []
            for _ in range(5):
                t0 = time.perf_counter()
                v.verify_into(pb, res)
                th.append((time.perf_counter() - t0) * 1e3)
            assert np.all(res.status == 1)
        finally:
            arena.close()
        out += f"  host entry pinned {np.median(th):7.3f} ms"
    print(out, flush=True)


for n in [int(x) for x in os.environ.get("AB_SIZES", "1000000").split(",")]:
    b = synth.events(n, n_creators=20, seed=21)
    fresh_items = int((np.asarray(b.item_key) == 0).sum())
    keys = [b.key(k) for k in range(b.n_keys)]
    print(f"{n} events, 20 creators, fresh key 0 signs {fresh_items} items", flush=True)
    os.environ["BV_KC_PARTIAL"] = "1"  # (read at context creation; off by default since this A/B)
    vc = Verifier(device=0, flags=native.F_KEY_CACHE)
    os.environ.pop("BV_KC_PARTIAL")
    vc.register_keys(keys[1:])
    run(vc, b, "key cache, partial (1 fresh of 20)")
    vc.close()
    vd = Verifier(device=0, flags=native.F_KEY_CACHE)
    vd.register_keys(keys[1:])
    run(vd, b, "key cache, 1 fresh, default (no partial)")
    vd.close()
    v0 = Verifier(device=0)
    run(v0, b, "per-batch tables (no cache)")
    v0.close()
    vf = Verifier(device=0, flags=native.F_KEY_CACHE)
    vf.register_keys(keys)
    run(vf, b, "key cache, all 20 registered")
    vf.close()
