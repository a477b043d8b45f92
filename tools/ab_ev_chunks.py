"""A/B of bv_verify_events' staging chunk size (BV_EV_CHUNK_MB, read at
bv_create; AB_LIB=<library variant> for same-box A/Bs of staging code) on
the bench's bulk events batch (1M C2 events, parents by known
hash), pageable and from bv_host_alloc memory: median wall ms of 5 calls
after a warm-up, h2d span, all statuses checked.

    python tools/ab_ev_chunks.py [sizes in MB ...]

A size may carry other knobs read at bv_create: "64:BV_QFIRST=0" (colon-
separated KEY=VAL after the size).  ROUNDS=n repeats the variant list.
Every variant runs in a fresh child process (a second Verifier in one
process measured ~0.7 ms slower per call, whatever the variant).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from babble_amd import native, synth  # noqa: E402

if os.environ.get("AB_LIB"):  # a library variant (tools/build_variant.sh)
    native.LIB_PATH = os.path.abspath(os.environ["AB_LIB"])
    native._lib = None
from babble_amd.verifier import PinnedArena, Verifier, VerifyResult  # noqa: E402

sizes = sys.argv[1:] or ["16", "32", "64"]  # BV_EV_CHUNK_MB values
if os.environ.get("AB_CHILD") is None:
    import subprocess

    for spec in sizes * int(os.environ.get("ROUNDS", "1")):
        subprocess.run([sys.executable, "-u", os.path.abspath(__file__), spec], env=dict(os.environ, AB_CHILD="1"),
                       check=True)
    sys.exit(0)
n = 1_000_000
_, wire = synth.event_fields(n, n_creators=64, seed=2, parents="hash")
arena = PinnedArena()
pw = arena.wire(wire)
res = VerifyResult(arena.array((n, 32), np.uint8), arena.array(n, np.uint8), arena.array((n + 63) // 64, np.uint64))
for spec in sizes:
    mb, *knobs = spec.split(":")
    os.environ["BV_EV_CHUNK_MB"] = mb
    for kv in knobs:
        k, val = kv.split("=")
        os.environ[k] = val
    v = Verifier(0)
    for kv in knobs:
        del os.environ[kv.split("=")[0]]
    for name, call in (("pinned", lambda: v.verify_events_into(pw, res)), ("pageable", lambda: v.verify_events(wire))):
        call()
        ts = []
        for _ in range(int(os.environ.get("CALLS", "5"))):
            t0 = time.perf_counter()
            r = call()
            ts.append((time.perf_counter() - t0) * 1e3)
        assert np.all(r.status == 1)
        t = v.timing()
        ms = float(np.median(ts))
        print(f"{os.environ.get('AB_LIB', 'HEAD'):>20s} chunk {spec:>14s} MB {name:8s} median {ms:.3f} ms ({n / ms / 1e3:.1f} M/s)  min {min(ts):.3f}  "
              f"h2d {t['ms_h2d']:.3f}  device {t['ms_total']:.3f}  host_prep {t['ms_host_prep']:.3f}", flush=True)
    v.close()
arena.close()
