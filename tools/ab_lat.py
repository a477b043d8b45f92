"""Same-box latency A/B of library variants or env knobs (development tool):
bv_verify_batch from host buffers, one call at a time, cold (no key cache),
median wall ms of 20 calls per size; each variant in its own child process,
variants interleaved, median of 3 rounds.

  AB_CREATORS=4 python tools/ab_lat.py "old:AB_LIB=gpurun_var/x.so" "new:" --sizes=1000,2000,4000
"""
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(sizes):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch  # noqa: F401

    from babble_amd import native, synth

    if os.environ.get("AB_LIB"):
        native.LIB_PATH = os.path.abspath(os.environ["AB_LIB"])
        native._lib = None
    from babble_amd.verifier import Verifier

    creators = int(os.environ.get("AB_CREATORS", "4"))
    v = Verifier(0)
    out = {}
    for n in sizes:
        b = synth.events(n, n_creators=min(creators, n), seed=900 + n)
        v.verify(b)
        ts = []
        for _ in range(20):
            t0 = time.perf_counter()
            r = v.verify(b)
            ts.append((time.perf_counter() - t0) * 1e3)
        assert np.all(r.status == 1)
        out[n] = [float(np.median(ts)), v.timing()["key_path"]]
    v.close()
    print("RESULT " + json.dumps(out), flush=True)


def main():
    sizes = [1000, 2000, 4000]
    for a in sys.argv[1:]:
        if a.startswith("--sizes="):
            sizes = [int(x) for x in a.split("=", 1)[1].split(",")]
    if "--child" in sys.argv:
        child(sizes)
        return
    variants = []
    for a in sys.argv[1:]:
        if a.startswith("--"):
            continue
        name, _, kv = a.partition(":")
        variants.append((name, dict(x.split("=", 1) for x in kv.split(",") if x)))
    res = {}
    for rnd in range(3):
        for name, env in variants:
            e = dict(os.environ)
            e.update(env)
            p = subprocess.run([sys.executable, "-u", __file__, "--child", "--sizes=" + ",".join(map(str, sizes))],
                               env=e, capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(p.stdout[-2000:], p.stderr[-3000:])
                sys.exit(p.returncode)
            line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")][-1]
            for n, (ms, kp) in json.loads(line[7:]).items():
                res.setdefault((int(n), name), []).append((ms, kp))
    for (n, name), xs in sorted(res.items()):
        print(f"events {n:6d} {name:10s} {statistics.median(x[0] for x in xs):7.3f} ms  key_path {xs[0][1]}  "
              f"{[round(x[0], 3) for x in xs]}", flush=True)


if __name__ == "__main__":
    main()
