"""Same-box A/B of process-level env knobs (development tool): each variant
runs in its own child process (the library reads the knobs once per process)
over cold device-resident C2 batches from 64 creators at several sizes, two
batches in flight as bench.py; variants interleaved, median of 3 rounds.

  python tools/ab_env.py "base:" "var:AB_LIB=gpurun_var/x.so" [--sizes=250000,1000000]
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(sizes):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch

    from babble_amd import native, synth

    if os.environ.get("AB_LIB"):  # a library variant (tools/build_variant.sh)
        native.LIB_PATH = os.path.abspath(os.environ["AB_LIB"])
        native._lib = None
    from babble_amd.verifier import Verifier

    out = {}
    for n in sizes:
        b = synth.events(n, n_creators=int(os.environ.get("AB_CREATORS", "64")), seed=2)
        v = Verifier(0)
        ds = [v.to_device(b) for _ in range(2)]
        for k in range(4):
            v.verify_device(ds[k % 2], stream=0, sync=False)
        torch.cuda.synchronize()
        v.sync()
        steps = max(20, int(30e6 // n))
        t0 = time.perf_counter()
        for k in range(steps):
            v.verify_device(ds[k % 2], stream=0, sync=False)
        v.sync()
        el = time.perf_counter() - t0
        assert np.all(ds[0].result().status == 1) and np.all(ds[1].result().status == 1)
        out[n] = n * steps / el / 1e6
        v.close()
        del ds, b
    print("RESULT " + json.dumps(out), flush=True)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    sizes = [250_000, 1_000_000]
    for a in sys.argv[1:]:
        if a.startswith("--sizes="):
            sizes = [int(x) for x in a.split("=", 1)[1].split(",")]
    if "--child" in sys.argv:
        child(sizes)
        return
    variants = []
    for a in args:
        name, _, kv = a.partition(":")
        env = dict(x.split("=", 1) for x in kv.split(",") if x)
        variants.append((name, env))
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
            for n, v in json.loads(line[7:]).items():
                res.setdefault((int(n), name), []).append(v)
            print(f"round {rnd} {name} {line[7:]}", flush=True)
    import statistics
    for (n, name), xs in sorted(res.items()):
        print(f"events {n:8d} {name:10s} {statistics.median(xs):7.1f} M/s  {[round(x, 1) for x in xs]}")


if __name__ == "__main__":
    main()
