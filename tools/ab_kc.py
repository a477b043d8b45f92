"""Same-box A/B of library variants on the key-cache path (development tool):
1M resident C2 events from 64 registered creators, two batches in flight as
bench.py's `warm` leg; verifies/s over 40 steps and k_verify_gq's span of a
batch alone.  Each variant in its own child process, interleaved, 3 rounds.

  python tools/ab_kc.py "base:" "var:AB_LIB=gpurun_var/x.so"
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, ROOT)
    import numpy as np  # noqa: F401
    import torch

    from babble_amd import native, synth

    if os.environ.get("AB_LIB"):
        native.LIB_PATH = os.path.abspath(os.environ["AB_LIB"])
        native._lib = None
    from babble_amd.verifier import Verifier

    b = synth.events(1_000_000, n_creators=64, seed=2)
    v = Verifier(0, flags=native.F_KEY_CACHE)
    v.register_keys([b.key(k) for k in range(b.n_keys)])
    ds = [v.to_device(b) for _ in range(2)]
    for k in range(4):
        v.verify_device(ds[k % 2], stream=0, sync=False)
    torch.cuda.synchronize()
    v.sync()
    steps = 40
    t0 = time.perf_counter()
    for k in range(steps):
        v.verify_device(ds[k % 2], stream=0, sync=False)
    v.sync()
    el = time.perf_counter() - t0
    spans = []
    for _ in range(3):
        v.verify_device(ds[0], sync=True)
        spans.append(v.timing()["ms_verify"])
    assert int((ds[0].result().status == 1).sum()) == b.n_items
    v.close()
    print(json.dumps({"value": b.n_items * steps / el, "k_verify_gq_ms": min(spans)}), flush=True)


if __name__ == "__main__":
    if os.environ.get("AB_CHILD"):
        child()
        sys.exit(0)
    variants = []
    for a in sys.argv[1:]:
        name, _, envs = a.partition(":")
        env = dict(os.environ, AB_CHILD="1")
        for kv in filter(None, envs.split(",")):
            k, _, val = kv.partition("=")
            env[k] = val
        variants.append((name, env))
    res = {n: [] for n, _ in variants}
    for rnd in range(3):
        for name, env in variants:
            p = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, capture_output=True, text=True,
                               timeout=300)
            line = [x for x in p.stdout.splitlines() if x.startswith("{")]
            if p.returncode != 0 or not line:
                print(name, "failed", p.stderr[-2000:], flush=True)
                sys.exit(1)
            r = json.loads(line[-1])
            res[name].append(r)
            print(f"round {rnd} {name:8s} {r['value'] / 1e6:7.1f} M/s  k_verify_gq {r['k_verify_gq_ms']:.3f} ms",
                  flush=True)
