"""Two contexts on one device (development tool): how long a small
cold verify on context B takes while context A runs back-to-back bulk
bv_verify_events calls, against B alone.  Each variant runs in its own child
process (the library reads its env knobs once), e.g.

  python tools/ab_twoctx.py "split:BV_EV_VERIFY_STREAM=1" "main:BV_EV_VERIFY_STREAM=0"

B's batch: 1000 C2 events from 64 creators through bv_verify_batch (key
tables built per call).  A's batch: 1M C2 events with parents by hash through
bv_verify_events.  Reported: B's median / p90 latency alone and under load,
and A's calls per second under load."""
import json
import os
import statistics
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, ROOT)
    import numpy as np

    from babble_amd import synth
    from babble_amd.verifier import Verifier

    small = synth.events(1000, n_creators=64, seed=5)
    _, wire = synth.event_fields(1_000_000, n_creators=64, seed=2, parents="hash")
    va, vb = Verifier(0), Verifier(0)
    va.verify_events(wire)
    for _ in range(5):
        vb.verify(small)

    def lat(n):
        xs = []
        for _ in range(n):
            t0 = time.perf_counter()
            r = vb.verify(small)
            xs.append((time.perf_counter() - t0) * 1e3)
            assert np.all(r.status == 1)
        return xs

    alone = lat(60)
    stop = threading.Event()
    calls = [0]

    def load():
        while not stop.is_set():
            va.verify_events(wire)
            calls[0] += 1

    th = threading.Thread(target=load)
    t0 = time.perf_counter()
    th.start()
    time.sleep(0.05)
    loaded = lat(60)
    stop.set()
    th.join()
    el = time.perf_counter() - t0

    def q(xs, p):
        return round(sorted(xs)[int(p * (len(xs) - 1))], 3)

    print("RESULT " + json.dumps({"alone_med": q(alone, 0.5), "alone_p90": q(alone, 0.9),
                                  "loaded_med": q(loaded, 0.5), "loaded_p90": q(loaded, 0.9),
                                  "A_calls_per_s": round(calls[0] / el, 1)}), flush=True)


def main():
    if "--child" in sys.argv:
        child()
        return
    res = {}
    for rnd in range(2):
        for a in sys.argv[1:]:
            name, _, kv = a.partition(":")
            e = dict(os.environ)
            e.update(dict(x.split("=", 1) for x in kv.split(",") if x))
            p = subprocess.run([sys.executable, "-u", __file__, "--child"], env=e, capture_output=True, text=True,
                               timeout=300)
            if p.returncode != 0:
                print(p.stdout[-2000:], p.stderr[-3000:])
                sys.exit(p.returncode)
            line = [x for x in p.stdout.splitlines() if x.startswith("RESULT ")][-1][7:]
            print(f"round {rnd} {name:8s} {line}", flush=True)
            res.setdefault(name, []).append(json.loads(line))
    for name, xs in res.items():
        print(name, {k: statistics.median(x[k] for x in xs) for k in xs[0]})


if __name__ == "__main__":
    main()
