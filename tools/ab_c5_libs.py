"""Same-box A/B of library variants on C5's host entry (development tool):
one bv_verify_batch of 10^4 BlockBodies + the Frame JSON (a 54 KB message,
hashed on the host) and 10^6 signatures from pageable host buffers, the 100
validators registered; median of 11 calls per round, variants interleaved.
python tools/ab_c5_libs.py a.so b.so"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from babble_amd import native, synth  # noqa: E402
from babble_amd.batch import PackedBatch  # noqa: E402

wb = synth.blocks(10_000, n_validators=100, seed=5)
b = wb.batch
fjson = bytes(range(256)) * 213  # a 54.5 KB item-less message in the Frame's place
off = np.concatenate([b.msg_off, [b.msg_off[-1] + len(fjson)]]).astype(np.uint64)
rb = PackedBatch(np.concatenate([b.msg_bytes, np.frombuffer(fjson, np.uint8)]), off, b.key_bytes, b.key_off,
                 b.item_msg, b.item_key, b.r_be, b.s_be, b.pre)
keys = [b.key(k) for k in range(b.n_keys)]
res = {}
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for lib in sys.argv[1:]:
        native.LIB_PATH = os.path.abspath(lib)
        native._lib = None
        from babble_amd import verifier as V

        v = V.Verifier(0, flags=native.F_KEY_CACHE)
        v.register_keys(keys)
        v.verify(rb)
        ts = []
        for _ in range(11):
            t0 = time.perf_counter()
            r = v.verify(rb)
            ts.append((time.perf_counter() - t0) * 1e3)
        assert np.all(r.status == 1)
        tm = v.timing()
        v.close()
        res.setdefault(lib, []).append(float(np.median(ts)))
        print(rnd, lib, round(float(np.median(ts)), 3), "prep", round(tm["ms_host_prep"], 3), flush=True)
for lib, xs in res.items():
    print(f"{lib:28s} {np.median(xs):7.3f} ms  {[round(x, 3) for x in xs]}")
