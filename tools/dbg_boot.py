"""Debug: the bootstrap test's batches through the host entry against the
C oracle, REPS times (development tool)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from babble_amd.batch import BatchBuilder  # noqa: E402
from babble_amd.verifier import Verifier  # noqa: E402
from oracle import coracle  # noqa: E402
from tests.test_bootstrap import make_db  # noqa: E402

evs = make_db(1200, bad={1111})
v = Verifier(0)
packs = []
for lo, hi in ((0, 500), (500, 1000), (1000, 1200)):
    bb = BatchBuilder()
    for ev in evs[lo:hi]:
        m = bb.add_msg(ev.Body.Marshal())
        k = bb.add_key(ev.Body.Creator or b"")
        bb.add_item(m, k, ev.Signature)
    p = bb.pack()
    packs.append((lo, p, coracle.verify_batch(p.as_dict())))
fails = 0
for rep in range(int(os.environ.get("REPS", "40"))):
    for lo, p, (h, st, _) in packs:
        res = v.verify(p)
        bad = np.flatnonzero(res.status != st)
        if bad.size:
            fails += 1
            print(f"rep {rep} batch@{lo} key_path {v.timing()['key_path']} mismatches {bad.size}: items {bad[:6] + lo} "
                  f"gpu {res.status[bad[:6]]} oracle {st[bad[:6]]}", flush=True)
print("failing calls", fails, flush=True)
v.close()
