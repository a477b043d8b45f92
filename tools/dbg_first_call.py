"""Debug: the first k_small call of fresh processes (the bootstrap test's
first batch) against the C oracle; PROCS children, sequential (development
tool)."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("CHILD") is None:
    bad = 0
    for p in range(int(os.environ.get("PROCS", "12"))):
        r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__)], env=dict(os.environ, CHILD="1"),
                           capture_output=True, text=True, timeout=120)
        line = [x for x in r.stdout.splitlines() if x.startswith("result")]
        print(p, r.returncode, line[-1] if line else r.stderr[-300:], flush=True)
        bad += 0 if line and line[-1].endswith("mismatches 0") else 1
    print("processes with mismatches or errors:", bad)
    sys.exit(0)
import numpy as np  # noqa: E402

from babble_amd import native  # noqa: E402
from babble_amd.batch import BatchBuilder  # noqa: E402

if os.environ.get("AB_LIB"):  # a library variant (tools/build_variant.sh)
    native.LIB_PATH = os.path.abspath(os.environ["AB_LIB"])
    native._lib = None
from babble_amd.verifier import Verifier  # noqa: E402
from oracle import coracle  # noqa: E402
from tests.test_bootstrap import make_db  # noqa: E402

evs = make_db(int(os.environ.get("N_EVENTS", "256")))  # <= 256: the cold k_small limit
bb = BatchBuilder()
for ev in evs:
    bb.add_item(bb.add_msg(ev.Body.Marshal()), bb.add_key(ev.Body.Creator or b""), ev.Signature)
p = bb.pack()
mode = os.environ.get("MODE", "cold")
if mode == "warm":
    v = Verifier(0, flags=native.F_KEY_CACHE)
    v.register_keys([evs[0].Body.Creator])
else:
    v = Verifier(0)
if os.environ.get("PRECALL") == "1":  # one unrelated device call first
    v.sha256([b"x" * 100])
elif os.environ.get("PRECALL") == "2":  # a different 500-event cold batch first
    bb2 = BatchBuilder()
    for ev in make_db(500, seed=77):
        bb2.add_item(bb2.add_msg(ev.Body.Marshal()), bb2.add_key(ev.Body.Creator or b""), ev.Signature)
    v.verify(bb2.pack())
h, st, _ = coracle.verify_batch(p.as_dict())
reps, nbad, items = int(os.environ.get("REPEAT", "1")), 0, []
for _ in range(reps):
    res = v.verify(p)
    bad = np.flatnonzero(res.status != st)
    nbad += int(bad.size > 0)
    items += bad[:3].tolist()
if reps > 1:
    print(f"repeat {reps} calls with mismatches {nbad} items {items[:12]}")
print(f"result key_path {v.timing()['key_path']} items {bad[:6].tolist()} gpu {res.status[bad[:6]].tolist()} "
      f"mismatches {bad.size}", flush=True)
v.close()
