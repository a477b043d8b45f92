import os, sys, ctypes, time
os.environ["BV_EVC_PROF"] = "1"
sys.path.insert(0, "/root/repo")
import numpy as np
from babble_amd import native, synth
from babble_amd.verifier import Verifier
_, dag = synth.event_fields(1000, n_creators=4, seed=31, parents="event")
vc = Verifier(0, flags=native.F_KEY_CACHE)
for i in range(4):
    t0 = time.perf_counter(); res = vc.verify_events(dag); print("ms", (time.perf_counter()-t0)*1e3)
L = native.lib(); out = (ctypes.c_uint64 * 8)()
L.bv_debug_evc_prof(out)
names = ["prologue", "A:stage+pf", "B:splice", "C:schedule", "D:rounds", "sync", "-", "-"]
tot = sum(out)
for n, v in zip(names, out): print(f"{n:12s} {v:10d} cycles  {v/2.4e3:8.1f} us  ({v/249/2.4e3:6.2f} us/level)")
