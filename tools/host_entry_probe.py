"""The pageable host entry (bv_verify_batch from ordinary buffers, C2's 1M
events) in one process, in the states the bench process passes through
(VERDICT r5 #3): (A) right after the batch is built, (B) with three more
contexts alive (the bench's later legs keep theirs), (C) after 30 resident
steps of the headline workload.  Per state: verifies/s over 5 calls, the
library's host breakdown, the cgroup's CPU throttling during the calls
(cpu.stat nr_throttled / throttled_usec), and the CPUs the process's
threads last ran on, with the GPU's NUMA node.  BV_HOST_STAMPS=1 adds the
library's per-call staging stamps on stderr."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from babble_amd import synth  # noqa: E402
from babble_amd.verifier import Verifier  # noqa: E402


def cpu_stat():
    try:
        return dict(line.split() for line in open("/sys/fs/cgroup/cpu.stat"))
    except OSError:
        return {}


def thread_cpus():
    cpus = []
    for tid in os.listdir("/proc/self/task"):
        try:
            f = open(f"/proc/self/task/{tid}/stat").read().rsplit(")", 1)[1].split()
            cpus.append(int(f[36]))  # field 39: processor
        except (OSError, IndexError, ValueError):
            pass
    return sorted(cpus)


def numa_of_cpu(c):
    base = "/sys/devices/system/node"
    try:
        for n in os.listdir(base):
            if n.startswith("node") and os.path.exists(f"{base}/{n}/cpu{c}"):
                return int(n[4:])
    except OSError:
        pass
    return None


def gpu_numa():
    out = []
    base = "/sys/class/drm"
    try:
        for d in sorted(os.listdir(base)):
            p = f"{base}/{d}/device/numa_node"
            if d.startswith("card") and "-" not in d and os.path.exists(p):
                out.append((d, open(p).read().strip()))
    except OSError:
        pass
    return out


def measure(v, batch, tag, reps=5, pause=0.0):
    v.verify(batch)
    time.sleep(pause)
    c0, t0, ru0 = cpu_stat(), time.perf_counter(), os.times()
    tms, per = [], []
    for _ in range(reps):
        t1 = time.perf_counter()
        v.verify(batch)
        per.append(round((time.perf_counter() - t1) * 1e3, 2))
        tms.append(v.timing())
    el = (time.perf_counter() - t0) / reps
    c1, ru1 = cpu_stat(), os.times()
    cpus = thread_cpus()
    nodes = {}
    for c in cpus:
        nodes[numa_of_cpu(c)] = nodes.get(numa_of_cpu(c), 0) + 1
    out = {"state": tag, "verifies_per_s": batch.n_items / el, "ms_per_call": el * 1e3, "per_call_ms": per,
           "ms_h2d": float(np.mean([t["ms_h2d"] for t in tms])),
           "ms_host": float(np.mean([t["ms_host"] for t in tms])),
           "cpu_s_per_call": ((ru1.user + ru1.system) - (ru0.user + ru0.system)) / reps,
           "throttled_per_call": {k: (int(c1.get(k, 0)) - int(c0.get(k, 0))) / reps
                                  for k in ("nr_periods", "nr_throttled", "throttled_usec")},
           "threads": len(cpus), "thread_numa_nodes": nodes}
    print(json.dumps(out), flush=True)
    return out


print(json.dumps({"gpu_numa": gpu_numa(), "main_cpu_numa": numa_of_cpu(thread_cpus()[0]) if thread_cpus() else None,
                  "affinity": len(os.sched_getaffinity(0))}), flush=True)
batch = synth.events(1_000_000, n_creators=64, seed=2)
v = Verifier(device=0)
measure(v, batch, "A fresh")
v.close()
v = Verifier(device=0)
measure(v, batch, "A2 new context, 0.5 s pause after the first call", pause=0.5)
v.close()
v = Verifier(device=0)
v.verify(batch)
measure(v, batch, "A3 new context, two untimed calls")
others = [Verifier(device=0) for _ in range(3)]
for o in others:
    o.verify(synth.events(1000, n_creators=4, seed=7))
measure(v, batch, "B three more contexts")
d = v.to_device(batch)
for _ in range(30):
    v.verify_device(d, sync=False)
torch.cuda.synchronize()
v.verify_device(d, sync=True)
measure(v, batch, "C after 30 resident steps")
for o in others:
    o.close()
measure(v, batch, "D contexts closed")
v.close()
