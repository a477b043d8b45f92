"""The N-GPU legs of bench.py.

`bench.py --gpus N` times one torch rank per GPU over device-resident C2
batches.  A Go caller reaches the GPUs differently: one process hands whole
batches to the library, which shards them over the node's devices itself
(bv_group_verify_batch: message-aligned shards, per-device staging from the
caller's host memory, ONE ncclAllGather of the accept bitmasks over xGMI).
This module measures that path and the shared host feed at N > 1:

  * `group` — rank 0's worker process runs bv_group_verify_batch over all N
    devices on C3-shaped input (seed 3, the same 64 creators,
    1M events per device per call, consecutive C3 chunks of one 10^8-event
    stream), built by the caller in bv_host_alloc memory, with the key cache
    on (the 64 creators admitted on their second batch, as a node's
    validator set) and cold (per-batch tables), every bitmask checked bit for
    bit; the other ranks wait at a store barrier (no GPU work, no collective
    kernel spinning on their devices).  Reference: the ingest loop
    src/node/core.go:214-245 and Bootstrap's batched replay
    src/hashgraph/hashgraph.go:1505-1531.
  * `concurrent` — every rank at once runs the two pinned host entries
    (bv_verify_batch of its 1M C2 events from bv_host_alloc memory, and
    bv_verify_events of 1M wire events), timed between store barriers, max
    over ranks: the aggregate rate the node's host memory and PCIe feed
    sustain with N devices busy.

Why a worker PROCESS for the group: its RCCL communicator (ncclCommInitAll)
and staging threads run beside the ranks' own contexts; a hang or crash in
them must not cost rank 0 its line.  The worker is started by rank 0 before
rank 0 touches a GPU (no exec from a GPU-initialised process), waits on its
stdin, and is killed (its own PID) if it overruns its time limit.

Barriers and the max-over-ranks use the rendezvous TCP store torch already
holds (no extra process group, no device collective).

`--dry-run` runs the same plumbing on CPU: the worker merges per-shard words
with the library's host helpers (bv_plan_shards, bv_merge_shard_bits) and
the concurrent legs time a CPU stand-in (tests/test_dist.py)."""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time
from datetime import timedelta

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GROUP_TIMEOUT_S = 420
STORE_TIMEOUT = timedelta(seconds=900)


# ---------------------------------------------------------------- barriers --

class StoreFence:
    """Barrier and max-over-ranks on the rendezvous store (CPU only)."""

    def __init__(self, rank: int, world: int):
        import torch.distributed.distributed_c10d as c10d

        self.store = c10d._get_default_store()
        self.rank, self.world = rank, world
        self.n = 0

    def barrier(self, tag: str = "b") -> None:
        self.n += 1
        key = f"bvfence/{tag}/{self.n}"
        self.store.set(f"{key}/{self.rank}", "1")
        self.store.wait([f"{key}/{q}" for q in range(self.world)], STORE_TIMEOUT)

    def max(self, x: float, tag: str = "m") -> float:
        self.n += 1
        key = f"bvmax/{tag}/{self.n}"
        self.store.set(f"{key}/{self.rank}", repr(float(x)))
        keys = [f"{key}/{q}" for q in range(self.world)]
        self.store.wait(keys, STORE_TIMEOUT)
        return max(float(self.store.get(k)) for k in keys)


class LocalFence:
    """World size 1: no-ops (the logical-shard rehearsal on one GPU)."""

    def barrier(self, tag: str = "b") -> None:
        pass

    def max(self, x: float, tag: str = "m") -> float:
        return float(x)


# ------------------------------------------------------------ group worker --

def start_group_worker(devices, events_per_device: int, reps: int, dry_run: bool):
    """Start the group worker (before this process touches a GPU).  It waits
    for "go" on stdin; EOF makes it exit without touching a GPU."""
    cmd = [sys.executable, os.path.abspath(__file__), "--worker", "--devices", ",".join(map(str, devices)),
           "--events-per-device", str(events_per_device), "--reps", str(reps)]
    if dry_run:
        cmd.append("--dry-run")
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK"):
        env.pop(k, None)  # the worker is not a rank
    return subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=env)


def run_group_worker(proc, timeout_s: float = GROUP_TIMEOUT_S) -> dict:
    """Release the worker and collect its JSON line (or the failure)."""
    t0 = time.perf_counter()
    try:
        out, _ = proc.communicate(input="go\n", timeout=timeout_s)
    except subprocess.TimeoutExpired:
        proc.kill()
        proc.communicate()
        return {"error": f"group worker exceeded {timeout_s:.0f}s and was killed"}
    lines = [ln for ln in (out or "").splitlines() if ln.startswith("{")]
    if proc.returncode != 0 or len(lines) != 1:
        return {"error": f"group worker exit {proc.returncode}", "stdout_tail": (out or "")[-800:]}
    res = json.loads(lines[0])
    res["worker_wall_s"] = time.perf_counter() - t0
    return res


def stop_group_worker(proc) -> None:
    """An unused worker: EOF on stdin, it exits without touching a GPU."""
    if proc is not None and proc.poll() is None:
        try:
            proc.communicate(input="", timeout=60)
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.communicate()


def concat_batches(parts):
    """One PackedBatch from chunks over the same key set (C3 chunks: seed 3,
    the same 64 creators): messages and items appended, offsets re-based."""
    import numpy as np

    from babble_amd.batch import PackedBatch

    k0 = parts[0]
    for b in parts[1:]:
        assert np.array_equal(b.key_bytes, k0.key_bytes) and np.array_equal(b.key_off, k0.key_off)
    offs, items, base_b, base_m = [], [], 0, 0
    for b in parts:
        offs.append(b.msg_off[:-1].astype(np.uint64) + np.uint64(base_b))
        items.append(b.item_msg.astype(np.uint32) + np.uint32(base_m))
        base_b += int(b.msg_off[-1])
        base_m += b.n_msgs
    offs.append(np.array([base_b], np.uint64))
    return PackedBatch(np.concatenate([b.msg_bytes[: int(b.msg_off[-1])] for b in parts]), np.concatenate(offs),
                       k0.key_bytes, k0.key_off, np.concatenate(items),
                       np.concatenate([b.item_key for b in parts]),
                       np.concatenate([b.r_be for b in parts]), np.concatenate([b.s_be for b in parts]),
                       np.concatenate([b.pre if b.pre is not None else np.zeros(b.n_items, np.uint8)
                                       for b in parts]))


def c3_group_input(n_dev: int, per_dev: int, first_chunk: int = 0):
    """n_dev consecutive C3 chunks of per_dev events (synth.c3_chunk: seed 3,
    64 creators, one timestamp stream, ~1 in 10^4 r-bit flips seeded by the
    chunk index), generated in parallel; returns (batch, rejected indices)."""
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np

    from babble_amd import synth

    with ThreadPoolExecutor(min(n_dev, 16)) as ex:
        chunks = list(ex.map(lambda i: synth.c3_chunk(first_chunk + i, per_dev), range(n_dev)))
    bad = np.concatenate([c[1] + i * per_dev for i, c in enumerate(chunks)])
    return concat_batches([c[0] for c in chunks]), bad


def _group_gpu(devices, per_dev: int, reps: int) -> dict:
    import numpy as np

    from babble_amd import native, synth
    from babble_amd.verifier import Group, PinnedArena, VerifyResult

    D = len(devices)
    logical = D > 1 and len(set(devices)) == 1
    t0 = time.perf_counter()
    batch, bad = c3_group_input(D, per_dev)
    gen_s = time.perf_counter() - t0
    n = batch.n_items
    want = synth.expected_bits(n, bad)
    arena = PinnedArena()
    out = {"devices": list(devices), "logical_shards": logical, "events_per_call": n, "events_per_device": per_dev,
           "input": "C3 chunks 0..%d (seed 3, 64 creators, consecutive timestamps), %d seeded r-bit flips; batch "
                    "built in bv_host_alloc memory, results into bv_host_alloc arrays" % (D - 1, len(bad)),
           "generate_s": gen_s,
           "collective": "device copies into shard 0 (logical shards of one device: RCCL needs distinct devices)"
           if logical else "ONE ncclAllGather of the shard bitmasks (ncclCommInitAll communicator over the devices)"}
    try:
        pb = arena.batch(batch)
        del batch
        res = VerifyResult(arena.array((pb.n_msgs, 32), np.uint8), arena.array(n, np.uint8),
                           arena.array((n + 63) // 64, np.uint64))
        for name, flags, warm in (("key_cache", native.F_KEY_CACHE, 3), ("cold", native.F_DEFAULT, 1)):
            t1 = time.perf_counter()
            g = Group(devices, flags=flags)
            create_ms = (time.perf_counter() - t1) * 1e3
            try:
                for _ in range(warm):
                    g.verify_into(pb, res)
                ts = []
                for _ in range(reps):
                    t1 = time.perf_counter()
                    g.verify_into(pb, res)
                    ts.append(time.perf_counter() - t1)
                if not np.array_equal(res.accept_bits, want):
                    raise SystemExit(f"group {name}: accept bitmask differs from the expected one")
                if not (np.all(res.status[bad] == native.REJECT) and
                        np.count_nonzero(res.status == native.ACCEPT) == n - len(bad)):
                    raise SystemExit(f"group {name}: statuses differ from the seeded rejections")
                el = float(sum(ts))
                tms = [g.timing(i) for i in range(D)]
                out[name] = {
                    "value": n * reps / el, "unit": "verifies/s", "ms_per_call": el / reps * 1e3,
                    "ms_per_call_min": min(ts) * 1e3, "calls": reps, "warmup_calls": warm,
                    "group_create_ms": create_ms,
                    "per_device": [{"device": devices[i], "ms_h2d": t["ms_h2d"], "ms_device": t["ms_total"],
                                    "ms_host_prep": t["ms_host_prep"], "ms_lib_call": t["ms_host"],
                                    "key_path": int(t["key_path"])} for i, t in enumerate(tms)],
                    "bitmask_check": f"exact: {n} events, {len(bad)} seeded rejections, every other item ACCEPT"}
            finally:
                g.close()
    finally:
        arena.close()
    return out


def _group_dry(devices, per_dev: int) -> dict:
    """CPU plumbing: the shard plan and the merge of per-shard words the
    library does after its all-gather (host helpers, no device)."""
    import numpy as np

    from babble_amd import native, synth
    from babble_amd.verifier import merge_shard_bits

    native.lib()  # loaded outside the timing
    D = len(devices)
    n = D * per_dev
    rng = np.random.default_rng(1000)
    bad = np.sort(rng.choice(n, max(1, n // 10_000), replace=False))
    want = synth.expected_bits(n, bad)
    bounds = [min(n, (n * d // D + 63) // 64 * 64) for d in range(D)] + [n]
    words = max((bounds[d + 1] - bounds[d] + 63) // 64 for d in range(D))
    ok = np.unpackbits(want.view(np.uint8), bitorder="little")[:n].astype(bool)
    gathered = np.zeros(words * D, np.uint64)
    for d in range(D):
        pk = np.packbits(ok[bounds[d]:bounds[d + 1]], bitorder="little")
        pk = np.concatenate([pk, np.zeros((-len(pk)) % 8, np.uint8)]).view(np.uint64)
        gathered[d * words: d * words + len(pk)] = pk
    t0 = time.perf_counter()
    merged = merge_shard_bits(gathered, words, bounds)
    el = time.perf_counter() - t0
    if not np.array_equal(merged, want):
        raise SystemExit("dry run: merged shard bits differ from the expected bitmask")
    return {"devices": list(devices), "dry_run": True, "events_per_call": n, "value": None,
            "merge_ms": el * 1e3, "bitmask_check": f"exact: {n} items over {D} shards merged by bv_merge_shard_bits"}


def worker_main(argv) -> int:
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--devices", required=True)
    ap.add_argument("--events-per-device", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--dry-run", action="store_true")
    a = ap.parse_args(argv)
    if sys.stdin.readline().strip() != "go":
        return 0  # not needed: exit before touching a GPU
    if a.dry_run and os.environ.get("BENCH_DRY_FAULT") == "worker_crash":  # (tests: a crashing group worker)
        os._exit(9)
    devices = [int(x) for x in a.devices.split(",")]
    res = _group_dry(devices, a.events_per_device) if a.dry_run else _group_gpu(devices, a.events_per_device, a.reps)
    print(json.dumps(res), flush=True)
    return 0


# -------------------------------------------------------- concurrent legs --

def concurrent_legs(fence, rank: int, world: int, batch, local: int, reps: int = 5, dry_run: bool = False) -> dict:
    """Every rank at once: its pinned host entries, timed between barriers,
    max over ranks.  Returns (on every rank) the aggregate rates."""
    legs = {}
    for name, prep in (("host_entry_pinned", _prep_host_pinned), ("events_bulk_pinned", _prep_events_pinned)):
        # every rank passes the same two fences whatever fails (a failed rank
        # reports an infinite time), so none waits for a rank that gave up
        err, run, n, close = None, None, 0, (lambda: None)
        try:
            run, n, close = _prep_dry(batch) if dry_run else prep(batch, local)
            run()  # warm-up (untimed)
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
        fence.barrier(name)
        mine = float("inf")
        if err is None:
            try:
                t0 = time.perf_counter()
                for _ in range(reps):
                    run()
                mine = time.perf_counter() - t0
            except Exception as e:  # noqa: BLE001
                err = f"{type(e).__name__}: {e}"
        el = fence.max(mine if err is None else 1e300, name)
        try:
            close()
        except Exception:  # noqa: BLE001
            pass
        if el >= 1e300:
            legs[name] = {"error": err or "another rank failed"}
            continue
        legs[name] = {"value": None if dry_run else world * n * reps / el, "unit": "verifies/s",
                      "ms_per_call_slowest_rank": el / reps * 1e3, "ranks": world, "events_per_rank_call": n,
                      "calls": reps}
    legs["note"] = ("every rank at once, each from its own bv_host_alloc arrays (bv_verify_batch: ~528 B per event "
                    "crosses PCIe; bv_verify_events: ~215 B); value = all ranks' events / the slowest rank's time")
    return legs


def _prep_host_pinned(batch, local: int):
    import numpy as np

    from babble_amd.verifier import PinnedArena, Verifier, VerifyResult

    arena = PinnedArena()
    v = Verifier(device=local)
    pb = arena.batch(batch)
    res = VerifyResult(arena.array((batch.n_msgs, 32), np.uint8), arena.array(batch.n_items, np.uint8),
                       arena.array((batch.n_items + 63) // 64, np.uint64))

    def close():
        v.close()
        arena.close()

    return (lambda: v.verify_into(pb, res)), batch.n_items, close


def _prep_events_pinned(batch, local: int):
    import numpy as np

    from babble_amd import synth
    from babble_amd.verifier import PinnedArena, Verifier, VerifyResult

    rank = int(os.environ.get("RANK", "0"))
    packed, wire = synth.event_fields(batch.n_items, n_creators=64, seed=2, parents="hash",
                                      ts0=synth.TS0 + rank * batch.n_items * 8)
    del packed
    arena = PinnedArena()
    v = Verifier(device=local)
    pw = arena.wire(wire)
    n = wire.n_events
    res = VerifyResult(arena.array((n, 32), np.uint8), arena.array(n, np.uint8), arena.array((n + 63) // 64, np.uint64))

    def run():
        v.verify_events_into(pw, res)
        if not np.all(res.status == 1):
            raise SystemExit("concurrent events leg: a valid signature was rejected")

    def close():
        v.close()
        arena.close()

    return run, n, close


def _prep_dry(batch):
    import hashlib

    buf = bytes(range(256)) * 4096

    def run():
        hashlib.sha256(buf).digest()

    return run, 0, (lambda: None)


if __name__ == "__main__":
    raise SystemExit(worker_main(sys.argv[1:]))
