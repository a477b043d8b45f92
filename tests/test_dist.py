"""Multi-rank path on CPU (gloo, world size 2 and 3): each rank verifies its
64-aligned shard (host build of the device code, tests/emu) and the accept
bitmasks are all-gathered; the global bitmask equals the oracle's."""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from babble_amd import shard, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_bounds_cover_and_align():
    for n in (0, 1, 63, 64, 65, 1000, 12_500_000):
        for world in (1, 2, 3, 8):
            spans = [shard.shard_bounds(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (lo, hi), (lo2, _) in zip(spans, spans[1:]):
                assert hi == lo2
            assert all(lo % 64 == 0 for lo, hi in spans if lo < hi)  # non-empty shards start on a word
            assert all(lo <= hi for lo, hi in spans)


def test_slice_batch_blocks_and_events():
    wb = synth.blocks(5, n_validators=7, seed=2)
    b = wb.batch
    sub = shard.slice_batch(b, 10, 30)
    assert sub.n_items == 20
    for j in range(20):
        assert sub.message(int(sub.item_msg[j])) == b.message(int(b.item_msg[10 + j]))
    e = synth.events(100, n_creators=3, seed=1)
    s2 = shard.slice_batch(e, 64, 100)
    assert s2.n_msgs == 36 and s2.message(0) == e.message(64)


def _worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    from tests.emu import emu

    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = synth.adversarial(1500, seed=41, n_creators=4, scale_per_million=dict(
        rflip=20000, sflip=20000, body=10000, highs=10000, range=8000, fmt=8000, key=12000))
    lo, hi = shard.shard_bounds(b.n_items, world, rank)
    sub = shard.slice_batch(b, lo, hi)
    _, st, bits, _ = emu.verify_batch(sub.as_dict(), n_threads=2)
    g = shard.allgather_bits(torch.from_numpy(bits.view(np.int64).copy()), b.n_items, world, rank)
    if rank == 0:
        out_q.put(g.numpy().view(np.uint64).copy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_allgather_matches_oracle(world):
    from oracle import coracle

    b = synth.adversarial(1500, seed=41, n_creators=4, scale_per_million=dict(
        rflip=20000, sflip=20000, body=10000, highs=10000, range=8000, fmt=8000, key=12000))
    _, _, want = coracle.verify_batch(b.as_dict())
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert np.array_equal(got, want)


def _worker_blocks(rank, world, port, out_q):
    """C5-shaped shard: a block's signatures never straddle ranks."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    from tests.emu import emu

    dist.init_process_group("gloo", rank=rank, world_size=world)
    wb = synth.blocks(9, n_validators=13, seed=44)
    b = wb.batch
    b.s_be[::7, 9] ^= 0x10  # every 7th signature invalid
    bounds = shard.plan_shards(b.item_msg, world)
    lo, hi = bounds[rank], bounds[rank + 1]
    assert len(set(b.item_msg[lo:hi].tolist()) & set(b.item_msg[:lo].tolist() + b.item_msg[hi:].tolist())) == 0
    sub = shard.slice_batch(b, lo, hi)
    _, st, bits, _ = emu.verify_batch(sub.as_dict(), n_threads=2) if hi > lo else (None, None,
                                                                                      np.zeros(1, np.uint64), 0)
    g = shard.allgather_bits_planned(torch.from_numpy(bits.view(np.int64).copy()), bounds, world)
    if rank == 0:
        out_q.put(g.copy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_block_aware_shards_match_oracle(world):
    from oracle import coracle

    wb = synth.blocks(9, n_validators=13, seed=44)
    b = wb.batch
    b.s_be[::7, 9] ^= 0x10
    _, _, want = coracle.verify_batch(b.as_dict())
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_blocks, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert np.array_equal(got, want)


def test_python_plan_equals_c_abi_plan():
    """shard.plan_shards == bv_plan_shards (the library's group sharding)."""
    from babble_amd.verifier import plan_shards

    rng = np.random.default_rng(5)
    for _ in range(50):
        reps = rng.integers(1, 120, size=rng.integers(1, 40))
        b = synth.blocks(1, n_validators=2, seed=1).batch
        im = np.repeat(np.arange(len(reps)), reps).astype(np.uint32)
        b.item_msg = im
        b.item_key = np.zeros(len(im), np.uint32)
        b.r_be = np.zeros((len(im), 32), np.uint8)
        b.s_be = np.zeros((len(im), 32), np.uint8)
        b.pre = None
        b.msg_off = np.zeros(len(reps) + 1, np.uint64)
        for w in (1, 2, 3, 8):
            assert shard.plan_shards(im, w) == plan_shards(b, w).tolist()


def test_merge_bits_shifts():
    rng = np.random.default_rng(9)
    for _ in range(20):
        n = int(rng.integers(1, 700))
        ok = rng.random(n) < 0.7
        bounds = sorted(set([0, n] + rng.integers(0, n, size=3).tolist()))
        parts = []
        for a, z in zip(bounds, bounds[1:]):
            pk = np.packbits(ok[a:z], bitorder="little")
            pk = np.concatenate([pk, np.zeros((-len(pk)) % 8, np.uint8)])
            parts.append(pk.view(np.uint64) if len(pk) else np.zeros(1, np.uint64))
        pk = np.packbits(ok, bitorder="little")
        want = np.concatenate([pk, np.zeros((-len(pk)) % 8, np.uint8)]).view(np.uint64)
        assert np.array_equal(shard.merge_bits(parts, bounds), want)


def _bench(args, env=None, timeout=240):
    import subprocess
    import sys

    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=e, capture_output=True,
                          text=True, timeout=timeout)


def test_bench_launcher_starts_n_ranks_dry_run():
    """`bench.py --gpus 2` outside torch.distributed.run starts
    two ranks itself (one child torch.distributed.run, rendezvous on
    127.0.0.1); in gloo dry-run mode rank 0 prints ONE line with n_gpus 2
    after the all-gathered bitmasks check out."""
    p = _bench(["--gpus", "2", "--dry-run", "--events", "5000"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["dry_run"] and line["config"]["parallelism"] == "shard2"
    # the N-GPU legs' plumbing — every rank's concurrent legs
    # passed the store barriers and max-over-ranks, rank 0's group worker
    # merged the shard words exactly while rank 1 waited
    conc = line["concurrent"]
    for leg in ("host_entry_pinned", "events_bulk_pinned"):
        assert conc[leg]["ranks"] == 2 and conc[leg]["ms_per_call_slowest_rank"] > 0, conc
    grp = line["group"]
    assert grp["devices"] == [0, 1] and grp["bitmask_check"].startswith("exact"), grp


def test_bench_group_logical_dry_run():
    """`--group-logical 2` at N = 1 (the one-GPU rehearsal of the group leg):
    the worker is started before any GPU use and released after the
    headline; in dry-run mode it merges two logical shards' words."""
    p = _bench(["--dry-run", "--group-logical", "2", "--events", "3000"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and "concurrent" not in line
    assert line["group"]["devices"] == [0, 0] and line["group"]["events_per_call"] == 6000


def test_group_input_concatenates_c3_chunks():
    """bench_multi.c3_group_input: N consecutive C3 chunks as one batch —
    messages, items and the seeded rejections re-based chunk by chunk."""
    import bench_multi

    b, bad = bench_multi.c3_group_input(2, 300)
    c0, bad0 = synth.c3_chunk(0, 300)
    c1, bad1 = synth.c3_chunk(1, 300)
    assert b.n_items == 600 and b.n_msgs == 600 and b.n_keys == 64
    assert np.array_equal(bad, np.concatenate([bad0, bad1 + 300]))
    for j in (0, 299, 300, 599):
        src, k = (c0, j) if j < 300 else (c1, j - 300)
        assert b.message(int(b.item_msg[j])) == src.message(int(src.item_msg[k]))
        assert b.key(int(b.item_key[j])) == src.key(int(src.item_key[k]))
        assert bytes(b.r_be[j]) == bytes(src.r_be[k]) and bytes(b.s_be[j]) == bytes(src.s_be[k])


def test_bench_rank_refuses_world_mismatch():
    """A rank whose WORLD_SIZE differs from --gpus exits non-zero and prints
    no line (never a one-GPU line labelled as N)."""
    p = _bench(["--gpus", "2", "--dry-run", "--events", "5000"], env={"WORLD_SIZE": "1", "RANK": "0",
                                                                       "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


# ------------------------------------------------ N > 1 failure paths --
# every way an N-GPU run can fail ends with a non-zero exit,
# no JSON line and no process left behind (the launcher's child
# torch.distributed.run, its ranks, rank 0's group worker).

def _leftovers(token: str):
    import psutil

    me = os.getpid()
    out = []
    for p in psutil.process_iter(["pid", "cmdline"]):
        try:
            cmd = p.info["cmdline"] or []
            line = " ".join(cmd)
            ours = any(x in line for x in ("bench.py", "bench_multi.py", "torch.distributed.run"))
            if p.info["pid"] != me and cmd and "python" in os.path.basename(cmd[0]) and ours and token in line:
                out.append((p.info["pid"], cmd))
        except psutil.Error:
            pass
    return out


def _assert_failed_cleanly(p, events: int):
    import time

    assert p.returncode != 0, p.stdout[-1000:]
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")], p.stdout
    deadline = time.time() + 30  # (a terminated rank may take a moment to be reaped)
    while _leftovers(f"--events {events}") and time.time() < deadline:
        time.sleep(0.5)
    assert not _leftovers(f"--events {events}")


def test_bench_fewer_gpus_than_ranks_fails_without_a_line():
    """Ranks that see fewer GPUs than --gpus exit 4 before any work; the
    launcher fails and prints nothing."""
    p = _bench(["--gpus", "2", "--dry-run", "--events", "5011"], env={"BENCH_DRY_VISIBLE_GPUS": "1"})
    _assert_failed_cleanly(p, 5011)
    assert "GPU(s) visible" in p.stderr


def test_bench_collective_init_failure_fails_without_a_line():
    """The ranks' collective initialisation failing (RCCL at N > 1) ends the
    run non-zero, no line, no child left."""
    p = _bench(["--gpus", "2", "--dry-run", "--events", "5012"], env={"BENCH_DRY_FAULT": "rccl_init"})
    _assert_failed_cleanly(p, 5012)
    assert "RCCL" in p.stderr


def test_bench_rank_crash_fails_without_a_line():
    """Rank 1 dying after the rendezvous (no cleanup): torch.distributed.run
    stops rank 0, rank 0's group worker sees EOF and exits, and the launcher
    exits non-zero without a line."""
    p = _bench(["--gpus", "2", "--dry-run", "--events", "5013"], env={"BENCH_DRY_FAULT": "rank_crash"})
    _assert_failed_cleanly(p, 5013)


def test_bench_group_worker_crash_is_recorded_and_reaped():
    """The group worker (bv_group_verify_batch over all N devices from one
    process) crashing is an extra leg's failure: the line records it as the
    group leg's error, the headline plumbing stands, and the worker is
    reaped."""
    p = _bench(["--gpus", "2", "--dry-run", "--events", "5014"], env={"BENCH_DRY_FAULT": "worker_crash"})
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    assert "error" in json.loads(lines[0])["group"]
    assert not _leftovers("--events-per-device 5014")


def test_group_create_more_devices_than_exist():
    """bv_group_create naming devices the process cannot see returns
    BV_E_NODEVICE (no context, no RCCL init, no crash)."""
    import ctypes

    import torch

    from babble_amd import native

    n = torch.cuda.device_count()
    g = ctypes.c_void_p()
    devs = (ctypes.c_int * 2)(0, n + 3)
    assert native.lib().bv_group_create(ctypes.byref(g), devs, 2, 0) == native.BV_E_NODEVICE and not g.value
