"""Benchmark: ECDSA event verifies/sec on MI355X (BASELINE.json metric).

    python bench.py --gpus N --steps K --warmup W

One step = one VerifyBatch over one batch of synthetic signed Events that is
already resident in HBM: SHA-256 of every canonical EventBody, pubkey decode
and per-key table build (rebuilt every step: no state is carried between
steps), batched s^-1, and the ECDSA verification of every signature,
producing status bytes and the accept bitmask (the SURVEY §8d C2 workload:
1M Events, 64 creators, one 64-byte transaction each).  With N > 1 ranks
(torch.distributed.run, one process per GPU) every rank verifies its own
1M-event shard (weak scaling) and the per-rank accept bitmasks are
all-gathered over RCCL inside the timed step.  Steps are issued back to
back as asynchronous calls on two alternating streams with two result
buffers (the library's two work-buffer slots), so two batches are in flight
and the host's per-call work overlaps the device's, as in a node verifying
a stream of SyncResponses; the timed region is closed by synchronize.

Rank 0 prints one JSON line.  `value` is the headline above.  Beside it:
  * `roofline` — the two verify kernels (k_verify_g + k_verify_q), timed with
    the library's HIP events on the stream they run on, for a batch alone on
    the chip (five synchronous calls after the timed region); see ROOFLINE;
  * `warm` — the same batches with BV_F_KEY_CACHE (validator tables kept in
    HBM across calls; Babble's validator set is stable), every other piece of
    work still done per step;
  * `host_entry` — bv_verify_batch from host (pageable) buffers, what a cgo
    caller sees: pinned staging, PCIe, kernels and copy-out in the timing;
  * `latency_ms` — bv_verify_batch at 1 / 100 / 1000 (SyncLimit,
    config.go:44) / 10^4 / 10^5 events, cold (no cache) and warm (key cache);
  * `shim_path` — the cgo shim's call sequence
    replayed in C (tests/cabi/shim_harness.c): one event, a 1000-event
    SyncResponse and a 1M-event replay with the batch built in pooled pinned
    arenas and the results copied out inside the clock, beside the
    library-only numbers;
  * `cpu_baseline` — the faster of two CPU legs on this host's cores, each on
    a bounded sample of the same batch: the C oracle (oracle/oracle.c, a
    restatement of the Go path) and the OpenSSL libcrypto proxy of SURVEY
    §8d (oracle/openssl_ref.c); both are reported;
  * at N > 1 (bench_multi.py): `concurrent` — every rank's pinned host
    entries at once (the node's shared host feed), and `group` — the
    library's own multi-GPU entry, bv_group_verify_batch over all N devices
    from one process on C3 chunks (one ncclAllGather), run by rank 0's
    worker process while the other ranks wait at a store barrier.
"""
from __future__ import annotations

import argparse
import json
import os

# HIP maps a process's streams onto GPU_MAX_HW_QUEUES hardware queues (4 by
# default) and streams sharing a queue run serially.  The library owns every
# stream a step uses — one lane per work slot, s^-1, the high-priority key
# tables; one set per device shared by all its contexts — so the headline
# holds at the default 4 queues (the bench creates no streams of its own).
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# ROOFLINE.  The verify kernels are VALU-integer bound (no MFMA, not HBM:
# ~2.1 KB of table gathers per item).  Work per item of the EXECUTED
# schedule, in 256-bit modular multiplications (squarings included), each
# 64 schoolbook 32x32 products + 16 reduction products = 80 IMUL32.  The
# accumulators are XYZZ (point.h gexz): a mixed addition is madd-2008-s,
# 8M + 2S = 10 modmuls:
#   u1 G:  10 signed windows of the 26-bit G table, the first lands on the
#          identity (a copy), the second adds to that affine entry with
#          mmadd-2008-s (4M + 2S = 6), 8 mixed additions x 10       =  86
#   u2 Q:  22 windows of the K12 GLV key tables, 22 x 10            = 220
#   u1 = e w (a Montgomery product) and the check X == r ZZ (1M)    ~   3
#   = 309 modmuls = 24,720 IMUL32 per item in k_verify_g + k_verify_q.
# u2 = r w and its GLV split (~2.8 modmuls) run in k_glv_split on the s^-1
# stream, beside SHA-256 and the key tables, outside these two spans.
# `achieved` = items x 24,720 / (k_verify_g + k_verify_q time); `peak` = the
# v_mad_u64_u32 rate measured on MI355X (tools/ubench_int.hip,
# profiles/r01_ubench_int.txt).  SURVEY §8d's canonical Strauss schedule
# (4,050 modmuls per verify) is reported only as `speedup_vs_canonical`.
MODMUL_PER_ITEM_EXEC = 309
IMUL32_PER_MODMUL = 80
# The same executed work per kernel (k_verify_g counted on
# its own).  k_verify_g: 86 (the G additions) + 1.6 (u1 = e w, an 8-limb
# Montgomery product mod N, 128 IMUL32) -> 87.6.  k_verify_q: 22 key-table
# additions x 10 + the final X == r ZZ check (1) -> 221.  (Rounded into the
# 309 above with the digit recoding and sign handling.)
MODMUL_G, MODMUL_Q = 87.6, 221
CANONICAL_MODMUL_PER_VERIFY = 4050
PEAK_IMUL32_PER_S = 31.76e12
# Measured gfx950 issue costs (profiles/r01_ubench_ops.txt): a wave64
# v_mad_u64_u32 holds its SIMD 5.39 cycles, a 32-bit VALU op 3.03.
CYC_MAD64, CYC_VALU32 = 5.39, 3.03
N_SIMD = 256 * 4


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 300 timed steps (~0.6 s of device time, two batches in flight) after 20
    # warm-up steps: sustained throughput; 30 steps (60 ms) read 1-4 % low and
    # noisier on the same box (profiles/r04_ab_bench_steps.log)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--events", type=int, default=1_000_000, help="events per GPU per step")
    ap.add_argument("--creators", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=9.0, help="target CPU-baseline sample duration (each leg)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="headline only (profiler passes)")
    ap.add_argument("--inflight", type=int, default=2, choices=(1, 2),
                    help="batches in flight: consecutive steps rotate over this many streams and result buffers")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / rank plumbing only, on CPU over gloo: no GPU, no verification (tests)")
    ap.add_argument("--group-logical", type=int, default=0,
                    help="N=1 rehearsal of the N-GPU group leg: bv_group over this many logical shards of GPU 0")
    ap.add_argument("--group-reps", type=int, default=5, help="timed bv_group_verify_batch calls per group leg")
    return ap.parse_args()


def launch_ranks(args) -> int:
    """`--gpus N` (N > 1) outside torch.distributed.run: start the N ranks as
    ONE child process (python -m torch.distributed.run, one rank per GPU,
    rendezvous on 127.0.0.1) before this process imports torch or touches a
    GPU, and return its exit code.  Ranks that find fewer than N GPUs exit
    non-zero without printing a line, so the launcher fails too."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def check_rank_env(args) -> int:
    """Inside a rank: the world must be exactly --gpus ranks and every rank
    needs its own GPU.  Returns the world size or exits non-zero."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: refusing to print a line", file=sys.stderr)
        raise SystemExit(3)
    if args.dry_run:  # (tests: a box with fewer GPUs than ranks, BENCH_DRY_VISIBLE_GPUS)
        visible = int(os.environ.get("BENCH_DRY_VISIBLE_GPUS", str(args.gpus)))
    else:
        import torch

        visible = torch.cuda.device_count()
    if visible < args.gpus:
        print(f"bench.py: --gpus {args.gpus} but {visible} GPU(s) visible", file=sys.stderr)
        raise SystemExit(4)
    return world


def dry_fault(where: str, rank: int) -> None:
    """Dry-run fault injection (tests/test_dist.py):
    BENCH_DRY_FAULT=rccl_init makes every rank's collective init fail (as
    dist.init_process_group("nccl") raising), rank_crash makes rank 1 die
    after the rendezvous (os._exit, no cleanup, as a segfaulting rank).
    Either way the launcher exits non-zero, no rank prints a line and no
    child process is left behind."""
    fault = os.environ.get("BENCH_DRY_FAULT", "")
    if where == "init" and fault == "rccl_init":
        raise RuntimeError("injected: collective (RCCL) initialisation failed")
    if where == "after_init" and fault == "rank_crash" and rank == 1:
        sys.stdout.flush()
        os._exit(7)


def dry_run(args, world: int, rank: int, worker) -> None:
    """The N-rank plumbing on CPU (gloo): each rank's expected accept bitmask
    of its shard, all-gathered and checked as the GPU run checks its own; the
    N-GPU legs' barriers, max-over-ranks and group worker (bench_multi) with
    CPU stand-ins; rank 0 prints a line with value null."""
    import numpy as np
    import torch
    import torch.distributed as dist

    dry_fault("init", rank)
    if world > 1:
        dist.init_process_group("gloo")
    dry_fault("after_init", rank)
    words = expected_words(rank, args.events)
    t0 = time.perf_counter()
    mine = torch.from_numpy(words.view(np.int64).copy())
    if world > 1:
        got = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(got, mine)
    else:
        got = [mine]
    for q in range(world):
        if not np.array_equal(got[q].numpy().view(np.uint64), expected_words(q, args.events)):
            raise SystemExit(f"rank {rank}: gathered bitmask of rank {q} differs")
    el = time.perf_counter() - t0
    extras = multi_gpu_legs(args, world, rank, worker, None, 0) if world > 1 or args.group_logical else {}
    if rank == 0:
        print(json.dumps(dict({"metric": "ECDSA event verifies/sec", "value": None, "unit": "verifies/s",
                               "n_gpus": world, "steps": 0, "warmup": 0, "ms_per_step": el * 1e3,
                               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
                               "data": "dry run (no GPU)", "dry_run": True,
                               "config": {"workload": "launcher plumbing only",
                                          "parallelism": f"shard{world}" if world > 1 else "single"}}, **extras)),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def multi_gpu_legs(args, world: int, rank: int, worker, batch, local: int) -> dict:
    """bench_multi's legs after the headline: every rank's
    pinned host entries at once, then the library's own multi-GPU entry
    (bv_group_verify_batch over all N devices from rank 0's worker process)
    while the other ranks wait at a store barrier.  Every rank runs the same
    barrier sequence whatever fails, so no rank waits for one that gave up."""
    import bench_multi as M

    fence = M.StoreFence(rank, world) if world > 1 else M.LocalFence()
    out = {}
    if world > 1:
        try:
            out["concurrent"] = M.concurrent_legs(fence, rank, world, batch, local, dry_run=args.dry_run)
        except Exception as e:  # noqa: BLE001 (the fences inside have all run: see concurrent_legs)
            out["concurrent"] = {"error": f"{type(e).__name__}: {e}"}
    fence.barrier("group")
    if rank == 0:
        out["group"] = M.run_group_worker(worker) if worker is not None else {"error": "no group worker"}
    fence.barrier("group-done")
    return out


def cpu_threads() -> int:
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit():
        cores = min(cores, int(omp))
    return cores


def _sample(batch, n):
    d = batch.as_dict()
    off = d["msg_off"][: n + 1]
    return dict(msg_bytes=d["msg_bytes"][: int(off[-1])], msg_off=off, key_bytes=d["key_bytes"],
                key_off=d["key_off"], item_msg=d["item_msg"][:n], item_key=d["item_key"][:n],
                r_be=d["r_be"][:n], s_be=d["s_be"][:n], pre=d["pre"][:n])


def cpu_baseline(batch, target_s: float) -> dict:
    """Time both CPU legs on a bounded sample of the same batch, all host
    cores this process may use; return the faster as the baseline.  Each
    sample is converted once (coracle.Prepared) and the C library keeps a
    persistent thread pool, so a timed call is the verification alone."""
    import numpy as np

    from oracle import coracle  # the checker, timed here as the CPU baseline

    cores = cpu_threads()

    def timed(leg):
        getattr(coracle.Prepared(_sample(batch, 64)), leg)(cores)  # one-time init outside the timing
        n = 128 * cores
        p = coracle.Prepared(_sample(batch, n))
        t0 = time.perf_counter()
        getattr(p, leg)(cores)
        rate = n / (time.perf_counter() - t0)
        n = int(min(batch.n_items, max(n, rate * target_s)))
        p = coracle.Prepared(_sample(batch, n))
        t0 = time.perf_counter()
        st = getattr(p, leg)(cores)
        dt = time.perf_counter() - t0
        return {"value": n / dt, "n": n, "seconds": dt, "accepted": int(np.count_nonzero(st == 1))}

    legs = {leg: timed(leg) for leg in ("port", "oracle", "openssl")}
    best = max(legs, key=lambda k: legs[k]["value"])
    what = {"port": "oracle/oracle.c port_verify_batch (C port of the reference stack's algorithms: Go 1.13 "
                    "ecdsa.Verify over btcec, i.e. byte-table ScalarBaseMult, GLV + NAF ScalarMult, mixed "
                    "additions, 3 affine conversions)",
            "oracle": "oracle/oracle.c oracle_verify_batch (the checker: byte tables for u1 G, 4-bit fixed "
                      "window for u2 Q)",
            "openssl": "oracle/openssl_ref.c (OpenSSL libcrypto SHA256 + o2i_ECPublicKey + ECDSA_do_verify, "
                       "the SURVEY §8d proxy)"}
    L = legs[best]
    return {"value": L["value"], "unit": "verifies/s", "cores": cores, "kind": "port",
            "sample": f"first {L['n']} events of the rank-0 batch, per item SHA-256 + pubkey decode + ECDSA "
                      f"verify, {L['seconds']:.1f}s on {cores} threads; {what[best]}",
            "accepted": L["accepted"],
            "legs": {k: {"value": v["value"], "sample_events": v["n"], "seconds": v["seconds"], "what": what[k]}
                     for k, v in legs.items()}}


def pmc_profile(n_items: int):
    """PMC counters of the headline verify kernels (the newest
    profiles/rNN_kverify_pmc.json: tools/gpu_pmc.sh + tools/pmc_summary.py on
    the same workload)."""
    import glob

    found = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_kverify_pmc.json")))
    if not found:
        return None
    path = found[-1]
    with open(path) as f:
        tj = json.load(f)
    tj["tracked_file"] = os.path.relpath(path, ROOT)  # the committed copy (tj["source"]: where it was written)
    return tj if tj.get("items_per_launch") == n_items else None


def corrupted(rank: int, n: int, buf: int = 0):
    """The seeded items of rank `rank`'s shard (in-flight buffer `buf`) whose
    r has a bit flipped: each buffer has its own set, so a race between two
    overlapping steps cannot write the other buffer's (identical) answer."""
    import numpy as np

    rng = np.random.default_rng(7919 + rank + 100_003 * buf)
    return np.sort(rng.choice(n, max(1, n // 10_000), replace=False))


def expected_words(rank: int, n: int, buf: int = 0):
    import numpy as np

    ok = np.ones(n, bool)
    ok[corrupted(rank, n, buf)] = False
    packed = np.packbits(ok, bitorder="little")
    words = (n + 63) // 64
    return np.concatenate([packed, np.zeros(words * 8 - len(packed), np.uint8)]).view(np.uint64)


def timed_steps(step, steps: int, warmup: int, world: int, dist, local: int, ver):
    """K steps issued back to back (each a full asynchronous VerifyBatch;
    the library orders a ctx's calls on the device per work-buffer slot, so
    with steps on two streams two batches are in flight and the host's
    launch work overlaps the device's), bracketed by barrier + synchronize.
    The last timed step's HIP events are read after the closing synchronize."""
    import torch

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    issue = 0.0
    for _ in range(steps):
        t1 = time.perf_counter()
        step()
        issue += time.perf_counter() - t1
    timed_steps.issue_ms_per_step = issue / max(steps, 1) * 1e3
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ver.sync()
    tms = [ver.timing()]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, tms


def mean(xs, k):
    import numpy as np

    return float(np.mean([x[k] for x in xs]))


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch_ranks(args))  # before torch is imported or a GPU touched
    world = check_rank_env(args)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    worker = None
    if rank == 0 and not args.no_extras and (world > 1 or args.group_logical > 1):
        import bench_multi

        # started before this process touches a GPU; it waits on its stdin
        devices = list(range(world)) if world > 1 else [0] * args.group_logical
        worker = bench_multi.start_group_worker(devices, args.events, args.group_reps, args.dry_run)
    try:
        if args.dry_run:
            return dry_run(args, world, rank, worker)
        return run(args, world, rank, local, worker)
    finally:
        if worker is not None:
            import bench_multi

            bench_multi.stop_group_worker(worker)


def run(args, world: int, rank: int, local: int, worker) -> None:
    import numpy as np
    import torch

    from babble_amd import native, synth
    from babble_amd.verifier import Verifier

    dist = None
    torch.cuda.set_device(local)
    torch.zeros(1, device=f"cuda:{local}")  # torch's default stream takes its queue first (idle while timed)
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    # Per-rank shard: same 64 creators (seeded keys), disjoint events.  One
    # item in 10^4 (seeded by rank and in-flight buffer) has an r bit flipped,
    # so every accept bitmask has known zeros and is checked bit for bit below.
    batch = synth.events(args.events, n_creators=args.creators, seed=2,
                         ts0=synth.TS0 + rank * args.events * 8)
    clean_r = batch.r_be.copy()
    v = Verifier(device=local)
    # BENCH_HOST_ENTRY_PROBE=1: the pageable host entry's rate at three
    # points of this process, printed to stderr
    probe = os.environ.get("BENCH_HOST_ENTRY_PROBE") == "1" and rank == 0 and world == 1
    if probe:
        host_entry_rate(v, batch, "before the headline steps")
    # Consecutive steps alternate two result buffers and the library's two
    # work slots, each slot on its own library lane (stream), so one batch's
    # key tables and hashing overlap the previous batch's k_verify_q tail — a
    # node verifying back-to-back SyncResponses.  Every step still verifies
    # its whole batch; the result of each buffer's last step is checked.
    devs = []
    for j in range(args.inflight):
        batch.r_be = clean_r.copy()
        batch.r_be[corrupted(rank, args.events, j), 31] ^= 1
        devs.append(v.to_device(batch))
    batch.r_be = clean_r
    batch.r_be[corrupted(rank, args.events, 0), 31] ^= 1  # the CPU baseline's sample = buffer 0's batch
    torch.cuda.synchronize()
    words = devs[0].accept_bits.numel()
    gathered = ([torch.empty(words * world, dtype=torch.int64, device=f"cuda:{local}") for _ in devs]
                if world > 1 else None)
    ext = {}
    k = [0]

    def step_with(ver):
        def step():
            j = k[0] % len(devs)
            k[0] += 1
            ver.verify_device(devs[j], stream=0, sync=False)  # on the library lane of the call's slot
            if world > 1:  # ordered after the verify: the gather is issued on the same lane
                h = ver.last_stream()
                if h not in ext:
                    ext[h] = torch.cuda.ExternalStream(h, device=f"cuda:{local}")
                with torch.cuda.stream(ext[h]):
                    dist.all_gather_into_tensor(gathered[j], devs[j].accept_bits)
        return step

    elapsed, tms = timed_steps(step_with(v), args.steps, args.warmup, world, dist, local, v)
    for j, dev in enumerate(devs):
        res = dev.result()
        if not np.array_equal(res.accept_bits, expected_words(rank, args.events, j)):
            raise SystemExit(f"rank {rank}: accept bitmask (buffer {j}) differs from the expected one")
        if world > 1:  # the all-gathered mask of the buffer's last step: every rank's shard, bit for bit
            got = gathered[j].cpu().numpy().view(np.uint64).reshape(world, -1)
            for q in range(world):
                if not np.array_equal(got[q], expected_words(q, args.events, j)):
                    raise SystemExit(f"rank {rank}: gathered bitmask of rank {q} differs from the expected one")

    # Kernel durations for the roofline: with two batches in flight the
    # kernels share the CUs with the other batch's, so their HIP-event spans
    # are stretched; the per-launch figures come from a batch alone on the
    # chip (synchronous calls, same workload), right after the timed region.
    iso = []
    for _ in range(5):
        v.verify_device(devs[0], sync=True)
        iso.append(v.timing())
    line = None
    if rank == 0:
        total_items = world * args.events * args.steps
        value = total_items / elapsed
        kq_ms, kg_ms = mean(iso, "ms_verify"), mean(iso, "ms_verify_g")
        kv_s = (kq_ms + kg_ms) * 1e-3
        achieved = args.events * MODMUL_PER_ITEM_EXEC * IMUL32_PER_MODMUL / kv_s
        roof = {
            "bound": "valu-int",
            "kernel": "k_verify_g<false, true> + k_verify_q<12, 11, false>",
            "achieved": achieved / 1e12,
            "peak": PEAK_IMUL32_PER_S / 1e12,
            "unit": f"T IMUL32/s (executed schedule: {MODMUL_PER_ITEM_EXEC} modmuls x 80 IMUL32 per item; "
                    "bench.py ROOFLINE)",
            "frac": achieved / PEAK_IMUL32_PER_S,
            "traffic": None,
            "speedup_vs_canonical": CANONICAL_MODMUL_PER_VERIFY / MODMUL_PER_ITEM_EXEC,
            "durations": "k_verify_g + k_verify_q HIP-event spans of a batch alone on the chip (breakdown_ms)",
            # the whole chip over the timed region (two batches in flight):
            # the verify kernels' executed IMUL32 at the headline rate
            "chip_frac": value / world * MODMUL_PER_ITEM_EXEC * IMUL32_PER_MODMUL / PEAK_IMUL32_PER_S,
            # per kernel, the same spans: each kernel's executed IMUL32 over its own time
            "per_kernel": {
                "k_verify_g": {"ms": kg_ms, "modmul_per_item": MODMUL_G,
                               "frac": args.events * MODMUL_G * IMUL32_PER_MODMUL / (kg_ms * 1e-3) / PEAK_IMUL32_PER_S},
                "k_verify_q": {"ms": kq_ms, "modmul_per_item": MODMUL_Q,
                               "frac": args.events * MODMUL_Q * IMUL32_PER_MODMUL / (kq_ms * 1e-3) / PEAK_IMUL32_PER_S},
            },
        }
        pmc = pmc_profile(args.events)
        if pmc:
            # physical utilisation from the PMC passes of the same workload:
            # v_mad_u64_u32 actually issued (SQ_INSTS_VALU_INT64) vs the mad
            # peak, and VALU issue occupancy with the measured per-class costs
            i64, ivalu = pmc["valu_int64_wave_insts"], pmc["valu_wave_insts"]
            roof["traffic"] = pmc["hbm_bytes_per_launch"]
            if "traffic_over_algorithmic" in pmc:  # FETCH_SIZE calibrated for the 64-B gathers
                roof["traffic_over_algorithmic"] = pmc["traffic_over_algorithmic"]
                roof["traffic_calibration"] = pmc.get("fetch_factor")
            roof["executed_frac"] = i64 * 64 / kv_s / PEAK_IMUL32_PER_S
            roof["valu_issue_frac"] = (i64 * CYC_MAD64 + (ivalu - i64) * CYC_VALU32) / (N_SIMD * 2.4e9 * kv_s)
            roof["pmc_source"] = pmc["tracked_file"]
        line = {
            "metric": "ECDSA event verifies/sec",
            "value": value,
            "unit": "verifies/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded DRBG keys, OpenSSL-signed canonical EventBody JSON; resident in HBM)",
            "config": {
                "workload": "C2: VerifyBatch of 1M signed Events per GPU (64 creators, 1x64-B tx, ~446-B bodies); "
                            "per-key tables rebuilt every step"
                            + ("; N GPUs = C2 weak scaling (1M events per GPU per step, bitmasks all-gathered "
                               "over RCCL), not C3's 10^8 (tests/test_gpu_c3.py)" if world > 1 else ""),
                "events_per_gpu": args.events,
                "creators": args.creators,
                "parallelism": f"shard{world}" if world > 1 else "single",
                "collective": "RCCL all_gather of accept bitmasks" if world > 1 else None,
                "batches_in_flight": args.inflight,
            },
            "breakdown_ms": {  # one batch alone on the chip (5 synchronous calls)
                "k_sha256": mean(iso, "ms_sha256"),
                "keyprep_stream": mean(iso, "ms_keyprep"),
                "k_sinv": mean(iso, "ms_scalar"),
                "k_verify_g": kg_ms,
                "k_verify_q": kq_ms,
                "device_total": mean(iso, "ms_total"),
            },
            # host time to issue one step (the library's launch work + Python):
            # when it reaches ms_per_step the run is host-bound, not device-bound
            "host_issue_ms_per_step": timed_steps.issue_ms_per_step,
            "in_flight_step_ms": {  # the last timed step's spans, overlapped with its neighbour
                "device_total": mean(tms, "ms_total"),
                "k_verify_g": mean(tms, "ms_verify_g"),
                "k_verify_q": mean(tms, "ms_verify"),
            },
            "roofline": roof,
            "bitmask_check": f"exact: {world} x {args.events} events, accept bits all-gathered and equal to the "
                             f"expected mask ({len(corrupted(0, args.events))} seeded r-bit flips per rank and "
                             f"in-flight buffer, a different set per buffer, rejected)",
            "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "default (4)"),
        }
    if probe:
        host_entry_rate(v, batch, "after the headline steps")
    if rank == 0 and world == 1 and not args.no_extras:
        line["warm"] = warm_leg(args, devs, world, dist, local, step_with)
        if probe:
            host_entry_rate(v, batch, "after the warm leg")
        line["host_entry"] = host_entry_leg(args, v, batch)
        line["host_entry_pinned"] = host_entry_pinned_leg(args, v, batch)
        line["latency_ms"] = latency_leg(args)
        line["events_entry"] = events_entry_leg(args)
        line["shim_path"] = guarded(shim_path_leg, args, line)
        line["tx_sweep"] = tx_sweep_leg(args, v, local)
        line["c5_fast_sync"] = guarded(c5_leg, args, local)
        line["c1_insert"] = guarded(c1_leg, args, local)
    if not args.no_extras and (world > 1 or args.group_logical > 1):
        extras = multi_gpu_legs(args, world, rank, worker, batch, local)
        if rank == 0:
            line.update(extras)
    if rank == 0:
        if world == 1 and not args.no_cpu:  # the CPU leg: rank 0 at N=1 only
            line["cpu_baseline"] = cpu_baseline(batch, args.cpu_seconds)
            line["gpu_over_cpu"] = line["value"] / line["cpu_baseline"]["value"]
        print(json.dumps(line), flush=True)
    v.close()
    if world > 1:
        dist.destroy_process_group()


def guarded(fn, *a):
    """An extra leg's failure is recorded in the line instead of losing it."""
    try:
        return fn(*a)
    except Exception as e:  # noqa: BLE001
        import traceback

        traceback.print_exc()
        return {"error": f"{type(e).__name__}: {e}"}


def warm_leg(args, devs, world, dist, local, step_with):
    """Same device-resident batches with BV_F_KEY_CACHE: the 64 creators are
    registered first (bv_kc_register builds their tables: register_ms), the
    timed steps reuse them; hashing, s^-1, u1 G, u2 Q and the decision run
    every step."""
    import numpy as np

    from babble_amd import native, synth
    from babble_amd.verifier import Verifier

    vc = Verifier(device=local, flags=native.F_KEY_CACHE)
    kb = synth.events(1, n_creators=args.creators, seed=2)  # the same seeded creator keys
    t0 = time.perf_counter()
    vc.register_keys([kb.key(k) for k in range(kb.n_keys)])
    reg_ms = (time.perf_counter() - t0) * 1e3
    builds = vc.timing()["kc_builds"]
    t0 = time.perf_counter()
    vc.verify_device(devs[0])
    cold_ms = (time.perf_counter() - t0) * 1e3
    elapsed, tms = timed_steps(step_with(vc), args.steps, 1, 1, None, local, vc)
    for j, dev in enumerate(devs):
        assert np.array_equal(dev.result().accept_bits, expected_words(0, args.events, j))
    out = {"value": args.events * args.steps / elapsed, "unit": "verifies/s",
           "ms_per_step": elapsed / args.steps * 1e3, "register_ms": reg_ms, "tables_built_by_register": builds,
           "first_call_ms": cold_ms,
           "key_path": int(tms[-1]["key_path"]),
           "breakdown_ms": {"k_sha256": mean(tms, "ms_sha256"), "k_sinv": mean(tms, "ms_scalar"),
                            "k_verify_g": mean(tms, "ms_verify_g"), "k_verify_q": mean(tms, "ms_verify"),
                            "device_total": mean(tms, "ms_total")}}
    vc.close()
    return out


# C5 roofline (key-cache path, k_verify_gq): 9 XYZZ adds from the G table
# (the first on window 0's affine entry: mmadd, 6 modmuls; 8 x 10) + 12 from
# the validator's KC table (6 per GLV half) at 10 modmuls each, the 6 beta x
# products of the phi half, ~7 for u1 / u2, the GLV split and the check:
# 219 modmuls x 80 IMUL32 per signature.
C5_MODMUL_PER_ITEM = 219


def c5_leg(args, local, reps=5):
    """SURVEY §8d C5 / BASELINE configs[4], fast-sync replay: 10^4 BlockBodies
    x 100 validators (seed 5, 16 x 64-B transactions, ~1.77 KB bodies), 5 %
    of the signatures corrupted.  One step = PeerSet.Hash of the 100
    validators (one device launch, the serial SHA chain of
    peer_set.go:104-115), then ONE bv_verify_batch from host buffers with
    every BlockBody (hashed once each, block.go:29-55) + the anchor Frame's
    canonical JSON (frame.go:35-46, an item-less message) and the 10^6
    signature items, then the host fold of CheckBlock (hashgraph.go:1599-1630:
    valid count > TrustCount per block) and the frame-hash comparison.  The
    validator set is registered with the key cache first (Babble knows its
    PeerSet before replaying).  Beside it: the C port on a bounded sample of
    the same items, all cores; and the device-resident rate of the same batch
    (bv_verify_batch_device, inputs in HBM) with its own roofline line."""
    import hashlib

    import numpy as np

    from babble_amd import frame as F
    from babble_amd import hashgraph as H
    from babble_amd import native, synth
    from babble_amd.batch import PackedBatch
    from babble_amd.verifier import Verifier

    wb = synth.blocks(10_000, n_validators=100, seed=5)
    b = wb.batch
    rng = np.random.default_rng(5)
    bad = rng.choice(b.n_items, size=b.n_items // 20, replace=False)
    b.s_be[bad, 7] ^= 0x40
    keys = [b.key(k) for k in range(b.n_keys)]
    peers = [H.Peer("172.77.%d.%d:1337" % (i // 250, i % 250 + 1), "0X" + k.hex().upper(), "node%d" % i)
             for i, k in enumerate(keys)]
    frame = F.Frame(Round=10_000, Peers=peers, Roots={p.PubKeyString(): F.Root(Events=None) for p in peers},
                    Events=None, PeerSets={0: peers}, Timestamp=1_600_000_000)
    fjson = frame.Marshal()
    fhash = hashlib.sha256(fjson).digest()
    off = np.concatenate([b.msg_off, [b.msg_off[-1] + len(fjson)]]).astype(np.uint64)
    rb = PackedBatch(np.concatenate([b.msg_bytes, np.frombuffer(fjson, np.uint8)]), off, b.key_bytes, b.key_off,
                     b.item_msg, b.item_key, b.r_be, b.s_be, b.pre)
    v = Verifier(device=local, flags=native.F_KEY_CACHE)
    t0 = time.perf_counter()
    v.register_keys(keys)
    reg_ms = (time.perf_counter() - t0) * 1e3
    tc = H.PeerSet(peers).TrustCount()

    def step():
        ph = v.peer_set_hash(keys)
        res = v.verify(rb)
        counts = (res.status == 1).reshape(wb.n_blocks, wb.n_validators).sum(axis=1)
        return ph, res, counts

    step()
    ts = []
    for _ in range(reps):
        t1 = time.perf_counter()
        ph, res, counts = step()
        ts.append(time.perf_counter() - t1)
    tm = v.timing()
    ok_blocks = int((counts > tc).sum())
    assert ph == wb.peers_hash, "PeerSet.Hash differs from the generator's chain"
    assert res.msg_hash[-1].tobytes() == fhash, "frame hash differs"
    want = np.ones(b.n_items, np.uint8)
    want[bad] = 0
    assert np.array_equal(res.status, want), "C5 statuses differ from the seeded corruption"
    el = float(np.median(ts))
    # device-resident: the blocks' batch in HBM, bv_verify_batch_device (the
    # 54 KB Frame left out: in HBM it would be one GPU lane's serial SHA chain,
    # which the host entry above hashes on the CPU instead)
    d = v.to_device(b)
    v.verify_device(d, sync=True)
    dts = []
    for _ in range(reps):
        t1 = time.perf_counter()
        v.verify_device(d, sync=True)
        dts.append(time.perf_counter() - t1)
    td = v.timing()
    assert np.array_equal(d.result().status, want)
    kv = td["ms_verify"] * 1e-3
    ach = b.n_items * C5_MODMUL_PER_ITEM * IMUL32_PER_MODMUL / kv if kv > 0 else 0.0
    out = {"value": b.n_items / el, "unit": "verifies/s", "ms_per_replay": el * 1e3, "blocks": wb.n_blocks,
           "validators": wb.n_validators, "items": b.n_items, "bytes_bodies": int(b.msg_off[-1]),
           "frame_json_bytes": len(fjson), "register_ms": reg_ms, "key_path": int(tm["key_path"]),
           "blocks_passing_check_block": ok_blocks, "trust_count": tc,
           "host_breakdown_ms": host_breakdown([tm]),
           "device_resident": {"value": b.n_items / float(np.median(dts)), "unit": "verifies/s",
                               "ms_per_call": float(np.median(dts)) * 1e3,
                               "breakdown_ms": {"k_sha256": td["ms_sha256"], "k_sinv": td["ms_scalar"],
                                                "k_verify_gq": td["ms_verify"], "device_total": td["ms_total"]}},
           "roofline": {"bound": "valu-int", "kernel": "k_verify_gq<false> (key cache)",
                        "achieved": ach / 1e12, "peak": PEAK_IMUL32_PER_S / 1e12,
                        "unit": f"T IMUL32/s ({C5_MODMUL_PER_ITEM} modmuls x 80 IMUL32 per signature)",
                        "frac": ach / PEAK_IMUL32_PER_S}}
    v.close()
    if not args.no_cpu:
        from oracle import coracle  # CPU baseline leg only

        from babble_amd import shard

        n = 20_000  # 200 blocks: their 200 bodies and 20,000 signatures
        prep = coracle.Prepared(shard.slice_batch(b, 0, n).as_dict())
        cores = cpu_threads()
        prep.port(cores)
        t1 = time.perf_counter()
        st = prep.port(cores)
        dt = time.perf_counter() - t1
        assert np.array_equal(st, want[:n])
        out["cpu"] = {"value": n / dt, "unit": "verifies/s", "cores": cores, "sample": f"first {n} items (200 blocks)",
                      "what": "oracle.c port_verify_batch (SHA-256 per item's body + decode + ECDSA), all cores"}
    return out


def tx_sweep_leg(args, v, local, steps=10):
    """SURVEY §8d C2's sweep over transactions per event, T in {0, 4, 16}
    (T = 1 is the headline): the headline's batch size and 64 creators, the
    same cold path (per-key tables rebuilt every step, two batches in
    flight); the body grows from 6 to 29 SHA-256 blocks while the ECDSA work
    per item stays fixed.  Every result is checked (all signatures valid).
    (At 250k events per batch the cold path is bound by the per-batch key
    tables instead: their serial base chain, ~0.6 ms per batch, sets a
    ~0.9 ms step whatever T is.)"""
    import numpy as np

    from babble_amd import synth

    n = args.events
    out = {}
    for t in (0, 4, 16):
        b = synth.events(n, n_creators=args.creators, seed=20 + t, n_tx=t)
        devs = [v.to_device(b) for _ in range(2)]
        k = [0]

        def step():
            v.verify_device(devs[k[0] % 2], stream=0, sync=False)
            k[0] += 1

        elapsed, _ = timed_steps(step, steps, 2, 1, None, local, v)
        for d in devs:
            if not np.all(d.result().status == 1):
                raise SystemExit(f"tx_sweep T={t}: a valid signature was rejected")
        v.verify_device(devs[0], sync=True)
        t_iso = v.timing()
        body = float(np.diff(b.msg_off).mean())
        out[str(t)] = {"value": n * steps / elapsed, "unit": "verifies/s", "ms_per_step": elapsed / steps * 1e3,
                       "events": n, "body_bytes_mean": body, "sha_blocks": int((body + 9 + 63) // 64),
                       "k_sha256_ms": t_iso["ms_sha256"], "k_verify_ms": t_iso["ms_verify_g"] + t_iso["ms_verify"]}
        del devs
    return out


def host_breakdown(ts):
    """Where a host-entry call's time goes (bv_timing): the library call's
    wall clock, its host prep (validation + staging copies until the last
    H2D is queued), the device span of the kernels, the result copy-out."""
    return {"lib_call": mean(ts, "ms_host"), "host_prep": mean(ts, "ms_host_prep"),
            "device_kernels": mean(ts, "ms_total"), "d2h_tail": mean(ts, "ms_d2h"),
            "host_out": mean(ts, "ms_host_out")}


def host_diag(batch) -> dict:
    """The host's state behind the pageable host entry: the
    CPUs this process may use (affinity, cgroup quota), and one thread's
    memcpy rate from the batch's pageable message bytes into page-locked
    memory in this process right now."""
    import numpy as np

    from babble_amd.verifier import PinnedArena

    out = {"affinity_cpus": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None}
    try:
        out["cgroup_cpu_max"] = open("/sys/fs/cgroup/cpu.max").read().strip()
    except OSError:
        out["cgroup_cpu_max"] = None
    try:  # the GPU's NUMA node (its PCI device's), and the main thread's now
        import torch

        pr = torch.cuda.get_device_properties(int(os.environ.get("LOCAL_RANK", "0")))
        bdf = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        out["gpu_numa_node"] = int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read())
    except (OSError, AttributeError, ValueError):
        out["gpu_numa_node"] = None
    out["msg_bytes_mapping"] = smaps_of(batch.msg_bytes.ctypes.data + batch.msg_bytes.nbytes // 2)
    try:
        out["thp"] = open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip()
    except OSError:
        out["thp"] = None
    arena = PinnedArena()
    try:
        src = batch.msg_bytes
        dst = arena.array(src.nbytes, np.uint8)
        np.copyto(dst, src)
        t0 = time.perf_counter()
        for _ in range(3):
            np.copyto(dst, src)
        out["memcpy_1thread_gb_s"] = 3 * src.nbytes / (time.perf_counter() - t0) / 1e9
        from concurrent.futures import ThreadPoolExecutor

        for nt in (8, 16):  # numpy releases the GIL for the copies
            step = (src.nbytes + nt - 1) // nt
            with ThreadPoolExecutor(nt) as ex:
                def part(k):
                    np.copyto(dst[k * step:(k + 1) * step], src[k * step:(k + 1) * step])
                list(ex.map(part, range(nt)))
                t0 = time.perf_counter()
                for _ in range(3):
                    list(ex.map(part, range(nt)))
                out[f"memcpy_{nt}threads_gb_s"] = 3 * src.nbytes / (time.perf_counter() - t0) / 1e9
    finally:
        arena.close()
    return out


def smaps_of(addr: int) -> dict:
    """The /proc/self/smaps entry of the mapping holding `addr`: its size and
    how much of it is backed by transparent huge pages (kB)."""
    cur = None
    try:
        for line in open("/proc/self/smaps"):
            f = line.split()
            if "-" in f[0] and len(f) >= 5:
                lo, hi = (int(x, 16) for x in f[0].split("-"))
                cur = {} if lo <= addr < hi else None
            elif cur is not None and f[0] in ("Size:", "Rss:", "AnonHugePages:"):
                cur[f[0][:-1]] = int(f[1])
                if len(cur) == 3:
                    return cur
    except (OSError, ValueError):
        pass
    return cur or {}


def numa_counters() -> dict:
    """Automatic NUMA balancing's activity: the sysctl, the host's hinting
    faults and page migrations (/proc/vmstat) and this process's
    (/proc/self/sched)."""
    out = {}
    try:
        out["numa_balancing"] = int(open("/proc/sys/kernel/numa_balancing").read())
    except (OSError, ValueError):
        pass
    try:
        for line in open("/proc/vmstat"):
            k, v = line.split()
            if k in ("numa_hint_faults", "numa_pages_migrated", "pgmigrate_success", "numa_pte_updates"):
                out["host_" + k] = int(v)
    except OSError:
        pass
    try:
        for line in open("/proc/self/sched"):
            if ":" in line:
                k, v = line.split(":", 1)
                k = k.strip()
                if k in ("numa_pages_migrated", "total_numa_faults"):
                    out["self_" + k] = int(float(v))
    except (OSError, ValueError):
        pass
    return out


def host_entry_rate(v, batch, tag, reps=5):
    """(diagnostic) bv_verify_batch from pageable buffers: verifies/s of
    `reps` calls after one untimed call, to stderr."""
    v.verify(batch)
    t0 = time.perf_counter()
    for _ in range(reps):
        v.verify(batch)
    rate = batch.n_items * reps / (time.perf_counter() - t0)
    print(f"host_entry_probe {tag}: {rate / 1e6:.1f} M verifies/s", file=sys.stderr, flush=True)
    return rate


def host_entry_leg(args, v, batch):
    """bv_verify_batch from pageable host buffers (the cgo entry point).
    `value` is the mean over the timed calls; `value_median_call` the median
    call's rate (1-2 calls in 10 wait 13-26 ms for their first DMA to start,
    DESIGN.md section 5)."""
    import resource

    import numpy as np

    msgs = batch.msg_bytes.nbytes
    staged = msgs + batch.msg_off.nbytes + batch.r_be.nbytes + batch.s_be.nbytes + batch.item_msg.nbytes * 2
    # two untimed calls (the first allocates the context's staging buffers)
    v.verify(batch)
    v.verify(batch)
    ts, per = [], []
    ru0, nb0 = resource.getrusage(resource.RUSAGE_SELF), numa_counters()
    t0 = time.perf_counter()
    reps = max(2, min(10, args.steps))
    for _ in range(reps):
        t1 = time.perf_counter()
        v.verify(batch)
        per.append(round((time.perf_counter() - t1) * 1e3, 2))
        ts.append(v.timing())
    elapsed = time.perf_counter() - t0
    ru1, nb1 = resource.getrusage(resource.RUSAGE_SELF), numa_counters()
    h2d = mean(ts, "ms_h2d")
    diag = host_diag(batch)
    diag.update({"minor_faults_per_call": (ru1.ru_minflt - ru0.ru_minflt) / reps,
                 "invol_ctx_switches_per_call": (ru1.ru_nivcsw - ru0.ru_nivcsw) / reps,
                 "host_cpu_s_per_call": ((ru1.ru_utime + ru1.ru_stime) - (ru0.ru_utime + ru0.ru_stime)) / reps,
                 "staging_gb_s": staged / (mean(ts, "ms_host_prep") * 1e-3) / 1e9,
                 "numa_per_call": {k: (nb1[k] - nb0.get(k, 0)) / reps for k in nb1 if k != "numa_balancing"},
                 "numa_balancing": nb1.get("numa_balancing")})
    return {"value": args.events * reps / elapsed, "unit": "verifies/s", "ms_per_call": elapsed / reps * 1e3,
            "per_call_ms": per, "value_median_call": args.events / (float(np.median(per)) * 1e-3),
            "ms_h2d": h2d, "ms_d2h_tail": mean(ts, "ms_d2h"), "host_breakdown_ms": host_breakdown(ts),
            "bytes_staged": staged,
            "pcie_gb_s": staged / (h2d * 1e-3) / 1e9 if h2d > 0 else None, "host_diag": diag,
            "note": "inputs in pageable host memory; staged through pinned chunks, hashing overlaps the transfer; "
                    "PCIe-bound (~520 B per event crosses the link)"}


def host_entry_pinned_leg(args, v, batch):
    """bv_verify_batch over a batch the caller built in bv_host_alloc memory
    (page-locked; the cgo shim allocates its arrays there instead of
    C.CBytes): the library DMAs the inputs from where they
    are and the digests / statuses straight into the caller's pinned result
    arrays — no staging copy, the call is the PCIe transfer overlapped with
    the kernels."""
    import numpy as np

    from babble_amd.verifier import PinnedArena, VerifyResult

    arena = PinnedArena()
    try:
        pb = arena.batch(batch)
        res = VerifyResult(arena.array((batch.n_msgs, 32), np.uint8), arena.array(batch.n_items, np.uint8),
                           arena.array((batch.n_items + 63) // 64, np.uint64))
        v.verify_into(pb, res)
        v.verify_into(pb, res)  # (two untimed calls, as host_entry)
        ts, per = [], []
        reps = max(2, min(10, args.steps))
        t0 = time.perf_counter()
        for _ in range(reps):
            t1 = time.perf_counter()
            v.verify_into(pb, res)
            per.append(round((time.perf_counter() - t1) * 1e3, 2))
            ts.append(v.timing())
        elapsed = time.perf_counter() - t0
        assert np.array_equal(res.accept_bits, expected_words(0, args.events, 0))
        h2d = mean(ts, "ms_h2d")
        staged = sum(a.nbytes for a in (pb.msg_bytes, pb.msg_off, pb.r_be, pb.s_be, pb.item_msg, pb.item_key))
        return {"value": args.events * reps / elapsed, "unit": "verifies/s", "ms_per_call": elapsed / reps * 1e3,
                "per_call_ms": per,
                "ms_h2d": h2d, "host_breakdown_ms": host_breakdown(ts), "bytes_staged": staged,
                "pcie_gb_s": staged / (h2d * 1e-3) / 1e9 if h2d > 0 else None,
                "note": "inputs and results in bv_host_alloc (pinned) memory: DMA'd in place, no staging copy"}
    finally:
        arena.close()


def events_entry_leg(args):
    """bv_verify_events: wire fields in, the device
    builds every canonical EventBody, hashes and verifies.  `bulk`: the C2
    events with every parent a known hash (a store replay, no in-batch
    dependency), host buffers in / results out; `sync_dag`: a SyncLimit
    (1000) SyncResponse from 4 creators whose parents are earlier events of
    the batch (333 DAG levels of 3 events hashed on the device), median latency, key
    cache warm."""
    import numpy as np

    from babble_amd import events as E
    from babble_amd import native, synth
    from babble_amd.verifier import Verifier

    local = int(os.environ.get("LOCAL_RANK", "0"))
    out = {}
    packed, wire = synth.event_fields(args.events, n_creators=args.creators, seed=2, parents="hash")
    del packed
    out["bulk_pinned"] = events_pinned(args, wire, local)
    v = Verifier(device=local)
    v.verify_events(wire)
    reps = max(2, min(5, args.steps))
    t0 = time.perf_counter()
    for _ in range(reps):
        res = v.verify_events(wire)
    el = (time.perf_counter() - t0) / reps
    assert np.all(res.status == 1)
    tm = v.timing()
    wb = E.wire_bytes(wire)
    out["bulk"] = {"value": args.events / el, "unit": "verifies/s", "ms_per_call": el * 1e3, "ms_h2d": tm["ms_h2d"],
                   "host_breakdown_ms": host_breakdown([tm]),
                   "bytes_staged": wb, "bytes_per_event": wb / args.events,
                   "pcie_gb_s": wb / (tm["ms_h2d"] * 1e-3) / 1e9 if tm["ms_h2d"] > 0 else None}
    v.close()
    dag_packed, dag = synth.event_fields(1000, n_creators=4, seed=31, parents="event")
    vc = Verifier(device=local, flags=native.F_KEY_CACHE)
    vc.register_keys([dag_packed.key(k) for k in range(dag_packed.n_keys)])
    vc.verify_events(dag)
    ts = []
    for _ in range(15):
        t0 = time.perf_counter()
        res = vc.verify_events(dag)
        ts.append((time.perf_counter() - t0) * 1e3)
    assert np.all(res.status == 1)
    # the same response carrying Signature text (decoded on the device), as the shim passes it
    from tests.cabi import harness
    dag_t = dag.with_signature_text(*harness.encode_signatures(dag.r_be, dag.s_be))
    vc.verify_events(dag_t)
    tt = []
    for _ in range(15):
        t0 = time.perf_counter()
        res = vc.verify_events(dag_t)
        tt.append((time.perf_counter() - t0) * 1e3)
    assert np.all(res.status == 1)
    vc.close()
    out["sync_dag_1000"] = {"ms_median": float(np.median(ts)), "ms_median_sig_text": float(np.median(tt)),
                            "creators": 4, "dag_levels": dag_levels(dag),
                            "cpu": None if args.no_cpu else cpu_sync_dag(dag_packed)}
    return out


def c1_leg(args, local) -> dict:
    """SURVEY §8d C1 / BASELINE configs[0]: 4 peers, 10k signed events in the
    hashgraph play order (each event's parents are earlier events of the
    batch: the in-batch DAG), through bv_verify_events as one batch, cold and
    with the 4 peers registered; beside the CPU ingesting the same events the
    way InsertEvent does (SHA-256 of every body in order, then ecdsa.Verify:
    the C port on one core, as the reference's serial InsertEvent, and on
    all cores)."""
    import numpy as np

    from babble_amd import native, synth
    from babble_amd.verifier import Verifier

    import hashlib

    packed, dag = synth.event_fields(10_000, n_creators=4, seed=1, parents="event")
    out = {"events": 10_000, "creators": 4, "dag_levels": dag_levels(dag)}
    for name, flags in (("cold", 0), ("warm", native.F_KEY_CACHE)):
        v = Verifier(device=local, flags=flags)
        if flags:
            v.register_keys([packed.key(k) for k in range(packed.n_keys)])
        v.verify_events(dag)
        ts = []
        for _ in range(9):
            t0 = time.perf_counter()
            res = v.verify_events(dag)
            ts.append((time.perf_counter() - t0) * 1e3)
        assert np.all(res.status == 1)
        assert res.msg_hash[-1].tobytes() == hashlib.sha256(packed.message(packed.n_msgs - 1)).digest()
        v.close()
        out[name] = {"ms_median": float(np.median(ts)), "value": 10_000 / (float(np.median(ts)) * 1e-3),
                     "unit": "verifies/s"}
    out["cpu"] = None if args.no_cpu else cpu_sync_dag(packed)
    return out


def events_pinned(args, wire, local) -> dict:
    """The bulk events batch built by the caller in bv_host_alloc memory
    (PinnedArena.wire; a cgo shim allocates its wire arrays there): the wire
    fields are DMA'd from where they are and the digests / statuses land in
    the caller's pinned result arrays — no staging copy on either side."""
    import numpy as np

    from babble_amd import events as E
    from babble_amd.verifier import PinnedArena, Verifier, VerifyResult

    arena = PinnedArena()
    v = Verifier(device=local)
    try:
        pw = arena.wire(wire)
        n = wire.n_events
        res = VerifyResult(arena.array((n, 32), np.uint8), arena.array(n, np.uint8),
                           arena.array((n + 63) // 64, np.uint64))
        v.verify_events_into(pw, res)
        reps = max(2, min(5, args.steps))
        ts = []
        t0 = time.perf_counter()
        for _ in range(reps):
            v.verify_events_into(pw, res)
            ts.append(v.timing())
        el = (time.perf_counter() - t0) / reps
        assert np.all(res.status == 1)
        wb = E.wire_bytes(wire)
        h2d = mean(ts, "ms_h2d")
        return {"value": n / el, "unit": "verifies/s", "ms_per_call": el * 1e3, "ms_h2d": h2d,
                "host_breakdown_ms": host_breakdown(ts), "bytes_staged": wb,
                "pcie_gb_s": wb / (h2d * 1e-3) / 1e9 if h2d > 0 else None,
                "note": "wire fields and results in bv_host_alloc (pinned) memory: DMA'd in place, no staging copy"}
    finally:
        v.close()
        arena.close()


def dag_levels(wire) -> int:
    """Number of levels of the in-batch parent DAG (level = 1 + the deepest
    in-batch parent's level): the serial hashing depth."""
    import numpy as np

    from babble_amd import events as E

    ref = np.asarray(wire.parent_ref).reshape(-1, 2)
    kind = np.asarray(wire.parent_kind).reshape(-1, 2)
    lvl = np.zeros(len(ref), np.int64)
    for e in range(len(ref)):
        for k in range(2):
            if kind[e, k] == E.PARENT_EVENT:
                lvl[e] = max(lvl[e], lvl[int(ref[e, k])] + 1)
    return int(lvl.max()) + 1 if len(ref) else 0


def cpu_sync_dag(packed) -> dict:
    """The same 1000-event SyncResponse on the host's cores, the way a CPU
    node ingests it (core.go:214-245): SHA-256 of every body in topological
    order (each body embeds its parents' hashes, so hashing is serial; the
    serialized bodies are GIVEN to the CPU — the library builds them from
    wire fields), then every signature verified by the C port (oracle/oracle.c
    port_verify_batch: Go's ecdsa.Verify over btcec) on all cores and on one.
    The batch is converted once; the port's thread pool persists across
    calls.  Median of 7 runs.  Returns ms."""
    import hashlib

    import numpy as np

    from oracle import coracle  # CPU baseline leg only

    cores = cpu_threads()
    bodies = [packed.message(m) for m in range(packed.n_msgs)]
    prep = coracle.Prepared(packed.as_dict())
    prep.port(cores)
    out = {}
    for name, nt in (("all_cores", cores), ("one_core", 1)):
        t_hash, t_ver = [], []
        for _ in range(7 if nt > 1 else 3):
            t0 = time.perf_counter()
            digests = [hashlib.sha256(b).digest() for b in bodies]  # topological order
            t1 = time.perf_counter()
            st = prep.port(nt)
            t2 = time.perf_counter()
            t_hash.append((t1 - t0) * 1e3)
            t_ver.append((t2 - t1) * 1e3)
        assert len(digests) == packed.n_msgs and np.all(st == 1)
        tot = [a + b for a, b in zip(t_hash, t_ver)]
        out[name] = {"ms_median": float(np.median(tot)), "hash_ms": float(np.median(t_hash)),
                     "verify_ms": float(np.median(t_ver)), "threads": nt}
    out["ms_median"] = out["all_cores"]["ms_median"]
    out["cores"] = cores
    out["what"] = "hashlib SHA-256 of the serialized bodies in order + oracle.c port_verify_batch"
    return out


def shim_path_leg(args, line):
    """The Go shim's path through the C harness
    (tests/cabi/shim_harness.c): the key-cache context, the creators
    registered as the PeerSet (bv_kc_register), batches built field by field
    in pooled pinned arenas, signature text copied (decoded on the device), results
    copied out — all inside the clock (the harness's own wall time).  Shapes:
    one event through bv_verify_batch (addSelfEvent, core.go:291), the
    SyncLimit SyncResponse of `events_entry.sync_dag_1000` (1000 events, 4
    creators, in-batch parents) and the C2 replay (1M events, store-hash
    parents) through bv_verify_events.  Each beside the library-only number
    of the same shape: for the SyncResponse measured in this leg, call for
    call alternating with the shim's."""
    import numpy as np

    from babble_amd import synth
    from tests.cabi import harness

    local = int(os.environ.get("LOCAL_RANK", "0"))
    out = {}
    sh = harness.Shim(device=local)
    try:
        one_packed, one = synth.event_fields(1, n_creators=1, seed=900 + 1, parents="hash")
        sh.set_peers([one_packed.key(0)])
        text, off = harness.encode_signatures(one.r_be, one.s_be)
        body, key, sig = one_packed.message(0), one_packed.key(0), harness.signature_text(text, off, 0)
        sh.verify_event(body, key, sig)
        ts = []
        for _ in range(31):
            _, st, ms = sh.verify_event(body, key, sig)
            assert st == 1
            ts.append(ms)
        lib1 = (line.get("latency_ms") or {}).get("1", {}).get("warm_key_cache")
        out["event_1"] = {"ms_median": float(np.median(ts)), "library_ms": lib1,
                          "over_library": float(np.median(ts)) / lib1 if lib1 else None}
        dag_packed, dag = synth.event_fields(1000, n_creators=4, seed=31, parents="event")
        dag_keys = [dag_packed.key(k) for k in range(dag_packed.n_keys)]
        sh.set_peers(dag_keys)
        sw, keep = sh.wire(dag)
        # the library's own call (Python ctypes, the same key-cache context
        # and Signature text) alternated with the shim's on this box: the
        # DAG path's host hashing makes separate legs' numbers drift
        from babble_amd import native
        from babble_amd.verifier import Verifier

        vc = Verifier(device=local, flags=native.F_KEY_CACHE)
        vc.register_keys(dag_keys)
        dag_t = dag.with_signature_text(*harness.encode_signatures(dag.r_be, dag.s_be))
        sh.sync(sw)
        vc.verify_events(dag_t)
        ts, tl, ph = [], [], []
        for _ in range(21):
            _, st, ms = sh.sync(sw)
            assert np.all(st == 1)
            ts.append(ms)
            ph.append(sh.phases())
            t0 = time.perf_counter()
            res = vc.verify_events(dag_t)
            tl.append((time.perf_counter() - t0) * 1e3)
            assert np.all(res.status == 1)
        vc.close()
        libd = float(np.median(tl))
        out["sync_dag_1000"] = {"ms_median": float(np.median(ts)), "library_ms": libd,
                                "over_library": float(np.median(ts)) / libd,
                                "library_ms_events_entry_leg": ((line.get("events_entry") or {}).get("sync_dag_1000")
                                                                or {}).get("ms_median"),
                                "phases_ms": {k: float(np.median([p[k] for p in ph])) for k in ph[0]}}
        del sw, keep
        packed, wire = synth.event_fields(args.events, n_creators=args.creators, seed=2, parents="hash")
        sh.set_peers([packed.key(k) for k in range(packed.n_keys)])
        del packed
        sw, keep = sh.wire(wire)
        sh.sync(sw)
        ts = []
        ph = []
        for _ in range(max(2, min(5, args.steps))):
            _, st, ms = sh.sync(sw)
            assert np.all(st == 1)
            ts.append(ms)
            ph.append(sh.phases())
        ms = float(np.median(ts))
        libb = ((line.get("events_entry") or {}).get("bulk_pinned") or {}).get("value")
        out["bulk_1m"] = {"events": args.events, "ms_median": ms, "value": args.events / (ms * 1e-3),
                          "unit": "verifies/s", "library_pinned_value": libb,
                          "phases_ms": {k: float(np.median([p[k] for p in ph])) for k in ph[0]}}
    finally:
        sh.close()
    return out


def latency_leg(args):
    """bv_verify_batch latency (host buffers in, results out) by batch size,
    beside the C port of the reference path on this host's cores."""
    import numpy as np

    from babble_amd import native, synth
    from babble_amd.verifier import Verifier

    out = {}
    vc = Verifier(device=int(os.environ.get("LOCAL_RANK", "0")), flags=native.F_KEY_CACHE)
    v0 = Verifier(device=int(os.environ.get("LOCAL_RANK", "0")))
    cores = cpu_threads()
    for n in (1, 100, 1000, 10_000, 100_000):
        b = synth.events(n, n_creators=min(4, n), seed=900 + n)
        row = {}
        if not args.no_cpu:  # the same batch on the host: the C port (SHA-256 + decode + verify)
            from oracle import coracle  # CPU baseline leg only

            prep = coracle.Prepared(b.as_dict())  # converted once: the timed call is the C call alone
            for name, nt in (("cpu_port_all_cores", cores), ("cpu_port_1core", 1)):
                if nt == 1 and n > 1000:
                    continue
                prep.port(nt)
                tc = []
                for _ in range(3 if n >= 10_000 else 7):
                    t0 = time.perf_counter()
                    prep.port(nt)
                    tc.append((time.perf_counter() - t0) * 1e3)
                row[name] = float(np.median(tc))
        for name, ver in (("cold", v0), ("warm_key_cache", vc)):
            if ver is vc:  # the creators are registered validators (their tables built here)
                ver.register_keys([b.key(k) for k in range(b.n_keys)])
            ver.verify(b)  # warm-up
            ts = []
            for _ in range(15):
                t0 = time.perf_counter()
                ver.verify(b)
                ts.append((time.perf_counter() - t0) * 1e3)
            row[name] = float(np.median(ts))
            row[name + "_key_path"] = int(ver.timing()["key_path"])
        out[str(n)] = row
    vc.close()
    v0.close()
    return out


if __name__ == "__main__":
    main()
