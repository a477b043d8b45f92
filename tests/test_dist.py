"""Multi-rank path on CPU (gloo, world size 2 and 3): each rank verifies its
64-aligned shard (host build of the device code, tests/emu) and the accept
bitmasks are all-gathered; the global bitmask equals the oracle's."""
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
