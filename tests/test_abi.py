"""The C-ABI library: builds, loads, exports every symbol include/*.h
declares, and fails loudly (no CPU fallback) without a gfx950 device."""
import ctypes
import glob
import os
import re
import subprocess

import pytest

from babble_amd import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b(bv_[a-z0-9_]+)\s*\(", src):
            names.add(m.group(1))
    return names


def test_header_declares_what_we_bind():
    assert declared_functions() == set(native.EXPORTS)


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", native.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = declared_functions() - exported
    assert not missing, missing


def test_abi_version_and_code_object():
    L = native.lib()
    assert L.bv_abi_version() == native.ABI_VERSION == 6
    # the library carries gfx950 device code (offload bundle entry name)
    blob = open(native.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_create_without_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    ctx = ctypes.c_void_p()
    rc = native.lib().bv_create(ctypes.byref(ctx), 0, 0)
    assert rc == native.BV_E_NODEVICE and not ctx.value


def test_null_args():
    L = native.lib()
    assert L.bv_verify_batch(None, None, None) == native.BV_E_ARGS
    assert L.bv_verify_batch_device(None, None, None, None, 0) == native.BV_E_ARGS
    assert L.bv_sha256_batch(None, 0, None, None, None) == native.BV_E_ARGS
    assert L.bv_get_timing(None, None) == native.BV_E_ARGS


def test_unknown_flags_rejected_before_any_device_call():
    ctx = ctypes.c_void_p()
    assert native.lib().bv_create(ctypes.byref(ctx), 0, 0x80) == native.BV_E_ARGS and not ctx.value
    g = ctypes.c_void_p()
    devs = (ctypes.c_int * 3)(0, 1, 0)  # a repeated device in a list of several devices
    assert native.lib().bv_group_create(ctypes.byref(g), devs, 3, 0) == native.BV_E_ARGS and not g.value


def test_group_null_args():
    L = native.lib()
    assert L.bv_group_verify_batch(None, None, None) == native.BV_E_ARGS
    assert L.bv_sync(None) == native.BV_E_ARGS
    assert L.bv_plan_shards(None, 2, None) == native.BV_E_ARGS


def test_plan_shards_balanced_and_message_aligned():
    """bv_plan_shards (the group's sharding): contiguous, covering, balanced,
    and never splitting the items of one message (C5: a block's 100
    signatures stay on one device)."""
    import numpy as np

    from babble_amd.batch import PackedBatch
    from babble_amd.verifier import plan_shards

    def batch(item_msg):
        n = len(item_msg)
        nm = int(item_msg.max()) + 1 if n else 0
        return PackedBatch(np.zeros(0, np.uint8), np.zeros(nm + 1, np.uint64), np.zeros(0, np.uint8),
                           np.zeros(2, np.uint64), np.asarray(item_msg, np.uint32), np.zeros(n, np.uint32),
                           np.zeros((n, 32), np.uint8), np.zeros((n, 32), np.uint8), None)

    # events: one item per message -> exact balance
    b = batch(np.arange(1000))
    assert plan_shards(b, 8).tolist() == [0, 125, 250, 375, 500, 625, 750, 875, 1000]
    # blocks: 100 items per message, 10^4 blocks over 8 devices
    im = np.repeat(np.arange(10_000), 100)
    bd = plan_shards(batch(im), 8)
    assert bd[0] == 0 and bd[-1] == im.size and np.all(np.diff(bd.astype(np.int64)) >= 0)
    for c in bd[1:-1]:
        assert im[c] != im[c - 1]  # a cut never splits a block
    sizes = np.diff(bd.astype(np.int64))
    assert sizes.max() - sizes.min() <= 100
    # ragged: more shards than messages, empty batch
    assert plan_shards(batch(np.repeat([0, 1], 5)), 4).tolist() == [0, 5, 5, 10, 10]
    assert plan_shards(batch(np.zeros(0, np.int64)), 3).tolist() == [0, 0, 0, 0]


def test_merge_shard_bits_equals_python_merge():
    """bv_merge_shard_bits (the host merge after bv_group's all-gather) equals
    shard.merge_bits on unaligned, empty and single-item shards; bits past a
    shard's end (padding garbage) never leak into the next shard."""
    import numpy as np

    from babble_amd import shard
    from babble_amd.verifier import merge_shard_bits

    rng = np.random.default_rng(11)
    for _ in range(300):
        n = int(rng.integers(0, 900))
        D = int(rng.integers(1, 9))
        cuts = sorted(rng.integers(0, n + 1, size=D - 1).tolist()) if n else [0] * (D - 1)
        bounds = [0] + cuts + [n]
        ok = rng.random(n) < 0.6
        words = max(1, max((bounds[d + 1] - bounds[d] + 63) // 64 for d in range(D)))
        g = rng.integers(0, 2**63, size=(D, words), dtype=np.int64).view(np.uint64)  # garbage everywhere
        parts = []
        for d in range(D):
            a, z = bounds[d], bounds[d + 1]
            pk = np.packbits(ok[a:z], bitorder="little")
            pk = np.concatenate([pk, np.zeros((-len(pk)) % 8, np.uint8)]).view(np.uint64)
            g[d, :len(pk)] = pk
            if z > a and (z - a) % 64:  # garbage above the last valid bit of the shard
                g[d, (z - a) // 64] |= ~np.uint64(0) << np.uint64((z - a) % 64)
            parts.append(g[d].copy())
        got = merge_shard_bits(g.reshape(-1), words, bounds)
        want = shard.merge_bits(parts, bounds)
        assert np.array_equal(got, want), (n, bounds)
        pk = np.packbits(ok, bitorder="little")
        full = np.concatenate([pk, np.zeros((-len(pk)) % 8, np.uint8)]).view(np.uint64)
        assert np.array_equal(got, full[: (n + 63) // 64])


def test_merge_shard_bits_rejects_bad_bounds():
    import numpy as np

    L = native.lib()
    g = np.zeros(4, np.uint64)
    out = np.zeros(4, np.uint64)
    for bounds in ([0, 70, 60], [1, 5, 9], [0, 200, 210]):  # non-monotone, not from 0, shard wider than 2 words
        b = np.asarray(bounds, np.uint64)
        assert L.bv_merge_shard_bits(g.ctypes.data, 2, 2, b.ctypes.data, out.ctypes.data) == native.BV_E_ARGS


def test_host_alloc_fails_loudly_or_frees():
    """bv_host_alloc needs the HIP runtime: without a device it reports an
    error (never a silent pageable fallback); bv_host_free ignores foreign
    pointers."""
    import torch

    L = native.lib()
    p = ctypes.c_void_p()
    rc = L.bv_host_alloc(4096, ctypes.byref(p))
    if torch.cuda.is_available():
        assert rc == native.BV_OK and p.value
    else:
        assert rc != native.BV_OK and not p.value
    L.bv_host_free(p)
    buf = ctypes.create_string_buffer(16)
    L.bv_host_free(ctypes.cast(buf, ctypes.c_void_p))  # not ours: ignored
    assert native.lib().bv_last_stream(None) is None


def test_plan_group_rejects_more_than_2_32_items():
    """the group plan keeps its permutation and sorted indices in
    u32; a batch claiming more than 2^32 items (or messages) is BV_E_ARGS
    before any array is read (the arrays here are tiny on purpose)."""
    import numpy as np

    L = native.lib()
    im = np.zeros(8, np.uint32)
    rs = np.zeros((8, 32), np.uint8)
    b = native.BvBatch()
    b.n_msgs = 1
    b.n_items = 2**32 + 5
    b.item_msg = b.item_key = im.ctypes.data
    b.r_be = b.s_be = rs.ctypes.data
    ib = np.zeros(3, np.uint64)
    mb = np.zeros(3, np.uint64)
    assert L.bv_plan_group(ctypes.byref(b), 2, ib.ctypes.data, mb.ctypes.data, None) == native.BV_E_ARGS
    b.n_items = 4
    b.n_msgs = 2**32 + 1
    assert L.bv_plan_group(ctypes.byref(b), 2, ib.ctypes.data, mb.ctypes.data, None) == native.BV_E_ARGS
