"""GPU parity for the key cache (BV_F_KEY_CACHE), the pinned host entry
point, call ordering across streams / async calls, the multi-device group
(bv_group_*, RCCL all-gather) and C5 at its full size — all through the C
ABI against the C oracle (bit-exact statuses, digests and accept bits)."""
import os

import numpy as np
import pytest

from babble_amd import native, synth
from oracle import coracle
from oracle import gosemantics as gs

pytestmark = pytest.mark.gpu

MIX = dict(rflip=20000, sflip=20000, body=10000, highs=10000, range=8000, fmt=8000, key=12000)


def oracle_check(res, b):
    h, st, bits = coracle.verify_batch(b.as_dict())
    assert np.array_equal(res.msg_hash, h), "digests differ from oracle"
    bad = np.flatnonzero(res.status != st)
    assert bad.size == 0, f"{bad.size} statuses differ, first {bad[:8]}: gpu {res.status[bad[:8]]} oracle {st[bad[:8]]}"
    assert np.array_equal(res.accept_bits, bits)
    return st


@pytest.fixture(scope="module")
def cached():
    from babble_amd.verifier import Verifier

    v = Verifier(device=0, flags=native.F_KEY_CACHE)
    yield v
    v.close()


@pytest.fixture(scope="module")
def verifier_default():
    from babble_amd.verifier import Verifier

    v = Verifier(device=0)
    yield v
    v.close()


def valid_keys(b):
    return [b.key(k) for k in range(b.n_keys) if gs.Unmarshal(b.key(k)) is not None]


def test_key_cache_admission_cold_then_warm(cached):
    """Admission: an unregistered valid key gets a KC table
    once it has been seen in 2 batches.  First call: per-batch tables, nothing
    built; second: a table per distinct valid key (malformed keys get none);
    third: every valid key hits and nothing is built.  All bit-exact."""
    b = synth.adversarial(30_000, seed=41, n_creators=6, scale_per_million=MIX)
    st = oracle_check(cached.verify(b), b)
    t = cached.timing()
    assert t["key_path"] in (8, 12) and t["kc_builds"] == 0
    n_valid = len(set(valid_keys(b)))
    assert 0 < n_valid < b.n_keys  # the mix carries malformed keys (and one repeated valid key)
    assert set(np.unique(st)) == {0, 1, 2, 3}
    oracle_check(cached.verify(b), b)
    t = cached.timing()
    assert t["key_path"] == 22 and t["kc_builds"] == n_valid and t["kc_hits"] == 0
    oracle_check(cached.verify(b), b)
    t = cached.timing()
    assert t["kc_builds"] == 0 and t["kc_hits"] == n_valid and t["key_path"] == 22


def test_key_cache_small_batches(cached):
    """Latency-sized batches (1, 100, 1000 = SyncLimit, config.go:44) of
    registered creators take the cached tables on the first call; same
    results as the oracle."""
    for n in (1, 100, 1000):
        b = synth.events(n, n_creators=4, seed=100 + n)
        cached.register_keys([b.key(k) for k in range(b.n_keys)])
        assert cached.timing()["kc_builds"] == b.n_keys
        oracle_check(cached.verify(b), b)
        t = cached.timing()
        assert t["key_path"] == 22 and t["kc_builds"] == 0 and t["kc_hits"] == b.n_keys


def test_key_cache_device_entry(cached):
    b = synth.adversarial(20_000, seed=42, n_creators=6, scale_per_million=MIX)
    d = cached.to_device(b)
    for call in range(2):
        cached.verify_device(d)
        oracle_check(d.result(), b)
    assert cached.timing()["key_path"] == 22


def test_key_cache_eviction(monkeypatch):
    """A 2.5 GB budget holds 3 tables (805 MB each): a batch with 2 new keys after a batch
    with 2 others evicts the least recently used; results stay exact."""
    from babble_amd.verifier import Verifier

    monkeypatch.setenv("BV_KEY_CACHE_GB", "2.5")
    monkeypatch.setenv("BV_KC_ADMIT", "1")
    v = Verifier(device=0, flags=native.F_KEY_CACHE)
    try:
        a = synth.events(3000, n_creators=2, seed=51)
        b = synth.events(3000, n_creators=2, seed=52)
        oracle_check(v.verify(a), a)
        assert v.timing()["kc_builds"] == 2
        oracle_check(v.verify(b), b)
        t = v.timing()
        assert t["kc_builds"] == 2 and t["kc_keys"] <= 3
        oracle_check(v.verify(a), a)
    finally:
        v.close()


def test_key_cache_register_beyond_budget(monkeypatch):
    """registering more validators than the budget holds
    builds the first ones that fit (2.5 GB: 3 tables of 805 MB) and returns
    BV_OK; the 2 left over never evict a registered table, so batches naming
    them take the per-batch path after their (already launched) key decode —
    the bail-out waits for that decode before the s^-1 stream decodes again —
    on the host entry, the device entry and the events entry, every result
    exact."""
    from babble_amd.verifier import Verifier

    monkeypatch.setenv("BV_KEY_CACHE_GB", "2.5")
    monkeypatch.setenv("BV_KC_ADMIT", "1")
    b = synth.adversarial(20_000, seed=46, n_creators=5, scale_per_million=MIX)
    keys = [b.key(k) for k in range(b.n_keys)]
    n_valid = len(set(valid_keys(b)))
    assert n_valid == 5
    v = Verifier(device=0, flags=native.F_KEY_CACHE)
    try:
        v.register_keys(keys)
        t = v.timing()
        assert t["kc_builds"] == 3 and t["kc_keys"] == 3, t
        for _ in range(2):
            oracle_check(v.verify(b), b)
            t = v.timing()
            assert t["key_path"] in (8, 12) and t["kc_keys"] == 3 and t["kc_builds"] == 0, t
        d = v.to_device(b)
        v.verify_device(d)
        oracle_check(d.result(), b)
        packed, wire = synth.event_fields(4000, n_creators=5, seed=46, parents="hash")
        res = v.verify_events(wire)
        h, st, bits = coracle.verify_batch(packed.as_dict())
        assert np.array_equal(res.msg_hash, h) and np.array_equal(res.status, st)
        assert np.array_equal(res.accept_bits, bits)
    finally:
        v.close()


@pytest.mark.parametrize("fail", ["alloc:3", "build:2"])
def test_key_cache_failure_leaves_no_unbuilt_slot(monkeypatch, fail):
    """a KC table allocation (the 3rd of a 64-key miss batch)
    or a build launch (the 2nd group of 8 keys) fails part-way.  The call
    either takes the per-batch path (allocation: results exact) or returns
    an error (launch); either way nothing is indexed, so the NEXT call on the
    same keys builds every table afresh and equals the oracle bit for bit,
    and the call after that hits all 64."""
    from babble_amd.verifier import Verifier

    monkeypatch.setenv("BV_KC_ADMIT", "1")
    monkeypatch.setenv("BV_KC_FAIL", fail)
    b = synth.adversarial(40_000, seed=44, n_creators=64, scale_per_million=MIX)
    n_valid = len(set(valid_keys(b)))
    v = Verifier(device=0, flags=native.F_KEY_CACHE)
    try:
        if fail.startswith("alloc"):
            oracle_check(v.verify(b), b)
            t = v.timing()
            assert t["key_path"] in (8, 12) and t["kc_keys"] == 0 and t["kc_builds"] == 0
        else:
            with pytest.raises(native.BvError):
                v.verify(b)
        oracle_check(v.verify(b), b)
        t = v.timing()
        assert t["key_path"] == 22 and t["kc_builds"] == n_valid and t["kc_keys"] == n_valid
        d = v.to_device(b)
        v.verify_device(d)
        oracle_check(d.result(), b)
        t = v.timing()
        assert t["kc_hits"] == n_valid and t["kc_builds"] == 0
    finally:
        v.close()


def _rss_mb() -> float:
    with open("/proc/self/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return int(line.split()[1]) / 1024
    return 0.0


def test_key_cache_admission_control():
    """with the 64 validators registered (bv_kc_register, the
    PeerSet), 10k distinct malformed 65-byte keys and 1k fresh valid keys
    (each seen once, as a flood of join requests would be) go through the
    same ctx: every result equals the oracle, no table is built for them,
    the 64 registered tables stay resident (the next validator batch hits all
    64 and builds nothing) and host memory stays bounded."""
    from babble_amd.batch import PackedBatch
    from babble_amd.verifier import Verifier

    vb = synth.events(20_000, n_creators=64, seed=2)
    v = Verifier(device=0, flags=native.F_KEY_CACHE)
    try:
        v.register_keys([vb.key(k) for k in range(vb.n_keys)])
        assert v.timing()["kc_builds"] == 64 and v.timing()["kc_keys"] == 64
        rng = np.random.default_rng(123)
        rss0 = None
        for j in range(5):  # 5 x 2000 distinct off-curve keys
            fb = synth.events(2000, n_creators=4, seed=300 + j)
            bad = np.concatenate([np.full((2000, 1), 4, np.uint8), rng.integers(0, 256, (2000, 64), dtype=np.uint8)],
                                 axis=1)
            mb = PackedBatch(fb.msg_bytes, fb.msg_off, bad.reshape(-1).copy(),
                             np.arange(2001, dtype=np.uint64) * 65, fb.item_msg, np.arange(2000, dtype=np.uint32),
                             fb.r_be, fb.s_be, fb.pre)
            st = oracle_check(v.verify(mb), mb)
            assert np.all(st == native.REF_PANIC)
            assert v.timing()["key_path"] == 22 and v.timing()["kc_builds"] == 0
            if rss0 is None:
                rss0 = _rss_mb()
        for j in range(4):  # 4 x 250 fresh valid creators, one batch each (16 events per creator)
            fb = synth.events(4000, n_creators=250, seed=400 + j)
            oracle_check(v.verify(fb), fb)
            t = v.timing()
            assert t["kc_builds"] == 0 and t["key_path"] == 8
        assert _rss_mb() - rss0 < 64, "host memory grew with attacker-chosen keys"
        oracle_check(v.verify(vb), vb)
        t = v.timing()
        assert t["kc_hits"] == 64 and t["kc_builds"] == 0 and t["kc_keys"] == 64 and t["key_path"] == 22
    finally:
        v.close()


def test_host_entry_equals_device_entry_1m(cached):
    """The pinned, chunked host entry point (digests hashed and items
    verified chunk by chunk as they land) at C2 size, with a seeded set of
    corrupted signatures spread over every chunk: all 1M digests, statuses
    and bits equal the C oracle's and the device
    entry's; the call reports its PCIe staging time."""
    from babble_amd.verifier import Verifier

    b = synth.events(1_000_000, n_creators=64, seed=2)
    bad = np.random.default_rng(99).choice(b.n_items, 5000, replace=False)
    b.s_be[bad, 11] ^= 0x04
    v = Verifier(device=0)
    try:
        res = v.verify(b)
        t = v.timing()
        assert t["ms_h2d"] > 0 and t["ms_host"] >= t["ms_h2d"]
        st = oracle_check(res, b)
        assert int((st != 1).sum()) == len(bad)
        d = v.to_device(b)
        v.verify_device(d)
        res2 = d.result()
        assert np.array_equal(res.msg_hash, res2.msg_hash)
        assert np.array_equal(res.status, res2.status)
        assert np.array_equal(res.accept_bits, res2.accept_bits)
    finally:
        v.close()


def test_async_calls_on_two_streams_are_ordered():
    """two async device calls on different streams share the ctx
    work buffers; the library orders them (ev_done), so both are exact."""
    import torch

    from babble_amd.verifier import Verifier

    v = Verifier(device=0)
    try:
        b1 = synth.adversarial(60_000, seed=61, n_creators=8, scale_per_million=MIX)
        b2 = synth.adversarial(50_000, seed=62, n_creators=8, scale_per_million=MIX)
        d1, d2 = v.to_device(b1), v.to_device(b2)
        s1, s2 = torch.cuda.Stream(0), torch.cuda.Stream(0)
        v.verify_device(d1, stream=s1.cuda_stream, sync=False)
        v.verify_device(d2, stream=s2.cuda_stream, sync=False)
        s1.synchronize()
        s2.synchronize()
        oracle_check(d1.result(), b1)
        oracle_check(d2.result(), b2)
        # async on the library's own stream: result() waits through bv_sync
        v.verify_device(d1, stream=0, sync=False)
        oracle_check(d1.result(), b1)
    finally:
        v.close()


@pytest.mark.parametrize("n_streams", [2, 3])
@pytest.mark.parametrize("flags", [0, native.F_KEY_CACHE], ids=["per_batch", "key_cache"])
def test_async_calls_two_in_flight(flags, n_streams):
    """Work-buffer slots: consecutive async device calls rotate over them and
    wait only for the slot's previous call (and for in-flight calls writing
    the same results), so calls on several streams overlap.  Seven calls over
    three batches of different sizes/keys on 2 or 3 streams (slots reused
    with other shapes, the same result buffers on different streams), then a
    host-entry call (waits for all) and one more async pair: every result
    exact."""
    import torch

    from babble_amd.verifier import Verifier

    v = Verifier(device=0, flags=flags)
    try:
        bs = [synth.adversarial(n, seed=63 + i, n_creators=c, scale_per_million=MIX)
              for i, (n, c) in enumerate([(70_000, 8), (9_000, 3), (40_000, 12)])]
        ds = [v.to_device(b) for b in bs]
        ss = [torch.cuda.Stream(0) for _ in range(n_streams)]
        torch.cuda.synchronize()
        for k in range(7):
            v.verify_device(ds[k % 3], stream=ss[k % n_streams].cuda_stream, sync=False)
        torch.cuda.synchronize()
        for d, b in zip(ds, bs):
            oracle_check(d.result(), b)
        oracle_check(v.verify(bs[1]), bs[1])
        v.verify_device(ds[2], stream=ss[0].cuda_stream, sync=False)
        v.verify_device(ds[0], stream=ss[1].cuda_stream, sync=False)
        oracle_check(ds[2].result(), bs[2])
        oracle_check(ds[0].result(), bs[0])
    finally:
        v.close()


def test_group_one_device():
    """bv_group over the box's device(s): shards, per-device staging and the
    RCCL all-gather of the bitmask; equal to the oracle."""
    import torch

    from babble_amd.verifier import Group

    g = Group(list(range(torch.cuda.device_count())))
    try:
        b = synth.adversarial(40_000, seed=71, n_creators=8, scale_per_million=MIX)
        oracle_check(g.verify(b), b)
        wb = synth.blocks(300, n_validators=100, seed=72)
        oracle_check(g.verify(wb.batch), wb.batch)
    finally:
        g.close()


def test_group_logical_shards():
    """The multi-shard path of bv_group on the box's one GPU: a device list
    naming device 0 three times makes three shards (three contexts, three
    concurrent staging threads, the shard plan and the shifted bit merge —
    the code an 8-GPU group runs, with device copies in place of the RCCL
    all-gather).  Batches whose shard bounds fall inside 64-item words
    (blocks of 30 signatures, shuffled items, item-less messages) and a
    bulk adversarial batch: statuses, bits and digests equal the oracle's
    and the single-context results."""
    from babble_amd.verifier import Group, plan_group

    b = synth.adversarial(150_001, seed=75, n_creators=8, scale_per_million=MIX)
    wb = synth.blocks(333, n_validators=30, seed=76)
    _, _, bounds, _ = plan_group(wb.batch, 3)
    assert any(int(x) % 64 for x in bounds[1:-1])  # unaligned shard starts
    g = Group([0, 0, 0])
    try:
        for batch in (b, wb.batch):
            r = g.verify(batch)
            oracle_check(r, batch)
            assert r.msg_hash.shape[0] == batch.n_msgs
        from babble_amd.verifier import Verifier
        v = Verifier(device=0)
        try:
            r1, r2 = g.verify(b), v.verify(b)
            assert np.array_equal(r1.msg_hash, r2.msg_hash) and np.array_equal(r1.status, r2.status)
            assert np.array_equal(r1.accept_bits, r2.accept_bits)
        finally:
            v.close()
    finally:
        g.close()


def test_group_rejects_repeated_devices_in_a_mixed_list():
    """A device may repeat only as logical shards of ONE device."""
    from babble_amd import native
    from babble_amd.verifier import Group

    with pytest.raises(native.BvError):
        Group([0, 1, 0])


@pytest.mark.parametrize("key_cache", [True, False])
def test_c5_full_size_check_block(cached, verifier_default, key_cache):
    """C5 as SURVEY §8d specifies it: 10^4 blocks x 100 validators (10^6
    signature items over 10^4 BlockBodies, each hashed once), 5 % invalid
    signatures; every status equal to the oracle, and the per-block valid
    counts decide CheckBlock (count > TrustCount, hashgraph.go:1599-1630)."""
    wb = synth.blocks(10_000, n_validators=100, seed=5)
    b = wb.batch
    rng = np.random.default_rng(5)
    bad = rng.choice(b.n_items, size=b.n_items // 20, replace=False)
    b.s_be[bad, 7] ^= 0x40
    v = cached if key_cache else verifier_default
    if key_cache:  # the validator set is registered, as CheckBlock's PeerSet is known
        v.register_keys([b.key(k) for k in range(b.n_keys)])
    res = v.verify(b)
    assert v.timing()["key_path"] == (22 if key_cache else 12)
    st = oracle_check(res, b)
    valid = (st == 1).reshape(wb.n_blocks, wb.n_validators).sum(axis=1)
    got = (res.status == 1).reshape(wb.n_blocks, wb.n_validators).sum(axis=1)
    assert np.array_equal(valid, got)
    tc = gs.trust_count(wb.n_validators)
    assert int(valid.sum()) == b.n_items - len(bad)
    assert np.all(valid > tc)


def test_group_item_less_messages_and_shuffled_items():
    """a group call hashes EVERY message (also messages no item
    names, as bv_verify_batch does) and takes items in any message order
    (stably sorted for sharding, results returned in the caller's order):
    digests, statuses and bits equal the oracle's."""
    import torch

    from babble_amd.batch import PackedBatch
    from babble_amd.verifier import Group, plan_group

    wb = synth.blocks(120, n_validators=30, seed=73)
    b = wb.batch
    rng = np.random.default_rng(73)
    b.s_be[rng.choice(b.n_items, 200, replace=False), 5] ^= 0x21
    # interleave item-less messages (before, between and after referenced ones)
    extra = [b"", b"x" * 55, b"y" * 64, b"{}\n" * 40]
    order = []  # new message index of each old message
    out = [extra[0]]
    for m in range(b.n_msgs):
        order.append(len(out))
        out.append(b.message(m))
        if m % 7 == 3:
            out.append(extra[1 + m % 3])
    out.append(extra[3])
    off = np.zeros(len(out) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in out])
    perm = rng.permutation(b.n_items)
    sb = PackedBatch(np.frombuffer(b"".join(out), np.uint8).copy(), off, b.key_bytes, b.key_off,
                     np.asarray(order, np.uint32)[b.item_msg[perm]], b.item_key[perm].copy(), b.r_be[perm].copy(),
                     b.s_be[perm].copy(), b.pre[perm].copy())
    permuted, _, _, mb = plan_group(sb, 3)
    assert permuted and mb[0] == 0 and mb[-1] == sb.n_msgs
    g = Group(list(range(torch.cuda.device_count())))
    try:
        oracle_check(g.verify(sb), sb)
        # the same batch through the single-device entry point: identical
        from babble_amd.verifier import Verifier
        v = Verifier(device=0)
        try:
            r1, r2 = g.verify(sb), v.verify(sb)
            assert np.array_equal(r1.msg_hash, r2.msg_hash) and np.array_equal(r1.status, r2.status)
            assert np.array_equal(r1.accept_bits, r2.accept_bits)
        finally:
            v.close()
    finally:
        g.close()


def test_pinned_host_entry_zero_copy():
    """bv_host_alloc memory: a batch whose arrays and result
    buffers are page-locked is DMA'd from / to them directly; results equal
    the pageable path and the oracle."""
    from babble_amd.verifier import PinnedArena, Verifier, VerifyResult

    b = synth.adversarial(50_000, seed=81, n_creators=8, scale_per_million=MIX)
    arena = PinnedArena()
    v = Verifier(device=0)
    try:
        pb = arena.batch(b)
        res = VerifyResult(arena.array((b.n_msgs, 32), np.uint8), arena.array(b.n_items, np.uint8),
                           arena.array((b.n_items + 63) // 64, np.uint64))
        v.verify_into(pb, res)
        t = v.timing()
        oracle_check(res, b)
        ref = v.verify(b)
        assert np.array_equal(ref.status, res.status) and np.array_equal(ref.msg_hash, res.msg_hash)
        assert t["ms_host_prep"] >= 0
    finally:
        v.close()
        arena.close()


@pytest.mark.parametrize("device_api", [False, True])
def test_key_cache_partial_batch(monkeypatch, device_api):
    """a batch whose keys are all cached but one fresh valid key
    (not registered, not yet admitted) keeps the key cache for the cached
    keys; the fresh key's items are left BV_DEFERRED by the KC kernels and
    finished by the generic path (bv_run_deferred).  Corrupted signatures
    on both kinds of key; every status, digest and bit equal to the oracle.
    With 3 fresh keys of 20 (more than 1 in 16) the batch takes the
    per-batch tables as before."""
    from babble_amd.verifier import Verifier

    monkeypatch.setenv("BV_KC_ADMIT", "1000")  # no fresh key gets a table during the test (read at bv_create)
    monkeypatch.setenv("BV_KC_PARTIAL", "1")  # partial mode is off by default (profiles/r06_ab_partial.log)
    b = synth.events(30_000, n_creators=20, seed=62)
    rng = np.random.default_rng(62)
    for i in rng.choice(b.n_items, 300, replace=False):
        b.r_be[i, int(rng.integers(0, 32))] ^= 1 << int(rng.integers(0, 8))
    keys = [b.key(k) for k in range(b.n_keys)]
    def run(v, batch):
        if device_api:
            d = v.to_device(batch)
            v.verify_device(d)
            return d.result()
        return v.verify(batch)

    for fresh, partial in ((1, True), (3, False)):
        v = Verifier(device=0, flags=native.F_KEY_CACHE)
        try:
            v.register_keys(keys[fresh:])
            # twice on one ctx: the second call finds the fresh
            # key remembered (no decode in bv_kc_prepare), so the deferred
            # items read the points bv_run_keys decoded on the s^-1 stream
            for rep in range(2):
                res = run(v, b)
                st = oracle_check(res, b)
                assert int((st == native.ACCEPT).sum()) == b.n_items - 300
                t = v.timing()
                assert (t["key_path"] == 22) == partial, (rep, t)
                if partial:
                    assert t["kc_hits"] == 20 - fresh and t["kc_builds"] == 0
        finally:
            v.close()
    # the deferred share is bounded by ITEMS too: one fresh key
    # of 20 that carries a fifth of the batch sends it to the per-batch tables
    skew = synth.events(30_000, n_creators=20, seed=63)
    skew.item_key = np.asarray(skew.item_key).copy()
    skew.item_key[::5] = 0
    v = Verifier(device=0, flags=native.F_KEY_CACHE)
    try:
        v.register_keys([skew.key(k) for k in range(1, 20)])
        oracle_check(run(v, skew), skew)
        assert v.timing()["key_path"] != 22
    finally:
        v.close()
    # the default (partial mode off): one fresh key of 20 sends the batch to
    # the per-batch tables, oracle-exact
    monkeypatch.delenv("BV_KC_PARTIAL")
    v = Verifier(device=0, flags=native.F_KEY_CACHE)
    try:
        v.register_keys(keys[1:])
        oracle_check(run(v, b), b)
        assert v.timing()["key_path"] != 22
    finally:
        v.close()


def test_key_cache_partial_batch_events_entry(monkeypatch):
    """the partial key-cache mode through bv_verify_events (the
    bulk wire path: key part first, the deferred tail on the split verify
    stream), one fresh creator of 20, twice on one context; digests,
    statuses and bits equal to the C oracle's."""
    from babble_amd.verifier import Verifier
    from oracle import coracle

    monkeypatch.setenv("BV_KC_ADMIT", "1000")
    monkeypatch.setenv("BV_KC_PARTIAL", "1")
    packed, wire = synth.event_fields(30_000, n_creators=20, seed=64, parents="hash")
    rng = np.random.default_rng(64)
    bad = rng.choice(packed.n_items, 200, replace=False)
    wire.s_be = np.asarray(wire.s_be).copy()
    wire.s_be[bad, 3] ^= 0x10
    packed.s_be[bad, 3] ^= 0x10
    h, st, bits = coracle.verify_batch(packed.as_dict())
    ko = np.asarray(wire.key_off, np.int64)
    keys = [wire.key_bytes[ko[k]:ko[k + 1]].tobytes() for k in range(len(ko) - 1)]
    v = Verifier(device=0, flags=native.F_KEY_CACHE)
    try:
        v.register_keys(keys[1:])
        for rep in range(2):
            res = v.verify_events(wire)
            assert np.array_equal(res.msg_hash, h), rep
            assert np.array_equal(res.status, st), rep
            assert np.array_equal(res.accept_bits, bits), rep
            assert v.timing()["key_path"] == 22, rep
        assert int((st != native.ACCEPT).sum()) == len(bad)
    finally:
        v.close()
