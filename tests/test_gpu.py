"""Parity tests proper: the gfx950 kernels through the C ABI against the
oracle (bit-exact statuses, digests and accept bits).  Run on the GPU box:
    python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
"""
import hashlib
import os
import threading

import numpy as np
import pytest

from babble_amd import native, synth
from babble_amd.batch import BatchBuilder
from oracle import coracle
from oracle import gosemantics as gs
from tests.helpers import bits_from_status, golden_items_batch, load

pytestmark = pytest.mark.gpu

MIX = dict(rflip=20000, sflip=20000, body=10000, highs=10000, range=8000, fmt=8000, key=12000)


@pytest.fixture(scope="module")
def verifier():
    from babble_amd.verifier import Verifier

    v = Verifier(device=0)
    yield v
    v.close()


def check_against_oracle(v, b, device_api=False):
    h, st, bits = coracle.verify_batch(b.as_dict())
    if device_api:
        d = v.to_device(b)
        v.verify_device(d)
        res = d.result()
    else:
        res = v.verify(b)
    assert np.array_equal(res.msg_hash, h), "digests differ from oracle"
    bad = np.flatnonzero(res.status != st)
    assert bad.size == 0, f"{bad.size} statuses differ, first {bad[:8]}: gpu {res.status[bad[:8]]} oracle {st[bad[:8]]}"
    assert np.array_equal(res.accept_bits, bits)
    return res


def test_golden_items(verifier):
    batch, expected, _ = golden_items_batch()
    res = verifier.verify(batch)
    assert np.array_equal(res.status, expected)
    assert np.array_equal(res.accept_bits, bits_from_status(expected))


def test_golden_items_from_signature_text(verifier):
    """Host path as the Go shim would drive it: signature text ->
    bv_decode_signature -> device."""
    items = load("golden_items.json")
    bb = BatchBuilder()
    for it in items:
        m = bb.add_msg(bytes.fromhex(it["body"]))
        k = bb.add_key(bytes.fromhex(it["pub"]))
        bb.add_item(m, k, it["sig"].encode("utf-8"))
    res = verifier.verify(bb.pack())
    assert np.array_equal(res.status, np.array([it["status"] for it in items], np.uint8))


def test_golden_sha256(verifier):
    fx = load("golden_sha256.json")
    msgs = [bytes.fromhex(e["msg"]) for e in fx]
    got = verifier.sha256(msgs)
    assert [g.hex() for g in got] == [e["digest"] for e in fx]


def test_sha256_boundaries_and_alignment(verifier):
    rng = np.random.default_rng(3)
    msgs = [rng.integers(0, 256, size=n, dtype=np.uint8).tobytes() for n in
            list(range(0, 300)) + [1 << 16, (1 << 20) + 3]]
    got = verifier.sha256(msgs)
    assert got == [hashlib.sha256(m).digest() for m in msgs]


def test_golden_events_digests(verifier):
    ev = load("golden_events.json")["events"]
    got = verifier.sha256([e["json"].encode("latin-1") for e in ev])
    assert [g.hex() for g in got] == [e["digest"] for e in ev]


def test_c1_hashgraph(verifier):
    b = synth.events(10_000, n_creators=4, seed=1)
    res = check_against_oracle(verifier, b)
    assert np.all(res.status == 1)


@pytest.mark.parametrize("device_api", [False, True])
def test_c4_adversarial_mix(verifier, device_api):
    b = synth.adversarial(20_000, seed=4, scale_per_million=MIX)
    res = check_against_oracle(verifier, b, device_api=device_api)
    assert set(np.unique(res.status)) == {0, 1, 2, 3}


def test_c4_adversarial_full_rate(verifier):
    """C4 at 10^5 items with the exact per-million corruption mix (~70 keys,
    ~1.4k items per key: the K8 chord-sum tables)."""
    b = synth.adversarial(100_000, seed=44)
    check_against_oracle(verifier, b)
    assert verifier.timing()["key_path"] == 8


def test_k8_tables_many_keys(monkeypatch):
    """More than 1024 keys (kMaxK12Keys): the 8-bit key tables, filled with
    the throughput point ops above 131072 items.  The many-key table
    threshold (192 items per key) is lowered to 16 so the oracle check stays
    at 140k items."""
    from babble_amd.verifier import Verifier

    monkeypatch.setenv("BV_TABLE_MIN_ITEMS_MANY", "16")  # read at bv_create
    verifier = Verifier(device=0)
    b = synth.adversarial(140_000, seed=45, n_creators=1100, scale_per_million=MIX)
    assert b.n_keys > 1024 and 16 * b.n_keys <= b.n_items < 2048 * b.n_keys and b.n_items > 131072
    check_against_oracle(verifier, b)
    assert verifier.timing()["key_path"] == 8
    verifier.close()


def test_generic_path_many_keys_few_items(verifier):
    """More than 1024 keys with fewer than 48 items each: the generic
    per-lane path, at 40k items (throughput variant) and 20k (latency)."""
    for n in (40_000, 20_000):
        b = synth.adversarial(n, seed=47, n_creators=1100, scale_per_million=MIX)
        assert b.n_keys > 1024 and b.n_items < 48 * b.n_keys
        check_against_oracle(verifier, b)
        assert verifier.timing()["key_path"] == 0


def test_k8_tables_many_keys_few_items(verifier):
    """200 keys with ~300 items each (above the latency rule's size, below
    K12's 8192 items per key): the K8 chord-sum tables."""
    b = synth.adversarial(60_000, seed=46, n_creators=200, scale_per_million=MIX)
    assert b.n_items > 4096 and b.n_items < 8192 * b.n_keys
    check_against_oracle(verifier, b)
    assert verifier.timing()["key_path"] == 8


def test_c4_adversarial_1m(verifier):
    """C4 exactly as SURVEY §8d specifies it: 10^6 events (seed 4, 64
    creators), the per-million corruption and malformed-key mix; every
    digest, status and accept bit equal to the C oracle's.  At 15.6k items
    per key this runs the signed-digit K12 tables (incl. digits 2^11 and the
    top-window carry at scale)."""
    b = synth.adversarial(1_000_000, seed=4)
    res = check_against_oracle(verifier, b)
    assert verifier.timing()["key_path"] == 12
    assert set(np.unique(res.status)) == {0, 1, 2, 3}


def test_k12_tables_adversarial(verifier):
    """>= 8192 items per key: 12-bit key tables (sub-table chord sums)."""
    b = synth.adversarial(120_000, seed=12, n_creators=8, scale_per_million=MIX)
    assert b.n_items >= 8192 * b.n_keys
    check_against_oracle(verifier, b)
    assert verifier.timing()["key_path"] == 12


def test_host_entry_item_order(monkeypatch):
    """bv_verify_batch verifies items chunk by chunk as their messages land
    when item_msg is non-decreasing, and after the whole transfer otherwise:
    the same batch (several 8 MB message chunks via BV_HOST_CHUNK_MB, K12
    tables, the C4 mix) in message order, shuffled, and with a run of 63
    items re-hitting an early message: every status equal to the oracle's."""
    import dataclasses

    from babble_amd.verifier import Verifier

    monkeypatch.setenv("BV_HOST_CHUNK_MB", "8")  # read at bv_create
    verifier = Verifier(device=0)
    b = synth.adversarial(120_000, seed=13, n_creators=8, scale_per_million=MIX)
    assert np.all(np.diff(b.item_msg.astype(np.int64)) >= 0)
    check_against_oracle(verifier, b)
    rng = np.random.default_rng(13)
    perm = rng.permutation(b.n_items)
    pre = None if b.pre is None else b.pre[perm]
    shuffled = dataclasses.replace(b, item_msg=b.item_msg[perm], item_key=b.item_key[perm], r_be=b.r_be[perm],
                                   s_be=b.s_be[perm], pre=pre)
    check_against_oracle(verifier, shuffled)
    late = b.item_msg.copy()
    late[-63:] = 0  # the last word's items point back at message 0: out of order
    check_against_oracle(verifier, dataclasses.replace(b, item_msg=late))
    verifier.close()


def test_host_entry_stamps_diagnostics(monkeypatch, capfd):
    """BV_HOST_STAMPS=1 (the host entry's phase stamps, the staging buffer's
    NUMA node and the per-call device timeline) prints
    its lines and changes no result: a 20k-event pageable host-entry call,
    twice, equal to the oracle."""
    from babble_amd.verifier import Verifier

    monkeypatch.setenv("BV_HOST_STAMPS", "1")  # read at bv_create
    b = synth.events(20_000, n_creators=8, seed=981)
    b.r_be[5, 31] ^= 1
    v = Verifier(device=0)
    try:
        for _ in range(2):
            res = check_against_oracle(v, b)
            assert int((res.status == 1).sum()) == b.n_items - 1
    finally:
        v.close()
    err = capfd.readouterr().err
    assert "bv_host_launch ms:" in err and "staging on NUMA node" in err
    assert "bv_host_finish ms:" in err and "device from E_CALL" in err


@pytest.mark.parametrize("qfirst", ["1", "0"])
def test_host_entry_key_part_order(monkeypatch, qfirst):
    """Host entries sum every item's k1 Q + k2 phi(Q) before its message is
    hashed (k_verify_qf over the batch, then k_verify_gf per hashed chunk;
    BV_QFIRST=0 keeps the device batches' order, u1 G first): both orders on
    K12 (8 keys, 8 MB message chunks) and K8 (200 keys) batches of the C4
    mix, ragged last word, bit-exact against the oracle."""
    from babble_amd.verifier import Verifier

    monkeypatch.setenv("BV_QFIRST", qfirst)  # read at bv_create
    monkeypatch.setenv("BV_HOST_CHUNK_MB", "8")
    verifier = Verifier(device=0)
    for n, keys, w in ((120_000 + 37, 8, 12), (60_000 + 5, 200, 8)):
        b = synth.adversarial(n, seed=15 + keys, n_creators=keys, scale_per_million=MIX)
        res = check_against_oracle(verifier, b)
        assert verifier.timing()["key_path"] == w
        assert set(np.unique(res.status)) == {0, 1, 2, 3}
    verifier.close()


def test_host_entry_single_copy_staging(verifier):
    """Host batches whose staging layout is <= 1 MB cross PCIe as one copy
    (bv_api.cpp kSmallStage): a ~0.8 MB adversarial batch in message order
    and shuffled (items verified after the whole transfer), and one just
    above the threshold (staged in pieces), all equal to the oracle."""
    import dataclasses

    b = synth.adversarial(1500, seed=71, n_creators=8, scale_per_million=MIX)
    assert b.msg_bytes.nbytes + 80 * b.n_items < (1 << 20)
    check_against_oracle(verifier, b)
    perm = np.random.default_rng(71).permutation(b.n_items)
    pre = None if b.pre is None else b.pre[perm]
    check_against_oracle(verifier, dataclasses.replace(b, item_msg=b.item_msg[perm], item_key=b.item_key[perm],
                                                       r_be=b.r_be[perm], s_be=b.s_be[perm], pre=pre))
    big = synth.adversarial(2600, seed=72, n_creators=8, scale_per_million=MIX)
    assert big.msg_bytes.nbytes > (1 << 20)
    check_against_oracle(verifier, big)


def test_throughput_variants_above_latency_threshold(verifier):
    """Batches of <= 128k items take the verify kernels' latency variants
    (zipped point ops), larger ones the throughput variants: just above the
    threshold (a ragged last word), the C4 mix, K12 tables, bit-exact."""
    b = synth.adversarial(131_072 + 64 + 5, seed=14, n_creators=8, scale_per_million=MIX)
    check_against_oracle(verifier, b)
    assert verifier.timing()["key_path"] == 12


def test_k8_tables_forced_by_flag():
    """BV_F_K8 keeps the 8-bit key tables on a batch that would take K12."""
    from babble_amd.verifier import Verifier

    v = Verifier(device=0, flags=native.F_K8)
    try:
        b = synth.adversarial(40_000, seed=13, n_creators=8, scale_per_million=MIX)
        check_against_oracle(v, b)
        assert v.timing()["key_path"] == 8
    finally:
        v.close()


def test_generic_path_few_items_per_key(verifier):
    """Keys with fewer than 8 items each take the per-lane path once the
    batch is past the latency rule (> 4096 items or > 256 keys)."""
    b = synth.adversarial(6000, seed=9, n_creators=1000, scale_per_million=MIX)
    assert 4096 < b.n_items < 8 * b.n_keys and b.n_keys <= 1024
    check_against_oracle(verifier, b)
    assert verifier.timing()["key_path"] == 0


def test_latency_rule_k8_for_small_many_key_batches(verifier):
    """A SyncResponse-sized batch from many creators (1000 events, 64 keys:
    < 16 items per key) takes per-batch K8 tables under the latency rule
    (2.6 -> 1.0 ms, profiles/r04_ab_lat_keys.log), bit-exact."""
    b = synth.adversarial(1000, seed=19, n_creators=64, scale_per_million=MIX)
    assert b.n_items < 16 * b.n_keys and b.n_keys <= 256
    check_against_oracle(verifier, b)
    assert verifier.timing()["key_path"] == 8


def test_small_batch_latency_rule_takes_k8_tables(monkeypatch):
    """With the small-batch kernel off (BV_SMALL=0), batches of <= 16 keys
    and <= 4096 items take the K8 tables even below 16 items per key (the
    per-lane generic path's 128 doublings + ~128 additions in one lane are
    the longer chain): a single event, and 40 events from 8 keys with
    adversarial items, both equal to the oracle."""
    from babble_amd.verifier import Verifier

    monkeypatch.setenv("BV_SMALL", "0")  # read at bv_create
    v = Verifier(device=0)
    try:
        b1 = synth.events(1, n_creators=1, seed=901)
        check_against_oracle(v, b1)
        assert v.timing()["key_path"] == 8
        b40 = synth.adversarial(40, seed=902, n_creators=8, scale_per_million=MIX)
        assert b40.n_keys <= 16 and b40.n_items < 16 * b40.n_keys
        check_against_oracle(v, b40)
        assert v.timing()["key_path"] == 8
    finally:
        v.close()


def test_small_batch_kernel_equals_oracle(monkeypatch):
    """k_small: a host batch of <= 256 items is one copy in,
    ONE launch (hash, s^-1, key decode, u1 G, k1 Q + k2 phi(Q) by
    wave-cooperative NAF chains on keys without a table, the decision table)
    and one copy out.  The golden items (every
    decision-table class, R = infinity, doubling cases) in chunks of <= 256
    items, a 40-item adversarial batch, single events and one BlockBody with
    100 signatures: digests, statuses and bits equal the oracle's, and equal
    the bulk pipeline's (BV_SMALL=0)."""
    from babble_amd import shard
    from babble_amd.verifier import Verifier

    verifier = Verifier(device=0)

    golden, expected, _ = golden_items_batch()
    batches = [shard.slice_batch(golden, lo, min(lo + 256, golden.n_items)) for lo in range(0, golden.n_items, 256)]
    batches += [synth.adversarial(40, seed=903, n_creators=8, scale_per_million=MIX),
                synth.events(1, n_creators=1, seed=904), synth.events(7, n_creators=3, seed=905),
                synth.blocks(1, n_validators=100, seed=906).batch]
    monkeypatch.setenv("BV_SMALL", "0")
    bulk = Verifier(device=0)
    try:
        got = []
        for b in batches:
            assert b.n_items <= 256
            res = check_against_oracle(verifier, b)
            t = verifier.timing()
            assert t["key_path"] == 0 and t["ms_total"] > 0  # the small kernel ran (no per-batch tables)
            ref = bulk.verify(b)
            assert np.array_equal(ref.status, res.status) and np.array_equal(ref.msg_hash, res.msg_hash)
            got.append(res.status)
        assert np.array_equal(np.concatenate(got[:len(got) - 4]), expected)
    finally:
        bulk.close()
        verifier.close()


def test_small_batch_host_records_equal_device_scalars(monkeypatch):
    """Latency batches (<= 4 items, or <= BV_HOST_SCALARS (16) items whose
    keys all have key-cache tables) carry host item records (hostscalar.h:
    s^-1 by one batch inversion, u1, u2 and u2's GLV split computed on the
    host with field.h's own functions, one 256-byte read per workgroup): the
    824 golden items (every
    decision-table class) in batches of 1-4 items and again in batches of
    16 / 9 / 5 / 13, single events and a 40-item adversarial batch in
    4-item slices, cold and with every valid key registered, equal to the
    oracle and, item for item, to the device-inversion path
    (BV_HOST_SCALARS=0)."""
    from babble_amd import shard
    from babble_amd.verifier import Verifier

    golden, expected, _ = golden_items_batch()
    rng = np.random.default_rng(77)
    cuts, lo = [], 0
    while lo < golden.n_items:
        hi = min(golden.n_items, lo + int(rng.integers(1, 5)))
        cuts.append((lo, hi))
        lo = hi
    batches = [shard.slice_batch(golden, a, c) for a, c in cuts]
    n_golden = len(batches)
    lo, k = 0, 0
    while lo < golden.n_items:  # larger batches: records when warm (every key cached), else the device
        hi = min(golden.n_items, lo + (16, 9, 5, 13)[k % 4])
        batches.append(shard.slice_batch(golden, lo, hi))
        lo, k = hi, k + 1
    batches += [synth.events(1, n_creators=1, seed=960 + i) for i in range(4)]
    adv = synth.adversarial(40, seed=970, n_creators=3, scale_per_million=MIX)
    batches += [shard.slice_batch(adv, lo, lo + 4) for lo in range(0, 40, 4)]
    good = []
    for b in batches:
        for k in range(b.n_keys):
            if gs.Unmarshal(b.key(k)) is not None and b.key(k) not in good:
                good.append(b.key(k))
    for flags in (0, native.F_KEY_CACHE):
        rec = Verifier(device=0, flags=flags)
        monkeypatch.setenv("BV_HOST_SCALARS", "0")  # read at bv_create
        dev = Verifier(device=0, flags=flags)
        monkeypatch.delenv("BV_HOST_SCALARS")
        try:
            if flags:
                rec.register_keys(good)  # every valid key: the 5-16-item batches take records too
                dev.register_keys(good)
            got = []
            for b in batches:
                r = check_against_oracle(rec, b)
                d = dev.verify(b)
                assert np.array_equal(d.status, r.status) and np.array_equal(d.msg_hash, r.msg_hash)
                got.append(r.status)
            assert np.array_equal(np.concatenate(got[:n_golden]), expected)
        finally:
            rec.close()
            dev.close()


def test_small_batch_kernel_warm_up_to_1024(monkeypatch):
    """A 1000-event batch whose keys all have key-cache tables takes k_small
    (no per-item NAF chain: BV_SMALL_WARM_MAX, 1024, above the cold limit
    BV_SMALL_MAX, 256); the same batch through the bulk pipeline (limits
    256).  Both equal to the oracle, corrupted signatures included."""
    from babble_amd.verifier import Verifier

    b = synth.events(1000, n_creators=6, seed=911)
    b.r_be[7, 31] ^= 1
    b.s_be[300, 0] ^= 0x40
    keys = [b.key(k) for k in range(b.n_keys)]
    for limit, small in (("1024", True), ("256", False)):
        monkeypatch.setenv("BV_SMALL_WARM_MAX", limit)  # read at bv_create
        monkeypatch.setenv("BV_SMALL_MAX", "256")
        v = Verifier(device=0, flags=native.F_KEY_CACHE)
        try:
            v.register_keys(keys)
            res = check_against_oracle(v, b)
            t = v.timing()
            assert t["key_path"] == 22 and (t["ms_sha256"] == 0) == small  # k_small has no separate hashing span
            assert int((res.status == 1).sum()) == 998
        finally:
            v.close()


def test_small_batch_first_call_in_fresh_processes():
    """The first k_small batch of a process (cold instruction and
    translation caches), in fresh child processes: 256 valid single-creator
    events (the cold k_small limit), every status equal to the oracle and
    the batch on k_small's cold path (key_path 0).  Round 5's right-to-left
    cold path gave a false REJECT on such first batches in ~1 process of 6
    (tools/dbg_first_call.py, profiles/r05_small_r2l_investigation.log)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CHILD="1", MODE="cold")
    for _ in range(6):
        r = subprocess.run([sys.executable, os.path.join(root, "tools", "dbg_first_call.py")], env=env,
                           capture_output=True, text=True, timeout=120)
        line = [x for x in r.stdout.splitlines() if x.startswith("result")]
        assert r.returncode == 0 and line, r.stderr[-2000:]
        assert line[-1].endswith("mismatches 0") and "key_path 0 " in line[-1], line[-1]


def test_small_batch_randomized_against_oracle():
    """k_small over randomized small adversarial batches (1..500 items, 1..9
    creators, the C4 mix of malformed keys and signatures), cold and with
    part of the valid keys registered (cached and uncached keys in one
    launch; batches above 256 items take k_small only when every key is
    cached): every status, digest and bit equal to the C oracle."""
    from babble_amd.verifier import Verifier

    rng = np.random.default_rng(2024)
    cold = Verifier(device=0)
    warm = Verifier(device=0, flags=native.F_KEY_CACHE)
    try:
        for it in range(14):
            n = int(rng.integers(1, 500))
            b = synth.adversarial(n, seed=3000 + it, n_creators=int(rng.integers(1, 10)), scale_per_million=MIX)
            good = sorted({b.key(k) for k in range(b.n_keys) if gs.Unmarshal(b.key(k)) is not None})
            warm.register_keys(good[: max(1, len(good) // 2)] if it % 2 else good)
            check_against_oracle(cold, b)
            check_against_oracle(warm, b)
    finally:
        cold.close()
        warm.close()


def test_small_batch_cold_path_many_batches():
    """The cold k_small path (no key-cache table: wave 2 doubles Q while
    waves 1 and 3 add the NAF digits of k1 / k2 in barrier-separated phases,
    kernels.hip SmallCold) over 48 batches of up to 256 valid events from 1-4
    creators with one corrupted signature each, in one process: ~12k items,
    every status and digest equal to the C oracle.  Each batch runs twice on
    the same context (the same statuses both times)."""
    from babble_amd.verifier import Verifier

    rng = np.random.default_rng(66)
    v = Verifier(device=0)
    try:
        for it in range(48):
            n = int(rng.integers(200, 257))
            b = synth.events(n, n_creators=int(rng.integers(1, 5)), seed=5000 + it)
            b.s_be[int(rng.integers(0, n)), 31] ^= 1
            res = check_against_oracle(v, b)
            assert v.timing()["key_path"] == 0
            assert int((res.status == 1).sum()) == n - 1
            again = v.verify(b)
            assert np.array_equal(again.status, res.status)
    finally:
        v.close()


def test_small_batch_kernel_key_cache(monkeypatch):
    """k_small with registered keys: every valid key registered -> the KC
    tables (6 lookups per GLV half; malformed keys need none); some keys
    registered -> cached and uncached keys (cooperative NAF chains) in one
    launch.  All equal to the oracle."""
    from babble_amd.verifier import Verifier

    b = synth.adversarial(200, seed=907, n_creators=6, scale_per_million=MIX)
    good = sorted({b.key(k) for k in range(b.n_keys) if gs.Unmarshal(b.key(k)) is not None})

    v = Verifier(device=0, flags=native.F_KEY_CACHE)
    try:
        v.register_keys(good)
        check_against_oracle(v, b)
        t = v.timing()
        # k_small (one launch that reads its inputs from host memory in
        # place: no staging copy, so no h2d span) with the cached tables
        assert t["key_path"] == 22 and t["kc_hits"] == len(good) and t["ms_h2d"] == 0 and t["ms_total"] > 0
        fresh = synth.events(30, n_creators=2, seed=908)  # unregistered: no table, the NAF chains
        check_against_oracle(v, fresh)
        assert v.timing()["key_path"] == 0
    finally:
        v.close()
    v = Verifier(device=0, flags=native.F_KEY_CACHE)
    try:
        v.register_keys(good[:3])
        check_against_oracle(v, b)
        t = v.timing()
        assert t["key_path"] == 22 and t["kc_hits"] == 3
    finally:
        v.close()


def test_c5_blocks_check_block(verifier):
    wb = synth.blocks(200, n_validators=100, seed=5)
    b = wb.batch
    rng = np.random.default_rng(5)
    bad = rng.choice(b.n_items, size=b.n_items // 20, replace=False)
    b.s_be[bad, 7] ^= 0x40
    res = check_against_oracle(verifier, b)
    valid = res.status.reshape(wb.n_blocks, wb.n_validators).astype(bool).sum(axis=1)
    tc = gs.trust_count(wb.n_validators)
    assert np.all(valid > tc)
    assert int(valid.sum()) == b.n_items - len(bad)


def test_edge_sizes(verifier):
    for n in (1, 63, 64, 65, 127, 129):
        b = synth.events(n, n_creators=2, seed=n)
        res = check_against_oracle(verifier, b)
        assert len(res.accept_bits) == (n + 63) // 64


def test_empty_batch(verifier):
    b = BatchBuilder().pack()
    res = verifier.verify(b)
    assert res.status.size == 0 and res.msg_hash.size == 0


def test_messages_without_items(verifier):
    bb = BatchBuilder()
    for n in (0, 5, 64, 200):
        bb.add_msg(os.urandom(n))
    res = verifier.verify(bb.pack())
    assert [res.msg_hash[i].tobytes() for i in range(4)] == [hashlib.sha256(bb._msgs[i]).digest() for i in range(4)]


def test_bad_index_rejected(verifier):
    b = synth.events(10, n_creators=2, seed=3)
    b.item_key[3] = 99
    with pytest.raises(native.BvError):
        verifier.verify(b)


def test_full_size_properties(verifier):
    """BASELINE size (1M events): every valid signature accepted, digests of a
    sample equal hashlib, a seeded corrupted subset rejected exactly, and ALL
    1M digests, statuses and accept bits equal the C oracle's (VERDICT r2
    weak #1: no longer a 3,000-item sample)."""
    b = synth.events(1_000_000, n_creators=64, seed=2)
    d = verifier.to_device(b)
    verifier.verify_device(d)
    res = d.result()
    assert np.all(res.status == 1)
    assert np.all(res.accept_bits == np.uint64(0xFFFFFFFFFFFFFFFF))
    for i in np.random.default_rng(0).choice(b.n_items, 50, replace=False):
        assert res.msg_hash[i].tobytes() == hashlib.sha256(b.message(int(i))).digest()
    rng = np.random.default_rng(11)
    bad = np.sort(rng.choice(b.n_items, 997, replace=False))
    b.r_be[bad, 17] ^= 0x10
    res2 = verifier.verify(b)
    assert np.array_equal(np.flatnonzero(res2.status != 1), bad)
    h, st, bits = coracle.verify_batch(b.as_dict())
    assert np.array_equal(res2.msg_hash, h)
    assert np.array_equal(res2.status, st)
    assert np.array_equal(res2.accept_bits, bits)


def test_reentrant_contexts():
    from babble_amd.verifier import Verifier

    b = synth.adversarial(3000, seed=31, n_creators=8, scale_per_million=MIX)
    _, st, _ = coracle.verify_batch(b.as_dict())
    out = {}

    def run(k):
        v = Verifier(0)
        for _ in range(3):
            out[k] = v.verify(b).status.copy()
        v.close()

    th = [threading.Thread(target=run, args=(k,)) for k in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for k in range(3):
        assert np.array_equal(out[k], st)


def test_shared_context_threads(verifier):
    b = synth.events(5000, n_creators=8, seed=12)
    errs = []

    def run():
        try:
            for _ in range(3):
                assert np.all(verifier.verify(b).status == 1)
        except Exception as e:  # pragma: no cover
            errs.append(e)

    th = [threading.Thread(target=run) for _ in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs


def test_native_library_is_the_one_loaded():
    maps = open("/proc/self/maps").read()
    assert native.LIB_PATH in maps


def test_bench_gpus_beyond_the_box_fails():
    """`bench.py --gpus N` with fewer than N GPUs exits
    non-zero without printing a line (it used to print a one-GPU line)."""
    import subprocess
    import sys

    import torch

    n = torch.cuda.device_count() + 1
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(n), "--steps", "1",
                        "--warmup", "0", "--events", "4096", "--no-cpu", "--no-extras"], env=env,
                       capture_output=True, text=True, timeout=180)
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_long_messages_hashed_on_host(verifier):
    """Host entry: messages longer than 16 KB (e.g. a Frame's JSON) are hashed
    on the host (SHA extensions) beside the device's hashing of the rest, and
    their digests put in place before the verify kernels: a batch mixing
    C2 bodies with 16 KB + 1, 20 KB and 100 KB messages (some signed, some
    item-less), in order and shuffled — digests, statuses and bits equal the
    oracle's."""
    import dataclasses

    from babble_amd.batch import PackedBatch

    b = synth.adversarial(3000, seed=31, n_creators=8, scale_per_million=MIX)
    rng = np.random.default_rng(31)
    msgs = [b.message(m) for m in range(b.n_msgs)]
    for pos_, size in ((5, 16 * 1024 + 1), (700, 20_000), (2999, 100_000), (1500, 64)):
        msgs[pos_] = rng.integers(0, 256, size, dtype=np.uint8).tobytes()  # signatures over them now fail
    msgs += [rng.integers(0, 256, 50_000, dtype=np.uint8).tobytes()]  # an item-less long message
    off = np.zeros(len(msgs) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in msgs])
    lb = PackedBatch(np.frombuffer(b"".join(msgs), np.uint8).copy(), off, b.key_bytes, b.key_off, b.item_msg,
                     b.item_key, b.r_be, b.s_be, b.pre)
    res = check_against_oracle(verifier, lb)
    assert res.msg_hash[-1].tobytes() == hashlib.sha256(msgs[-1]).digest()
    perm = rng.permutation(lb.n_items)
    check_against_oracle(verifier, dataclasses.replace(lb, item_msg=lb.item_msg[perm], item_key=lb.item_key[perm],
                                                       r_be=lb.r_be[perm], s_be=lb.s_be[perm], pre=lb.pre[perm]))
