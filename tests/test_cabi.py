"""The cgo shim's call sequence replayed through
the C ABI by a C harness (tests/cabi/shim_harness.c): the process context
with the key cache, bv_kc_register from core.setPeers, batch builders whose
pinned arenas (bv_arena_*) are reused across calls, bv_verify_events for a
SyncResponse after ReadWireBatch and bv_verify_batch for one event.

CPU: the harness builds, exports its entry points and encodes signatures as
keys.EncodeSignature (the oracle's restatement).  GPU: every digest and
status against the C oracle."""
import subprocess

import numpy as np
import pytest

from babble_amd import synth
from oracle import gosemantics as gs
from tests.cabi import harness


def test_harness_exports():
    out = subprocess.run(["nm", "-D", "--defined-only", harness.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    names = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert {"shim_open", "shim_close", "shim_set_peers", "shim_sync", "shim_verify_event",
            "shim_encode_signatures"} <= names
    # it calls the library only through the C ABI (no HIP symbol of its own)
    und = subprocess.run(["nm", "-D", "--undefined-only", harness.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    assert not [x for x in und.split() if x.startswith("hip")]
    assert "bv_arena_reserve" in und and "bv_verify_events" in und and "bv_kc_register" in und


def test_encode_signatures_equals_go_text():
    rng = np.random.default_rng(5)
    r = rng.integers(0, 256, (200, 32), dtype=np.uint8)
    s = rng.integers(0, 256, (200, 32), dtype=np.uint8)
    r[0] = 0
    s[1, :31] = 0
    text, off = harness.encode_signatures(r, s)
    for i in range(200):
        want = gs.EncodeSignature(int.from_bytes(r[i].tobytes(), "big"), int.from_bytes(s[i].tobytes(), "big"))
        assert harness.signature_text(text, off, i) == want.encode(), i


def _oracle(packed):
    from oracle import coracle

    return coracle.verify_batch(packed.as_dict())


@pytest.mark.gpu
def test_shim_sync_and_single_event_against_oracle():
    """The shim path end to end: peers registered, a 1000-event SyncResponse
    whose parents are earlier events of the response (in-batch DAG), a
    20k-event replay whose parents are store hashes (bulk), each twice on the
    pooled arenas (the second call reuses them), 1% corrupted signatures;
    then single events (addSelfEvent) through bv_verify_batch, valid and
    corrupted.  Digests and statuses equal the oracle's."""
    sh = harness.Shim(device=0)
    try:
        dag_packed, dag = synth.event_fields(1000, n_creators=4, seed=71, parents="event")
        sh.set_peers([dag_packed.key(k) for k in range(dag_packed.n_keys)])
        for packed, wire in ((dag_packed, dag), synth.event_fields(20_000, n_creators=8, seed=72, parents="hash")):
            n = packed.n_items
            rng = np.random.default_rng(n)
            bad = rng.choice(n, max(1, n // 100), replace=False)
            wire.s_be = np.asarray(wire.s_be).copy()
            wire.s_be[bad, 9] ^= 4
            packed.s_be[bad, 9] ^= 4
            h, st, _ = _oracle(packed)
            sw, keep = sh.wire(wire)
            for rep in range(2):
                dig, got, ms = sh.sync(sw)
                assert ms > 0
                assert np.array_equal(dig, h), (n, rep)
                assert np.array_equal(got, st), (n, rep, np.flatnonzero(got != st)[:8])
            assert int((st != 1).sum()) >= len(bad) // 2
        one_packed, one = synth.event_fields(3, n_creators=1, seed=73, parents="hash")
        text, off = harness.encode_signatures(one.r_be, one.s_be)
        h, st, _ = _oracle(one_packed)
        for i in range(3):
            d, s, ms = sh.verify_event(one_packed.message(i), one_packed.key(0), harness.signature_text(text, off, i))
            assert d == h[i].tobytes() and s == st[i] == 1, i
        good = harness.signature_text(text, off, 0)
        bad_sig = good[:-1] + (b"1" if good.endswith(b"0") else b"0")
        _, s, _ = sh.verify_event(one_packed.message(0), one_packed.key(0), bad_sig)
        assert s == 0
        _, s, _ = sh.verify_event(one_packed.message(0), one_packed.key(0), b"only-one-part")
        assert s == 2  # DecodeSignature's error
    finally:
        sh.close()


@pytest.mark.gpu
def test_arena_reserve_keeps_contents_and_reuses_blocks():
    """bv_arena_reserve: growth keeps the first `keep` bytes and at least
    doubles; a reserve within the capacity returns the same block; bad
    slots and keeps are BV_E_ARGS."""
    import ctypes

    from babble_amd import native

    L = native.lib()
    a = ctypes.c_void_p()
    assert L.bv_arena_create(ctypes.byref(a)) == 0
    try:
        p, cap = ctypes.c_void_p(), ctypes.c_size_t()
        assert L.bv_arena_reserve(a, 3, 100, 0, ctypes.byref(p), ctypes.byref(cap)) == 0 and cap.value == 100
        ctypes.memmove(p, bytes(range(100)), 100)
        first = p.value
        assert L.bv_arena_reserve(a, 3, 80, 100, ctypes.byref(p), ctypes.byref(cap)) == 0 and p.value == first
        assert L.bv_arena_reserve(a, 3, 150, 100, ctypes.byref(p), ctypes.byref(cap)) == 0
        assert cap.value == 200 and ctypes.string_at(p, 100) == bytes(range(100))
        assert L.bv_arena_reserve(a, 3, 10, 300, ctypes.byref(p), None) == native.BV_E_ARGS  # keep > capacity
        assert L.bv_arena_reserve(a, native.ARENA_SLOTS, 10, 0, ctypes.byref(p), None) == native.BV_E_ARGS
    finally:
        L.bv_arena_destroy(a)
