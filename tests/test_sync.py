"""core.sync as one batch (babble_amd/sync.py): the
level-scheduled ReadWireInfo rebuilds exactly the bodies the sequential Go
loop (core.go:210-271 + hashgraph.go:1538-1595) would, and the batch verify
decisions equal the oracle's Event.Verify.

The generator below IS the sequential restatement: it walks the
SyncResponse in order, resolving parents through a store that gains each
event's hash as it is "inserted", and signs each body with the oracle."""
import hashlib
import random

import pytest

from babble_amd import hashgraph as H
from babble_amd import sync as S
from oracle import gosemantics as gs
from tests.test_mirror import Signer


class HashlibStub:
    """Test-only stand-in for the device SHA-256 (CPU tests of the level
    scheduling); the product path uses the Verifier."""
    calls = 0

    def sha256(self, msgs):
        HashlibStub.calls += 1
        return [hashlib.sha256(bytes(m)).digest() for m in msgs]


def make_sync(seed=1, n=120, n_peers=4, corrupt=(), bad_creator_at=None, bad_parent_at=None):
    sg = Signer(seed)
    rng = sg.rng
    keys = [sg.key() for _ in range(n_peers)]
    rep = {i: H.Peer("10.0.0.%d:1337" % i, gs.EncodeToString(k[1]), "node%d" % i) for i, k in enumerate(keys)}
    pk = {i: rep[i].PubKeyString() for i in rep}
    store0 = {}
    last = {}
    for c in range(n_peers):  # events already in the store before the sync
        pre = rng.randrange(0, 4)
        for idx in range(pre):
            store0[(pk[c], idx)] = gs.EncodeToString(rng.randbytes(32))
        last[c] = pre - 1
    store = dict(store0)
    wevents, bodies = [], []
    for t in range(n):
        c = rng.randrange(n_peers)
        index = last[c] + 1
        others = [o for o in range(n_peers) if o != c and last[o] >= 0]
        if others and rng.random() < 0.9:
            o = rng.choice(others)
            opi = rng.randint(max(0, last[o] - 2), last[o])
        else:
            o, opi = 0, -1
        if bad_parent_at == t:
            o, opi = (c + 1) % n_peers, last[(c + 1) % n_peers] + 5
        wb = S.WireBody(Transactions=[rng.randbytes(rng.randrange(1, 80)) for _ in range(rng.randrange(3))] or None,
                        CreatorID=c if bad_creator_at != t else 99, OtherParentCreatorID=o, Index=index,
                        SelfParentIndex=index - 1, OtherParentIndex=opi, Timestamp=1_600_000_000 + t)
        if t % 9 == 4:
            wb.BlockSignatures = [S.WireBlockSignature(Index=3, Signature="abc|def")]
        parents = [store.get((pk[c], index - 1), "") if index > 0 else "",
                   store.get((pk[o], opi), "") if opi >= 0 else ""]
        body = gs.EventBody(Transactions=wb.Transactions, Parents=parents, Creator=keys[c][1], Index=index,
                            BlockSignatures=[gs.BlockSignature(keys[c][1], 3, "abc|def")] if wb.BlockSignatures
                            else None, Timestamp=wb.Timestamp)
        sig = sg.sign(keys[c][0], body.Hash())
        if t in corrupt:
            r, s = sig.split("|")
            sig = r + "|" + gs.go_big_text36(int(gs.go_big_setstring36(s)) ^ 2)
        wevents.append(S.WireEvent(Body=wb, Signature=sig))
        bodies.append((body, sig))
        store[(pk[c], index)] = gs.EncodeToString(body.Hash())
        last[c] = index
    return wevents, bodies, rep, (lambda p, i: store0.get((p, i)))


def test_read_wire_batch_rebuilds_sequential_bodies():
    wevents, bodies, rep, pe = make_sync(seed=3, n=150)
    HashlibStub.calls = 0
    reads, levels = S.read_wire_batch(wevents, rep, pe, verifier=HashlibStub())
    assert all(r.err is None and r.event is not None for r in reads)
    for r, (b, _) in zip(reads, bodies):
        assert r.event.Body.Marshal() == b.Marshal()
    assert max(levels) >= 5                     # a real in-batch dependency chain
    assert HashlibStub.calls <= max(levels)     # one hash batch per level (leaves skipped)


def test_read_wire_batch_stops_at_first_error():
    wevents, bodies, rep, pe = make_sync(seed=4, n=40, bad_creator_at=17)
    reads, levels = S.read_wire_batch(wevents, rep, pe, verifier=HashlibStub())
    assert reads[17].err == "Creator 99 not found"
    assert all(r.event is None and r.err is None for r in reads[18:]) and levels[18:] == [-1] * 22
    for r, (b, _) in zip(reads[:17], bodies):
        assert r.event.Body.Marshal() == b.Marshal()
    wevents, _, rep, pe = make_sync(seed=5, n=30, bad_parent_at=20)
    reads, _ = S.read_wire_batch(wevents, rep, pe, verifier=HashlibStub())
    assert reads[20].err.startswith("OtherParent (creator:")


def test_genesis_parents_and_nil_block_signatures():
    wevents, bodies, rep, pe = make_sync(seed=6, n=12)
    reads, _ = S.read_wire_batch(wevents, rep, pe, verifier=HashlibStub())
    first = {}
    for we, r in zip(wevents, reads):
        if we.Body.Index == 0:
            assert r.event.Body.Parents[0] == ""
        if we.Body.BlockSignatures is None:
            assert r.event.Body.BlockSignatures is None   # nil stays null in the JSON
        first.setdefault(we.Body.CreatorID, r)


@pytest.mark.gpu
def test_sync_verify_matches_oracle():
    corrupt = {7, 33, 90}
    wevents, bodies, rep, pe = make_sync(seed=7, n=160, corrupt=corrupt)
    events, outcomes, read_err = S.sync_verify(wevents, rep, pe)
    assert read_err is None and len(events) == len(wevents)
    for t, (ev, o, (b, sig)) in enumerate(zip(events, outcomes, bodies)):
        want = gs.event_status(b, sig)
        assert o.ok == (want == gs.EV_ACCEPT) and o.ok == (t not in corrupt), (t, want, o)
        assert ev.Hash() == b.Hash()


@pytest.mark.gpu
def test_sync_verify_read_error_prefix():
    wevents, bodies, rep, pe = make_sync(seed=8, n=50, bad_creator_at=30)
    events, outcomes, read_err = S.sync_verify(wevents, rep, pe)
    assert read_err == "Creator 99 not found" and len(events) == 30
    assert all(o.ok for o in outcomes)


def test_self_parent_store_error_text_passes_through():
    """ReadWireInfo returns the store's error unchanged for a missing
    self-parent (hashgraph.go:1556-1559): common.StoreErr text
    "<dataType>, <key>, <kind>" (store_errors.go:46-63); a TooLate stands
    even if the index is in the batch, a KeyNotFound can be satisfied by an
    event inserted earlier in the same sync."""
    wevents, bodies, rep, pe = make_sync(seed=9, n=40)
    # the 12th event's self-parent: make the pre-sync store report TooLate
    t = next(i for i, we in enumerate(wevents) if we.Body.SelfParentIndex >= 0 and i > 10)
    we = wevents[t]
    cpk = rep[we.Body.CreatorID].PubKeyString()

    def pe_late(p, i):
        if p == cpk and i == we.Body.SelfParentIndex:
            return S.StoreError("ParticipantEvents[%d]" % we.Body.CreatorID, S.StoreError.TOO_LATE, str(i))
        return pe(p, i)

    reads, _ = S.read_wire_batch(wevents, rep, pe_late, verifier=HashlibStub())
    assert reads[t].err == "ParticipantEvents[%d], %d, Too Late" % (we.Body.CreatorID, we.Body.SelfParentIndex)
    assert all(r.err is None for r in reads[:t])
    # an explicit KeyNotFound (or None) for an in-batch self-parent is resolved in the batch
    reads, _ = S.read_wire_batch(wevents, rep, lambda p, i: pe(p, i) or S.StoreError(
        "ParticipantEvents[0]", S.StoreError.KEY_NOT_FOUND, str(i)), verifier=HashlibStub())
    assert all(r.err is None for r in reads)


def test_missing_self_parent_not_found_text():
    wevents, bodies, rep, pe = make_sync(seed=10, n=30)
    t = next(i for i, we in enumerate(wevents) if we.Body.SelfParentIndex >= 0)
    we = wevents[t]
    cpk = rep[we.Body.CreatorID].PubKeyString()
    we.Body.SelfParentIndex += 1000  # nowhere: not in the store, not in the batch
    reads, _ = S.read_wire_batch(wevents, rep, pe, verifier=HashlibStub())
    assert reads[t].err == "ParticipantEvents, %d, Not Found" % we.Body.SelfParentIndex
    del cpk


@pytest.mark.gpu
@pytest.mark.parametrize("bad", [None, 33])
def test_sync_verify_device_equals_host_path(bad):
    """sync_verify_device (one bv_verify_events call: the library builds the
    bodies from wire fields and, for this in-batch DAG, hashes them on the
    host in topological order with SHA-NI while the device decodes keys and
    inverts s; the device then verifies) == sync_verify (the mirror's host
    bodies, per-level hashing): same bodies, digests, outcomes and first read
    error."""
    import time

    from babble_amd.verifier import Verifier

    corrupt = {5, 64, 100}
    wevents, bodies, rep, pe = make_sync(seed=17, n=160, corrupt=corrupt, bad_creator_at=bad)
    v = Verifier(0)
    try:
        t0 = time.perf_counter()
        ev_h, out_h, err_h = S.sync_verify(wevents, rep, pe, v)
        t1 = time.perf_counter()
        ev_d, out_d, err_d = S.sync_verify_device(wevents, rep, pe, v)
        t2 = time.perf_counter()
        print(f"host-level path {1e3 * (t1 - t0):.1f} ms, device path {1e3 * (t2 - t1):.1f} ms")
        assert err_h == err_d and len(ev_h) == len(ev_d)
        for a, b, (body, _) in zip(ev_h, ev_d, bodies):
            assert a.Body.Marshal() == b.Body.Marshal() == body.Marshal()
            assert a.Hash() == b.Hash() == body.Hash()
        assert [(o.ok, o.err, o.panic) for o in out_h] == [(o.ok, o.err, o.panic) for o in out_d]
        assert [t for t, o in enumerate(out_d) if not o.ok] == sorted(c for c in corrupt if c < len(out_d))
    finally:
        v.close()
