"""bv_verify_events: canonical EventBody JSON built from wire fields
(babble_amd/csrc/evjson.h) and in-batch DAG hashing.

CPU: the device's per-event code run by the host emulator equals Go
encoding/json as restated by the oracle (oracle/gosemantics.py EventBody,
event.go:38-45) on the synthetic hashgraph and on random edge cases (nil
and empty transaction lists, nil transactions, ITX / BlockSignature
fragments, negative Index / Timestamp, HASH / EVENT / no parents, odd key
lengths), digests included.  GPU: the same through the C ABI, with the
signatures verified, against the oracle.
"""
import hashlib
import random

import numpy as np
import pytest

from babble_amd import events as E
from babble_amd import synth
from oracle import gosemantics as gs
from tests.emu import emu


def random_wire(seed, n=300, in_batch=True):
    """(EventWireBatch, oracle EventBodies, signatures as (pre, r, s)):
    parents reference earlier events of the batch (unless not `in_batch`)
    or known hashes."""
    rng = random.Random(seed)
    b = E.EventBatchBuilder()
    keys = [bytes(rng.getrandbits(8) for _ in range(rng.choice([65, 65, 65, 33, 0, 70]))) for _ in range(5)]
    kidx = [b.add_key(k) for k in keys]
    bodies, digests = [], []
    for e in range(n):
        c = rng.randrange(len(keys))
        parents, pstr = [], []
        for _ in range(2):
            r = rng.random()
            if r < 0.2 or e == 0:
                parents.append(None)
                pstr.append("")
            elif r < 0.5 or not in_batch:
                h = bytes(rng.getrandbits(8) for _ in range(32))
                parents.append(("hash", h))
                pstr.append(gs.EncodeToString(h))
            else:
                j = rng.randrange(max(0, e - 8), e)
                parents.append(("event", j))
                pstr.append(gs.EncodeToString(digests[j]))
        r = rng.random()
        txs = None if r < 0.15 else ([] if r < 0.25 else [
            None if rng.random() < 0.1 else bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 80)))
            for _ in range(rng.randrange(1, 4))])
        itxs = None
        if rng.random() < 0.1:
            itxs = [gs.InternalTransaction(gs.InternalTransactionBody(rng.randrange(2), gs.Peer(
                "h:%d" % e, "0X04AB", "<m&>")), "r|s")]
        bsigs = None
        if rng.random() < 0.1:
            bsigs = [gs.BlockSignature(keys[c], rng.randrange(9), "a| b")] if rng.random() < 0.5 else []
        idx = rng.choice([0, 1, 7, -5, 2**62, -(2**63)])
        ts = rng.choice([0, 1600000000 + e, -1, 2**63 - 1])
        body = gs.EventBody(Transactions=txs, InternalTransactions=itxs, Parents=pstr, Creator=keys[c], Index=idx,
                            BlockSignatures=bsigs, Timestamp=ts)
        raw = body.Marshal()
        b.add_event(kidx[c], idx, ts, parents, txs, (0, b"\1" * 32, b"\2" * 32),
                    itx_json=frag_json(itxs), bsig_json=frag_json(bsigs))
        bodies.append(raw)
        digests.append(hashlib.sha256(raw).digest())
    return b.pack(), bodies, digests


def frag_json(xs):
    """encoding/json of a slice of ITX / BlockSignature (b"" = nil)."""
    if xs is None:
        return b""
    return gs.json_list(xs, lambda t: t.json())


@pytest.mark.parametrize("parents", ["event", "hash"])
def test_emu_bodies_equal_synth_hashgraph(parents):
    packed, wire = synth.event_fields(600, n_creators=5, seed=7, parents=parents)
    bodies, dig = emu.ev_bodies(wire)
    for i in range(packed.n_items):
        assert bodies[i] == packed.message(i), i
        assert dig[i].tobytes() == hashlib.sha256(bodies[i]).digest()


def test_emu_bodies_equal_oracle_edge_cases():
    for seed in (1, 2, 3):
        wire, want, wd = random_wire(seed)
        bodies, dig = emu.ev_bodies(wire)
        assert bodies == want
        assert [d.tobytes() for d in dig] == wd


def test_emu_streaming_body_hash_equals_hashlib():
    """k_ev_body_hash's streaming serialise-and-hash (no body in memory), run
    by the emulator: equal to hashlib over the oracle's bodies for batches
    without in-batch parents, over bodies of every length mod 64 (the
    padding's block-boundary cases) and the edge cases of random_wire."""
    seen = set()
    for seed in (4, 5, 6, 7):
        wire, want, wd = random_wire(seed, n=160, in_batch=False)
        assert emu.ev_body_hash(wire).tolist() == [list(d) for d in wd]
        seen |= {len(x) % 64 for x in want}
    assert len(seen) == 64
    packed, wire = synth.event_fields(300, n_creators=5, seed=8, parents="hash")
    dig = emu.ev_body_hash(wire)
    for i in range(packed.n_items):
        assert dig[i].tobytes() == hashlib.sha256(packed.message(i)).digest(), i


def test_no_transactions_and_wire_bytes():
    packed, wire = synth.event_fields(50, n_creators=3, seed=9, n_tx=0)
    bodies, _ = emu.ev_bodies(wire)
    assert bodies == [packed.message(i) for i in range(50)]
    assert b'"Transactions":null' in bodies[0]
    # the wire form is much smaller than the serialized bodies
    p2, w2 = synth.event_fields(1000, n_creators=4, seed=3)
    assert E.wire_bytes(w2) * 2 < p2.msg_bytes.nbytes + p2.r_be.nbytes + p2.s_be.nbytes


@pytest.mark.gpu
@pytest.mark.parametrize("parents,n", [("event", 2000), ("hash", 200_000)])
def test_verify_events_matches_oracle(parents, n):
    from babble_amd.verifier import Verifier
    from oracle import coracle

    packed, wire = synth.event_fields(n, n_creators=8, seed=11, parents=parents)
    rng = np.random.default_rng(3)
    bad = rng.choice(n, size=max(1, n // 100), replace=False)
    wire.s_be[bad, 5] ^= 0x20
    packed.s_be[bad, 5] ^= 0x20
    v = Verifier(0)
    try:
        res = v.verify_events(wire)
        h, st, bits = coracle.verify_batch(packed.as_dict())
        assert np.array_equal(res.msg_hash, h)
        assert np.array_equal(res.status, st) and np.array_equal(res.accept_bits, bits)
        assert int((st != 1).sum()) == len(bad)
    finally:
        v.close()


@pytest.mark.gpu
def test_verify_events_edge_cases_digests():
    from babble_amd.verifier import Verifier

    v = Verifier(0)
    try:
        for seed in (4, 5):
            wire, want, wd = random_wire(seed, n=500)
            res = v.verify_events(wire)
            assert [d.tobytes() for d in res.msg_hash] == wd
    finally:
        v.close()


@pytest.mark.gpu
def test_verify_events_chunk_boundaries(monkeypatch):
    """Bulk batches (no in-batch parents) stage their per-event fields in
    event chunks (bv_events.cpp); a tiny chunk size puts chunk boundaries
    through nil / empty transaction lists, nil transactions and ITX /
    BlockSignature fragments.  Digests, statuses and bits equal the C
    oracle's over the oracle-serialized bodies (no
    longer compared with a one-chunk run of the same kernels); a signed
    C2-shaped batch with corrupted signatures crosses chunks the same way."""
    from babble_amd.batch import PackedBatch
    from babble_amd.verifier import Verifier
    from oracle import coracle

    monkeypatch.setenv("BV_EV_CHUNK_MB", "0.001")  # 256-event chunks (read at bv_create)
    v = Verifier(0)
    try:
        for seed in (6, 7):
            wire, bodies, wd = random_wire(seed, n=1100, in_batch=False)
            many = v.verify_events(wire)
            assert [d.tobytes() for d in many.msg_hash] == wd
            n = wire.n_events
            off = np.zeros(n + 1, np.uint64)
            off[1:] = np.cumsum([len(x) for x in bodies])
            packed = PackedBatch(np.frombuffer(b"".join(bodies), np.uint8).copy(), off, wire.key_bytes,
                                 wire.key_off, np.arange(n, dtype=np.uint32), wire.creator.astype(np.uint32),
                                 wire.r_be, wire.s_be,
                                 wire.pre if wire.pre is not None else np.zeros(n, np.uint8))
            h, st, bits = coracle.verify_batch(packed.as_dict())
            assert np.array_equal(many.status, st) and np.array_equal(many.accept_bits, bits)
        packed, wire = synth.event_fields(3000, n_creators=8, seed=19, parents="hash")
        bad = np.random.default_rng(19).choice(3000, 40, replace=False)
        wire.s_be[bad, 3] ^= 0x08
        packed.s_be[bad, 3] ^= 0x08
        res = v.verify_events(wire)
        h, st, bits = coracle.verify_batch(packed.as_dict())
        assert np.array_equal(res.msg_hash, h)
        assert np.array_equal(res.status, st) and np.array_equal(res.accept_bits, bits)
        assert int((st != 1).sum()) == len(bad)
    finally:
        v.close()


@pytest.mark.gpu
def test_verify_events_sync_sized_dag_depth():
    """A SyncLimit-sized batch (config.go:44) from 4 creators: 333 DAG levels
    of 3, bodies built and hashed in topological order on the host
    (hostdag.cpp) while the device verifies: digests and statuses equal the
    oracle's over the generator's bodies."""
    from babble_amd.verifier import Verifier
    from oracle import coracle

    packed, wire = synth.event_fields(1000, n_creators=4, seed=12, parents="event")
    v = Verifier(0)
    try:
        res = v.verify_events(wire)
        h, st, _ = coracle.verify_batch(packed.as_dict())
        assert np.array_equal(res.msg_hash, h) and np.all(res.status == 1)
    finally:
        v.close()


@pytest.mark.gpu
def test_verify_events_rejects_forward_reference():
    from babble_amd import native
    from babble_amd.verifier import Verifier

    _, wire = synth.event_fields(10, n_creators=2, seed=13)
    wire.parent_kind[3, 0] = E.PARENT_EVENT
    wire.parent_ref[3, 0] = 5
    v = Verifier(0)
    try:
        with pytest.raises(native.BvError):
            v.verify_events(wire)
    finally:
        v.close()


@pytest.mark.gpu
def test_verify_events_from_pinned_buffers(monkeypatch):
    """Wire fields and results in bv_host_alloc memory (PinnedArena.wire):
    the library DMAs them in place, chunk by chunk (small chunks here), and
    the digests / statuses land in the pinned result arrays — equal to the
    oracle on a signed bulk batch with corruptions and to the pageable call
    on the edge-case wire batches (nil / empty lists, fragments, in-batch
    parents)."""
    from babble_amd.verifier import PinnedArena, Verifier, VerifyResult
    from oracle import coracle

    monkeypatch.setenv("BV_EV_CHUNK_MB", "0.05")
    v = Verifier(0)
    arena = PinnedArena()
    try:
        packed, wire = synth.event_fields(5000, n_creators=8, seed=23, parents="hash")
        bad = np.random.default_rng(23).choice(5000, 50, replace=False)
        wire.s_be[bad, 9] ^= 0x04
        packed.s_be[bad, 9] ^= 0x04
        pw = arena.wire(wire)
        res = VerifyResult(arena.array((5000, 32), np.uint8), arena.array(5000, np.uint8),
                           arena.array((5000 + 63) // 64, np.uint64))
        v.verify_events_into(pw, res)
        h, st, bits = coracle.verify_batch(packed.as_dict())
        assert np.array_equal(res.msg_hash, h)
        assert np.array_equal(res.status, st) and np.array_equal(res.accept_bits, bits)
        for seed in (8, 9):
            w2, _, wd = random_wire(seed, n=700)
            n = w2.n_events
            r2 = VerifyResult(arena.array((n, 32), np.uint8), arena.array(n, np.uint8),
                              arena.array((n + 63) // 64, np.uint64))
            v.verify_events_into(arena.wire(w2), r2)
            assert [d.tobytes() for d in r2.msg_hash] == wd
            ref = v.verify_events(w2)
            assert np.array_equal(r2.status, ref.status) and np.array_equal(r2.accept_bits, ref.accept_bits)
    finally:
        v.close()
        arena.close()


# ---------------------------------------------------------------------------
# The host DAG hasher (babble_amd/csrc/hostdag.cpp + hostsha.cpp): the path
# bv_verify_events takes for batches with in-batch parents, run here on the
# CPU through the emulator library, which links the same source.
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("portable", [False, True], ids=["sha_ext", "portable"])
def test_host_sha256_every_padding_boundary(portable):
    if not portable and not emu.host_sha_accelerated():
        pytest.skip("no SHA extensions on this CPU")
    rng = np.random.default_rng(5)
    for n in list(range(0, 200)) + [447, 448, 1000, 4095, 4096, 65537]:
        m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert emu.host_sha256(m, portable) == hashlib.sha256(m).digest(), n
    assert emu.host_sha256(b"abc", portable).hex() == \
        "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"  # FIPS 180-4 B.1


@pytest.mark.parametrize("threads,portable", [(1, False), (4, False), (1, True)])
def test_host_dag_hash_equals_synth_and_oracle(threads, portable):
    """SyncResponse-shaped DAGs (in-batch parents by index, 333 levels of 3
    events) and the random edge-case batches (nil / empty lists, nil
    transactions, fragments, negative Index / Timestamp, odd key lengths,
    HASH / EVENT / no parents): every digest equals hashlib over the
    generator's bodies / the Go-semantics restatement's."""
    packed, wire = synth.event_fields(1000, n_creators=4, seed=31, parents="event")
    dig = emu.host_dag_hash(wire, threads, portable)
    for i in range(packed.n_items):
        assert dig[i].tobytes() == hashlib.sha256(packed.message(i)).digest(), i
    for seed in (1, 2, 3):
        w, _, wd = random_wire(seed, n=400)
        assert [d.tobytes() for d in emu.host_dag_hash(w, threads, portable)] == wd


def test_host_dag_hash_wide_levels():
    """Levels wider than the parallel threshold (128 events): 300 creators
    give 11 levels of 300 events, hashed on 6 threads."""
    packed, wire = synth.event_fields(3000, n_creators=300, seed=33, parents="event")
    dig = emu.host_dag_hash(wire, threads=6)
    assert all(dig[i].tobytes() == hashlib.sha256(packed.message(i)).digest() for i in range(3000))


KCW = 22  # timing key_path of a batch served by key-cache tables (geometry.h BV_KCW)


def _oracle_bodies(wire):
    """The canonical bodies of a synth-shaped wire batch (one list of
    non-nil transactions, no ITX / BlockSignature fragments) restated by the
    oracle (gosemantics.EventBody.Marshal, event.go:38-45), parents resolved
    in order as ReadWireInfo does (hashgraph.go:1555-1578)."""
    n = wire.n_events
    kind = np.asarray(wire.parent_kind).reshape(n, 2)
    ref = np.asarray(wire.parent_ref).reshape(n, 2)
    ph = np.asarray(wire.parent_hashes).reshape(-1, 32)
    ko = np.asarray(wire.key_off, np.int64)
    bodies, digests = [], []
    for i in range(n):
        ps = []
        for k in range(2):
            if kind[i, k] == E.PARENT_HASH:
                ps.append(gs.EncodeToString(ph[int(ref[i, k])].tobytes()))
            elif kind[i, k] == E.PARENT_EVENT:
                ps.append(gs.EncodeToString(digests[int(ref[i, k])]))
            else:
                ps.append("")
        t0, t1 = int(wire.tx_start[i]), int(wire.tx_start[i + 1])
        txs = [wire.tx_bytes[int(wire.tx_off[t]):int(wire.tx_off[t + 1])].tobytes() for t in range(t0, t1)]
        c = int(wire.creator[i])
        body = gs.EventBody(Transactions=txs, InternalTransactions=None, Parents=ps,
                            Creator=wire.key_bytes[ko[c]:ko[c + 1]].tobytes(), Index=int(wire.index[i]),
                            BlockSignatures=None, Timestamp=int(wire.timestamp[i])).Marshal()
        bodies.append(body)
        digests.append(hashlib.sha256(body).digest())
    return bodies, digests


def _adversarial_kc_wire(parents, n, seed, fresh_key=None):
    """A signed synth wire batch (6 creators) with every key class the key
    cache must keep apart: 2 % corrupted s; events re-assigned to a 65-byte
    key off the curve (a creator's key with y changed), to its compressed
    33-byte form and to an empty key; optionally to a `fresh_key` (valid,
    never seen by the cache).  Returns (wire, oracle statuses, digests, bits,
    the valid creator keys)."""
    from babble_amd.batch import PackedBatch
    from oracle import coracle

    _, wire = synth.event_fields(n, n_creators=6, seed=seed, parents=parents)
    ko = np.asarray(wire.key_off, np.int64)
    keys = [wire.key_bytes[ko[k]:ko[k + 1]].tobytes() for k in range(len(ko) - 1)]
    off_curve = bytearray(keys[0])
    off_curve[64] ^= 1
    extra = [bytes(off_curve), bytes([2 + (keys[1][64] & 1)]) + keys[1][1:33], b""]
    if fresh_key is not None:
        extra.append(fresh_key)
    allk = keys + extra
    wire.key_bytes = np.frombuffer(b"".join(allk), np.uint8).copy()
    wire.key_off = np.concatenate([[0], np.cumsum([len(k) for k in allk])]).astype(np.uint64)
    rng = np.random.default_rng(seed)
    # re-assigned events come from the batch's tail: a re-assigned body's
    # in-batch descendants no longer match their signatures
    rows = n - 1 - rng.choice(n // 8, size=4 * len(extra) * max(1, n // 400), replace=False)
    wire.creator = np.asarray(wire.creator, np.uint32).copy()
    wire.creator[rows] = len(keys) + np.arange(len(rows)) % len(extra)
    bad = rng.choice(np.setdiff1d(np.arange(n), rows), size=max(1, n // 50), replace=False)
    wire.s_be = np.asarray(wire.s_be).copy()
    wire.s_be[bad, 11] ^= 0x02
    bodies, digests = _oracle_bodies(wire)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum([len(b) for b in bodies])
    packed = PackedBatch(np.frombuffer(b"".join(bodies), np.uint8).copy(), off, wire.key_bytes, wire.key_off,
                         np.arange(n, dtype=np.uint32), wire.creator, wire.r_be, wire.s_be,
                         wire.pre if wire.pre is not None else np.zeros(n, np.uint8))
    h, st, bits = coracle.verify_batch(packed.as_dict())
    assert [d.tobytes() for d in h] == digests
    assert {0, 1, 3} <= set(np.unique(st).tolist())  # rejects, accepts and the empty / malformed-key panics
    return wire, st, h, bits, keys


@pytest.mark.gpu
@pytest.mark.parametrize("parents,n", [("event", 1500), ("hash", 6000)])
def test_verify_events_key_cache_matches_oracle(parents, n):
    """bv_verify_events on a BV_F_KEY_CACHE context, with
    in-batch parents (host-hashed DAG path) and without (bulk path), through
    every cache state — cold (unknown keys decoded, valid ones remembered:
    per-batch tables), admitted on the second batch (KC tables built, then
    used), warm (hits), registered (tables from bv_kc_register before the
    first batch) and blocked (a fresh valid key keeps the batch on the
    per-batch path) — over corrupted s, an off-curve key, a compressed and an
    empty key: digests, statuses and bits equal to the C oracle's over the
    oracle-serialized bodies and to a Verifier without the cache."""
    from babble_amd import native
    from babble_amd.verifier import Verifier

    wire, st, h, bits, keys = _adversarial_kc_wire(parents, n, seed=61)

    def check(res, what):
        assert np.array_equal(res.msg_hash, h), what
        assert np.array_equal(res.status, st), what
        assert np.array_equal(res.accept_bits, bits), what

    v0 = Verifier(0)
    vc = Verifier(0, flags=native.F_KEY_CACHE)
    vr = Verifier(0, flags=native.F_KEY_CACHE)
    try:
        check(v0.verify_events(wire), "no cache")
        check(vc.verify_events(wire), "cold")
        assert vc.timing()["key_path"] != KCW, "first sight: keys not admitted yet"
        check(vc.verify_events(wire), "admitted")
        t = vc.timing()
        assert t["key_path"] == KCW and t["kc_builds"] == len(keys), t
        check(vc.verify_events(wire), "warm")
        t = vc.timing()
        assert t["key_path"] == KCW and t["kc_builds"] == 0 and t["kc_hits"] == len(keys), t
        vr.register_keys(keys)
        check(vr.verify_events(wire), "registered")
        assert vr.timing()["key_path"] == KCW
        # a fresh valid key (never seen): the batch takes the per-batch path
        # on the warm ctx, statuses still exact
        fresh = synth.events(1, n_creators=1, seed=62).key(0)
        w2, st2, h2, bits2, _ = _adversarial_kc_wire(parents, n, seed=61, fresh_key=fresh)
        res = vc.verify_events(w2)
        assert np.array_equal(res.msg_hash, h2) and np.array_equal(res.status, st2)
        assert np.array_equal(res.accept_bits, bits2)
        assert vc.timing()["key_path"] != KCW, "blocked by the fresh key"
    finally:
        v0.close()
        vc.close()
        vr.close()


@pytest.mark.gpu
@pytest.mark.parametrize("parents,n", [("event", 1200), ("hash", 30_000)])
def test_verify_events_signature_text_decoded_on_device(parents, n):
    """bv_event_batch.sig_text: the Signature TEXT of every event, decoded on
    the device (k_sig_decode) instead of r / s / pre from the host.  A fifth
    of the events carry adversarial texts (the host fuzzer's corpus: wrong
    part counts, signs, non-digits, values at and past N, 2^288+), the rest
    their real signatures.  Statuses, digests and bits equal the same batch
    with r / s / pre from bv_decode_signature (host) and the C oracle."""
    import random as _random

    from babble_amd import native
    from babble_amd.verifier import Verifier
    from oracle import coracle
    from tests.cabi import harness
    from tests.test_hostfuzz import _sig_cases

    packed, wire = synth.event_fields(n, n_creators=6, seed=81, parents=parents)
    text, off = harness.encode_signatures(wire.r_be, wire.s_be)
    sigs = [harness.signature_text(text, off, i) for i in range(n)]
    rng = _random.Random(n)
    corpus = _sig_cases(_random.Random(7))
    for i in rng.sample(range(n), n // 5):
        sigs[i] = rng.choice(corpus)
    dec = [native.decode_signature(s) for s in sigs]
    pre = np.array([d[0] for d in dec], np.uint8)
    r = np.frombuffer(b"".join(d[1] for d in dec), np.uint8).reshape(n, 32).copy()
    s = np.frombuffer(b"".join(d[2] for d in dec), np.uint8).reshape(n, 32).copy()
    wire.r_be, wire.s_be, wire.pre = r, s, pre
    packed.r_be, packed.s_be, packed.pre = r.copy(), s.copy(), pre.copy()
    h, st, bits = coracle.verify_batch(packed.as_dict())
    toff = np.zeros(n + 1, np.uint64)
    toff[1:] = np.cumsum([len(x) for x in sigs])
    twire = wire.with_signature_text(np.frombuffer(b"".join(sigs), np.uint8).copy(), toff)
    v = Verifier(0)
    try:
        ref = v.verify_events(wire)
        got = v.verify_events(twire)
        for res in (ref, got):
            assert np.array_equal(res.msg_hash, h)
            assert np.array_equal(res.status, st), np.flatnonzero(res.status != st)[:8]
            assert np.array_equal(res.accept_bits, bits)
        assert set(np.unique(st).tolist()) >= {0, 1, 2, 3}
    finally:
        v.close()
