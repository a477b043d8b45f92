"""The reference's own test scenarios for the verification path, reproduced
through the product (the host mirror babble_amd/hashgraph.py, sync.py,
frame.py over libbabbleverify.so's gfx950 kernels), one named test per
reference test.  SURVEY §8c: the reference pins no values on this path (no
golden vectors, Go and btcd absent here), only these properties — so these
tests pin behaviour, and parity of values stays "unpinned" beyond them
(DESIGN.md §6).  Signatures are made by a pure-Python signer (test-side,
independent of the device and of the C oracle).
"""
import hashlib
import random

import pytest

from babble_amd import hashgraph as H
from babble_amd import native
from oracle import gosemantics as gs
from tests.test_mirror import Signer

pytestmark = pytest.mark.gpu

N = gs.N


@pytest.fixture(scope="module")
def v():
    from babble_amd.verifier import Verifier

    ver = Verifier(0)
    yield ver
    ver.close()


def _keys_verify(v, pub: bytes, msg: bytes, sig: str) -> int:
    """keys.Verify(pub, SHA256(msg), DecodeSignature(sig)) as one device item."""
    from babble_amd.batch import BatchBuilder

    bb = BatchBuilder()
    bb.add_item(bb.add_msg(msg), bb.add_key(pub), sig)
    return int(v.verify(bb.pack()).status[0])


def test_keys_TestSignatureEncoding(v):
    """/root/reference/src/crypto/keys/keys_test.go:53-80: a signature over
    SHA256("J'aime mieux forger mon ame que la meubler") survives
    EncodeSignature -> DecodeSignature (r and s equal) — here through the
    product's bv_decode_signature — and verifies.  64 fresh keys."""
    msg = "J'aime mieux forger mon ame que la meubler".encode()
    digest = H.SHA256(msg, v)
    assert digest == hashlib.sha256(msg).digest()
    sg = Signer(53)
    for _ in range(64):
        d, pub = sg.key()
        sig = sg.sign(d, digest)
        r, s = (gs.go_big_setstring36(x) for x in sig.split("|"))
        pre, rb, sb = native.decode_signature(sig)
        assert pre == 0 and int.from_bytes(rb, "big") == r and int.from_bytes(sb, "big") == s
        assert _keys_verify(v, pub, msg, sig) == native.ACCEPT


def _dummy_event_body(creator: bytes) -> H.EventBody:
    """createDummyEventBody (event_test.go:10-24) with Creator set to the
    signer's key as TestSignEvent does; the BlockSignature's Validator keeps
    the dummy []byte("public key") it was given before."""
    return H.EventBody(Transactions=[b"abc", b"def"], InternalTransactions=[], Parents=["self", "other"],
                       Creator=creator,
                       BlockSignatures=[H.BlockSignature(Validator=b"public key", Index=0, Signature="r|s")])


def _sign_event(sg: Signer, d: int, ev: H.Event) -> None:
    """Event.Sign (event.go:201-215): keys.Sign over Body.Hash()."""
    ev.Signature = sg.sign(d, gs.SHA256(ev.Body.Marshal()))


def test_event_TestSignEvent(v):
    """/root/reference/src/hashgraph/event_test.go:57-76: sign the dummy
    event body, Event.Verify() returns (true, nil).  Also what must fail: the
    same signature after a body change, and by another key."""
    sg = Signer(57)
    d, pub = sg.key()
    ev = H.Event(Body=_dummy_event_body(pub))
    _sign_event(sg, d, ev)
    assert ev.Verify(v) == (True, None)
    assert ev.Hash(v) == gs.SHA256(ev.Body.Marshal())
    bad = H.Event(Body=_dummy_event_body(pub), Signature=ev.Signature)
    bad.Body.Transactions = [b"abc", b"deg"]
    assert bad.Verify(v) == (False, None)
    _, other = sg.key()
    assert H.Event(Body=_dummy_event_body(other), Signature=ev.Signature).Verify(v) == (False, None)


def _test_block() -> H.Block:
    """createTestBlock (block_test.go:11-33): NewBlock(0, 1, "framehash", no
    peers, [abc def ghi], [PEER_ADD peer1, PEER_REMOVE peer2], 0) with an
    accepted receipt per internal transaction.  NewBlock (block.go:161-192):
    StateHash []byte{}, PeersHash = the empty peer set's hash ([]byte{})."""
    itxs = [H.InternalTransaction(Body=H.InternalTransactionBody(Type=0, Peer=H.Peer(
                NetAddr="paris", PubKeyHex="peer1", Moniker="peer1"))),
            H.InternalTransaction(Body=H.InternalTransactionBody(Type=1, Peer=H.Peer(
                NetAddr="london", PubKeyHex="peer2", Moniker="peer2")))]
    body = H.BlockBody(Index=0, RoundReceived=1, Timestamp=0, StateHash=b"", FrameHash=b"framehash",
                       PeersHash=H.PeerSet([]).Hash(), Transactions=[b"abc", b"def", b"ghi"],
                       InternalTransactions=itxs,
                       InternalTransactionReceipts=[H.InternalTransactionReceipt(t, True) for t in itxs])
    return H.Block(Body=body)


def _block_sign(sg: Signer, d: int, pub: bytes, block: H.Block) -> H.BlockSignature:
    """Block.Sign (block.go:318-334)."""
    return H.BlockSignature(Validator=pub, Index=block.Index(), Signature=sg.sign(d, gs.SHA256(block.Body.Marshal())))


def test_block_TestSignBlock(v):
    """/root/reference/src/hashgraph/block_test.go:36-54."""
    sg = Signer(36)
    d, pub = sg.key()
    block = _test_block()
    assert block.Body.Marshal() == gs.BlockBody(
        Index=0, RoundReceived=1, Timestamp=0, StateHash=b"", FrameHash=b"framehash", PeersHash=b"",
        Transactions=[b"abc", b"def", b"ghi"],
        InternalTransactions=[gs.InternalTransaction(Body=gs.InternalTransactionBody(Type=t, Peer=gs.Peer(a, k, m)))
                              for t, a, k, m in ((0, "paris", "peer1", "peer1"), (1, "london", "peer2", "peer2"))],
        InternalTransactionReceipts=[gs.InternalTransactionReceipt(gs.InternalTransaction(
            Body=gs.InternalTransactionBody(Type=t, Peer=gs.Peer(a, k, m))), True)
            for t, a, k, m in ((0, "paris", "peer1", "peer1"), (1, "london", "peer2", "peer2"))]).Marshal()
    sig = _block_sign(sg, d, pub, block)
    assert block.Verify(sig, v) == (True, None)


def test_block_TestAppendSignature(v):
    """/root/reference/src/hashgraph/block_test.go:56-82: SetSignature, then
    GetSignature(PublicKeyHex) round-trips through the validator hex and
    still verifies."""
    sg = Signer(56)
    d, pub = sg.key()
    block = _test_block()
    block.SetSignature(_block_sign(sg, d, pub, block))
    bs = [s for s in block.GetSignatures() if s.ValidatorHex() == gs.EncodeToString(pub)]
    assert len(bs) == 1 and bs[0].Validator == pub and bs[0].Index == 0
    assert block.Verify(bs[0], v) == (True, None)


# initRoundHashgraph's plays (hashgraph_test.go:403-416): (creator, index,
# self-parent, other-parent, name, transactions)
_PLAYS = [(0, 0, "", "", "e0", None), (1, 0, "", "", "e1", None), (2, 0, "", "", "e2", None),
          (1, 1, "e1", "e0", "e10", None), (2, 1, "e2", "", "s20", None), (0, 1, "e0", "", "s00", None),
          (2, 2, "s20", "e10", "e21", None), (0, 2, "s00", "e21", "e02", None), (1, 2, "e10", "", "s10", None),
          (1, 3, "s10", "e02", "f1", None), (1, 4, "f1", "", "s11", [b"abc"])]


def _round_hashgraph(sg: Signer):
    """The events of initRoundHashgraph, signed: NewEvent (event.go:123-142)
    bodies with Parents [index[self], index[other]] ("" for none)."""
    nodes = [sg.key() for _ in range(3)]
    index, events, by_name = {"": ""}, [], {}
    for k, (c, i, sp, op, name, txs) in enumerate(_PLAYS):
        ev = H.Event(Body=H.EventBody(Transactions=txs, Parents=[index[sp], index[op]], Creator=nodes[c][1],
                                      Index=i, Timestamp=1_600_000_000 + k))
        _sign_event(sg, nodes[c][0], ev)
        index[name] = gs.EncodeToString(gs.SHA256(ev.Body.Marshal()))
        events.append((name, c, sp, op, ev))
        by_name[name] = (c, i)
    return nodes, index, events, by_name


def test_hashgraph_TestReadWireInfo(v):
    """/root/reference/src/hashgraph/hashgraph_test.go:575-608: every event of
    initRoundHashgraph, ToWire -> ReadWireInfo: Body and Signature equal
    the original and Verify is true.  Here the whole set goes through the
    product's core.sync path (sync.sync_verify_device: the device rebuilds
    every EventBody from wire fields, hashes and verifies), once with every
    parent in the store (the reference test's situation) and once with an
    empty store (every parent resolved in-batch, the DAG hashed level by
    level on the device)."""
    from babble_amd import sync as S

    sg = Signer(575)
    nodes, index, events, by_name = _round_hashgraph(sg)
    peers = {100 + c: H.Peer(PubKeyHex=gs.EncodeToString(pub)) for c, (_, pub) in enumerate(nodes)}
    wevents = []
    for name, c, sp, op, ev in events:  # Event.ToWire (event.go:390-405)
        wevents.append(S.WireEvent(Body=S.WireBody(
            Transactions=ev.Body.Transactions, InternalTransactions=ev.Body.InternalTransactions,
            BlockSignatures=None, CreatorID=100 + c,
            OtherParentCreatorID=100 + by_name[op][0] if op else 0, Index=ev.Body.Index,
            SelfParentIndex=by_name[sp][1] if sp else -1, OtherParentIndex=by_name[op][1] if op else -1,
            Timestamp=ev.Body.Timestamp), Signature=ev.Signature))
    store = {(gs.EncodeToString(ev.Body.Creator), ev.Body.Index): index[name] for name, _, _, _, ev in events}
    for participant_event in (lambda pk, i: store.get((pk, i)), lambda pk, i: None):
        got, outcomes, read_err = S.sync_verify_device(wevents, peers, participant_event, v)
        assert read_err is None and len(got) == len(events)
        for (name, _, _, _, ev), g, o in zip(events, got, outcomes):
            assert g.Body == ev.Body, name
            assert g.Signature == ev.Signature
            assert (o.ok, o.err) == (True, None), name
            assert g.Hex() == index[name]


def test_hashgraph_TestInsertEvent_BlockSignatureNotFromCreator(v):
    """/root/reference/src/hashgraph/hashgraph_test.go:1017-1046: an event of
    node 0 carrying a block signature made by a key outside the peer set is
    inserted (its own signature is valid) but the block signature is not
    appended to the block.  Here: the event verifies; ProcessSigPool
    (hashgraph.go:1295-1367) skips the foreign validator, and the same
    signature claimed for node 0 fails Block.Verify and is skipped too — the
    block keeps its 3 signatures."""
    sg = Signer(1017)
    nodes = [sg.key() for _ in range(3)]
    ps = H.PeerSet([H.Peer(PubKeyHex=gs.EncodeToString(pub)) for _, pub in nodes])
    body = H.BlockBody(Index=0, RoundReceived=1, Timestamp=5, StateHash=b"", FrameHash=b"f" * 32,
                       PeersHash=ps.Hash(v), Transactions=[b"abc"], InternalTransactions=[])
    block = H.Block(Body=body)
    for d, pub in nodes:
        block.SetSignature(_block_sign(sg, d, pub, block))
    bad_d, bad_pub = sg.key()
    bad_sig = _block_sign(sg, bad_d, bad_pub, block)
    ev = H.Event(Body=H.EventBody(Parents=["", ""], Creator=nodes[0][1], Index=2, Timestamp=9,
                                  BlockSignatures=[bad_sig]))
    _sign_event(sg, nodes[0][0], ev)
    assert H.insert_event_verify(ev, verifier=v) is None  # the event itself is inserted
    claimed = H.BlockSignature(Validator=nodes[0][1], Index=0, Signature=bad_sig.Signature)
    appended, err = H.process_sig_pool([bad_sig, claimed], lambda i: block if i == 0 else None, lambda r: ps, v)
    assert appended == [] and err is None
    assert len(block.Signatures) == 3


def test_core_TestCoreFastForward_not_enough_signatures(v):
    """/root/reference/src/node/core_test.go:492-550: 4 peers; an anchor
    block with only 1 signature makes fastForward fail, with all 3 others'
    signatures it succeeds (core.fastForward's checks, core.go:367-388:
    CheckBlock then the frame hash)."""
    from babble_amd import frame as F

    sg = Signer(492)
    keys = [sg.key() for _ in range(4)]
    peers = [H.Peer(NetAddr="127.0.0.1:%d" % (1337 + i), PubKeyHex=gs.EncodeToString(pub), Moniker="node%d" % i)
             for i, (_, pub) in enumerate(keys)]
    frame = F.Frame(Round=1, Peers=peers, Timestamp=1_600_000_000)
    ps = H.PeerSet(peers)
    body = H.BlockBody(Index=0, RoundReceived=1, Timestamp=1_600_000_000, StateHash=b"", FrameHash=frame.Hash(v),
                       PeersHash=ps.Hash(v), Transactions=[b"tx0", b"tx1"], InternalTransactions=[])
    sigs = [_block_sign(sg, d, pub, H.Block(Body=body)) for d, pub in keys[1:]]
    block = H.Block(Body=body)
    block.SetSignature(sigs[0])
    assert F.fast_forward_check(block, frame, v) == "Not enough valid signatures: got 1, need 2"
    for s in sigs[1:]:
        block.SetSignature(s)
    assert F.fast_forward_check(block, frame, v) is None


def test_decode_signature_error_passes_through_unchanged(v):
    """ProcessSigPool and InsertEvent return keys.DecodeSignature's error
    unchanged (hashgraph.go:1331-1337, :672-687; signature.go:33-35): the
    mirror surfaces Go's exact text with the part count."""
    sg = Signer(1331)
    d, pub = sg.key()
    ev = H.Event(Body=H.EventBody(Parents=["", ""], Creator=pub, Index=0, Timestamp=1))
    for sig, parts in (("abc", 1), ("a|b|c", 3), ("", 1), ("||||", 5)):
        ev.Signature = sig
        ev._hash = None
        assert H.insert_event_verify(ev, verifier=v) == "wrong number of values in signature: got %d, want 2" % parts


def test_reference_usage_peers_keys_panic_on_device(v):
    """the four PubKeyHex values of the reference's own
    docs/usage.rst:166-181 (lowercase "0x" prefix) are reference-held
    vectors for common.DecodeFromString -> keys.ToPublicKey: each decodes
    (bv_hex_decode) to 65 bytes with prefix 0x04 but lies off the curve, so
    elliptic.Unmarshal leaves X nil and ecdsa.Verify panics in ScalarMult
    for any item whose r and s pass the range checks (REF_PANIC); items
    stopped earlier keep their earlier outcome (r = 0: REJECT; parts != 2:
    REJECT_ERR).  Statuses equal the C oracle's."""
    from babble_amd.batch import BatchBuilder
    from oracle import coracle
    from tests.helpers import load

    peers = load("reference_usage_peers.json")["peers"]
    sg = Signer(181)
    bb = BatchBuilder()
    want = []
    for p in peers:
        pub = native.hex_decode(p["PubKeyHex"])
        assert pub == gs.DecodeFromString(p["PubKeyHex"]) and len(pub) == 65 and pub[0] == 4
        assert gs.Unmarshal(pub) is None
        k = bb.add_key(pub)
        msg = p["Moniker"].encode()
        d, _ = sg.key()
        sig = sg.sign(d, hashlib.sha256(msg).digest())
        m = bb.add_msg(msg)
        for s, st in ((sig, native.REF_PANIC), ("0|" + sig.split("|")[1], native.REJECT), ("abc", native.REJECT_ERR)):
            bb.add_item(m, k, s)
            want.append(st)
    b = bb.pack()
    res = v.verify(b)
    assert res.status.tolist() == want
    _, st, _ = coracle.verify_batch(b.as_dict())
    assert st.tolist() == want
