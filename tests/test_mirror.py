"""The host-side mirror of the reference interface (babble_amd/hashgraph.py):
its JSON equals the oracle's encoding/json restatement (CPU), and its
Verify / CheckBlock / ProcessSigPool decisions equal the oracle's (GPU)."""
import dataclasses
import hashlib
import random

import pytest

from babble_amd import hashgraph as H
from oracle import gosemantics as gs

N = gs.N


def to_mirror(obj):
    """Convert an oracle dataclass tree into the mirror's (same field names)."""
    if dataclasses.is_dataclass(obj):
        cls = getattr(H, type(obj).__name__)
        return cls(**{f.name: to_mirror(getattr(obj, f.name)) for f in dataclasses.fields(obj)})
    if isinstance(obj, list):
        return [to_mirror(x) for x in obj]
    return obj


class Signer:
    def __init__(self, seed):
        self.rng = random.Random(seed)

    def key(self):
        d = self.rng.randrange(1, N)
        return d, gs.Marshal(gs.scalar_mult(d, gs.G))

    def sign(self, d, digest):
        k = self.rng.randrange(1, N)
        r = gs.scalar_mult(k, gs.G)[0] % N
        s = pow(k, -1, N) * (int.from_bytes(digest, "big") + r * d) % N
        return gs.EncodeSignature(r, s)


STRINGS = ["plain", "<b>&amp;</b>", 'q"\\', "ctl\x01\t\n", "é ☃ 😀", "  ", b"\xff\xfe", b"\xe2\x82",
           b"\xed\xa0\x80x"]


def make_events(seed=1, n=48):
    sg = Signer(seed)
    keys = [sg.key() for _ in range(4)]
    peers = [gs.Peer("10.0.0.%d:1337" % i, gs.EncodeToString(k[1]), "node%d" % i) for i, k in enumerate(keys)]
    evs = []
    for i in range(n):
        v = i % 8
        b = gs.EventBody(Transactions=[bytes(sg.rng.randrange(256) for _ in range(sg.rng.randrange(70)))
                                       for _ in range(sg.rng.randrange(3))] if v != 1 else None,
                         Parents=["", ""] if i % 5 == 0 else [gs.EncodeToString(bytes(32)), "0XAB"],
                         Creator=keys[0][1], Index=i, Timestamp=1_600_000_000 + i)
        if v == 2:
            b.Transactions, b.InternalTransactions, b.Parents, b.BlockSignatures = [], [], [], []
        if v in (3, 5, 7):
            t = gs.InternalTransaction(Body=gs.InternalTransactionBody(Type=v % 2, Peer=gs.Peer(
                STRINGS[i % len(STRINGS)], peers[1].PubKeyHex, STRINGS[(i + 3) % len(STRINGS)])))
            sig = sg.sign(keys[1][0], t.Body.Hash())
            t.Signature = sig if v == 3 else (sig + "1" if v == 5 else "nope")
            b.InternalTransactions = [t]
        if v == 4:
            b.BlockSignatures = [gs.BlockSignature(keys[0][1], 3, "r|s"), gs.BlockSignature(None, 0, STRINGS[i % 9])]
        if v == 6:
            b.InternalTransactions = [gs.InternalTransaction(Body=gs.InternalTransactionBody(
                Peer=gs.Peer("x", "0" if i % 16 == 6 else "0X04ZZ", "m")), Signature="1|1")]
        if i % 11 == 10:
            b.Creator = None
        sig = sg.sign(keys[0][0], b.Hash())
        if i % 7 == 3:
            sig = sig.split("|")[0] + "|" + gs.go_big_text36(int(gs.go_big_setstring36(sig.split("|")[1])) ^ 4)
        if i % 13 == 12:
            sig = sig + "|x"
        evs.append((b, sig))
    return evs


def test_mirror_json_equals_oracle_json():
    for b, _ in make_events(seed=3, n=64):
        assert to_mirror(b).Marshal() == b.Marshal()
        for t in b.InternalTransactions or []:
            assert to_mirror(t).Body.Marshal() == t.Body.Marshal()


@pytest.mark.parametrize("s", STRINGS + ["", "\x7f", "\U0010ffff", b"\xf4\x90\x80\x80", b"\xc0\x80"])
def test_gojson_string_equals_oracle(s):
    from babble_amd import gojson

    assert gojson.string(s) == gs.json_string(s)


def test_block_json_and_trust_count():
    ob = gs.BlockBody(Index=4, RoundReceived=9, Timestamp=7, StateHash=b"", FrameHash=None, PeersHash=b"\x01\x02",
                      Transactions=[b"a" * 64] * 3, InternalTransactions=[], InternalTransactionReceipts=None)
    assert to_mirror(ob).Marshal() == ob.Marshal()
    for n in (0, 1, 2, 3, 10, 100):
        peers = [H.Peer(PubKeyHex="0X%02X" % i) for i in range(n)]
        assert H.PeerSet(peers).TrustCount() == gs.trust_count(n)


@pytest.mark.gpu
def test_verify_events_matches_oracle():
    evs = make_events(seed=5, n=96)
    mirror = [H.Event(Body=to_mirror(b), Signature=s) for b, s in evs]
    outs = H.verify_events(mirror)
    codes = {gs.EV_ACCEPT: (True, False), gs.EV_REJECT: (False, False), gs.EV_ERR: (False, False),
             gs.EV_ITX_INVALID: (False, False), gs.EV_PANIC: (False, True)}
    seen = set()
    for (b, s), ev, o in zip(evs, mirror, outs):
        want = gs.event_status(b, s)
        seen.add(want)
        assert (o.ok, o.panic) == codes[want], (want, o)
        if want == gs.EV_ERR:  # signature.go:34: Go's text with the part count, passed up unchanged
            assert o.err == gs.event_verify_error(b, s) and o.err.endswith(", want 2"), o.err
        if want == gs.EV_ITX_INVALID:
            assert o.err == "invalid signature on internal transaction"
        assert ev.Hash() == hashlib.sha256(b.Marshal()).digest()  # digest filled by the batch
    assert seen == {gs.EV_ACCEPT, gs.EV_REJECT, gs.EV_ERR, gs.EV_ITX_INVALID, gs.EV_PANIC}


@pytest.mark.gpu
def test_single_event_verify_and_panic():
    evs = make_events(seed=6, n=24)
    for b, s in evs:
        ev = H.Event(Body=to_mirror(b), Signature=s)
        want = gs.event_status(b, s)
        if want == gs.EV_PANIC:
            with pytest.raises(H.ReferencePanic):
                ev.Verify()
        else:
            ok, err = ev.Verify()
            assert ok == (want == gs.EV_ACCEPT)
            msg = H.insert_event_verify(ev)
            assert (msg is None) == ok


def _signed_block(sg, vals, peers_hash, n_bad, idx=1):
    ob = gs.BlockBody(Index=idx, RoundReceived=idx + 1, Timestamp=1, StateHash=b"s" * 32, FrameHash=b"f" * 32,
                      PeersHash=peers_hash, Transactions=[b"t" * 64] * 4, InternalTransactions=[],
                      InternalTransactionReceipts=None)
    digest = ob.Hash()
    sigs = {}
    for i, (d, pub) in enumerate(vals):
        s = sg.sign(d, digest)
        if i < n_bad:
            s = s[:-1] + ("1" if s[-1] != "1" else "2")
        sigs[gs.EncodeToString(pub)] = s
    return ob, sigs


@pytest.mark.gpu
@pytest.mark.parametrize("n_bad", [0, 5, 6, 7, 10])
def test_check_block_matches_oracle(n_bad):
    sg = Signer(100 + n_bad)
    vals = [sg.key() for _ in range(10)]
    opeers = [gs.Peer(PubKeyHex=gs.EncodeToString(v[1])) for v in vals]
    ph = gs.peer_set_hash(opeers)
    ob, sigs = _signed_block(sg, vals, ph, n_bad)
    outsider = sg.key()
    sigs[gs.EncodeToString(outsider[1])] = sg.sign(outsider[0], ob.Hash())  # not a member: skipped
    ok, valid = gs.check_block(ob, list(sigs.items()), opeers)
    ps = H.PeerSet([H.Peer(PubKeyHex=p.PubKeyHex) for p in opeers])
    assert ps.Hash() == ph
    err = H.check_block(H.Block(Body=to_mirror(ob), Signatures=dict(sigs)), ps)
    assert (err is None) == ok
    if not ok:
        assert err == "Not enough valid signatures: got %d, need %d" % (valid, 4)
    wrong = H.Block(Body=to_mirror(dataclasses.replace(ob, PeersHash=b"x")), Signatures=dict(sigs))
    assert H.check_block(wrong, ps) == "Wrong PeerSet"


@pytest.mark.gpu
def test_process_sig_pool_order_and_abort():
    sg = Signer(7)
    vals = [sg.key() for _ in range(5)]
    ps = H.PeerSet([H.Peer(PubKeyHex=gs.EncodeToString(v[1])) for v in vals])
    ob, sigs = _signed_block(sg, vals, ps.Hash(), n_bad=1)
    blk = H.Block(Body=to_mirror(ob), Signatures={})
    pending = [H.BlockSignature(DecodeFromStringHex(k), 1, s) for k, s in sigs.items()]
    pending.insert(3, H.BlockSignature(vals[2][1], 1, "broken"))  # parts != 2 -> abort here
    pending.insert(1, H.BlockSignature(sg.key()[1], 1, "a|b"))    # not a member: skipped
    pending.insert(0, H.BlockSignature(vals[0][1], 99, "a|b"))    # unknown block: skipped
    appended, err = H.process_sig_pool(pending, lambda i: blk if i == 1 else None, lambda r: ps)
    assert err == "wrong number of values in signature: got 1, want 2"  # signature.go:34 ("broken")
    # the first signature (index 0 of sigs) is the corrupted one; two valid ones precede the abort
    assert [a.Signature for a in appended] == [s for s in list(sigs.values())[1:3]]
    assert set(blk.Signatures) == {a.ValidatorHex() for a in appended}


def DecodeFromStringHex(h):
    return gs.DecodeFromString(h)
