"""Go-semantics restatement (oracle/gosemantics.py) and the product's host
parsing helpers (bv_decode_signature / bv_hex_decode in libbabbleverify.so,
no device needed) agree on the rules the reference inherits from the Go
1.13 stdlib.  CPU only."""
import random

import pytest

from oracle import gosemantics as gs

N = gs.N


# ----------------------------------------------------------------------------
# math/big SetString(s, 36) and keys.DecodeSignature (signature.go:31-39)
# ----------------------------------------------------------------------------
@pytest.mark.parametrize("s,val", [
    ("0", 0), ("-0", 0), ("+0", 0), ("z", 35), ("Z", 35), ("10", 36), ("-10", -36), ("+10", 36),
    ("00012", 38), ("", None), ("+", None), ("-", None), ("1_0", None), (" 1", None), ("1 ", None),
    ("1\n", None), ("--1", None), ("+-1", None), ("1.5", None), ("0x1f", 42819), ("é", None), ("a|b", None),
])
def test_setstring36(s, val):
    assert gs.go_big_setstring36(s) == val


def test_text36_roundtrip():
    rng = random.Random(1)
    for _ in range(300):
        v = rng.getrandbits(rng.choice([1, 8, 64, 255, 256, 300]))
        assert gs.go_big_setstring36(gs.go_big_text36(v)) == v
        assert gs.go_big_text36(v) == gs.go_big_text36(v).lower()


def test_decode_signature_parts():
    assert gs.DecodeSignature("a|b") == (10, 11, True)
    assert gs.DecodeSignature("r|s") == (27, 28, True)  # event_test.go dummy body
    assert gs.DecodeSignature("a") == (None, None, False)
    assert gs.DecodeSignature("a|b|c") == (None, None, False)
    assert gs.DecodeSignature("") == (None, None, False)
    assert gs.DecodeSignature("|") == (None, None, True)
    assert gs.DecodeSignature("a|") == (10, None, True)


def _fuzz_sigs():
    rng = random.Random(7)
    alphabet = "0123456789abcdefghijklmnopqrstuvwxyzABCXYZ+-|_ .\x00é"
    out = ["", "|", "||", "a|b", "0|0", "-1|1", gs.go_big_text36(N) + "|1", gs.go_big_text36(N - 1) + "|1",
           "1|" + gs.go_big_text36(N + 1), gs.go_big_text36(2**256) + "|5", gs.go_big_text36(2**400) + "|5",
           "+" + gs.go_big_text36(12345) + "|" + gs.go_big_text36(N - 2).upper()]
    for _ in range(3000):
        k = rng.randrange(0, 60)
        out.append("".join(rng.choice(alphabet) for _ in range(k)))
    for _ in range(500):
        out.append(gs.EncodeSignature(rng.randrange(-5, N + 5), rng.randrange(-5, 2**257)))
    return out


def test_bv_decode_signature_matches_go_semantics():
    from babble_amd import native

    for sig in _fuzz_sigs():
        pre, rb, sb = native.decode_signature(sig)
        r, s, ok = gs.DecodeSignature(sig)
        if not ok:
            assert pre == 0x80 and rb == bytes(32) and sb == bytes(32), sig
            continue
        rc, sc = gs.scalar_class(r), gs.scalar_class(s)
        assert pre == rc | (sc << 2), (sig, pre, rc, sc)
        assert rb == (r.to_bytes(32, "big") if rc == gs.SC_OK else bytes(32))
        assert sb == (s.to_bytes(32, "big") if sc == gs.SC_OK else bytes(32))


# ----------------------------------------------------------------------------
# common.DecodeFromString / hex.DecodeString (hex.go:15-17)
# ----------------------------------------------------------------------------
@pytest.mark.parametrize("s,out", [
    ("0X", b""), ("0X04", b"\x04"), ("0Xab", b"\xab"), ("0XABc", b"\xab"), ("0X0g12", b""),
    ("0X12zz34", b"\x12"), ("xx0102", b"\x01\x02"), ("0X1", b""), ("0X123", b"\x12"),
])
def test_decode_from_string(s, out):
    from babble_amd import native

    assert gs.DecodeFromString(s) == out
    assert native.hex_decode(s) == out


def test_decode_from_string_panics_short():
    from babble_amd import native

    for s in ("", "0"):
        with pytest.raises(gs.ReferencePanic):
            gs.DecodeFromString(s)
        with pytest.raises(native.ReferencePanic):
            native.hex_decode(s)


def test_encode_to_string():
    assert gs.EncodeToString(b"\x04\xab") == "0X04AB"
    assert gs.EncodeToString(b"") == "0X"


# ----------------------------------------------------------------------------
# encoding/json (Go 1.13, json.Encoder with HTML escaping) for hashed structs
# ----------------------------------------------------------------------------
@pytest.mark.parametrize("s,enc", [
    ("abc", b'"abc"'), ("<a>&", b'"\\u003ca\\u003e\\u0026"'), ('q"b\\', b'"q\\"b\\\\"'),
    ("\n\r\t", b'"\\n\\r\\t"'), ("\x00\x01\x1f\x7f", b'"\\u0000\\u0001\\u001f\x7f"'),
    ("\x08\x0c", b'"\\u0008\\u000c"'), ("é", '"é"'.encode()), ("  ", b'"\\u2028\\u2029"'),
    (b"\xff", b'"\\ufffd"'), (b"\xe2\x82", b'"\\ufffd\\ufffd"'), (b"\xed\xa0\x80", b'"\\ufffd\\ufffd\\ufffd"'),
    ("�", '"�"'.encode()), ("😀", '"😀"'.encode()), (b"\xf4\x90\x80\x80", b'"' + b"\\ufffd" * 4 + b'"'),
])
def test_json_string(s, enc):
    assert gs.json_string(s) == enc


def test_event_body_nil_vs_empty():
    b = gs.EventBody()
    assert b.Marshal() == (b'{"Transactions":null,"InternalTransactions":null,"Parents":null,"Creator":null,'
                           b'"Index":0,"BlockSignatures":null,"Timestamp":0}\n')
    b = gs.EventBody(Transactions=[], InternalTransactions=[], Parents=[], Creator=b"", BlockSignatures=[])
    assert b.Marshal() == (b'{"Transactions":[],"InternalTransactions":[],"Parents":[],"Creator":"",'
                           b'"Index":0,"BlockSignatures":[],"Timestamp":0}\n')


def test_dummy_event_body_of_reference_test():
    """createDummyEventBody (event_test.go:10-24) encodes as Go would."""
    body = gs.EventBody(Transactions=[b"abc", b"def"], InternalTransactions=[], Parents=["self", "other"],
                        Creator=b"public key",
                        BlockSignatures=[gs.BlockSignature(Validator=b"public key", Index=0, Signature="r|s")])
    assert body.Marshal() == (
        b'{"Transactions":["YWJj","ZGVm"],"InternalTransactions":[],"Parents":["self","other"],'
        b'"Creator":"cHVibGljIGtleQ==","Index":0,"BlockSignatures":[{"Validator":"cHVibGljIGtleQ==",'
        b'"Index":0,"Signature":"r|s"}],"Timestamp":0}\n')


def test_itx_and_block_body_field_order():
    itx = gs.InternalTransaction(Body=gs.InternalTransactionBody(Type=1, Peer=gs.Peer("a:1", "0X04", "m")),
                                 Signature="x|y")
    assert itx.Body.Marshal() == b'{"Type":1,"Peer":{"NetAddr":"a:1","PubKeyHex":"0X04","Moniker":"m"}}\n'
    bb = gs.BlockBody(Index=1, RoundReceived=2, Timestamp=3, StateHash=b"", FrameHash=None, PeersHash=b"\x01",
                      Transactions=[], InternalTransactions=[itx], InternalTransactionReceipts=None)
    assert bb.Marshal() == (
        b'{"Index":1,"RoundReceived":2,"Timestamp":3,"StateHash":"","FrameHash":null,"PeersHash":"AQ==",'
        b'"Transactions":[],"InternalTransactions":[{"Body":{"Type":1,"Peer":{"NetAddr":"a:1","PubKeyHex":"0X04",'
        b'"Moniker":"m"}},"Signature":"x|y"}],"InternalTransactionReceipts":null}\n')


def test_trust_count():
    assert [gs.trust_count(n) for n in (0, 1, 2, 3, 4, 10, 100)] == [0, 0, 1, 1, 2, 4, 34]


def test_item_status_order():
    """parse error before panic, empty-key panic before r/s
    checks, r checks before s checks, malformed key only after r/s pass."""
    good = gs.Marshal(gs.scalar_mult(5, gs.G))
    d = bytes(32)
    assert gs.item_status(b"", d, None, None, False) == gs.REJECT_ERR
    assert gs.item_status(b"", d, 1, 1) == gs.REF_PANIC
    assert gs.item_status(b"\x04", d, None, 1) == gs.REF_PANIC
    assert gs.item_status(b"\x04", d, 0, None) == gs.REJECT
    assert gs.item_status(b"\x04", d, 1, None) == gs.REF_PANIC
    assert gs.item_status(b"\x04", d, 1, -1) == gs.REJECT
    assert gs.item_status(b"\x04", d, N, 1) == gs.REJECT
    assert gs.item_status(b"\x04", d, 1, N) == gs.REJECT
    assert gs.item_status(b"\x04", d, 1, 1) == gs.REF_PANIC
    assert gs.item_status(good, d, 1, 1) == gs.REJECT


def test_check_block_deepequal_nil_vs_empty_peers_hash():
    """CheckBlock compares with reflect.DeepEqual (hashgraph.go:1605):
    PeerSet.Hash of an empty set is []byte{} (peer_set.go:104-115), which
    equals an empty PeersHash ("" in JSON) but not a nil one (null)."""
    from oracle import gosemantics as gs

    empty = gs.BlockBody(Index=1, RoundReceived=1, Timestamp=1, StateHash=b"", FrameHash=b"", PeersHash=b"",
                         Transactions=None, InternalTransactions=None, InternalTransactionReceipts=None)
    nil = gs.BlockBody(Index=1, RoundReceived=1, Timestamp=1, StateHash=b"", FrameHash=b"", PeersHash=None,
                       Transactions=None, InternalTransactions=None, InternalTransactionReceipts=None)
    # empty set: count 0 > TrustCount 0 is false either way, but only the nil
    # hash fails at the PeerSet comparison (valid count not reached)
    assert gs.peer_set_hash([]) == b""
    assert gs.check_block(empty, [], []) == (False, 0)
    assert gs.check_block(nil, [], []) == (False, 0)


def test_mirror_check_block_wrong_peerset_for_nil_hash():
    from babble_amd import hashgraph as H

    nil_block = H.Block(Body=H.BlockBody(Index=1, RoundReceived=1, Timestamp=1, StateHash=b"", FrameHash=b"",
                                         PeersHash=None), Signatures={})
    empty_block = H.Block(Body=H.BlockBody(Index=1, RoundReceived=1, Timestamp=1, StateHash=b"", FrameHash=b"",
                                           PeersHash=b""), Signatures={})
    ps = H.PeerSet([])
    assert H.check_block(nil_block, ps) == "Wrong PeerSet"
    assert H.check_block(empty_block, ps) == "Not enough valid signatures: got 0, need 0"
