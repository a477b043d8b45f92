"""Frame.Marshal / Frame.Hash (ugorji canonical JSON, frame.go:35-69) and the
verification half of core.fastForward (core.go:367-388).

CPU: the product mirror's encoder (babble_amd/frame.py) against the oracle's
schema-driven restatement (oracle/gosemantics.py ugorji_*) on random frames,
canonical-JSON properties, the committed golden frames, and the reference's
own property (hashgraph_test.go:1729-1740: Marshal -> Unmarshal -> equal).
GPU: frame digests and fast_forward_check through the device.
"""
import json
import random

import pytest

from babble_amd import frame as F
from oracle import gosemantics as gs
from tests.frame_spec import ProductNS, frame_spec, to_types
from tests.helpers import load


def test_product_encoder_equals_oracle_restatement():
    rng = random.Random(11)
    P = ProductNS()
    for _ in range(300):
        spec = frame_spec(rng)
        a = to_types(spec, P).Marshal()
        b = gs.frame_marshal(to_types(spec, gs))
        assert a == b


def _keys_in_order(raw: bytes):
    """Every JSON object's keys, in output order (object_pairs_hook)."""
    orders = []

    def hook(pairs):
        orders.append([k for k, _ in pairs])
        return dict(pairs)

    json.loads(raw.decode("utf-8"), object_pairs_hook=hook)
    return orders


def test_output_is_canonical_json():
    """Valid JSON, no whitespace, every object's keys sorted (struct fields by
    name, string map keys by bytes, int map keys numerically), no newline."""
    rng = random.Random(12)
    P = ProductNS()
    for _ in range(200):
        f = to_types(frame_spec(rng), P)
        raw = f.Marshal()
        assert not raw.endswith(b"\n")
        for keys in _keys_in_order(raw):
            if keys and all(k.lstrip("-").isdigit() for k in keys):
                assert [int(k) for k in keys] == sorted(int(k) for k in keys)
            else:
                assert keys == sorted(keys, key=lambda k: k.encode("utf-8"))
    top = _keys_in_order(F.Frame().Marshal())[-1]
    assert top == ["Events", "PeerSets", "Peers", "Roots", "Round", "Timestamp"]
    assert F.Frame().Marshal() == (b'{"Events":null,"PeerSets":null,"Peers":null,"Roots":null,"Round":0,'
                                   b'"Timestamp":0}')


def test_marshal_unmarshal_round_trip_property():
    """hashgraph_test.go:1729-1740 / 2270-2281: a marshalled frame parses back
    to the same structure; re-encoding the parsed value gives the same bytes."""
    rng = random.Random(13)
    P = ProductNS()
    for _ in range(100):
        spec = frame_spec(rng)
        raw = to_types(spec, P).Marshal()
        parsed = json.loads(raw.decode("utf-8"))
        assert parsed["Round"] == spec["Round"] and parsed["Timestamp"] == spec["Timestamp"]
        if spec["PeerSets"] is not None:
            assert sorted(int(k) for k in parsed["PeerSets"]) == sorted(spec["PeerSets"])
        if spec["Roots"] is not None:
            assert set(parsed["Roots"]) == set(spec["Roots"])


def test_golden_frames():
    fx = load("golden_frames.json")
    assert len(fx) >= 20
    P = ProductNS()
    for g in fx:
        f = to_types(g["spec"], P)
        raw = f.Marshal()
        assert raw.hex() == g["marshal"]
        assert gs.SHA256(raw).hex() == g["hash"]
        assert gs.frame_hash(to_types(g["spec"], gs)).hex() == g["hash"]


@pytest.mark.gpu
def test_frame_hashes_on_device():
    from babble_amd.verifier import Verifier

    rng = random.Random(14)
    P = ProductNS()
    frames = [to_types(frame_spec(rng), P) for _ in range(300)]
    v = Verifier(0)
    try:
        got = F.frame_hashes(frames, v)
        assert got == [gs.SHA256(f.Marshal()) for f in frames]
        # a long frame (many blocks on one lane)
        big = to_types(frame_spec(rng), P)
        big.Events = [F.FrameEvent(Round=i, LamportTimestamp=i) for i in range(3000)]
        assert big.Hash(v) == gs.SHA256(big.Marshal())
    finally:
        v.close()


@pytest.mark.gpu
def test_peer_set_hash_on_device():
    """bv_peer_set_hash (one launch) == the sequential chain of peer_set.go."""
    from babble_amd.verifier import Verifier

    rng = random.Random(15)
    v = Verifier(0)
    try:
        for n in (0, 1, 2, 5, 100):
            pks = [bytes(rng.getrandbits(8) for _ in range(rng.choice([65, 65, 33, 0, 70]))) for _ in range(n)]
            want = b""
            for pk in pks:
                want = gs.SimpleHashFromTwoHashes(want, pk)
            assert v.peer_set_hash(pks) == want
    finally:
        v.close()


@pytest.mark.gpu
def test_fast_forward_check():
    """core.fastForward's checks on a real anchor: 100 validators signing a
    BlockBody whose FrameHash is the frame's hash -> None; a wrong frame ->
    "Invalid Frame Hash"; too few valid signatures -> CheckBlock's error; a
    nil PeersHash -> "Wrong PeerSet" (reflect.DeepEqual)."""
    from babble_amd import hashgraph as H
    from babble_amd.verifier import Verifier
    from tests.test_mirror import Signer

    sg = Signer(1000)
    keys = [sg.key() for _ in range(100)]
    peers = [H.Peer(NetAddr="n%d" % i, PubKeyHex=gs.EncodeToString(pub), Moniker="m%d" % i)
             for i, (_, pub) in enumerate(keys)]
    rng = random.Random(16)
    frame = to_types(frame_spec(rng), ProductNS())
    frame.Peers = peers
    v = Verifier(0)
    try:
        ps = H.PeerSet(peers)
        body = H.BlockBody(Index=7, RoundReceived=3, Timestamp=11, StateHash=b"s" * 32, FrameHash=frame.Hash(v),
                           PeersHash=ps.Hash(v), Transactions=[b"t" * 64] * 4, InternalTransactions=[])
        digest = gs.SHA256(body.Marshal())
        block = H.Block(Body=body, Signatures={gs.EncodeToString(pub): sg.sign(priv, digest)
                                               for priv, pub in keys})
        assert F.fast_forward_check(block, frame, v) is None
        other = to_types(frame_spec(rng), ProductNS())
        other.Peers = peers
        assert F.fast_forward_check(block, other, v) == "Invalid Frame Hash"
        weak = H.Block(Body=body, Signatures=dict(list(block.Signatures.items())[:34]))
        assert F.fast_forward_check(weak, frame, v) == "Not enough valid signatures: got 34, need 34"
        nilph = H.Block(Body=H.BlockBody(**{**body.__dict__, "PeersHash": None}), Signatures=block.Signatures)
        assert F.fast_forward_check(nilph, frame, v) == "Wrong PeerSet"
    finally:
        v.close()
