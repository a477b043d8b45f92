"""The synthetic workload generator produces exactly the canonical bytes the
Go encoders would (checked with the oracle's encoding/json restatement) and
valid signatures (checked with the oracle)."""
import base64
import json

import numpy as np

from babble_amd import synth
from oracle import coracle
from oracle import gosemantics as gs


def test_event_bodies_are_canonical_json():
    b = synth.events(300, n_creators=4, seed=1)
    for m in (0, 1, 3, 4, 5, 77, 299):
        raw = b.message(m)
        d = json.loads(raw)
        body = gs.EventBody(Transactions=[base64.b64decode(x) for x in d["Transactions"]], InternalTransactions=None,
                            Parents=d["Parents"], Creator=base64.b64decode(d["Creator"]), Index=d["Index"],
                            BlockSignatures=None, Timestamp=d["Timestamp"])
        assert body.Marshal() == raw
    # parents are the 0X-hex hashes of the creator's previous event and of the
    # other creator's latest event (hashgraph_test.go play pattern)
    d5 = json.loads(b.message(5))
    assert d5["Parents"][0] == gs.EncodeToString(gs.SHA256(b.message(1)))
    assert d5["Parents"][1] == gs.EncodeToString(gs.SHA256(b.message(2)))
    assert json.loads(b.message(0))["Parents"] == ["", ""]
    assert 445 <= len(b.message(100)) <= 449  # T=1 body size


def test_events_all_valid():
    b = synth.events(500, n_creators=8, seed=2)
    _, st, _ = coracle.verify_batch(b.as_dict())
    assert np.all(st == 1)


def test_t0_and_t16_bodies():
    for n_tx, lo, hi in ((0, 300, 400), (16, 1700, 1900)):
        b = synth.events(20, n_creators=2, seed=3, n_tx=n_tx)
        assert lo <= len(b.message(10)) <= hi
        _, st, _ = coracle.verify_batch(b.as_dict())
        assert np.all(st == 1)


def test_blocks_canonical_and_peers_hash():
    wb = synth.blocks(3, n_validators=7, seed=5)
    b = wb.batch
    peers = [gs.Peer(PubKeyHex=gs.EncodeToString(b.key(k))) for k in range(7)]
    assert gs.peer_set_hash(peers) == wb.peers_hash
    raw = b.message(1)
    d = json.loads(raw)
    body = gs.BlockBody(Index=d["Index"], RoundReceived=d["RoundReceived"], Timestamp=d["Timestamp"],
                        StateHash=base64.b64decode(d["StateHash"]), FrameHash=base64.b64decode(d["FrameHash"]),
                        PeersHash=base64.b64decode(d["PeersHash"]),
                        Transactions=[base64.b64decode(x) for x in d["Transactions"]], InternalTransactions=[],
                        InternalTransactionReceipts=None)
    assert body.Marshal() == raw
    _, st, _ = coracle.verify_batch(b.as_dict())
    assert np.all(st == 1)


def test_adversarial_mix_counts():
    b = synth.adversarial(100_000, seed=4)
    _, st, _ = coracle.verify_batch(b.as_dict())
    counts = np.bincount(st, minlength=4)
    # REJECT_ERR = the parts errors: half of the 50 format cases at 10^5 items
    assert counts[2] == 26
    assert counts[1] > 98_000 and counts[0] > 500 and counts[3] > 100
