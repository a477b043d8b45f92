"""Random Frame specs (plain JSON-able dicts) and their conversion into the
product mirror's types (babble_amd.frame) and the oracle's
(oracle.gosemantics) — shared by tests/test_frame.py and the golden-fixture
generator.  Byte strings are hex in the spec; None stays None (nil)."""
from __future__ import annotations

import random

STRINGS = ["", "node0:1337", "<script>&amp;", "tab\there\nnl", "  ", "é😀", "q\"b\\s", "\x01\x1f\x7f"]


def _hx(rng, n):
    return bytes(rng.getrandbits(8) for _ in range(n)).hex()


def peer_spec(rng):
    return {"NetAddr": rng.choice(STRINGS), "PubKeyHex": "0X" + _hx(rng, 65).upper(), "Moniker": rng.choice(STRINGS)}


def body_spec(rng):
    def maybe(f):
        r = rng.random()
        return None if r < 0.3 else ([] if r < 0.4 else f())

    return {
        "Transactions": maybe(lambda: [None if rng.random() < 0.1 else _hx(rng, rng.randrange(0, 70))
                                       for _ in range(rng.randrange(1, 4))]),
        "InternalTransactions": maybe(lambda: [{"Type": rng.randrange(2), "Peer": peer_spec(rng),
                                                "Signature": rng.choice(STRINGS + ["r|s"])}
                                               for _ in range(rng.randrange(1, 3))]),
        "Parents": rng.choice([None, ["", ""], ["0X" + _hx(rng, 32).upper(), ""],
                               ["0X" + _hx(rng, 32).upper(), "0X" + _hx(rng, 32).upper()]]),
        "Creator": None if rng.random() < 0.1 else _hx(rng, 65),
        "Index": rng.randrange(-2, 10**6),
        "BlockSignatures": maybe(lambda: [{"Validator": None if rng.random() < 0.2 else _hx(rng, 65),
                                           "Index": rng.randrange(100), "Signature": rng.choice(STRINGS)}
                                          for _ in range(rng.randrange(1, 3))]),
        "Timestamp": rng.randrange(-10**10, 10**10),
    }


def frame_event_spec(rng):
    if rng.random() < 0.05:
        return None
    return {"Core": None if rng.random() < 0.05 else {"Body": body_spec(rng), "Signature": rng.choice(STRINGS)},
            "Round": rng.randrange(-1, 50), "LamportTimestamp": rng.randrange(-1, 500),
            "Witness": rng.random() < 0.5}


def frame_spec(rng: random.Random):
    peers = [peer_spec(rng) for _ in range(rng.randrange(0, 6))]
    r = rng.random()
    roots = None if r < 0.15 else {
        ("0X" + _hx(rng, 65).upper() if rng.random() < 0.8 else rng.choice(STRINGS)):
            (None if rng.random() < 0.1 else {"Events": None if rng.random() < 0.1 else
                                              [frame_event_spec(rng) for _ in range(rng.randrange(0, 3))]})
        for _ in range(rng.randrange(0, 5))}
    psets = None if rng.random() < 0.15 else {
        rng.randrange(-3, 120): (None if rng.random() < 0.1 else
                                 [None if rng.random() < 0.05 else peer_spec(rng) for _ in range(rng.randrange(0, 4))])
        for _ in range(rng.randrange(0, 6))}
    return {"Round": rng.randrange(-1, 10**5),
            "Peers": None if rng.random() < 0.1 else [None if rng.random() < 0.05 else p for p in peers],
            "Roots": roots,
            "Events": None if rng.random() < 0.1 else [frame_event_spec(rng) for _ in range(rng.randrange(0, 5))],
            "PeerSets": psets,
            "Timestamp": rng.randrange(-10**12, 10**12)}


def _b(h):
    return None if h is None else bytes.fromhex(h)


def to_types(spec, m):
    """spec -> Frame of module namespace `m` (babble_amd.frame + hashgraph
    names, or oracle.gosemantics)."""
    P = lambda p: None if p is None else m.Peer(NetAddr=p["NetAddr"], PubKeyHex=p["PubKeyHex"],  # noqa: E731
                                                Moniker=p["Moniker"])

    def body(b):
        itxs = None if b["InternalTransactions"] is None else [
            m.InternalTransaction(Body=m.InternalTransactionBody(Type=t["Type"], Peer=P(t["Peer"])),
                                  Signature=t["Signature"]) for t in b["InternalTransactions"]]
        bs = None if b["BlockSignatures"] is None else [
            m.BlockSignature(Validator=_b(s["Validator"]), Index=s["Index"], Signature=s["Signature"])
            for s in b["BlockSignatures"]]
        txs = None if b["Transactions"] is None else [_b(t) for t in b["Transactions"]]
        return m.EventBody(Transactions=txs, InternalTransactions=itxs, Parents=b["Parents"], Creator=_b(b["Creator"]),
                           Index=b["Index"], BlockSignatures=bs, Timestamp=b["Timestamp"])

    def fe(e):
        if e is None:
            return None
        core = None if e["Core"] is None else m.Event(Body=body(e["Core"]["Body"]), Signature=e["Core"]["Signature"])
        return m.FrameEvent(Core=core, Round=e["Round"], LamportTimestamp=e["LamportTimestamp"], Witness=e["Witness"])

    def plist(ps):
        return None if ps is None else [P(p) for p in ps]

    roots = None if spec["Roots"] is None else {
        k: (None if r is None else m.Root(Events=None if r["Events"] is None else [fe(e) for e in r["Events"]]))
        for k, r in spec["Roots"].items()}
    psets = None if spec["PeerSets"] is None else {int(k): plist(v) for k, v in spec["PeerSets"].items()}
    return m.Frame(Round=spec["Round"], Peers=plist(spec["Peers"]), Roots=roots,
                   Events=None if spec["Events"] is None else [fe(e) for e in spec["Events"]], PeerSets=psets,
                   Timestamp=spec["Timestamp"])


class ProductNS:
    """The product mirror's type namespace (frame.py + hashgraph.py)."""

    def __init__(self):
        from babble_amd import frame as F
        from babble_amd import hashgraph as H

        for n in ("Peer", "InternalTransaction", "InternalTransactionBody", "BlockSignature", "EventBody", "Event"):
            setattr(self, n, getattr(H, n))
        for n in ("FrameEvent", "Root", "Frame"):
            setattr(self, n, getattr(F, n))
