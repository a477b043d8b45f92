"""Host-side mirror of the reference's Go interface for the verification path.

Same type names, fields and method semantics as sikoba/babble v0.8.4:
  Peer / PeerSet                 src/peers/peer.go, peer_set.go
  InternalTransaction(Body)      src/hashgraph/internal_transaction.go
  BlockBody / Block / BlockSignature  src/hashgraph/block.go
  EventBody / Event              src/hashgraph/event.go
  check_block / process_sig_pool / insert_event_verify / bootstrap
                                 src/hashgraph/hashgraph.go:1599-1630, 1295-1367, 672-687,
                                 1481-1536
Every hash and every signature check goes through libbabbleverify.so
(`Verifier`); there is no CPU path.  Go's panics are raised as
`ReferencePanic` by the single-object methods and reported as `panic=True`
outcomes by the batch functions (a batch cannot panic half way).

Batch entry points (what the cgo shim in INTEGRATION.md exposes to Go):
  verify_events(events)            -> [Outcome]   (Event.Verify for each)
  verify_block_signatures(b, sigs) -> [Outcome]   (Block.Verify for each)
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import gojson as J
from .batch import BatchBuilder
from .native import ACCEPT, REF_PANIC, REJECT, REJECT_ERR, ReferencePanic, hex_decode

_default = None


def default_verifier():
    """Process-wide Verifier on device 0 (created on first use)."""
    global _default
    if _default is None:
        from .verifier import Verifier

        _default = Verifier(0)
    return _default


def SHA256(data: bytes, verifier=None) -> bytes:
    """crypto.SHA256 (src/crypto/hash.go:8) on the device."""
    return (verifier or default_verifier()).sha256([data])[0]


def EncodeToString(b: bytes) -> str:
    """common.EncodeToString (src/common/hex.go:10-12)."""
    return "0X" + bytes(b).hex().upper()


def DecodeFromString(s) -> bytes:
    """common.DecodeFromString (hex.go:15-17) via bv_hex_decode; len < 2 panics."""
    return hex_decode(s)


@dataclass
class Outcome:
    """Result of one reference Verify call: (ok, err) or a Go panic."""
    ok: bool
    err: Optional[str] = None
    panic: bool = False


# ----------------------------------------------------------------------------
# peers
# ----------------------------------------------------------------------------
@dataclass
class Peer:
    NetAddr: str = ""
    PubKeyHex: str = ""
    Moniker: str = ""

    def PubKeyBytes(self) -> bytes:
        return DecodeFromString(self.PubKeyHex)

    def PubKeyString(self) -> str:
        return self.PubKeyHex.upper() if isinstance(self.PubKeyHex, str) else self.PubKeyHex.decode().upper()

    def json(self) -> bytes:
        return J.struct(("NetAddr", J.string(self.NetAddr)), ("PubKeyHex", J.string(self.PubKeyHex)),
                        ("Moniker", J.string(self.Moniker)))


class PeerSet:
    """peers.PeerSet: ordered peers + ByPubKey index (peer_set.go)."""

    def __init__(self, peers: Sequence[Peer]):
        self.Peers = list(peers)
        self.ByPubKey: Dict[str, Peer] = {p.PubKeyString(): p for p in self.Peers}
        self._hash: Optional[bytes] = None

    def Len(self) -> int:
        return len(self.ByPubKey)

    def Hash(self, verifier=None) -> bytes:
        """peer_set.go:104-115: h = SHA256(h || pubkey) over the peers in order."""
        if self._hash is None and not self.Peers:
            self._hash = b""  # h := []byte{} with nothing to chain
        if self._hash is None:
            v = verifier or default_verifier()
            pks = [p.PubKeyBytes() for p in self.Peers]
            if hasattr(v, "peer_set_hash"):  # the whole chain in one device launch
                self._hash = v.peer_set_hash(pks)
            else:
                h = b""
                for pk in pks:
                    h = SHA256(h + pk, v)
                self._hash = h
        return self._hash

    def TrustCount(self) -> int:
        """peer_set.go:168-177: ceil(n/3) when there is more than one peer."""
        return int(math.ceil(self.Len() / 3.0)) if len(self.Peers) > 1 else 0


# ----------------------------------------------------------------------------
# internal transactions, block signatures, blocks, events
# ----------------------------------------------------------------------------
@dataclass
class InternalTransactionBody:
    Type: int = 0
    Peer: Peer = field(default_factory=Peer)

    def Marshal(self) -> bytes:
        return J.struct(("Type", J.integer(self.Type)), ("Peer", self.Peer.json())) + b"\n"

    def Hash(self, verifier=None) -> bytes:
        return SHA256(self.Marshal(), verifier)


@dataclass
class InternalTransaction:
    Body: InternalTransactionBody = field(default_factory=InternalTransactionBody)
    Signature: str = ""

    def json(self) -> bytes:
        return J.struct(("Body", J.struct(("Type", J.integer(self.Body.Type)), ("Peer", self.Body.Peer.json()))),
                        ("Signature", J.string(self.Signature)))

    def Verify(self, verifier=None) -> Tuple[bool, Optional[str]]:
        """internal_transaction.go:139-154 (raises ReferencePanic where Go panics)."""
        return _single(verify_itxs([self], verifier)[0])


@dataclass
class InternalTransactionReceipt:
    InternalTransaction: InternalTransaction = field(default_factory=InternalTransaction)
    Accepted: bool = False

    def json(self) -> bytes:
        return J.struct(("InternalTransaction", self.InternalTransaction.json()),
                        ("Accepted", J.boolean(self.Accepted)))


@dataclass
class BlockSignature:
    Validator: Optional[bytes] = None
    Index: int = 0
    Signature: str = ""

    def ValidatorHex(self) -> str:
        return EncodeToString(self.Validator or b"")

    def Key(self) -> str:
        return "%d-%s" % (self.Index, self.ValidatorHex())

    def json(self) -> bytes:
        return J.struct(("Validator", J.byteslice(self.Validator)), ("Index", J.integer(self.Index)),
                        ("Signature", J.string(self.Signature)))


@dataclass
class BlockBody:
    Index: int = 0
    RoundReceived: int = 0
    Timestamp: int = 0
    StateHash: Optional[bytes] = None
    FrameHash: Optional[bytes] = None
    PeersHash: Optional[bytes] = None
    Transactions: Optional[List[Optional[bytes]]] = None
    InternalTransactions: Optional[List[InternalTransaction]] = None
    InternalTransactionReceipts: Optional[List[InternalTransactionReceipt]] = None

    def Marshal(self) -> bytes:
        return J.struct(
            ("Index", J.integer(self.Index)), ("RoundReceived", J.integer(self.RoundReceived)),
            ("Timestamp", J.integer(self.Timestamp)), ("StateHash", J.byteslice(self.StateHash)),
            ("FrameHash", J.byteslice(self.FrameHash)), ("PeersHash", J.byteslice(self.PeersHash)),
            ("Transactions", J.slice_(self.Transactions, J.byteslice)),
            ("InternalTransactions", J.slice_(self.InternalTransactions, lambda t: t.json())),
            ("InternalTransactionReceipts", J.slice_(self.InternalTransactionReceipts, lambda t: t.json())),
        ) + b"\n"

    def Hash(self, verifier=None) -> bytes:
        return SHA256(self.Marshal(), verifier)


@dataclass
class Block:
    Body: BlockBody = field(default_factory=BlockBody)
    Signatures: Dict[str, str] = field(default_factory=dict)  # validator hex -> signature

    def Index(self) -> int:
        return self.Body.Index

    def PeersHash(self) -> Optional[bytes]:
        return self.Body.PeersHash

    def GetSignatures(self) -> List[BlockSignature]:
        """block.go:241-253 (map iteration order: Python dict order here)."""
        return [BlockSignature(Validator=DecodeFromString(v), Index=self.Index(), Signature=s)
                for v, s in self.Signatures.items()]

    def SetSignature(self, bs: BlockSignature) -> None:
        self.Signatures[bs.ValidatorHex()] = bs.Signature

    def Verify(self, sig: BlockSignature, verifier=None) -> Tuple[bool, Optional[str]]:
        """block.go:343-357 (raises ReferencePanic where Go panics)."""
        return _single(verify_block_signatures(self, [sig], verifier)[0])


@dataclass
class EventBody:
    Transactions: Optional[List[Optional[bytes]]] = None
    InternalTransactions: Optional[List[InternalTransaction]] = None
    Parents: Optional[List[str]] = None
    Creator: Optional[bytes] = None
    Index: int = 0
    BlockSignatures: Optional[List[BlockSignature]] = None
    Timestamp: int = 0

    def Marshal(self) -> bytes:
        """EventBody.Marshal (event.go:38-45)."""
        return J.struct(
            ("Transactions", J.slice_(self.Transactions, J.byteslice)),
            ("InternalTransactions", J.slice_(self.InternalTransactions, lambda t: t.json())),
            ("Parents", J.slice_(self.Parents, J.string)), ("Creator", J.byteslice(self.Creator)),
            ("Index", J.integer(self.Index)), ("BlockSignatures", J.slice_(self.BlockSignatures, lambda t: t.json())),
            ("Timestamp", J.integer(self.Timestamp)),
        ) + b"\n"

    def Hash(self, verifier=None) -> bytes:
        return SHA256(self.Marshal(), verifier)


@dataclass
class Event:
    Body: EventBody = field(default_factory=EventBody)
    Signature: str = ""
    _hash: Optional[bytes] = None

    def Hash(self, verifier=None) -> bytes:
        if not self._hash:
            self._hash = self.Body.Hash(verifier)
        return self._hash

    def Hex(self, verifier=None) -> str:
        return EncodeToString(self.Hash(verifier))

    def Verify(self, verifier=None) -> Tuple[bool, Optional[str]]:
        """event.go:219-247 (raises ReferencePanic where Go panics)."""
        return _single(verify_events([self], verifier)[0])


def _single(o: Outcome) -> Tuple[bool, Optional[str]]:
    if o.panic:
        raise ReferencePanic(o.err or "reference panic")
    return o.ok, o.err


# ----------------------------------------------------------------------------
# batch verification (one bv_verify_batch per call)
# ----------------------------------------------------------------------------
def parts_error(sig) -> str:
    """keys.DecodeSignature's error (signature.go:31-35): strings.Split on
    "|" gave len(values) != 2.  The device reports only the status
    (REJECT_ERR); the part count is the host's, as in Go."""
    if isinstance(sig, (bytes, bytearray)):
        sig = bytes(sig).decode("utf-8", errors="surrogateescape")
    return "wrong number of values in signature: got %d, want 2" % (sig.count("|") + 1)


def _item_outcome(st: int, sig="") -> Outcome:
    """One item status as Go's (ok, err) / panic; `sig` is the item's
    signature text (for the REJECT_ERR message)."""
    if st == ACCEPT:
        return Outcome(True)
    if st == REJECT:
        return Outcome(False)
    if st == REJECT_ERR:
        return Outcome(False, parts_error(sig))
    return Outcome(False, "reference panic (nil pointer dereference)", panic=True)


def _add_itx(bb: BatchBuilder, itx: InternalTransaction) -> Optional[int]:
    """Item index for the ITX, or None if PubKeyBytes panics (len < 2)."""
    try:
        pub = itx.Body.Peer.PubKeyBytes()
    except ReferencePanic:
        return None
    m = bb.add_msg(itx.Body.Marshal())
    return bb.add_item(m, bb.add_key(pub), itx.Signature)


def verify_itxs(itxs: Sequence[InternalTransaction], verifier=None) -> List[Outcome]:
    bb = BatchBuilder()
    idx = [_add_itx(bb, t) for t in itxs]
    res = (verifier or default_verifier()).verify(bb.pack()) if bb._item_msg else None
    out = []
    for t, k in zip(itxs, idx):
        if k is None:
            out.append(Outcome(False, "slice bounds out of range", panic=True))
        else:
            out.append(_item_outcome(int(res.status[k]), t.Signature))
    return out


def verify_events(events: Sequence[Event], verifier=None) -> List[Outcome]:
    """Event.Verify for every event in one device batch.  Each event's digest
    is stored in its `_hash` (so Hex() does not hash again, cf. the second
    JSON+SHA-256 in initEventCoordinates, hashgraph.go:474-479)."""
    bb = BatchBuilder()
    plan = []  # per event: ([itx item or None], event item, msg index)
    for ev in events:
        itx_items = [_add_itx(bb, t) for t in (ev.Body.InternalTransactions or [])]
        m = bb.add_msg(ev.Body.Marshal())
        k = bb.add_key(ev.Body.Creator or b"")
        plan.append((itx_items, bb.add_item(m, k, ev.Signature), m))
    res = (verifier or default_verifier()).verify(bb.pack())
    out = []
    for ev, (itx_items, item, m) in zip(events, plan):
        ev._hash = res.msg_hash[m].tobytes()
        itx_st = [None if k is None else int(res.status[k]) for k in itx_items]
        out.append(compose_event_outcome(itx_st, int(res.status[item]),
                                         [t.Signature for t in (ev.Body.InternalTransactions or [])], ev.Signature))
    return out


def compose_event_outcome(itx_statuses: Sequence[Optional[int]], event_status: int,
                          itx_sigs: Sequence = (), event_sig="") -> Outcome:
    """Event.Verify's order (event.go:219-247): each ITX in order, the first
    failure wins (None = PubKeyBytes panicked); then the event signature.
    An ITX's DecodeSignature error is returned unchanged (event.go:223-225)."""
    for j, st in enumerate(itx_statuses):  # event.go:222-230
        if st is None:
            return Outcome(False, "slice bounds out of range", panic=True)
        if st == ACCEPT:
            continue
        if st in (REJECT_ERR, REF_PANIC):
            return _item_outcome(st, itx_sigs[j] if j < len(itx_sigs) else "")
        return Outcome(False, "invalid signature on internal transaction")
    return _item_outcome(event_status, event_sig)


def verify_block_signatures(block: Block, sigs: Sequence[BlockSignature], verifier=None) -> List[Outcome]:
    """Block.Verify for every signature: the body is hashed once, not per
    signature (block.go:344 re-hashes on every call)."""
    if not sigs:
        return []
    bb = BatchBuilder()
    m = bb.add_msg(block.Body.Marshal())
    items = [bb.add_item(m, bb.add_key(s.Validator or b""), s.Signature) for s in sigs]
    res = (verifier or default_verifier()).verify(bb.pack())
    return [_item_outcome(int(res.status[k]), s.Signature) for s, k in zip(sigs, items)]


def check_block(block: Block, peer_set: PeerSet, verifier=None) -> Optional[str]:
    """Hashgraph.CheckBlock (hashgraph.go:1599-1630): None or the error text."""
    # reflect.DeepEqual(psh, block.PeersHash()) (hashgraph.go:1605): the
    # computed hash is never nil ([]byte{} for an empty set), so a nil
    # PeersHash never matches, while an empty one matches an empty set
    bph = block.PeersHash()
    if bph is None or peer_set.Hash(verifier) != bph:
        return "Wrong PeerSet"
    sigs = [s for s in block.GetSignatures() if s.ValidatorHex() in peer_set.ByPubKey]
    outcomes = verify_block_signatures(block, sigs, verifier)
    if any(o.panic for o in outcomes):
        raise ReferencePanic("Block.Verify panics")
    valid = sum(1 for o in outcomes if o.ok)
    if valid <= peer_set.TrustCount():
        return "Not enough valid signatures: got %d, need %d" % (valid, peer_set.TrustCount())
    return None


def process_sig_pool(pending: Sequence[BlockSignature], get_block: Callable[[int], Optional[Block]],
                     get_peer_set: Callable[[int], Optional[PeerSet]], verifier=None):
    """Hashgraph.ProcessSigPool (hashgraph.go:1295-1367) over `pending` in the
    given (map) order.  Returns (appended signatures, error or None); a
    DecodeSignature error aborts the pool at that signature, as in Go.
    All candidate signatures are verified in one device batch first."""
    cands = []
    for bs in pending:
        blk = get_block(bs.Index)
        if blk is None:
            continue
        ps = get_peer_set(blk.Body.RoundReceived)
        if ps is None or bs.ValidatorHex() not in ps.ByPubKey:
            continue
        cands.append((bs, blk))
    bb = BatchBuilder()
    msg_of = {}
    items = []
    for bs, blk in cands:
        if id(blk) not in msg_of:
            msg_of[id(blk)] = bb.add_msg(blk.Body.Marshal())
        items.append(bb.add_item(msg_of[id(blk)], bb.add_key(bs.Validator or b""), bs.Signature))
    res = (verifier or default_verifier()).verify(bb.pack()) if items else None
    appended = []
    for (bs, blk), k in zip(cands, items):
        o = _item_outcome(int(res.status[k]), bs.Signature)
        if o.panic:
            raise ReferencePanic("Block.Verify panics")
        if o.err:
            return appended, o.err
        if not o.ok:
            continue
        blk.SetSignature(bs)
        appended.append(bs)
    return appended, None


def insert_event_verify(event: Event, outcome: Optional[Outcome] = None, verifier=None) -> Optional[str]:
    """The verify step of Hashgraph.InsertEvent (hashgraph.go:672-687):
    None if the event may be inserted, else the error text."""
    o = outcome or verify_events([event], verifier)[0]
    if o.panic:
        raise ReferencePanic(o.err or "reference panic")
    if not o.ok:
        return o.err if o.err else "Invalid Event signature %s" % event.Hex(verifier)
    return None


def bootstrap(topological_events: Callable[[int, int], List[Event]],
              insert_and_run_consensus: Callable[[Event], Optional[str]],
              process_sig_pool_step: Callable[[], Optional[str]], batch_size: int = 100,
              verify_window: int = 100_000, verifier=None) -> Optional[str]:
    """The event replay of Hashgraph.Bootstrap (hashgraph.go:1481-1536) with
    batched verification.  Go reads the DB in batches of 100 topological
    events, inserts each (InsertEventAndRunConsensus -> InsertEvent, whose
    first step is Event.Verify, hashgraph.go:672-687) and runs
    ProcessSigPool after every DB batch, returning the first error.

    Here DB batches are read ahead until `verify_window` events are pending
    and verified in ONE device batch; insertion, ProcessSigPool calls and
    the error that ends the replay happen in exactly Go's order (a DB read is
    a pure function of (offset, limit), so reading ahead changes nothing).
    `insert_and_run_consensus(ev)` is the caller's non-verify part of the
    insert (ancestry checks, consensus); it returns an error text or None.
    """
    index = 0
    done = False
    while not done:
        window: List[List[Event]] = []
        n = 0
        while n < verify_window:  # read ahead whole DB batches
            evs = topological_events(index * batch_size, batch_size)
            window.append(evs)
            n += len(evs)
            index += 1
            if len(evs) < batch_size:
                done = True
                break
        flat = [e for evs in window for e in evs]
        outcomes = verify_events(flat, verifier) if flat else []
        k = 0
        for evs in window:
            for ev in evs:
                err = insert_event_verify(ev, outcomes[k], verifier)
                k += 1
                if err is None:
                    err = insert_and_run_consensus(ev)
                if err is not None:
                    return err
            err = process_sig_pool_step()
            if err is not None:
                return err
    return None
