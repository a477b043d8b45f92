"""core.sync ingest as one verification batch.

Reference semantics (sikoba/babble v0.8.4):
  core.sync                 src/node/core.go:210-271
  Hashgraph.ReadWireInfo    src/hashgraph/hashgraph.go:1538-1595
  WireBody / WireEvent      src/hashgraph/event.go:413-449
  InsertEvent verify step   src/hashgraph/hashgraph.go:672-687

`core.sync` walks a SyncResponse's WireEvents in (topological) order:
ReadWireInfo rebuilds each EventBody, resolving the two parent indices to
parent hex hashes through `Store.ParticipantEvent(creator, index)` — which
includes events inserted earlier in the same loop — and InsertEvent then
verifies the event (JSON + SHA-256 + ECDSA).  The first error ends the sync.

The body of an event embeds its parents' hashes, so hashing inside one
SyncResponse is ordered by DAG depth.  `read_wire_batch` resolves it level by
level: an event whose parents are all in the store is level 0; otherwise its
level is one more than its deepest in-batch parent.  Each level's bodies are
hashed in ONE device SHA-256 batch (bv_sha256_batch), and only events that
are parents of later events in the batch are hashed here at all.  Then
`sync_verify` verifies every rebuilt event in ONE bv_verify_batch (which
also returns the digests, stored in each Event so Hex() does not re-hash).

Parent resolution order: the store as it was before the sync, then earlier
events of the batch.  This equals the sequential loop: an in-batch event j
is only visible to a later event i in Go if j was inserted, which (short of
a NormalSelfParentError, i.e. the store already held that (creator, index))
means it was new to the store.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from . import gojson as J
from .hashgraph import (BlockSignature, Event, EventBody, InternalTransaction, Outcome, Peer, DecodeFromString,
                        EncodeToString, _item_outcome, default_verifier, verify_events, verify_itxs)


@dataclass
class WireBlockSignature:
    """event.go WireBlockSignature: Index + Signature (validator implied)."""
    Index: int = 0
    Signature: str = ""


@dataclass
class WireBody:
    """event.go:413-423."""
    Transactions: Optional[List[Optional[bytes]]] = None
    InternalTransactions: Optional[List[InternalTransaction]] = None
    BlockSignatures: Optional[List[WireBlockSignature]] = None
    CreatorID: int = 0
    OtherParentCreatorID: int = 0
    Index: int = 0
    SelfParentIndex: int = -1
    OtherParentIndex: int = -1
    Timestamp: int = 0


@dataclass
class WireEvent:
    """event.go:427-430."""
    Body: WireBody = field(default_factory=WireBody)
    Signature: str = ""

    def BlockSignatures(self, validator: bytes) -> Optional[List[BlockSignature]]:
        """event.go:433-449: nil stays nil."""
        if self.Body.BlockSignatures is None:
            return None
        return [BlockSignature(Validator=validator, Index=b.Index, Signature=b.Signature)
                for b in self.Body.BlockSignatures]


# participant_event(pubkey_string, index) -> hex hash or None (not found);
# the Store.ParticipantEvent of inmem_store.go:143-145 before the sync.
class StoreError(Exception):
    """common.StoreErr (src/common/store_errors.go:29-63): its Error() text is
    "<dataType>, <key>, <kind>" and ReadWireInfo returns it unchanged for a
    missing self-parent (hashgraph.go:1556-1559)."""

    KEY_NOT_FOUND, TOO_LATE, SKIPPED_INDEX, UNKNOWN_PARTICIPANT, EMPTY, KEY_ALREADY_EXISTS = range(6)
    _KIND = ("Not Found", "Too Late", "Skipped Index", "Unknown Participant", "Empty", "Key Already Exists")

    def __init__(self, data_type: str, err_type: int, key: str):
        super().__init__(data_type, err_type, key)
        self.data_type, self.err_type, self.key = data_type, err_type, key

    def __str__(self) -> str:
        return "%s, %s, %s" % (self.data_type, self.key, self._KIND[self.err_type])


# Store.ParticipantEvent (inmem_store.go:143-145 -> caches.go:84-95 ->
# rolling_index.go:55-66) before the sync: the hex hash, or the StoreError
# the store returns (None = a plain KeyNotFound).
ParticipantEvent = Callable[[str, int], object]


@dataclass
class WireRead:
    """ReadWireInfo outcome for one WireEvent: the Event or the error."""
    event: Optional[Event] = None
    err: Optional[str] = None


def _body(we: WireEvent, creator_bytes: bytes, self_parent: str, other_parent: str) -> EventBody:
    """hashgraph.go:1577-1588 (exported fields; the unexported wire ids are
    not part of the JSON)."""
    return EventBody(Transactions=we.Body.Transactions, InternalTransactions=we.Body.InternalTransactions,
                     BlockSignatures=we.BlockSignatures(creator_bytes), Parents=[self_parent, other_parent],
                     Creator=creator_bytes, Index=we.Body.Index, Timestamp=we.Body.Timestamp)


def read_wire_batch(wevents: Sequence[WireEvent], repertoire_by_id: Dict[int, Peer],
                    participant_event: ParticipantEvent, verifier=None) -> Tuple[List[WireRead], List[int]]:
    """ReadWireInfo for a whole SyncResponse.  Returns (reads, levels): one
    WireRead per WireEvent up to and including the first ReadWireInfo error
    (events after it are never read by core.sync and are returned as
    WireRead(None, None)), and each event's hashing level (-1 if not read)."""
    v = verifier or default_verifier()
    n = len(wevents)
    reads = [WireRead() for _ in range(n)]
    levels = [-1] * n
    pending, has_child, err_at, err = _resolve_batch(wevents, repertoire_by_id, participant_event)
    if err_at is not None:
        reads[err_at].err = err
    for i in range(n):
        if pending[i] is None:
            continue
        lvl = 0
        for p in pending[i][1]:
            if isinstance(p, int):
                lvl = max(lvl, levels[p] + 1)
        levels[i] = lvl

    hexes: Dict[int, str] = {}
    n_levels = max(levels) + 1 if n else 0
    for lvl in range(n_levels):
        idx = [i for i in range(n) if levels[i] == lvl]
        for i in idx:
            cb, ps = pending[i]
            ps = [hexes[p] if isinstance(p, int) else p for p in ps]
            reads[i].event = Event(Body=_body(wevents[i], cb, ps[0], ps[1]), Signature=wevents[i].Signature)
        need = [i for i in idx if has_child[i]]
        if need:  # one device SHA-256 batch per DAG level
            digests = v.sha256([reads[i].event.Body.Marshal() for i in need])
            for i, d in zip(need, digests):
                reads[i].event._hash = d
                hexes[i] = EncodeToString(d)
    return reads, levels


def _resolve_batch(wevents: Sequence[WireEvent], repertoire_by_id: Dict[int, Peer],
                   participant_event: ParticipantEvent):
    """ReadWireInfo's lookups for a whole SyncResponse, without hashing:
    (pending, has_child, err_at, err) where pending[i] = (creator bytes,
    [self, other]) with each parent "" / a store hex / an in-batch index, up
    to the first error (event err_at with Go's text err)."""
    n = len(wevents)
    pending: List[Optional[Tuple[bytes, List[object]]]] = [None] * n
    in_batch: Dict[Tuple[str, int], int] = {}
    has_child = [False] * n
    for i, we in enumerate(wevents):
        creator = repertoire_by_id.get(we.Body.CreatorID)
        if creator is None:
            return pending, has_child, i, "Creator %d not found" % we.Body.CreatorID
        cpk = creator.PubKeyString()
        creator_bytes = DecodeFromString(cpk)
        parents: List[object] = ["", ""]
        err = None
        if we.Body.SelfParentIndex >= 0:
            parents[0] = _resolve(cpk, we.Body.SelfParentIndex, participant_event, in_batch)
            if isinstance(parents[0], StoreError):
                err = str(parents[0])  # returned unchanged (hashgraph.go:1556-1559)
        if err is None and we.Body.OtherParentIndex >= 0:
            opc = repertoire_by_id.get(we.Body.OtherParentCreatorID)
            if opc is None:
                err = "Participant %d not found" % we.Body.OtherParentCreatorID
            else:
                parents[1] = _resolve(opc.PubKeyString(), we.Body.OtherParentIndex, participant_event, in_batch)
                if isinstance(parents[1], StoreError):
                    err = "OtherParent (creator: %d, index: %d) not found" % (we.Body.OtherParentCreatorID,
                                                                              we.Body.OtherParentIndex)
        if err is not None:
            return pending, has_child, i, err
        for p in parents:
            if isinstance(p, int):
                has_child[p] = True
        pending[i] = (creator_bytes, parents)
        in_batch.setdefault((cpk, we.Body.Index), i)
    return pending, has_child, None, None


def _resolve(pk: str, index: int, participant_event: ParticipantEvent, in_batch: Dict[Tuple[str, int], int]):
    """hex hash (store), in-batch event index, or the StoreError Go would see.
    Only a KeyNotFound can be satisfied by an event inserted earlier in the
    same sync; TooLate / UnknownParticipant stand as they are."""
    h = participant_event(pk, index)
    if isinstance(h, str):
        return h
    if h is None:
        h = StoreError("ParticipantEvents", StoreError.KEY_NOT_FOUND, str(index))
    if h.err_type == StoreError.KEY_NOT_FOUND and (pk, index) in in_batch:
        return in_batch[(pk, index)]
    return h


def sync_verify(wevents: Sequence[WireEvent], repertoire_by_id: Dict[int, Peer], participant_event: ParticipantEvent,
                verifier=None) -> Tuple[List[Event], List[Outcome], Optional[str]]:
    """The verification half of core.sync over one SyncResponse: returns
    (events, outcomes, read_err).  `events`/`outcomes` cover the WireEvents
    read before the first ReadWireInfo error (`read_err`, None if all were
    read); outcomes are Event.Verify results from ONE device batch, each
    event's digest cached in it.  The caller inserts in order and stops at
    the first non-ok outcome, as InsertEvent (hashgraph.go:672-687) and
    core.sync (core.go:214-231) do."""
    reads, _ = read_wire_batch(wevents, repertoire_by_id, participant_event, verifier)
    events: List[Event] = []
    read_err = None
    for r in reads:
        if r.err is not None:
            read_err = r.err
            break
        if r.event is None:
            break
        events.append(r.event)
    if not events:
        return [], [], read_err
    cached = [e._hash for e in events]
    outcomes = verify_events(events, verifier)
    for e, h in zip(events, cached):
        assert h is None or h == e._hash, "level hash disagrees with the verify batch digest"
    return events, outcomes, read_err


_HEX_RE = re.compile(r"0X[0-9A-F]{64}")


def sync_verify_device(wevents: Sequence[WireEvent], repertoire_by_id: Dict[int, Peer],
                       participant_event: ParticipantEvent,
                       verifier=None) -> Tuple[List[Event], List[Outcome], Optional[str]]:
    """sync_verify with the bodies built ON THE DEVICE (bv_verify_events): the
    resolved wire fields cross PCIe, the device serializes every EventBody,
    hashes the in-batch DAG level by level (narrow levels in one launch) and
    verifies every signature; events carrying InternalTransactions get their
    ITX items verified in one more bv_verify_batch (Event.Verify's order,
    event.go:222-230).  Same results as sync_verify (tests/test_sync.py).
    Falls back to sync_verify if a store hash is not a canonical Event.Hex()."""
    from .events import EventBatchBuilder

    v = verifier or default_verifier()
    pending, _, err_at, read_err = _resolve_batch(wevents, repertoire_by_id, participant_event)
    n = err_at if err_at is not None else len(wevents)
    if n == 0:
        return [], [], read_err
    if any(isinstance(p, str) and p and not _HEX_RE.fullmatch(p) for i in range(n) for p in pending[i][1]):
        return sync_verify(wevents, repertoire_by_id, participant_event, verifier)
    eb = EventBatchBuilder()
    bsigs = []
    for i in range(n):
        we = wevents[i]
        cb, ps = pending[i]
        par = [None if p == "" else ("event", p) if isinstance(p, int) else ("hash", bytes.fromhex(p[2:])) for p in ps]
        itxs = we.Body.InternalTransactions
        bs = we.BlockSignatures(cb)
        bsigs.append(bs)
        eb.add_event(eb.add_key(cb), we.Body.Index, we.Body.Timestamp, par, we.Body.Transactions, we.Signature,
                     itx_json=b"" if itxs is None else J.slice_(itxs, lambda t: t.json()),
                     bsig_json=b"" if bs is None else J.slice_(bs, lambda t: t.json()))
    res = v.verify_events(eb.pack())
    digests = [res.msg_hash[i].tobytes() for i in range(n)]
    itx_events = [i for i in range(n) if wevents[i].Body.InternalTransactions]
    itx_out = {}
    if itx_events:
        flat = [t for i in itx_events for t in wevents[i].Body.InternalTransactions]
        outs = verify_itxs(flat, v)
        k = 0
        for i in itx_events:
            m = len(wevents[i].Body.InternalTransactions)
            itx_out[i] = outs[k:k + m]
            k += m
    events, outcomes = [], []
    for i in range(n):
        cb, ps = pending[i]
        ps = [EncodeToString(digests[p]) if isinstance(p, int) else p for p in ps]
        we = wevents[i]
        ev = Event(Body=EventBody(Transactions=we.Body.Transactions, InternalTransactions=we.Body.InternalTransactions,
                                  BlockSignatures=bsigs[i], Parents=ps, Creator=cb, Index=we.Body.Index,
                                  Timestamp=we.Body.Timestamp), Signature=we.Signature)
        ev._hash = digests[i]
        events.append(ev)
        o = _item_outcome(int(res.status[i]), we.Signature)
        for io in itx_out.get(i, []):  # event.go:222-230: the first ITX failure wins
            if not io.ok or io.panic:
                o = io if (io.panic or io.err) else Outcome(False, "invalid signature on internal transaction")
                break
        outcomes.append(o)
    return events, outcomes, read_err
