"""Fast-sync Frame hashing and the verification half of core.fastForward
 — host mirror of the Go types over the device verifier.

Reference (sikoba/babble v0.8.4):
  Frame / Frame.Marshal / Frame.Hash   src/hashgraph/frame.go:12-69
  Root                                 src/hashgraph/root.go:11-14
  FrameEvent                           src/hashgraph/event.go:455-463
  core.fastForward                     src/node/core.go:367-402
  Hashgraph.CheckBlock                 src/hashgraph/hashgraph.go:1599-1630
  PeerSet.Hash                         src/peers/peer_set.go:104-115

Frame.Marshal is NOT encoding/json: it is github.com/ugorji/go/codec v1.1.7
(go.mod:24) with a JsonHandle and Canonical = true.  Its output, restated
here for the types a Frame holds:
  * a struct is a JSON object of its exported fields ordered by field NAME
    (ugorji encodes struct-as-map from the name-sorted field list), e.g.
    Frame -> Events, PeerSets, Peers, Roots, Round, Timestamp;
  * a map is an object with its keys sorted (Canonical): map[string] by the
    key bytes, map[int] numerically, int keys written as quoted decimals;
  * nil pointer / slice / map -> null; []byte -> padded StdEncoding base64
    string (nil -> null); ints in decimal; bools true / false;
  * strings: `"` `\\` -> escaped, \\n \\r \\t \\b \\f short escapes, other
    bytes < 0x20 and the HTML characters < > & as \\u00XX, U+2028/U+2029 as
    \\u2028/\\u2029, invalid UTF-8 bytes -> \\ufffd;
  * no whitespace and no trailing newline (Encoder.Encode on a JsonHandle
    with TermWhitespace unset).
The oracle restates the same codec independently (schema-driven,
oracle/gosemantics.py: ugorji_*); tests/test_frame.py checks the two agree,
that the output is canonical JSON, and the committed golden frames.
Parity with ugorji itself is UNPINNED: no Go toolchain or ugorji module
exists in this container and the reference ships no serialized Frame.

The fast-forward check runs as ONE device batch: the anchor Block's body
with its validator signatures (CheckBlock) and the Frame's JSON (hashed only)
go to bv_verify_batch together; the PeerSet hash chain is one device launch
(bv_peer_set_hash).
"""
from __future__ import annotations

import base64
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

from . import gojson as J
from .batch import BatchBuilder
from .hashgraph import (Block, BlockSignature, Event, EventBody, InternalTransaction, Peer, PeerSet, ReferencePanic,
                        default_verifier, _item_outcome)

_HEX = b"0123456789abcdef"
_SHORT = {0x22: b'\\"', 0x5C: b"\\\\", 0x0A: b"\\n", 0x0D: b"\\r", 0x08: b"\\b", 0x0C: b"\\f", 0x09: b"\\t"}


def ustring(s) -> bytes:
    """ugorji jsonEncDriver string quoting (HTMLCharsAsIs = false)."""
    b = s.encode("utf-8") if isinstance(s, str) else bytes(s)
    out = bytearray(b'"')
    i = 0
    while i < len(b):
        c = b[i]
        if c < 0x80:
            if c in _SHORT:
                out += _SHORT[c]
            elif c < 0x20 or c in b"<>&":
                out += b"\\u00" + bytes([_HEX[c >> 4], _HEX[c & 15]])
            else:
                out.append(c)
            i += 1
            continue
        n = J._rune_len(b, i)
        if n == 0:
            out += b"\\ufffd"
            i += 1
        elif b[i:i + 3] in (b"\xe2\x80\xa8", b"\xe2\x80\xa9"):
            out += b"\\u2028" if b[i + 2] == 0xA8 else b"\\u2029"
            i += 3
        else:
            out += b[i:i + n]
            i += n
    out += b'"'
    return bytes(out)


def ubytes(b: Optional[bytes]) -> bytes:
    return b"null" if b is None else b'"' + base64.b64encode(bytes(b)) + b'"'


def uint(v: int) -> bytes:
    return b"%d" % int(v)


def ubool(v: bool) -> bytes:
    return b"true" if v else b"false"


def ulist(items, enc) -> bytes:
    return b"null" if items is None else b"[" + b",".join(enc(x) for x in items) + b"]"


def uptr(x, enc) -> bytes:
    return b"null" if x is None else enc(x)


def ustruct(**fields: bytes) -> bytes:
    """Exported fields as a JSON object in NAME order (ugorji sfiSort)."""
    return b"{" + b",".join(b'"' + k.encode() + b'":' + fields[k] for k in sorted(fields)) + b"}"


def upeer(p: Peer) -> bytes:
    return ustruct(NetAddr=ustring(p.NetAddr), PubKeyHex=ustring(p.PubKeyHex), Moniker=ustring(p.Moniker))


def uitx(t: InternalTransaction) -> bytes:
    return ustruct(Body=ustruct(Type=uint(t.Body.Type), Peer=upeer(t.Body.Peer)), Signature=ustring(t.Signature))


def ubsig(s: BlockSignature) -> bytes:
    return ustruct(Validator=ubytes(s.Validator), Index=uint(s.Index), Signature=ustring(s.Signature))


def ubody(b: EventBody) -> bytes:
    return ustruct(Transactions=ulist(b.Transactions, ubytes), InternalTransactions=ulist(b.InternalTransactions, uitx),
                   Parents=ulist(b.Parents, ustring), Creator=ubytes(b.Creator), Index=uint(b.Index),
                   BlockSignatures=ulist(b.BlockSignatures, ubsig), Timestamp=uint(b.Timestamp))


def uevent(e: Event) -> bytes:
    return ustruct(Body=ubody(e.Body), Signature=ustring(e.Signature))


@dataclass
class FrameEvent:
    """event.go:455-463."""
    Core: Optional[Event] = None
    Round: int = 0
    LamportTimestamp: int = 0
    Witness: bool = False

    def json(self) -> bytes:
        return ustruct(Core=uptr(self.Core, uevent), Round=uint(self.Round),
                       LamportTimestamp=uint(self.LamportTimestamp), Witness=ubool(self.Witness))


@dataclass
class Root:
    """root.go:11-14."""
    Events: Optional[List[Optional[FrameEvent]]] = None

    def json(self) -> bytes:
        return ustruct(Events=ulist(self.Events, lambda fe: uptr(fe, FrameEvent.json)))


def _peers(ps) -> bytes:
    return ulist(ps, lambda p: uptr(p, upeer))


@dataclass
class Frame:
    """frame.go:12-20."""
    Round: int = 0
    Peers: Optional[List[Optional[Peer]]] = None
    Roots: Optional[Dict[str, Optional[Root]]] = None
    Events: Optional[List[Optional[FrameEvent]]] = None
    PeerSets: Optional[Dict[int, Optional[List[Optional[Peer]]]]] = None
    Timestamp: int = 0

    def Marshal(self) -> bytes:
        """Frame.Marshal (frame.go:35-46): ugorji JsonHandle, Canonical."""
        roots = b"null" if self.Roots is None else b"{" + b",".join(
            ustring(k) + b":" + uptr(self.Roots[k], Root.json)
            for k in sorted(self.Roots, key=lambda k: k.encode("utf-8") if isinstance(k, str) else bytes(k))) + b"}"
        psets = b"null" if self.PeerSets is None else b"{" + b",".join(
            b'"%d":' % k + _peers(self.PeerSets[k]) for k in sorted(self.PeerSets)) + b"}"
        return ustruct(Round=uint(self.Round), Peers=_peers(self.Peers), Roots=roots,
                       Events=ulist(self.Events, lambda fe: uptr(fe, FrameEvent.json)), PeerSets=psets,
                       Timestamp=uint(self.Timestamp))

    def Hash(self, verifier=None) -> bytes:
        """Frame.Hash (frame.go:63-69): SHA256 of Marshal, on the device."""
        return (verifier or default_verifier()).sha256([self.Marshal()])[0]


def fast_forward_check(block: Block, frame: Frame, verifier=None) -> Optional[str]:
    """The verification half of core.fastForward (core.go:367-388): the
    Block's signatures against the Frame's peer set (Hashgraph.CheckBlock),
    then Frame.Hash against Block.FrameHash (reflect.DeepEqual).  Returns the
    first error text Go would return, or None (then Go goes on to
    Hashgraph.Reset).  One device batch carries the block body, every
    signature by a validator of the set, and the frame JSON."""
    v = verifier or default_verifier()
    peer_set = PeerSet([p for p in (frame.Peers or []) if p is not None])
    bph = block.PeersHash()
    if bph is None or peer_set.Hash(v) != bph:
        return "Wrong PeerSet"
    sigs = [s for s in block.GetSignatures() if s.ValidatorHex() in peer_set.ByPubKey]
    bb = BatchBuilder()
    m_block = bb.add_msg(block.Body.Marshal())
    m_frame = bb.add_msg(frame.Marshal())
    for s in sigs:
        bb.add_item(m_block, bb.add_key(s.Validator or b""), s.Signature)
    res = v.verify(bb.pack())
    outcomes = [_item_outcome(int(st), s.Signature) for st, s in zip(res.status, sigs)]
    if any(o.panic for o in outcomes):
        raise ReferencePanic("Block.Verify panics")
    valid = sum(1 for o in outcomes if o.ok)
    if valid <= peer_set.TrustCount():
        return "Not enough valid signatures: got %d, need %d" % (valid, peer_set.TrustCount())
    if block.Body.FrameHash is None or res.msg_hash[m_frame].tobytes() != block.Body.FrameHash:
        return "Invalid Frame Hash"
    return None


def frame_hashes(frames: Sequence[Frame], verifier=None) -> List[bytes]:
    """Frame.Hash of many frames in one device SHA-256 batch (one lane per
    frame), e.g. a replay that checks a frame per block."""
    return (verifier or default_verifier()).sha256([f.Marshal() for f in frames])
