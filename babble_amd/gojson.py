"""Go encoding/json (1.13) for the structs Babble hashes — host side.

In the Go integration these bytes come from Go itself (`json.Encoder.Encode`
in EventBody.Marshal, event.go:38-45; BlockBody.Marshal, block.go:29-36;
InternalTransactionBody.Marshal, internal_transaction.go:46-57).  This module
lets the Python mirror (babble_amd/hashgraph.py) produce the identical bytes:
exported fields in declaration order, `[]byte` as padded StdEncoding base64,
nil slice -> null / empty -> [] or "", strings HTML-escaped (<, >, & ->
\\u003c ...), U+2028/2029 escaped, invalid UTF-8 -> \\ufffd, trailing '\\n'.
tests/test_mirror.py checks it against the oracle's independent restatement.
"""
from __future__ import annotations

import base64
from typing import Callable, Optional, Sequence, Union

GoStr = Union[str, bytes]
_HEX = b"0123456789abcdef"
_SAFE = bytes(c for c in range(0x20, 0x80) if c not in b'"\\<>&')


def _rune_len(b: bytes, i: int) -> int:
    """Length of the valid UTF-8 sequence at b[i] (>= 2), or 0 if invalid."""
    c = b[i]
    if 0xC2 <= c <= 0xDF:
        n, lo, hi = 2, 0x80, 0xBF
    elif 0xE0 <= c <= 0xEF:
        n = 3
        lo, hi = {0xE0: (0xA0, 0xBF), 0xED: (0x80, 0x9F)}.get(c, (0x80, 0xBF))
    elif 0xF0 <= c <= 0xF4:
        n = 4
        lo, hi = {0xF0: (0x90, 0xBF), 0xF4: (0x80, 0x8F)}.get(c, (0x80, 0xBF))
    else:
        return 0
    if i + n > len(b) or not (lo <= b[i + 1] <= hi):
        return 0
    if any(not (0x80 <= b[i + k] <= 0xBF) for k in range(2, n)):
        return 0
    return n


def string(s: GoStr) -> bytes:
    b = s.encode("utf-8") if isinstance(s, str) else bytes(s)
    out = bytearray(b'"')
    i = 0
    while i < len(b):
        c = b[i]
        if c < 0x80:
            if c in _SAFE:
                out.append(c)
            elif c in (0x22, 0x5C):
                out += b"\\" + bytes([c])
            elif c == 0x0A:
                out += b"\\n"
            elif c == 0x0D:
                out += b"\\r"
            elif c == 0x09:
                out += b"\\t"
            else:
                out += b"\\u00" + bytes([_HEX[c >> 4], _HEX[c & 15]])
            i += 1
            continue
        n = _rune_len(b, i)
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


def byteslice(b: Optional[bytes]) -> bytes:
    return b"null" if b is None else b'"' + base64.b64encode(bytes(b)) + b'"'


def integer(v: int) -> bytes:
    return b"%d" % int(v)


def boolean(v: bool) -> bytes:
    return b"true" if v else b"false"


def slice_(items: Optional[Sequence], enc: Callable) -> bytes:
    return b"null" if items is None else b"[" + b",".join(enc(x) for x in items) + b"]"


def struct(*fields) -> bytes:
    """fields: (name, encoded value bytes) in declaration order."""
    return b"{" + b",".join(b'"' + n.encode() + b'":' + v for n, v in fields) + b"}"
