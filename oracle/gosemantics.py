"""CPU ORACLE — test infrastructure only, never the product path.

Pure-Python restatement of the Go semantics that decide Babble's
event-ingestion verification (reference v0.8.4 at /root/reference, Go).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker.

Parity status:
  * SHA-256: pinned by FIPS 180-4 known answers + hashlib (tests/test_oracle.py).
  * secp256k1 ECDSA math: pinned against OpenSSL libcrypto (independent
    implementation of the same standard) on every well-formed golden item.
  * Go-specific edge semantics (encoding/json, math/big base-36, hex decode,
    elliptic.Unmarshal, ecdsa.Verify panic/short-circuit order): restated from
    the pinned upstream versions (Go 1.13 stdlib, btcec 16327141da8c); the
    reference ships no golden vectors and Go is absent here, so these rows are
    "parity unpinned" by the reference itself.

Reference call sites followed (paths relative to /root/reference):
  src/crypto/hash.go:8-22                SHA256, SimpleHashFromTwoHashes
  src/crypto/keys/signature.go:20-39     Verify, EncodeSignature, DecodeSignature
  src/crypto/keys/public_key.go:14-20    ToPublicKey (elliptic.Unmarshal)
  src/crypto/keys/curve.go:13-22         secp256k1N, curve()
  src/common/hex.go:10-17                EncodeToString / DecodeFromString
  src/hashgraph/event.go:21-64,219-247   EventBody JSON/Hash, Event.Verify
  src/hashgraph/internal_transaction.go:40-65,139-154
  src/hashgraph/block.go:16-66,343-357   BlockBody JSON/Hash, Block.Verify
  src/hashgraph/hashgraph.go:1295-1367,1599-1630  ProcessSigPool, CheckBlock
  src/peers/peer.go:51-54, peer_set.go:104-115,168-177
"""
from __future__ import annotations

import base64
import hashlib
import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple, Union

# ----------------------------------------------------------------------------
# secp256k1 constants (btcec S256(); curve.go:13 for N)
# ----------------------------------------------------------------------------
P = 2**256 - 2**32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8
B = 7

# Item statuses (SURVEY §8a-9 decision table); shared with include/babbleverify.h
REJECT = 0
ACCEPT = 1
REJECT_ERR = 2   # DecodeSignature returned an error (parts != 2)
REF_PANIC = 3    # the Go reference would panic (nil deref / slice bounds)

# Host pre-class of one r or s value (bv_batch.pre encoding, see babbleverify.h)
SC_OK = 0        # parsed, 0 < v < N
SC_NIL = 1       # big.Int SetString failed -> nil pointer
SC_NONPOS = 2    # parsed, v <= 0
SC_GE_N = 3      # parsed, v >= N (possibly > 2^256)

GoStr = Union[str, bytes]


def _b(s: GoStr) -> bytes:
    return s.encode("utf-8") if isinstance(s, str) else bytes(s)


# ----------------------------------------------------------------------------
# crypto.SHA256 (src/crypto/hash.go:8) — FIPS 180-4, restated in pure Python
# so the oracle does not depend on the thing it is checked against.
# ----------------------------------------------------------------------------
_K256 = [
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2,
]
_H0 = [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19]


def sha256_fips(data: bytes) -> bytes:
    def rotr(x, n):
        return ((x >> n) | (x << (32 - n))) & 0xFFFFFFFF

    msg = bytes(data) + b"\x80"
    msg += b"\x00" * ((56 - len(msg) % 64) % 64)
    msg += (8 * len(data)).to_bytes(8, "big")
    h = list(_H0)
    for off in range(0, len(msg), 64):
        w = [int.from_bytes(msg[off + 4 * i: off + 4 * i + 4], "big") for i in range(16)]
        for i in range(16, 64):
            s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3)
            s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10)
            w.append((w[i - 16] + s0 + w[i - 7] + s1) & 0xFFFFFFFF)
        a, b_, c, d, e, f, g, hh = h
        for i in range(64):
            s1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)
            ch = (e & f) ^ (~e & g)
            t1 = (hh + s1 + ch + _K256[i] + w[i]) & 0xFFFFFFFF
            s0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)
            maj = (a & b_) ^ (a & c) ^ (b_ & c)
            t2 = (s0 + maj) & 0xFFFFFFFF
            hh, g, f, e, d, c, b_, a = g, f, e, (d + t1) & 0xFFFFFFFF, c, b_, a, (t1 + t2) & 0xFFFFFFFF
        h = [(x + y) & 0xFFFFFFFF for x, y in zip(h, [a, b_, c, d, e, f, g, hh])]
    return b"".join(x.to_bytes(4, "big") for x in h)


def SHA256(data: bytes) -> bytes:
    """crypto.SHA256 (hash.go:8-13). hashlib for speed; sha256_fips pins it in tests."""
    return hashlib.sha256(data).digest()


def SimpleHashFromTwoHashes(left: bytes, right: bytes) -> bytes:
    """crypto.SimpleHashFromTwoHashes (hash.go:17-22)."""
    return hashlib.sha256(bytes(left) + bytes(right)).digest()


# ----------------------------------------------------------------------------
# common/hex.go:10-17 and Go encoding/hex (1.13) DecodeString
# ----------------------------------------------------------------------------
def EncodeToString(b: bytes) -> str:
    """common.EncodeToString: "0X" + UPPERCASE hex (hex.go:10-12)."""
    return "0X" + bytes(b).hex().upper()


def _from_hex_char(c: int) -> Optional[int]:
    if 0x30 <= c <= 0x39:
        return c - 0x30
    if 0x61 <= c <= 0x66:
        return c - 0x61 + 10
    if 0x41 <= c <= 0x46:
        return c - 0x41 + 10
    return None


def go_hex_decode_string(s: GoStr) -> Tuple[bytes, bool]:
    """encoding/hex.DecodeString: returns (bytes decoded before the first error, ok).

    Go returns src[:n] together with the error; callers in Babble ignore the
    error (peer.go:51-54), so the partial prefix is what they use.
    """
    src = _b(s)
    out = bytearray()
    for i in range(len(src) // 2):
        a = _from_hex_char(src[2 * i])
        if a is None:
            return bytes(out), False
        b_ = _from_hex_char(src[2 * i + 1])
        if b_ is None:
            return bytes(out), False
        out.append((a << 4) | b_)
    if len(src) % 2 == 1:
        return bytes(out), False
    return bytes(out), True


class ReferencePanic(Exception):
    """Raised where the Go reference would panic (unrecovered in Babble)."""


def DecodeFromString(s: GoStr) -> bytes:
    """common.DecodeFromString (hex.go:15-17): hex.DecodeString(s[2:]).

    len(s) < 2 panics in Go (slice bounds out of range).
    """
    sb = _b(s)
    if len(sb) < 2:
        raise ReferencePanic("slice bounds out of range in DecodeFromString")
    return go_hex_decode_string(sb[2:])[0]


# ----------------------------------------------------------------------------
# math/big Int.SetString(s, 36) (Go 1.13 natconv.go / intconv.go)
# ----------------------------------------------------------------------------
def go_big_setstring36(s: GoStr) -> Optional[int]:
    """Returns the parsed integer, or None where Go returns (nil, false).

    Rules: optional single leading '+'/'-'; digits 0-9a-zA-Z (case-insensitive
    for base <= 36); no underscores (only legal for base 0); at least one digit;
    the whole string must be consumed.
    """
    sb = _b(s)
    if len(sb) == 0:
        return None  # scanSign: ReadByte -> io.EOF -> error
    i = 0
    neg = False
    if sb[0] == 0x2D:  # '-'
        neg = True
        i = 1
    elif sb[0] == 0x2B:  # '+'
        i = 1
    val = 0
    count = 0
    while i < len(sb):
        c = sb[i]
        if 0x30 <= c <= 0x39:
            d = c - 0x30
        elif 0x61 <= c <= 0x7A:
            d = c - 0x61 + 10
        elif 0x41 <= c <= 0x5A:
            d = c - 0x41 + 10
        else:
            break
        val = val * 36 + d
        count += 1
        i += 1
    if count == 0:
        return None  # errNoDigits
    if i != len(sb):
        return None  # entire content must be consumed
    return -val if (neg and val != 0) else val


def go_big_text36(v: int) -> str:
    """big.Int.Text(36): lowercase, no leading zeros, '-' for negatives."""
    if v == 0:
        return "0"
    digs = "0123456789abcdefghijklmnopqrstuvwxyz"
    neg = v < 0
    v = abs(v)
    out = []
    while v:
        v, r = divmod(v, 36)
        out.append(digs[r])
    return ("-" if neg else "") + "".join(reversed(out))


def EncodeSignature(r: int, s: int) -> str:
    """keys.EncodeSignature (signature.go:25-27)."""
    return go_big_text36(r) + "|" + go_big_text36(s)


def DecodeSignature(sig: GoStr) -> Tuple[Optional[int], Optional[int], bool]:
    """keys.DecodeSignature (signature.go:31-39) -> (r, s, parts_ok).

    strings.Split on '|' must give exactly 2 parts, else an error (parts_ok
    False). Each part: SetString(part, 36) with the error ignored (None = nil).
    """
    parts = _b(sig).split(b"|")
    if len(parts) != 2:
        return None, None, False
    return go_big_setstring36(parts[0]), go_big_setstring36(parts[1]), True


def DecodeSignatureError(sig: GoStr) -> Optional[str]:
    """The error value of keys.DecodeSignature (signature.go:33-35), None when
    strings.Split gives exactly 2 parts."""
    n = len(_b(sig).split(b"|"))
    return None if n == 2 else "wrong number of values in signature: got %d, want 2" % n


def scalar_class(v: Optional[int]) -> int:
    if v is None:
        return SC_NIL
    if v <= 0:
        return SC_NONPOS
    if v >= N:
        return SC_GE_N
    return SC_OK


# ----------------------------------------------------------------------------
# secp256k1 group law (btcec S256 semantics: infinity represented as (0,0))
# ----------------------------------------------------------------------------
INF = None


def _inv(a: int, m: int) -> int:
    return pow(a, -1, m)


def point_add(p1, p2):
    """Affine group law incl. P+P (doubling) and P+(-P)=inf (btcec Add semantics)."""
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    x1, y1 = p1
    x2, y2 = p2
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = (3 * x1 * x1) * _inv(2 * y1, P) % P
    else:
        lam = (y2 - y1) * _inv(x2 - x1, P) % P
    x3 = (lam * lam - x1 - x2) % P
    y3 = (lam * (x1 - x3) - y1) % P
    return (x3, y3)


def _jac_double(X, Y, Z):
    if Z == 0 or Y == 0:
        return (0, 1, 0)
    A = X * X % P
    Bv = Y * Y % P
    C = Bv * Bv % P
    D = 2 * ((X + Bv) ** 2 - A - C) % P
    E = 3 * A % P
    F = E * E % P
    X3 = (F - 2 * D) % P
    Y3 = (E * (D - X3) - 8 * C) % P
    Z3 = 2 * Y * Z % P
    return (X3, Y3, Z3)


def _jac_add_affine(X1, Y1, Z1, x2, y2):
    if Z1 == 0:
        return (x2, y2, 1)
    Z1Z1 = Z1 * Z1 % P
    U2 = x2 * Z1Z1 % P
    S2 = y2 * Z1 * Z1Z1 % P
    H = (U2 - X1) % P
    R = (S2 - Y1) % P
    if H == 0:
        if R == 0:
            return _jac_double(X1, Y1, Z1)
        return (0, 1, 0)
    HH = H * H % P
    HHH = H * HH % P
    V = X1 * HH % P
    X3 = (R * R - HHH - 2 * V) % P
    Y3 = (R * (V - X3) - Y1 * HHH) % P
    Z3 = Z1 * H % P
    return (X3, Y3, Z3)


def scalar_mult(k: int, pt):
    """k*pt for an affine point (None = infinity); returns affine or None."""
    if pt is None or k % N == 0:
        return None
    X, Y, Z = 0, 1, 0
    for bit in bin(k)[2:]:
        X, Y, Z = _jac_double(X, Y, Z)
        if bit == "1":
            X, Y, Z = _jac_add_affine(X, Y, Z, pt[0], pt[1])
    if Z == 0:
        return None
    zi = _inv(Z, P)
    return (X * zi * zi % P, Y * zi * zi * zi % P)


G = (GX, GY)


def is_on_curve(x: int, y: int) -> bool:
    return (y * y - (x * x * x + B)) % P == 0


def Unmarshal(pub: bytes) -> Optional[Tuple[int, int]]:
    """elliptic.Unmarshal(btcec.S256(), b) (Go 1.13): (x, y) or None for (nil, nil)."""
    pub = bytes(pub)
    if len(pub) != 65 or pub[0] != 4:
        return None
    x = int.from_bytes(pub[1:33], "big")
    y = int.from_bytes(pub[33:65], "big")
    if x >= P or y >= P:
        return None
    if not is_on_curve(x, y):
        return None
    return (x, y)


def Marshal(pt: Tuple[int, int]) -> bytes:
    """elliptic.Marshal uncompressed form (keys.FromPublicKey, public_key.go:25-30)."""
    return b"\x04" + pt[0].to_bytes(32, "big") + pt[1].to_bytes(32, "big")


# ----------------------------------------------------------------------------
# The verification decision, one signature item.
# ----------------------------------------------------------------------------
def ecdsa_math(q: Tuple[int, int], digest: bytes, r: int, s: int) -> bool:
    """ecdsa.Verify steps 4-10 (Go 1.13 generic path over btcec): r, s in [1, N-1]."""
    e = int.from_bytes(digest, "big")  # hashToInt: 256-bit digest, no truncation, no reduction
    w = _inv(s, N)
    u1 = e * w % N
    u2 = r * w % N
    p1 = scalar_mult(u1, G)      # ScalarBaseMult(u1.Bytes()); u1 = 0 -> (0,0)
    p2 = scalar_mult(u2, q)      # ScalarMult(Q, u2.Bytes())
    R = point_add(p1, p2)        # btcec Add: inf identity, doubling, P+(-P)=inf
    if R is None:
        return False             # x.Sign()==0 && y.Sign()==0
    return R[0] % N == r


def item_status(pub: bytes, digest: bytes, r: Optional[int], s: Optional[int],
                parts_ok: bool = True) -> int:
    """Final status of one (pubkey bytes, digest, decoded r, s) item.

    Order (event.go:219-247 -> signature.go:20 -> ecdsa.Verify):
      DecodeSignature error                 -> REJECT_ERR (returned before Verify)
      len(pub)==0 -> ToPublicKey nil        -> panic at pub.Curve
      r nil -> r.Sign() nil deref           -> panic;  r<=0 -> false
      s nil                                  -> panic;  s<=0 -> false
      r>=N || s>=N                           -> false
      pub malformed (X nil) -> ScalarMult   -> panic
      R = inf -> false; x(R) mod N == r.
    """
    if not parts_ok:
        return REJECT_ERR
    if len(pub) == 0:
        return REF_PANIC
    if r is None:
        return REF_PANIC
    if r <= 0:
        return REJECT
    if s is None:
        return REF_PANIC
    if s <= 0:
        return REJECT
    if r >= N or s >= N:
        return REJECT
    q = Unmarshal(pub)
    if q is None:
        return REF_PANIC
    return ACCEPT if ecdsa_math(q, digest, r, s) else REJECT


def item_status_from_sigstr(pub: bytes, digest: bytes, sig: GoStr) -> int:
    r, s, ok = DecodeSignature(sig)
    return item_status(pub, digest, r, s, ok)


def status_from_classes(pub: bytes, digest: bytes, parts_ok: bool, rc: int, sc: int,
                        r_val: int, s_val: int) -> int:
    """Same decision, from the pre-class encoding the C-ABI carries."""
    if not parts_ok:
        return REJECT_ERR
    if len(pub) == 0:
        return REF_PANIC
    if rc == SC_NIL:
        return REF_PANIC
    if rc == SC_NONPOS:
        return REJECT
    if sc == SC_NIL:
        return REF_PANIC
    if sc == SC_NONPOS:
        return REJECT
    if rc == SC_GE_N or sc == SC_GE_N:
        return REJECT
    q = Unmarshal(pub)
    if q is None:
        return REF_PANIC
    return ACCEPT if ecdsa_math(q, digest, r_val, s_val) else REJECT


# ----------------------------------------------------------------------------
# Go encoding/json (1.13) restatement for the hashed structs.
# ----------------------------------------------------------------------------
_HEX = b"0123456789abcdef"


def json_string(s: GoStr) -> bytes:
    """encodeState.string with escapeHTML=true (json.Encoder default)."""
    src = _b(s)
    out = bytearray(b'"')
    i = 0
    n = len(src)
    while i < n:
        c = src[i]
        if c < 0x80:
            if c >= 0x20 and c not in (0x22, 0x5C, 0x3C, 0x3E, 0x26):
                out.append(c)
            elif c == 0x22:
                out += b'\\"'
            elif c == 0x5C:
                out += b"\\\\"
            elif c == 0x0A:
                out += b"\\n"
            elif c == 0x0D:
                out += b"\\r"
            elif c == 0x09:
                out += b"\\t"
            else:
                out += b"\\u00" + bytes([_HEX[c >> 4], _HEX[c & 0xF]])
            i += 1
            continue
        # multi-byte: decode one rune the way utf8.DecodeRune does
        size, ok = _utf8_rune(src, i)
        if not ok:
            out += b"\\ufffd"
            i += 1
            continue
        rune_bytes = src[i:i + size]
        if rune_bytes == b"\xe2\x80\xa8":
            out += b"\\u2028"
        elif rune_bytes == b"\xe2\x80\xa9":
            out += b"\\u2029"
        else:
            out += rune_bytes
        i += size
    out += b'"'
    return bytes(out)


def _utf8_rune(src: bytes, i: int) -> Tuple[int, bool]:
    """utf8.DecodeRune validity (RuneError, size 1 on invalid)."""
    c0 = src[i]
    n = len(src)
    if c0 < 0xC2 or c0 > 0xF4:
        return 1, False
    if c0 < 0xE0:
        need, lo, hi = 1, 0x80, 0xBF
    elif c0 < 0xF0:
        need = 2
        lo, hi = (0xA0, 0xBF) if c0 == 0xE0 else ((0x80, 0x9F) if c0 == 0xED else (0x80, 0xBF))
    else:
        need = 3
        lo, hi = (0x90, 0xBF) if c0 == 0xF0 else ((0x80, 0x8F) if c0 == 0xF4 else (0x80, 0xBF))
    if i + need >= n:  # truncated sequence
        return 1, False
    c1 = src[i + 1]
    if not (lo <= c1 <= hi):
        return 1, False
    for k in range(2, need + 1):
        if not (0x80 <= src[i + k] <= 0xBF):
            return 1, False
    return need + 1, True


def json_bytes(b: Optional[bytes]) -> bytes:
    """[]byte: nil -> null, else StdEncoding base64 with padding."""
    if b is None:
        return b"null"
    return b'"' + base64.b64encode(bytes(b)) + b'"'


def json_int(v: int) -> bytes:
    return str(int(v)).encode()


def json_list(items: Optional[Sequence], enc) -> bytes:
    if items is None:
        return b"null"
    return b"[" + b",".join(enc(x) for x in items) + b"]"


@dataclass
class Peer:
    """peers.Peer (peer.go:13-23); id is unexported and not serialized."""
    NetAddr: GoStr = ""
    PubKeyHex: GoStr = ""
    Moniker: GoStr = ""

    def PubKeyBytes(self) -> bytes:
        return DecodeFromString(self.PubKeyHex)

    def json(self) -> bytes:
        return (b'{"NetAddr":' + json_string(self.NetAddr) + b',"PubKeyHex":' + json_string(self.PubKeyHex)
                + b',"Moniker":' + json_string(self.Moniker) + b"}")


@dataclass
class InternalTransactionBody:
    Type: int = 0
    Peer: Peer = field(default_factory=Peer)

    def json(self) -> bytes:
        return b'{"Type":' + json_int(self.Type) + b',"Peer":' + self.Peer.json() + b"}"

    def Marshal(self) -> bytes:
        return self.json() + b"\n"

    def Hash(self) -> bytes:
        return SHA256(self.Marshal())


@dataclass
class InternalTransaction:
    Body: InternalTransactionBody = field(default_factory=InternalTransactionBody)
    Signature: GoStr = ""

    def json(self) -> bytes:
        return b'{"Body":' + self.Body.json() + b',"Signature":' + json_string(self.Signature) + b"}"


@dataclass
class InternalTransactionReceipt:
    InternalTransaction: InternalTransaction = field(default_factory=InternalTransaction)
    Accepted: bool = False

    def json(self) -> bytes:
        return (b'{"InternalTransaction":' + self.InternalTransaction.json() + b',"Accepted":'
                + (b"true" if self.Accepted else b"false") + b"}")


@dataclass
class BlockSignature:
    Validator: Optional[bytes] = None
    Index: int = 0
    Signature: GoStr = ""

    def json(self) -> bytes:
        return (b'{"Validator":' + json_bytes(self.Validator) + b',"Index":' + json_int(self.Index)
                + b',"Signature":' + json_string(self.Signature) + b"}")


@dataclass
class EventBody:
    """hashgraph.EventBody (event.go:21-35); exported fields in declaration order."""
    Transactions: Optional[List[Optional[bytes]]] = None
    InternalTransactions: Optional[List[InternalTransaction]] = None
    Parents: Optional[List[GoStr]] = None
    Creator: Optional[bytes] = None
    Index: int = 0
    BlockSignatures: Optional[List[BlockSignature]] = None
    Timestamp: int = 0

    def Marshal(self) -> bytes:
        """EventBody.Marshal (event.go:38-45): json.Encoder.Encode -> trailing '\\n'."""
        return (b'{"Transactions":' + json_list(self.Transactions, json_bytes)
                + b',"InternalTransactions":' + json_list(self.InternalTransactions, lambda t: t.json())
                + b',"Parents":' + json_list(self.Parents, json_string)
                + b',"Creator":' + json_bytes(self.Creator)
                + b',"Index":' + json_int(self.Index)
                + b',"BlockSignatures":' + json_list(self.BlockSignatures, lambda t: t.json())
                + b',"Timestamp":' + json_int(self.Timestamp) + b"}\n")

    def Hash(self) -> bytes:
        return SHA256(self.Marshal())


@dataclass
class BlockBody:
    """hashgraph.BlockBody (block.go:16-26)."""
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
        return (b'{"Index":' + json_int(self.Index) + b',"RoundReceived":' + json_int(self.RoundReceived)
                + b',"Timestamp":' + json_int(self.Timestamp)
                + b',"StateHash":' + json_bytes(self.StateHash)
                + b',"FrameHash":' + json_bytes(self.FrameHash)
                + b',"PeersHash":' + json_bytes(self.PeersHash)
                + b',"Transactions":' + json_list(self.Transactions, json_bytes)
                + b',"InternalTransactions":' + json_list(self.InternalTransactions, lambda t: t.json())
                + b',"InternalTransactionReceipts":'
                + json_list(self.InternalTransactionReceipts, lambda t: t.json()) + b"}\n")

    def Hash(self) -> bytes:
        return SHA256(self.Marshal())


# ----------------------------------------------------------------------------
# Composite verifications (reference control flow)
# ----------------------------------------------------------------------------
EV_REJECT = 0       # (false, nil)
EV_ACCEPT = 1       # (true, nil)
EV_ERR = 2          # (false, err) from DecodeSignature (event or ITX)
EV_PANIC = 3        # reference panics
EV_ITX_INVALID = 4  # (false, "invalid signature on internal transaction")


def itx_status(itx: InternalTransaction) -> int:
    """InternalTransaction.Verify (internal_transaction.go:139-154)."""
    try:
        pub = itx.Body.Peer.PubKeyBytes()       # may panic (len(PubKeyHex) < 2)
    except ReferencePanic:
        return REF_PANIC
    digest = itx.Body.Hash()
    return item_status_from_sigstr(pub, digest, itx.Signature)


def event_status(body: EventBody, signature: GoStr) -> int:
    """Event.Verify (event.go:219-247) folded to one code."""
    for itx in body.InternalTransactions or []:
        st = itx_status(itx)
        if st == ACCEPT:
            continue
        if st == REJECT_ERR:
            return EV_ERR
        if st == REF_PANIC:
            return EV_PANIC
        return EV_ITX_INVALID
    pub = body.Creator if body.Creator is not None else b""
    st = item_status_from_sigstr(pub, body.Hash(), signature)
    return {ACCEPT: EV_ACCEPT, REJECT: EV_REJECT, REJECT_ERR: EV_ERR, REF_PANIC: EV_PANIC}[st]


def event_verify_error(body: EventBody, signature: GoStr) -> Optional[str]:
    """The error Event.Verify returns for EV_ERR (event.go:222-247): the
    first failing ITX's DecodeSignature error, else the event's own."""
    for itx in body.InternalTransactions or []:
        st = itx_status(itx)
        if st == ACCEPT:
            continue
        return DecodeSignatureError(itx.Signature) if st == REJECT_ERR else None
    return DecodeSignatureError(signature)


def peer_set_hash(peers: Sequence[Peer]) -> bytes:
    """PeerSet.Hash (peer_set.go:104-115): h = SHA256(h || pubkey) over peers in order."""
    h = b""
    for p in peers:
        h = SimpleHashFromTwoHashes(h, p.PubKeyBytes())
    return h


def trust_count(n_peers: int) -> int:
    """PeerSet.TrustCount (peer_set.go:168-177)."""
    return int(math.ceil(n_peers / 3.0)) if n_peers > 1 else 0


def check_block(body: BlockBody, signatures: Sequence[Tuple[str, GoStr]], peers: Sequence[Peer]) -> Tuple[bool, int]:
    """Hashgraph.CheckBlock (hashgraph.go:1599-1630) -> (ok, valid_count).

    `signatures` is the Block.Signatures map as (validatorHex, sig) pairs in the
    iteration order the caller chose (the count does not depend on the order,
    since errors count as invalid). A panicking Verify would crash the node;
    it is reported as ReferencePanic.
    """
    # reflect.DeepEqual(psh, block.PeersHash()) (hashgraph.go:1605):
    # psh is []byte{} (non-nil) for an empty set, so a nil PeersHash never
    # matches and an empty one matches only the empty set
    if body.PeersHash is None or peer_set_hash(peers) != body.PeersHash:
        return False, 0
    by_pub = {EncodeToString(p.PubKeyBytes()) for p in peers}
    digest = body.Hash()
    valid = 0
    for vhex, sig in signatures:
        validator = DecodeFromString(vhex)
        if EncodeToString(validator) not in by_pub:
            continue
        st = item_status_from_sigstr(validator, digest, sig)
        if st == REF_PANIC:
            raise ReferencePanic("Block.Verify panics")
        if st == ACCEPT:
            valid += 1
    return valid > trust_count(len(peers)), valid


# ----------------------------------------------------------------------------
# github.com/ugorji/go/codec v1.1.7 JsonHandle{Canonical: true} (go.mod:24),
# as used by Frame.Marshal (src/hashgraph/frame.go:35-46).  Restated from the
# published codec (encode.go kStruct / kMapCanonical, json.go quoteStr),
# schema-driven: every Go type the Frame graph holds is described by its
# type string below, and one recursive encoder walks values against it.
# PARITY UNPINNED: neither Go nor the ugorji module is in this container and
# the reference holds no serialized Frame.
# ----------------------------------------------------------------------------
@dataclass
class Event:
    """hashgraph.Event exported fields (event.go:102-105)."""
    Body: EventBody = field(default_factory=EventBody)
    Signature: GoStr = ""


@dataclass
class FrameEvent:
    """event.go:455-463."""
    Core: Optional[Event] = None
    Round: int = 0
    LamportTimestamp: int = 0
    Witness: bool = False


@dataclass
class Root:
    """root.go:11-14."""
    Events: Optional[list] = None


@dataclass
class Frame:
    """frame.go:12-20."""
    Round: int = 0
    Peers: Optional[list] = None
    Roots: Optional[dict] = None
    Events: Optional[list] = None
    PeerSets: Optional[dict] = None
    Timestamp: int = 0


UGORJI_SCHEMA = {
    "Frame": [("Round", "int"), ("Peers", "[]*Peer"), ("Roots", "map[string]*Root"), ("Events", "[]*FrameEvent"),
              ("PeerSets", "map[int][]*Peer"), ("Timestamp", "int64")],
    "Root": [("Events", "[]*FrameEvent")],
    "FrameEvent": [("Core", "*Event"), ("Round", "int"), ("LamportTimestamp", "int"), ("Witness", "bool")],
    "Event": [("Body", "EventBody"), ("Signature", "string")],
    "EventBody": [("Transactions", "[][]byte"), ("InternalTransactions", "[]InternalTransaction"),
                  ("Parents", "[]string"), ("Creator", "[]byte"), ("Index", "int"),
                  ("BlockSignatures", "[]BlockSignature"), ("Timestamp", "int64")],
    "InternalTransaction": [("Body", "InternalTransactionBody"), ("Signature", "string")],
    "InternalTransactionBody": [("Type", "uint8"), ("Peer", "Peer")],
    "BlockSignature": [("Validator", "[]byte"), ("Index", "int"), ("Signature", "string")],
    "Peer": [("NetAddr", "string"), ("PubKeyHex", "string"), ("Moniker", "string")],
}


def ugorji_string(s: GoStr) -> bytes:
    """json.go quoteStr (HTMLCharsAsIs false): short escapes for " \\ \\n \\r
    \\b \\f \\t, \\u00XX for other bytes < 0x20 and < > &, U+2028/2029
    escaped, each invalid UTF-8 byte -> \\ufffd."""
    b = _b(s)
    out = bytearray(b'"')
    i = 0
    short = {ord('"'): b'\\"', ord("\\"): b"\\\\", ord("\n"): b"\\n", ord("\r"): b"\\r", 8: b"\\b", 12: b"\\f",
             ord("\t"): b"\\t"}
    while i < len(b):
        c = b[i]
        if c < 0x80:
            if c in short:
                out += short[c]
            elif c < 0x20 or c in (ord("<"), ord(">"), ord("&")):
                out += b"\\u%04x" % c
            else:
                out.append(c)
            i += 1
            continue
        n, ok = _utf8_rune(b, i)
        if not ok:
            out += b"\\ufffd"
            i += 1
            continue
        if b[i:i + 3] in (b"\xe2\x80\xa8", b"\xe2\x80\xa9"):
            out += b"\\u%04x" % (0x2000 + (b[i + 2] - 0x80))
        else:
            out += b[i:i + n]
        i += n
    out += b'"'
    return bytes(out)


def ugorji_encode(v, gotype: str) -> bytes:
    """Encode value `v` of Go type `gotype` (a UGORJI_SCHEMA type string)."""
    if gotype.startswith("*"):
        return b"null" if v is None else ugorji_encode(v, gotype[1:])
    if gotype == "[]byte":
        return b"null" if v is None else b'"' + base64.b64encode(bytes(v)) + b'"'
    if gotype.startswith("[]"):
        if v is None:
            return b"null"
        return b"[" + b",".join(ugorji_encode(x, gotype[2:]) for x in v) + b"]"
    if gotype.startswith("map["):
        if v is None:
            return b"null"
        ktype, vtype = gotype[4:].split("]", 1)
        if ktype == "string":  # Canonical: keys sorted by their bytes
            keys = sorted(v, key=_b)
            kenc = ugorji_string
        else:  # integer keys: numeric order, written as quoted decimals
            keys = sorted(v)
            kenc = lambda k: b'"%d"' % k  # noqa: E731
        return b"{" + b",".join(kenc(k) + b":" + ugorji_encode(v[k], vtype) for k in keys) + b"}"
    if gotype in ("int", "int64", "uint8"):
        return b"%d" % v
    if gotype == "bool":
        return b"true" if v else b"false"
    if gotype == "string":
        return ugorji_string(v)
    # struct: exported fields, name-sorted (encode.go kStruct: toMap uses sfiSort)
    fields = sorted(UGORJI_SCHEMA[gotype], key=lambda f: f[0])
    return b"{" + b",".join(b'"' + n.encode() + b'":' + ugorji_encode(getattr(v, n), t) for n, t in fields) + b"}"


def frame_marshal(f: Frame) -> bytes:
    """Frame.Marshal (frame.go:35-46)."""
    return ugorji_encode(f, "Frame")


def frame_hash(f: Frame) -> bytes:
    """Frame.Hash (frame.go:63-69)."""
    return SHA256(frame_marshal(f))
