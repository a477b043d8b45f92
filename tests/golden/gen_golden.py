"""Generate the committed golden fixtures (tests/golden/*.json).

Run in the build container only (needs OpenSSL libcrypto through ctypes):
    python tests/golden/gen_golden.py

Every expected value comes from the pure-Python restatement of the Go path
(oracle/gosemantics.py) and is cross-checked before it is written:
  * digests against hashlib AND the from-scratch FIPS 180-4 restatement;
  * ECDSA outcomes of well-formed items against OpenSSL (independent
    implementation of the same verification equation);
  * every status against the C oracle (oracle/oracle.c).
The reference itself (Go) cannot run here (no toolchain, no module cache), so
these fixtures pin our restatement, not a Go run; the Go-specific parsing
rules they encode are documented in DESIGN.md §Oracle.

Outputs:
  golden_items.json   ~2.5k signature items across every SURVEY §8a-9 class:
                      {pub_hex, body_hex, sig (text), pre, r, s, status}
  golden_events.json  EventBodies (incl. ITXs, block signatures, HTML/UTF-8
                      escapes, nil vs empty slices) with canonical JSON,
                      digest, signature text and Event.Verify outcome
  golden_blocks.json  BlockBodies with validator signatures and CheckBlock
                      results (valid counts vs TrustCount)
  golden_sha256.json  SHA-256 known answers at every padding boundary
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import coracle, openssl_xcheck  # noqa: E402
from oracle import gosemantics as gs  # noqa: E402
from oracle.gosemantics import N, P  # noqa: E402


class Drbg:
    def __init__(self, seed: bytes):
        self.key = hashlib.sha256(b"golden:" + seed).digest()
        self.ctr = 0

    def bytes(self, n: int) -> bytes:
        out = b""
        while len(out) < n:
            out += hashlib.sha256(self.key + self.ctr.to_bytes(8, "big")).digest()
            self.ctr += 1
        return out[:n]

    def scalar(self) -> int:
        while True:
            v = int.from_bytes(self.bytes(32), "big")
            if 0 < v < N:
                return v

    def below(self, n: int) -> int:
        return int.from_bytes(self.bytes(8), "big") % n


def sign(d: int, digest: bytes, k: int):
    R = gs.scalar_mult(k, gs.G)
    r = R[0] % N
    s = pow(k, -1, N) * (int.from_bytes(digest, "big") + r * d) % N
    return r, s


def pre_of(sig: str):
    r, s, ok = gs.DecodeSignature(sig)
    if not ok:
        return 0x80, 0, 0
    rc, sc = gs.scalar_class(r), gs.scalar_class(s)
    rb = r if rc == gs.SC_OK else 0
    sb = s if sc == gs.SC_OK else 0
    return rc | (sc << 2), rb, sb


def make_keys(dr: Drbg, n: int):
    out = []
    for _ in range(n):
        d = dr.scalar()
        out.append((d, gs.Marshal(gs.scalar_mult(d, gs.G))))
    return out


def items_fixture(dr: Drbg):
    keys = make_keys(dr, 8)
    items = []

    def add(pub: bytes, body: bytes, sig: str, tag: str):
        digest = gs.SHA256(body)
        pre, r, s = pre_of(sig)
        st = gs.item_status_from_sigstr(pub, digest, sig)
        items.append(dict(tag=tag, pub=pub.hex(), body=body.hex(), sig=sig, pre=pre, r="%064x" % r,
                          s="%064x" % s, status=st))

    def body():
        return dr.bytes(1 + dr.below(300))

    t36 = gs.go_big_text36
    # valid, high-S, wrong digest, bit flips
    for i in range(600):
        d, pub = keys[i % len(keys)]
        b = body()
        r, s = sign(d, gs.SHA256(b), dr.scalar())
        kind = i % 6
        if kind == 0:
            add(pub, b, gs.EncodeSignature(r, s), "valid")
        elif kind == 1:
            add(pub, b, gs.EncodeSignature(r, N - s), "high_s")
        elif kind == 2:
            add(pub, b + b"x", gs.EncodeSignature(r, s), "wrong_digest")
        elif kind == 3:
            add(pub, b, gs.EncodeSignature(r ^ (1 << dr.below(256)), s), "r_flip")
        elif kind == 4:
            add(pub, b, gs.EncodeSignature(r, s ^ (1 << dr.below(256))), "s_flip")
        else:
            add(keys[(i + 1) % len(keys)][1], b, gs.EncodeSignature(r, s), "wrong_key")
    # range edge cases on r and s
    d, pub = keys[0]
    b = body()
    r, s = sign(d, gs.SHA256(b), dr.scalar())
    specials = ["0", "-0", "+0", t36(N), t36(N + 1), t36(N - 1), "-" + t36(r), t36(2**256), t36(2**300),
                "-1", "1", "00000" + t36(r), "+" + t36(r)]
    for sp in specials:
        add(pub, b, sp + "|" + t36(s), "r_special")
        add(pub, b, t36(r) + "|" + sp, "s_special")
    # text format: parts, empty parts, bad chars, case, underscores, spaces
    fmts = [t36(r), t36(r) + "|" + t36(s) + "|", "|", "", "||", t36(r) + "|", "|" + t36(s),
            t36(r).upper() + "|" + t36(s).upper(), t36(r) + "_|" + t36(s), " " + t36(r) + "|" + t36(s),
            t36(r) + "|" + t36(s) + "\n", t36(r) + "|" + t36(s)[:-1] + "!", "+|" + t36(s), "-|" + t36(s),
            t36(r) + "|+", "0x" + t36(r) + "|" + t36(s), t36(r) + "|é", "r|s"]
    for f in fmts:
        add(pub, b, f, "format")
    # public key encodings
    x = int.from_bytes(pub[1:33], "big")
    y = int.from_bytes(pub[33:], "big")
    badkeys = [b"", b"\x04", pub[:64], pub + b"\x00", bytes([2 + (y & 1)]) + pub[1:33], b"\x06" + pub[1:],
               b"\x07" + pub[1:], b"\x00" + pub[1:], b"\x04" + P.to_bytes(32, "big") + pub[33:],
               b"\x04" + pub[1:33] + (y + P).to_bytes(33, "big")[1:] if y + P < 2**256 else b"\x04" + pub[1:33] + P.to_bytes(32, "big"),
               b"\x04" + pub[1:33] + (y ^ 1).to_bytes(32, "big"),
               b"\x04" + pub[1:33] + (P - y).to_bytes(32, "big")]  # (x, -y): valid point, wrong key
    for bk in badkeys:
        for sg in (gs.EncodeSignature(r, s), "0|" + t36(s), t36(r) + "|" + t36(N), "nope", "|"):
            add(bk, b, sg, "key")
    # exceptional group-law cases: Q = G (u1 G + u2 G), Q = -G, small multiples
    for qk in (1, N - 1, 2, 3, N - 2):
        Q = gs.scalar_mult(qk, gs.G)
        qpub = gs.Marshal(Q)
        for _ in range(8):
            bb = body()
            e = int.from_bytes(gs.SHA256(bb), "big")
            rr, ss = sign(qk, gs.SHA256(bb), dr.scalar())
            add(qpub, bb, gs.EncodeSignature(rr, ss), "small_key")
            # forge r so that u1 G == -u2 Q (R = inf): pick w, u1 = e w, need r w = -e w / qk
            w = dr.scalar()
            u1 = e * w % N
            u2 = (-u1 * pow(qk, -1, N)) % N
            rr2 = u2 * pow(w, -1, N) % N
            ss2 = pow(w, -1, N)
            if 0 < rr2 < N:
                add(qpub, bb, gs.EncodeSignature(rr2, ss2), "r_inf")
            # forge u1 G == u2 Q (doubling inside Add)
            u2b = u1 * pow(qk, -1, N) % N
            rr3 = u2b * pow(w, -1, N) % N
            if 0 < rr3 < N:
                add(qpub, bb, gs.EncodeSignature(rr3, ss2), "r_double")
    return items


def json_event_bodies(dr: Drbg, keys):
    d0, pub0 = keys[0]
    evs = []
    peers = [gs.Peer(NetAddr="127.0.0.1:%d" % (1337 + i), PubKeyHex=gs.EncodeToString(k[1]), Moniker="node%d" % i)
             for i, k in enumerate(keys[:4])]

    def itx(kind, peer, signer_d, corrupt=None):
        t = gs.InternalTransaction(Body=gs.InternalTransactionBody(Type=kind, Peer=peer))
        r, s = sign(signer_d, t.Body.Hash(), dr.scalar())
        t.Signature = gs.EncodeSignature(r, s) if corrupt is None else corrupt(r, s)
        return t

    strings = ["plain", "<html>&amp;", "quote\"back\\slash", "ctl\x01\x1f\t\n\r", "utf8 é ☃ 😀",
               "line sep ", b"bad\xff\xfeutf8", b"trunc\xe2\x82", "�", b"\xed\xa0\x80surrogate"]
    for i in range(40):
        variant = i % 8
        body = gs.EventBody(
            Transactions=[dr.bytes(dr.below(100)) for _ in range(dr.below(4))] if variant != 1 else None,
            InternalTransactions=None,
            Parents=["", ""] if i % 5 == 0 else [gs.EncodeToString(dr.bytes(32)), gs.EncodeToString(dr.bytes(32))],
            Creator=pub0, Index=i, BlockSignatures=None, Timestamp=1_600_000_000 + i)
        if variant == 2:
            body.Transactions = []
        if variant == 3:
            body.InternalTransactions = [itx(0, gs.Peer("10.0.0.1:1", peers[1].PubKeyHex, strings[i % len(strings)]),
                                             keys[1][0])]
            body.InternalTransactions[0].Body.Peer.PubKeyHex = peers[1].PubKeyHex
            # ITX signature is by the joining peer over its own body
            t = body.InternalTransactions[0]
            r, s = sign(keys[1][0], t.Body.Hash(), dr.scalar())
            t.Signature = gs.EncodeSignature(r, s)
        if variant == 4:
            body.InternalTransactions = []
            body.BlockSignatures = [gs.BlockSignature(Validator=pub0, Index=7, Signature="r|s"),
                                    gs.BlockSignature(Validator=None, Index=0, Signature=strings[i % 10])]
        if variant == 5:  # ITX with a bad signature then a good one
            t1 = itx(1, peers[2], keys[2][0], corrupt=lambda r, s: gs.EncodeSignature(r, s ^ 1))
            body.InternalTransactions = [t1]
        if variant == 6:  # ITX whose PubKeyHex is too short (Go panics) / malformed
            body.InternalTransactions = [gs.InternalTransaction(
                Body=gs.InternalTransactionBody(Type=0, Peer=gs.Peer("x", "0" if i % 2 else "0X04ZZ", "m")),
                Signature="1|1")]
        if variant == 7:
            body.InternalTransactions = [itx(0, peers[3], keys[3][0], corrupt=lambda r, s: "bad")]
        digest = body.Hash()
        r, s = sign(d0, digest, dr.scalar())
        sig = gs.EncodeSignature(r, s) if i % 7 else gs.EncodeSignature(r, s ^ 2)
        evs.append(dict(json=body.Marshal().decode("latin-1"), digest=digest.hex(), sig=sig,
                        verify=gs.event_status(body, sig)))
    return evs


def blocks_fixture(dr: Drbg):
    vals = make_keys(dr, 10)
    peers = [gs.Peer(NetAddr="", PubKeyHex=gs.EncodeToString(k[1]), Moniker="") for k in vals]
    ph = gs.peer_set_hash(peers)
    out = []
    for bi in range(12):
        body = gs.BlockBody(Index=bi, RoundReceived=bi + 3, Timestamp=1_600_000_000 + bi, StateHash=dr.bytes(32),
                            FrameHash=dr.bytes(32), PeersHash=ph if bi != 5 else dr.bytes(32),
                            Transactions=[dr.bytes(64) for _ in range(16)], InternalTransactions=[],
                            InternalTransactionReceipts=None)
        digest = body.Hash()
        sigs = []
        n_bad = bi % 8  # 0..7 invalid among 10 -> counts around TrustCount = 4
        for vi, (d, pub) in enumerate(vals):
            r, s = sign(d, digest, dr.scalar())
            sg = gs.EncodeSignature(r, s) if vi >= n_bad else gs.EncodeSignature(r, (s + 1) % N)
            sigs.append((gs.EncodeToString(pub), sg))
        foreign = make_keys(dr, 1)[0]
        r, s = sign(foreign[0], digest, dr.scalar())
        sigs.append((gs.EncodeToString(foreign[1]), gs.EncodeSignature(r, s)))  # not a member: skipped
        ok, valid = gs.check_block(body, sigs, peers)
        out.append(dict(json=body.Marshal().decode("latin-1"), digest=digest.hex(), peers_hash=ph.hex(),
                        sigs=sigs, check_ok=ok, valid=valid, trust_count=gs.trust_count(len(peers))))
    return dict(validators=[k[1].hex() for k in vals], blocks=out)


def sha_fixture(dr: Drbg):
    out = []
    for n in list(range(0, 130)) + [183, 191, 192, 447, 448, 449, 1000, 1771, 4096, 65537]:
        m = dr.bytes(n)
        h = hashlib.sha256(m).digest()
        assert gs.sha256_fips(m) == h == coracle.sha256(m)
        out.append(dict(msg=m.hex(), digest=h.hex()))
    # FIPS 180-4 examples
    for m, h in [(b"abc", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"),
                 (b"", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
                 (b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
                  "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1")]:
        assert hashlib.sha256(m).hexdigest() == h == gs.sha256_fips(m).hex()
        out.append(dict(msg=m.hex(), digest=h))
    return out


def main():
    dr = Drbg(b"v1")
    items = items_fixture(dr)
    # cross-checks
    n_ossl = 0
    for it in items:
        pub = bytes.fromhex(it["pub"])
        digest = gs.SHA256(bytes.fromhex(it["body"]))
        c = coracle.item_status(pub, digest, it["pre"], bytes.fromhex(it["r"]), bytes.fromhex(it["s"]))
        assert c == it["status"], (it, c)
        if it["pre"] == 0 and gs.Unmarshal(pub) is not None:
            o = openssl_xcheck.verify(pub, digest, int(it["r"], 16), int(it["s"], 16))
            if it["tag"] == "r_inf":
                # u1 G + u2 Q = infinity: OpenSSL reports an error (-1) where
                # Go's Verify returns false; both reject.
                assert o is None and it["status"] == gs.REJECT, (it, o)
            else:
                assert o is not None and (o == (it["status"] == gs.ACCEPT)), (it, o)
            n_ossl += 1
    counts = {}
    for it in items:
        counts[it["status"]] = counts.get(it["status"], 0) + 1
    print(f"items: {len(items)} statuses {counts}; {n_ossl} cross-checked with OpenSSL")
    keys = make_keys(dr, 4)
    evs = json_event_bodies(dr, keys)
    print("events:", len(evs), "outcomes", sorted({e["verify"] for e in evs}))
    blocks = blocks_fixture(dr)
    print("blocks:", [(b["valid"], b["check_ok"]) for b in blocks["blocks"]])
    sha = sha_fixture(dr)
    with open(os.path.join(HERE, "golden_items.json"), "w") as f:
        json.dump(items, f, indent=0)
    with open(os.path.join(HERE, "golden_events.json"), "w") as f:
        json.dump(dict(keys=[k[1].hex() for k in keys], events=evs), f, indent=0)
    with open(os.path.join(HERE, "golden_blocks.json"), "w") as f:
        json.dump(blocks, f, indent=0)
    with open(os.path.join(HERE, "golden_sha256.json"), "w") as f:
        json.dump(sha, f, indent=0)


if __name__ == "__main__":
    main()
