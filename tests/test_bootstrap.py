"""Hashgraph.Bootstrap's replay with batched verification
(babble_amd/hashgraph.py:bootstrap, hashgraph.go:1481-1536): the same
insert / ProcessSigPool call sequence and the same first error as the
sequential Go loop, with one device verify per read-ahead window."""
import types

import numpy as np
import pytest

from babble_amd import hashgraph as H
from oracle import coracle
from oracle import gosemantics as gs
from tests.test_mirror import Signer, to_mirror


class OracleVerifier:
    """Test-only CPU stand-in for the device batch (the C oracle), so the
    host ordering logic is covered without a GPU."""
    calls = 0

    def verify(self, packed):
        OracleVerifier.calls += 1
        h, st, _ = coracle.verify_batch(packed.as_dict())
        return types.SimpleNamespace(status=st, msg_hash=h)


def make_db(n, bad=(), seed=2):
    sg = Signer(seed)
    d, pub = sg.key()
    evs = []
    for i in range(n):
        b = gs.EventBody(Transactions=[sg.rng.randbytes(40)], Parents=["", ""] if i == 0 else
                         [gs.EncodeToString(sg.rng.randbytes(32)), ""], Creator=pub, Index=i,
                         Timestamp=1_600_000_000 + i)
        sig = sg.sign(d, b.Hash())
        if i in bad:
            r, s = sig.split("|")
            sig = gs.go_big_text36((int(gs.go_big_setstring36(r)) + 1) % gs.N) + "|" + s
        evs.append(H.Event(Body=to_mirror(b), Signature=sig))
    return evs


def run(evs, window, verifier, fail_insert_at=None):
    log = []

    def db(off, limit):
        log.append(("read", off))
        return evs[off:off + limit]

    def insert(ev):
        log.append(("insert", ev.Body.Index))
        if ev.Body.Index == fail_insert_at:
            return "Other-parent not known"
        return None

    def sig_pool():
        log.append(("sigpool",))
        return None

    err = H.bootstrap(db, insert, sig_pool, batch_size=100, verify_window=window, verifier=verifier)
    return err, log


def go_sequence(n, stop_at=None):
    """The call sequence of the sequential Go loop (reads, inserts, pools)."""
    out = []
    index = 0
    while True:
        out.append(("read", index * 100))
        batch = list(range(index * 100, min(n, index * 100 + 100)))
        for i in batch:
            if i == stop_at:
                return out, True
            out.append(("insert", i))
        out.append(("sigpool",))
        if len(batch) < 100:
            return out, False
        index += 1


@pytest.mark.parametrize("window", [100, 250, 100_000])
def test_bootstrap_order_and_first_error(window):
    evs = make_db(430, bad={311})
    OracleVerifier.calls = 0
    err, log = run(evs, window, OracleVerifier())
    want, _ = go_sequence(430, stop_at=311)
    assert err == "Invalid Event signature %s" % evs[311].Hex()
    # the read-ahead may read further DB batches than Go; everything else is identical
    assert [x for x in log if x[0] != "read"] == [x for x in want if x[0] != "read"]
    assert OracleVerifier.calls <= 5


def test_bootstrap_all_valid_and_insert_error():
    evs = make_db(300)
    err, log = run(evs, 1000, OracleVerifier())
    want, _ = go_sequence(300)
    assert err is None  # 300 = 3 full batches + an empty read
    assert [x for x in log if x[0] != "read"] == [x for x in want if x[0] != "read"]
    assert [x for x in log if x[0] == "read"] == [x for x in want if x[0] == "read"]
    err, log = run(evs, 1000, OracleVerifier(), fail_insert_at=150)
    assert err == "Other-parent not known"
    assert log[-1] == ("insert", 150)


class CheckedVerifier:
    """The default device Verifier, each batch also checked against the C
    oracle (a wrong status is reported as such, not as a replay error)."""

    def __init__(self):
        self.mismatches = []

    def verify(self, packed):
        res = H.default_verifier().verify(packed)
        h, st, _ = coracle.verify_batch(packed.as_dict())
        bad = np.flatnonzero(res.status != st)
        if bad.size or not np.array_equal(res.msg_hash, h):
            self.mismatches.append((packed.n_items, bad[:8].tolist(), res.status[bad[:8]].tolist(),
                                    st[bad[:8]].tolist(), H.default_verifier().timing()))
        return res

    def sha256(self, msgs):
        return H.default_verifier().sha256(msgs)


@pytest.mark.gpu
def test_bootstrap_on_device():
    evs = make_db(1200, bad={1111})
    cv = CheckedVerifier()
    err, log = run(evs, 500, cv)
    assert not cv.mismatches, f"device statuses differ from the oracle: {cv.mismatches}"
    assert err == "Invalid Event signature %s" % evs[1111].Hex()
    assert sum(1 for x in log if x[0] == "insert") == 1111
    assert all(e._hash is not None for e in evs[:1112])
