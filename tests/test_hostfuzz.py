"""The product's host-only C++ under AddressSanitizer + UBSan, fuzzed
(VERDICT r2 #8): hostparse.cpp (bv_decode_signature, bv_hex_decode — the
signature text and PubKeyHex are attacker-controlled; processJoinRequest
reaches them outside coreLock, /root/reference/src/node/node_rpc.go:250-260)
and hostplan.cpp (bv_plan_shards, bv_plan_group, bv_merge_shard_bits — the
multi-device group's host side).  tests/hostfuzz builds them with the fuzz
driver (plain clang, host only); every input is copied into an exactly-sized
heap buffer, so an over-read aborts the run.  Results are compared with the
Go-semantics restatement (oracle/gosemantics.py: keys.DecodeSignature,
big.Int.SetString(., 36), common.DecodeFromString) and with babble_amd/shard.py.
CPU only."""
import os
import random
import subprocess

import numpy as np
import pytest

from babble_amd import shard
from oracle import gosemantics as gs

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hostfuzz")
EXE = os.path.join(HERE, "_build", "hostfuzz")


@pytest.fixture(scope="module")
def run():
    subprocess.run(["make", "-s", "-C", HERE], check=True)

    def go(lines):
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
                   UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
        p = subprocess.run([EXE], input="\n".join(lines) + "\n", capture_output=True, text=True, env=env,
                           timeout=600)
        assert p.returncode == 0, p.stderr[-3000:]
        assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-3000:]
        out = p.stdout.splitlines()
        assert len(out) == len(lines)
        return out
    return go


def _hx(b: bytes) -> str:
    return b.hex() or "-"


def _sig_cases(rng):
    N = gs.N
    t36 = gs.go_big_text36
    out = [b"", b"|", b"||", b"a|b", b"0|0", b"-1|1", b"+|-", b"-|+", b"--1|1", b"+-1|1", b"1|1|", b"|1|",
           (t36(N) + "|1").encode(), (t36(N - 1) + "|1").encode(), ("1|" + t36(N + 1)).encode(),
           (t36(2**288) + "|5").encode(), (t36(2**288 - 1) + "|5").encode(), (t36(2**300) + "|" + t36(2**512)).encode(),
           ("-" + t36(2**288) + "|5").encode(), (t36(N - 2).upper() + "|" + t36(3)).encode(),
           b"0" * 400 + b"1|2", b"1|" + b"z" * 300, b"\xff|\xfe", b"a\x00|b"]
    alphabet = b"0123456789abcdefghijklmnopqrstuvwxyzABCXYZ+-|_ .\x00\xc3\xa9\xff"
    for _ in range(6000):
        k = rng.randrange(0, 90)
        out.append(bytes(rng.choice(alphabet) for _ in range(k)))
    for _ in range(2000):  # well-formed texts around the range limits, plus signs
        a = rng.choice([rng.randrange(-5, 6), rng.randrange(N - 5, N + 5), rng.getrandbits(rng.choice([64, 256, 257, 289, 400]))])
        b = rng.choice([rng.randrange(-5, 6), rng.randrange(N - 5, N + 5), rng.getrandbits(rng.choice([64, 256, 257, 289, 400]))])
        sa = (rng.choice(["", "+"]) if a >= 0 else "-") + t36(abs(a))
        sb = (rng.choice(["", "+"]) if b >= 0 else "-") + t36(abs(b))
        if rng.random() < 0.3:
            sa = sa.upper()
        out.append((sa + "|" + sb).encode())
    for _ in range(500):
        out.append(bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 200))))
    return out


def test_decode_signature_fuzz_sanitized(run):
    rng = random.Random(2024)
    cases = _sig_cases(rng)
    res = run(["S " + _hx(c) for c in cases])
    for c, line in zip(cases, res):
        _, pre, rh, sh = line.split()
        pre = int(pre)
        r, s, ok = gs.DecodeSignature(c)
        if not ok:
            assert pre == 0x80 and rh == sh == "00" * 32, c
            continue
        rc, sc = gs.scalar_class(r), gs.scalar_class(s)
        assert pre == rc | (sc << 2), (c, pre, rc, sc)
        assert rh == (r.to_bytes(32, "big").hex() if rc == gs.SC_OK else "00" * 32), c
        assert sh == (s.to_bytes(32, "big").hex() if sc == gs.SC_OK else "00" * 32), c


def test_hex_decode_fuzz_sanitized(run):
    rng = random.Random(99)
    hexch = b"0123456789abcdefABCDEF"
    cases = [b"", b"0", b"0X", b"0X1", b"0X12", b"0Xg", b"0X1g", b"0Xg1", b"0X123", b"0X12zz"]
    for _ in range(5000):
        n = rng.randrange(0, 140)  # odd and even lengths
        body = bytes(rng.choice(hexch) for _ in range(n))
        if rng.random() < 0.4 and n:  # one bad character somewhere
            i = rng.randrange(n)
            body = body[:i] + bytes([rng.choice(b"gz \x00\xff-")]) + body[i + 1:]
        cases.append(rng.choice([b"0X", b"0x", b"xx", b""]) + body)
    res = run(["H " + _hx(c) for c in cases])
    for c, line in zip(cases, res):
        _, n, oh = line.split()
        n = int(n)
        if len(c) < 2:
            assert n == -1, c  # Go panics on s[2:]
            continue
        want = gs.DecodeFromString(c)
        assert n == len(want) and (oh == "-" if not want else oh == want.hex()), c


def test_plan_group_fuzz_sanitized(run):
    rng = np.random.default_rng(5)
    cases = []
    for t in range(1500):
        n_msgs = int(rng.integers(0, 60))
        n = int(rng.integers(0, 200)) if n_msgs else 0
        im = np.sort(rng.integers(0, n_msgs, size=n)) if n else np.zeros(0, np.int64)
        if t % 2 and n:
            im = rng.permutation(im)  # shuffled items: the group sorts them stably
        D = int(rng.integers(1, 10))
        cases.append((D, n_msgs, im))
    res = run([f"G {D} {nm} {','.join(map(str, im.tolist())) or '-'}" for D, nm, im in cases])
    for (D, n_msgs, im), line in zip(cases, res):
        f = line.split()
        permuted, perm, ib, mb = shard.plan_group(im, n_msgs, D)
        assert int(f[1]) == int(permuted)
        got_perm = [] if f[2] == "-" else [int(x) for x in f[2].split(",")]
        assert got_perm == list(map(int, perm))
        assert [int(x) for x in f[3].split(",")] == list(ib)
        got_mb = [int(x) for x in f[4].split(",")]
        assert got_mb == list(mb)
        # properties: messages partitioned, every shard's items inside its range
        assert got_mb[0] == 0 and got_mb[-1] == n_msgs and all(a <= b for a, b in zip(got_mb, got_mb[1:]))
        srt = im[np.asarray(got_perm, dtype=np.int64)] if len(im) else im
        for d in range(D):
            seg = srt[ib[d]:ib[d + 1]]
            assert np.all((seg >= got_mb[d]) & (seg < got_mb[d + 1]))
    # out-of-range message index: refused, not read out of bounds
    assert run(["G 2 3 0,1,3"]) == ["G -1"]


def test_merge_shard_bits_fuzz_sanitized(run):
    rng = np.random.default_rng(8)
    cases, wants = [], []
    for _ in range(800):
        n = int(rng.integers(0, 700))
        D = int(rng.integers(1, 9))
        bounds = [0] + sorted(rng.integers(0, n + 1, size=D - 1).tolist()) + [n]
        words = max(1, max((bounds[d + 1] - bounds[d] + 63) // 64 for d in range(D)))
        g = rng.integers(0, 2**63, size=(D, words), dtype=np.int64).astype(np.uint64)
        g |= rng.integers(0, 2, size=(D, words)).astype(np.uint64) << np.uint64(63)
        cases.append(f"M {words} {D} {','.join(map(str, bounds))} {','.join('%x' % int(x) for x in g.reshape(-1))}")
        wants.append(shard.merge_bits([g[d] for d in range(D)], bounds))
    for line, want in zip(run(cases), wants):
        f = line.split()
        assert f[1] == "0"
        got = [] if f[2] == "-" else [int(x, 16) for x in f[2].split(",")]
        assert got == [int(x) for x in want]
    assert run(["M 1 2 0,70,80 0,0"])[0] == "M -1"  # a shard wider than words_per_shard


LAMBDA = 0x5363AD4CC05C30E0A5261C028812645A122E22EA20816678DF02967C1B23BD72  # phi's eigenvalue mod N


def test_host_item_record_sanitized(run):
    """hostscalar.cpp bv_host_item_record (the latency batch's item record):
    u1 = e s^-1 mod N and u2 = r s^-1 = k1 + k2 lambda (mod N) with
    |k1|, |k2| < 2^129, the key / r / s / pre / table fields in place, and
    all-zero scalars whenever s is unusable (pre != 0, s = 0, s >= N) — on
    random and edge values, under ASan + UBSan."""
    rng = random.Random(11)
    N = gs.N
    cases = []
    for i in range(400):
        e = rng.getrandbits(256)
        r = rng.getrandbits(256) if i % 7 else rng.choice([0, 1, N - 1, N, 2 ** 256 - 1])
        s = rng.randrange(1, N) if i % 5 else rng.choice([0, 1, 2, N - 1, N, N + 1, 2 ** 256 - 1])
        pre = 0 if i % 11 else rng.choice([1, 4, 5, 0x40])
        klen = 65 if i % 13 else rng.choice([0, 33, 64, 66, 100])
        key = bytes([4] + [rng.getrandbits(8) for _ in range(klen - 1)]) if klen else b""
        cases.append((e, r, s, pre, key))
    out = run([f"R {e:064x} {r:064x} {s:064x} {pre} {key.hex() or '-'}" for e, r, s, pre, key in cases])

    def limbs(w, a, n):
        return sum(int(w[a + i], 16) << (32 * i) for i in range(n))

    for (e, r, s, pre, key), line in zip(cases, out):
        w = line.split()[1:]
        assert len(w) == 64
        raw = b"".join(int(x, 16).to_bytes(4, "little") for x in w)
        kl = min(len(key), 66)
        assert int(w[18], 16) == kl and int(w[19], 16) == pre
        assert raw[:65] == (key if kl == 65 else bytes(65))
        assert raw[80:112] == r.to_bytes(32, "big") and raw[112:144] == s.to_bytes(32, "big")
        assert limbs(w, 54, 2) == 0x1122334455667788
        u1, k1, k2, signs = limbs(w, 36, 8), limbs(w, 44, 4), limbs(w, 48, 4), int(w[52], 16)
        if pre or s == 0 or s >= N:
            assert u1 == k1 == k2 == signs == 0
            continue
        si = pow(s, -1, N)
        assert u1 == e * si % N
        k1s = -k1 if signs & 1 else k1
        k2s = -k2 if signs & 2 else k2
        assert (k1s + k2s * LAMBDA - r * si) % N == 0
        assert k1 < 2 ** 129 and k2 < 2 ** 129 and signs < 4
