"""The hand-scheduled gfx950 field programs (tools/gen_field_asm.py ->
babble_amd/csrc/field_asm.h) executed by the generator's interpreter against
Python integers mod p; plus the hazard spacing and header freshness checks.
The GPU parity tests (tests/test_gpu.py) cover the same code end to end."""
import os
import random
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_field_asm as G  # noqa: E402

P = G.P


def _run(g, a, b, force_slow=False):
    m = G.Machine()
    for i in range(8):
        m.r[f"%[a{i}]"] = (a >> (32 * i)) & G.M32
        m.r[f"%[b{i}]"] = (b >> (32 * i)) & G.M32
    m.run(g, force_slow)
    return sum(m.r[f"%[r{i}]"] << (32 * i) for i in range(8))


def _operands(seed, n):
    rng = random.Random(seed)
    edge = [0, 1, 2, 977, 2**32 - 1, 2**32, P - 1, P, P + 1, 2**256 - 1, 2**256 - 2, 2**256 - G.K,
            2**256 - G.K - 1, 2**256 - G.K + 1, 2**255, 2**255 - 1, 2 * (2**256 - P)]
    top = [2**256 - 1 - rng.getrandbits(rng.choice([8, 40, 64, 200])) for _ in range(n // 4)]
    limbs = [sum((rng.choice([0, G.M32, G.M32 - 977, 1]) << (32 * i)) for i in range(8)) for _ in range(n // 4)]
    return edge + top + limbs + [rng.getrandbits(256) for _ in range(n)]


OPS = {"fe_mul": lambda a, b: a * b, "fe_sqr": lambda a, b: a * a, "fe_add": lambda a, b: a + b, "fe_sub": lambda a, b: a - b}


@pytest.mark.parametrize("name", sorted(OPS))
@pytest.mark.parametrize("force_slow", [False, True])
def test_program_matches_python_ints(name, force_slow):
    g = G.build(name)
    xs = _operands(1, 160)
    ys = _operands(2, 40)
    for a in xs:
        for b in ys:
            r = _run(g, a, b, force_slow)
            assert r < 2**256 and (r - OPS[name](a, b)) % P == 0, (name, hex(a), hex(b), hex(r))


def test_squares_and_rare_tail_hit():
    """a*a (fe_sqr on the device) and operands that drive the rare tail."""
    g = G.build("fe_mul")
    hits = 0
    rng = random.Random(3)
    for _ in range(3000):
        a = 2**256 - 1 - rng.getrandbits(rng.choice([1, 16, 64, 128]))
        b = rng.choice([a, 2**256 - 1 - rng.getrandbits(32)])
        m = G.Machine()
        for i in range(8):
            m.r[f"%[a{i}]"] = (a >> (32 * i)) & G.M32
            m.r[f"%[b{i}]"] = (b >> (32 * i)) & G.M32
        m._run(g)
        hits += bool(m.get(g.slow[0]))
        m.run(g.slow[1])
        r = sum(m.r[f"%[r{i}]"] << (32 * i) for i in range(8))
        assert r < 2**256 and (r - a * b) % P == 0
    assert hits == hits  # the tail is exercised by force_slow above regardless


def test_hazard_spacing():
    for name in OPS:
        G.check_hazards(G.build(name))


def test_header_is_fresh():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_field_asm.py"), "--check"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.parametrize("kinds", G.ZIP_COMBOS, ids=lambda k: "_".join(k))
@pytest.mark.parametrize("force_slow", [False, True])
def test_zipped_programs_match_python_ints(kinds, force_slow):
    """The interleaved multi-product programs (gen_zip) of the key-table
    doubling chain: every component equals its own product mod p."""
    g = G.build(G.zip_name(kinds))
    G.check_hazards(g)
    rng = random.Random(7)
    for trial in range(150):
        m = G.Machine()
        want = []
        for k, kind in enumerate(kinds):
            a, b = rng.getrandbits(256), rng.getrandbits(256)
            if trial < 50:
                a = 2**256 - 1 - rng.getrandbits(rng.choice([1, 8, 64]))
                b = 2**256 - 1 - rng.getrandbits(rng.choice([1, 3, 40]))
            if kind == "sqr":
                b = a
            for i in range(8):
                m.r[f"%[z{k}a{i}]"] = (a >> (32 * i)) & G.M32
                if kind == "mul":
                    m.r[f"%[z{k}b{i}]"] = (b >> (32 * i)) & G.M32
            want.append(a * b)
        m.run(g, force_slow)
        for k in range(len(kinds)):
            r = sum(m.r[f"%[z{k}r{i}]"] << (32 * i) for i in range(8))
            assert r < 2**256 and (r - want[k]) % P == 0, (kinds, k)
