"""A digit-level Python model of coop.h's cooperative field arithmetic
(mul, norm, tail: one 16-lane DPP row, the same DPP reads, 32/64-bit
truncations and carry-lookahead as the device code) that asserts, at every
step, the bounds the device code's exactness rests on: u_k < 2^34, the
unresolved digits E_k < 2^32 + 3, the folded columns < 2^42, the carry-save
digits < 2^32 + 2^20, no 64-bit wrap, no carry leaving the row, and after
tail()'s rare second fold no carry out of limb 7.  Results are compared with
Python integers mod p over edge-heavy operands (limbs 0 / 2^32 - 1 /
2^32 - 977 / 2^31, values near p and 2^256), and the rare branch is driven
on purpose.  CPU only: the GPU check of the same functions on hardware is
tests/test_gpu_field.py::test_coop_mul_norm_match_python_ints."""
import random

import pytest

P = 2**256 - 2**32 - 977
M32 = 2**32 - 1
M64 = 2**64 - 1
F977 = [977, 1] + [0] * 14
M4 = [0x1FFFFF0BC, 0x1FFFFFFFA] + [0x1FFFFFFFE] * 6 + [2] + [0] * 7


def shr(x, n=1):  # row_shr:n (lane k reads k - n; zeros in)
    return [0] * n + x[:16 - n]


def shl(x, n):  # row_shl:n (lane k reads k + n; zeros past the row)
    return x[n:] + [0] * n


def bcast(x, n):  # row_newbcast:n
    return [x[n]] * 16


def resolve(v, gen, stats):
    assert all(0 <= x <= M32 for x in v)
    G = sum(1 << k for k in range(16) if gen[k])
    Pm = sum(1 << k for k in range(16) if v[k] == M32)
    C = ((G << 1) + Pm) ^ Pm
    assert C >> 16 == 0, "carry out of the row"
    stats["resolves"] += 1
    return [(v[k] + ((C >> k) & 1)) & M32 for k in range(16)]


def tail(w, stats):
    """coop::tail: lanes 0..8 hold w_k < 2^32 + 2^20, lanes 9..15 zero."""
    assert all(x < 2**32 + 2**20 for x in w[:9]) and not any(w[9:]), w
    w8 = bcast(w, 8)
    z = [(w[k] if k < 8 else 0) + w8[k] * F977[k] for k in range(16)]
    assert all(x <= M64 for x in z) and all(x < 2**43 for x in z)
    y = [(z[k] & M32) + shr([x >> 32 for x in z])[k] for k in range(16)]
    assert all(x < 2**33 for x in y) and y[8] <= 1 and not any(y[9:])
    d = resolve([x & M32 for x in y], [x >> 32 != 0 for x in y], stats)
    assert d[8] <= 1 and not any(d[9:])
    if d[8]:
        stats["rare"] += 1
        o = bcast(d, 8)
        z2 = [(d[k] if k < 8 else 0) + o[k] * F977[k] for k in range(16)]
        y2 = [(z2[k] & M32) + shr([x >> 32 for x in z2])[k] for k in range(16)]
        d = resolve([x & M32 for x in y2], [x >> 32 != 0 for x in y2], stats)
        assert d[8] == 0, "carry out of limb 7 after the second fold"
    assert not any(d[8:]), "tail() returns without masking: lanes 8..15 must be 0"
    return d


def norm(w, stats):
    """coop::norm: WIDE lanes 0..8 (< 2^40), lanes 9..15 zero."""
    assert all(0 <= x < 2**40 for x in w[:9]) and not any(w[9:])
    v = [(w[k] & M32) + shr([x >> 32 for x in w])[k] for k in range(16)]
    assert v[9] == 0
    return tail(v, stats)


def mul(a, b, stats):
    """coop::mul: a, b NORMAL (lanes 0..7 limbs, 8..15 zero)."""
    acc, cnt, bs = [0] * 16, [0] * 16, list(b)
    for s in range(8):
        as_ = bcast(a, s)
        if s:
            bs = shr(bs)
        for k in range(16):
            n = acc[k] + as_[k] * bs[k]
            cnt[k] += n >> 64
            acc[k] = n & M64
    lo, hi = [x & M32 for x in acc], [x >> 32 for x in acc]
    h1, c2 = shr(hi), shr(cnt, 2)
    u = [lo[k] + h1[k] + c2[k] for k in range(16)]
    assert all(x < 2**34 for x in u) and sum(x << (32 * k) for k, x in enumerate(u)) == to_int(a) * to_int(b)
    v = [(u[k] & M32) + shr([x >> 32 for x in u])[k] for k in range(16)]
    assert all(x < 2**32 + 3 for x in v) and v[15] <= M32
    vl, vh = [x & M32 for x in v], [x >> 32 for x in v]
    assert all(x <= 1 for x in vh)
    e8 = [(h << 32) | l for h, l in zip(shl(vh, 8), shl(vl, 8))]
    m7 = [0 if (k == 0 or k > 8) else M32 for k in range(16)]
    e7 = [((h & m) << 32) | (l & m) for h, l, m in zip(shl(vh, 7), shl(vl, 7), m7)]
    t = [(v[k] if k < 8 else 0) + e8[k] * 977 + e7[k] for k in range(16)]
    assert all(x < 2**42 for x in t) and t[8] <= M32 and not any(t[9:])
    w = [(t[k] & M32) + shr([x >> 32 for x in t])[k] for k in range(16)]
    assert all(x < 2**32 + 2**10 for x in w)
    return tail(w, stats)


def limbs(x):
    return [(x >> (32 * k)) & M32 for k in range(8)] + [0] * 8


def to_int(r):
    return sum(x << (32 * k) for k, x in enumerate(r[:8]))


def negw(b):  # coop::negw: M4 - b
    return [M4[k] - b[k] for k in range(16)]


def _operands(seed, n):
    rng = random.Random(seed)
    K = 2**32 + 977
    edge = [0, 1, 2, 977, M32, 2**32, P - 1, P, P + 1, 2**256 - 1, 2**256 - 2, 2**256 - K, 2**256 - K - 1,
            2**256 - K + 1, 2**255, 2**255 - 1, 2 * K]
    top = [2**256 - 1 - rng.getrandbits(rng.choice([1, 8, 16, 40, 64, 128, 200])) for _ in range(n // 4)]
    pat = [sum(rng.choice([0, M32, M32 - 977, M32 - 976, 1, 2**31]) << (32 * i) for i in range(8))
           for _ in range(n // 4)]
    return edge + top + pat + [rng.getrandbits(256) for _ in range(n)]


def test_m4_is_4p():
    assert sum(x << (32 * k) for k, x in enumerate(M4)) == 4 * P
    assert all(x >= 2**32 for x in M4[:8])


def test_mul_model_exact_on_edge_operands():
    stats = {"resolves": 0, "rare": 0}
    xs, ys = _operands(1, 600), _operands(2, 600)
    rng = random.Random(3)
    pairs = [(x, y) for x in xs[:17] for y in ys[:17]] + [(rng.choice(xs), rng.choice(ys)) for _ in range(3000)]
    for x, y in pairs:
        r = to_int(mul(limbs(x), limbs(y), stats))
        assert r < 2**256 and (r - x * y) % P == 0, (hex(x), hex(y))
    assert stats["resolves"] == len(pairs) + stats["rare"]  # one resolve a product (+1 on the rare fold)


def test_tail_rare_branch_exact():
    """Drive tail()'s rare fold: lanes 0..7 near 2^256 with the redundant
    bits set, w_8 at its largest — the resolved lane 8 is 1 and the second
    fold must not carry."""
    stats = {"resolves": 0, "rare": 0}
    rng = random.Random(7)
    for _ in range(2000):
        w = [M32 - rng.choice([0, 0, 1, 977, rng.getrandbits(12)]) + rng.choice([0, 0, 1, rng.getrandbits(10)])
             for _ in range(8)]
        w.append(rng.choice([0, 1, M32, 2**32 + 2**10 - 1, rng.getrandbits(33) % (2**32 + 2**10)]))
        w += [0] * 7
        value = sum(x << (32 * k) for k, x in enumerate(w))
        r = to_int(tail(w, stats))
        assert r < 2**256 and (r - value) % P == 0
    assert stats["rare"] > 100, stats


def test_norm_model_exact_on_wide_combinations():
    """Every WIDE form coop.h feeds norm(): 2Y, 3X^2, 4Y^2, a + (M4 - b),
    2 (W + (M4 - A) + (M4 - C)), F + 2 (M4 - D), m + 8 (M4 - C),
    RR + (M4 - HHH) + 2 (M4 - V), 3S + (M4 - M^2), 3Q + PPP + (M4 - R^2)."""
    stats = {"resolves": 0, "rare": 0}
    xs = _operands(11, 400)
    rng = random.Random(12)

    def pick():
        return limbs(rng.choice(xs) % 2**256)

    for _ in range(1500):
        a, b, c = pick(), pick(), pick()
        forms = [
            ([2 * x for x in a], 2 * to_int(a)),
            ([3 * x for x in a], 3 * to_int(a)),
            ([x + y for x, y in zip(a, negw(b))], to_int(a) - to_int(b)),
            ([2 * (x + y + z) for x, y, z in zip(a, negw(b), negw(c))], 2 * (to_int(a) - to_int(b) - to_int(c))),
            ([x + 2 * y for x, y in zip(a, negw(b))], to_int(a) - 2 * to_int(b)),
            ([x + 8 * y for x, y in zip(a, negw(b))], to_int(a) - 8 * to_int(b)),
            ([x + y + 2 * z for x, y, z in zip(a, negw(b), negw(c))], to_int(a) - to_int(b) - 2 * to_int(c)),
            ([4 * x for x in a], 4 * to_int(a)),
            ([3 * x + y for x, y in zip(a, negw(b))], 3 * to_int(a) - to_int(b)),
            ([3 * x + y + z for x, y, z in zip(a, b, negw(c))], 3 * to_int(a) + to_int(b) - to_int(c)),
        ]
        for w, want in forms:
            r = to_int(norm(w, stats))
            assert r < 2**256 and (r - want) % P == 0


@pytest.mark.parametrize("seed", [21, 22])
def test_mul_chain_model(seed):
    """Dependent chains (results fed back as operands, as the doubling chain
    does): outputs are NORMAL and stay exact."""
    stats = {"resolves": 0, "rare": 0}
    rng = random.Random(seed)
    x, y = rng.getrandbits(256), rng.getrandbits(256)
    a, b = limbs(x), limbs(y)
    for _ in range(300):
        r = mul(a, b, stats)
        x = x * y % P
        assert to_int(r) % P == x
        a = r
