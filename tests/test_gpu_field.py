"""Device field / scalar primitives (the generated gfx950 inline asm of
babble_amd/csrc/field_asm.h, through tests/fieldcheck/libfieldcheck.so)
checked against Python integers: fe_mul / fe_sqr / fe_add / fe_sub mod p
(weakly reduced: < 2^256 and congruent), sc_mont (a b 2^-256 mod N, < N) and
fe_inv_var.  Operands include limb patterns that drive every rare block of
the programs (fold carry-outs, tails), so the hardware's carry / hazard
behaviour is exercised, not just the generator's interpreter."""
import ctypes
import os
import random

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "fieldcheck", "libfieldcheck.so")
P = 2**256 - 2**32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
M32 = 2**32 - 1
OPS = {"mul": 0, "sqr": 1, "add": 2, "sub": 3, "mont": 4, "inv": 5,
       "zssm0": 6, "zssm1": 7, "zssm2": 8, "zsss0": 9, "zsss1": 10, "zsss2": 11, "cneg": 12}

pytestmark = pytest.mark.gpu


def _lib():
    if not os.path.exists(LIB):
        pytest.fail("tests/fieldcheck/libfieldcheck.so missing: run __graft_entry__.build()")
    import torch  # noqa: F401  (bind the same HIP runtime torch uses, as babble_amd.native does)

    L = ctypes.CDLL(LIB)
    L.fc_run.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.fc_run.restype = ctypes.c_int
    return L


def _pack(xs):
    out = np.zeros((len(xs), 8), dtype=np.uint32)
    for i, x in enumerate(xs):
        for k in range(8):
            out[i, k] = (x >> (32 * k)) & M32
    return out


def _unpack(arr):
    return [sum(int(arr[i, k]) << (32 * k) for k in range(8)) for i in range(arr.shape[0])]


def _run(op, a, b):
    A, B = _pack(a), _pack(b)
    R = np.zeros_like(A)
    rc = _lib().fc_run(OPS[op], len(a), A.ctypes.data, B.ctypes.data, R.ctypes.data)
    assert rc == 0, rc
    return _unpack(R)


def _operands(seed, n):
    rng = random.Random(seed)
    K = 2**32 + 977
    edge = [0, 1, 2, 977, M32, 2**32, P - 1, P, P + 1, 2**256 - 1, 2**256 - 2, 2**256 - K, 2**256 - K - 1,
            2**256 - K + 1, 2**255, 2**255 - 1, 2 * K, N - 1, N, N + 1]
    top = [2**256 - 1 - rng.getrandbits(rng.choice([1, 8, 16, 40, 64, 128, 200])) for _ in range(n // 4)]
    limbs = [sum(rng.choice([0, M32, M32 - 977, M32 - 976, 1, 2**31]) << (32 * i) for i in range(8))
             for _ in range(n // 4)]
    return edge + top + limbs + [rng.getrandbits(256) for _ in range(n)]


def _pairs(n=4000, seed=11):
    xs = _operands(seed, n // 2)
    ys = _operands(seed + 1, n // 2)
    rng = random.Random(seed + 2)
    a = [rng.choice(xs) for _ in range(n)] + xs
    b = [rng.choice(ys) for _ in range(n)] + [rng.choice(ys) for _ in xs]
    return a, b


@pytest.mark.parametrize("op", ["mul", "sqr", "add", "sub"])
def test_field_ops_match_python_ints(op):
    a, b = _pairs()
    if op == "sqr":
        b = a
    r = _run(op, a, b)
    want = {"mul": lambda x, y: x * y, "sqr": lambda x, y: x * x, "add": lambda x, y: x + y,
            "sub": lambda x, y: x - y}[op]
    bad = [(hex(x), hex(y), hex(z)) for x, y, z in zip(a, b, r) if z >= 2**256 or (z - want(x, y)) % P]
    assert not bad, bad[:5]


def test_fold_carry_blocks_are_hit_and_exact():
    """Products whose high limbs are near 2^32 make Y_i = w_i + (2^32+977) w_(i+8)
    carry out of 64 bits (fe_mul's rare mid block) and R_8 wrap (c9)."""
    rng = random.Random(5)
    a, b = [], []
    for _ in range(4096):
        x = 2**256 - 1 - rng.getrandbits(rng.choice([1, 4, 12, 33, 70]))
        y = 2**256 - 1 - rng.getrandbits(rng.choice([1, 4, 12, 33, 70]))
        a.append(x)
        b.append(y)
    for op in ("mul", "sqr"):
        bb = a if op == "sqr" else b
        r = _run(op, a, bb)
        for x, y, z in zip(a, bb, r):
            assert z < 2**256 and (z - x * y) % P == 0, (op, hex(x), hex(y), hex(z))


def test_add_sub_carry_propagation_blocks_are_exact():
    """fe_add / fe_sub apply K = 2^32 + 977 to limbs 0..1 after a wrap and
    propagate the carry through limbs 2..7 in a rare block: operand pairs
    whose wrapped sum / difference has limbs 0..1 within K of 2^64 (and
    limbs 2..7 all ones, which wrap a second time) enter it."""
    rng = random.Random(9)
    K = 2**32 + 977
    a_add, b_add, a_sub, b_sub = [], [], [], []
    for _ in range(4096):
        lo = 2**64 - 1 - rng.randrange(K + 8)             # low 64 bits of the wrapped value
        hi = rng.choice([rng.getrandbits(192), 2**192 - 1, 2**192 - 2, 0])
        w = (hi << 64) | lo                                # the wrapped value, < 2^256
        a = rng.getrandbits(256)
        if w + 2**256 - a < 2**256:                        # a + b = 2^256 + w
            a_add.append(a)
            b_add.append(w + 2**256 - a)
        lo2 = rng.randrange(K + 8)                         # a - b + 2^256 = w2, limbs 0..1 < K
        w2 = (rng.choice([rng.getrandbits(192), 0, 2**192 - 1]) << 64) | lo2
        b = rng.getrandbits(256)
        if b >= 2**256 - w2 and b + w2 - 2**256 < b:       # a = b + w2 - 2^256 >= 0, a < b
            a_sub.append(b + w2 - 2**256)
            b_sub.append(b)
    assert len(a_add) > 1000 and len(a_sub) > 1000
    for op, xs, ys, f in (("add", a_add, b_add, lambda x, y: x + y), ("sub", a_sub, b_sub, lambda x, y: x - y)):
        r = _run(op, xs, ys)
        bad = [(hex(x), hex(y), hex(z)) for x, y, z in zip(xs, ys, r) if z >= 2**256 or (z - f(x, y)) % P]
        assert not bad, (op, bad[:5])


def test_cneg_canon_matches_python_ints():
    """fe_cneg_canon (the signed-digit table lookups' y negation) on
    canonical operands, including limb patterns that borrow past limb 1."""
    rng = random.Random(13)
    xs = [0, 1, P - 1, P - 2, 2**64 - 1, 2**64, 2**64 - 977, 2**32 + 976, 2**32 + 977, 2**32 + 978]
    xs += [(rng.getrandbits(192) << 64) | rng.choice([0xFFFFFFFFFFFFFFFF, 0xFFFFFFFF00000000 | rng.getrandbits(32),
                                                        0xFFFFFFFEFFFFFC2F, rng.getrandbits(64)])
           for _ in range(3000)]
    xs = [x % P for x in xs]
    flags = [rng.getrandbits(1) for _ in xs]
    r = _run("cneg", xs, flags)
    bad = [(hex(x), f, hex(z)) for x, f, z in zip(xs, flags, r)
           if z >= 2**256 or (z - (-x if f else x)) % P or (not f and z != x)]
    assert not bad, bad[:5]


def test_sc_mont_matches_python_ints():
    a, b = _pairs(3000, 21)
    b = [y % N for y in b]
    r = _run("mont", a, b)
    rinv = pow(2**256, -1, N)
    bad = [(hex(x), hex(y), hex(z)) for x, y, z in zip(a, b, r) if z >= N or z != x * y * rinv % N]
    assert not bad, bad[:5]


def test_fe_inv_var_matches_python_ints():
    a, _ = _pairs(2000, 31)
    a = [x for x in a if x % P]
    r = _run("inv", a, a)
    bad = [(hex(x), hex(z)) for x, z in zip(a, r) if (z * x - 1) % P]
    assert not bad, bad[:5]


@pytest.mark.parametrize("combo", ["zssm", "zsss"])
def test_zipped_programs_match_python_ints(combo):
    """The interleaved multi-product programs of the key-table doubling chain
    (gen_zip: fe_sqr_sqr_mul_zip / fe_sqr_sqr_sqr_zip), every component, on
    operands that also drive each program's rare blocks."""
    a, b = _pairs(3000, 41)
    rng = random.Random(43)
    for _ in range(1500):  # near-2^256 limbs: fold carry-outs in all three programs at once
        a.append(2**256 - 1 - rng.getrandbits(rng.choice([1, 4, 12, 33, 70])))
        b.append(2**256 - 1 - rng.getrandbits(rng.choice([1, 4, 12, 33, 70])))
    want = {"zssm": [lambda x, y: x * x, lambda x, y: y * y, lambda x, y: x * y],
            "zsss": [lambda x, y: x * x, lambda x, y: y * y, lambda x, y: (x ^ y) ** 2]}[combo]
    for k in range(3):
        r = _run(f"{combo}{k}", a, b)
        bad = [(hex(x), hex(y), hex(z)) for x, y, z in zip(a, b, r) if z >= 2**256 or (z - want[k](x, y)) % P]
        assert not bad, (k, bad[:5])


def _ec_add(p1, p2):
    """Affine secp256k1 addition over Python ints (None = identity)."""
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    (x1, y1), (x2, y2) = p1, p2
    if x1 == x2 and (y1 + y2) % P == 0:
        return None
    if p1 == p2:
        lam = 3 * x1 * x1 * pow(2 * y1, -1, P) % P
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, P) % P
    x3 = (lam * lam - x1 - x2) % P
    return x3, (lam * (x1 - x3) - y1) % P


def _ec_mul(k, pt):
    acc = None
    for bit in bin(k)[2:]:
        acc = _ec_add(acc, acc)
        if bit == "1":
            acc = _ec_add(acc, pt)
    return acc


@pytest.mark.parametrize("lat", [0, 1], ids=["gexz_add_ge", "gexz_add_ge_lat"])
def test_xyzz_mixed_add_exceptional_cases(lat):
    """the XYZZ mixed addition of the verify kernels (point.h,
    madd-2008-s; the zipped latency variant too) on the device, against
    Python integers, with the accumulator in random projective form (X = x
    z^2, Y = y z^3, ZZ = z^2, ZZZ = z^3): generic sums, P + P (the
    dbl-2008-s-1 doubling branch), P + (-P) (the identity) and the identity
    plus a point.  Results compared as affine points (X / ZZ, Y / ZZZ)."""
    G = (0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
         0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8)
    rng = random.Random(17 + lat)
    accs, pts, want = [], [], []
    for i in range(256):
        a = _ec_mul(rng.randrange(1, N), G)
        kind = i % 4
        b = a if kind == 1 else ((a[0], P - a[1]) if kind == 2 else _ec_mul(rng.randrange(1, N), G))
        z = rng.randrange(1, P)
        zz, zzz = z * z % P, z * z * z % P
        if kind == 3:
            accs.append([0, 0, 0, 0, 1])
            want.append(b)
        else:
            accs.append([a[0] * zz % P, a[1] * zzz % P, zz, zzz, 0])
            want.append(_ec_add(a, b))
        pts.append(b)
    A = np.zeros((len(accs), 33), np.uint32)
    Q = np.zeros((len(pts), 16), np.uint32)
    for i, (acc, pt) in enumerate(zip(accs, pts)):
        for j in range(4):
            A[i, 8 * j:8 * j + 8] = _pack([acc[j]])[0]
        A[i, 32] = acc[4]
        Q[i, :8], Q[i, 8:] = _pack([pt[0]])[0], _pack([pt[1]])[0]
    R = np.zeros_like(A)
    L = _lib()
    L.fc_xyzz.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.fc_xyzz.restype = ctypes.c_int
    assert L.fc_xyzz(lat, len(accs), A.ctypes.data, Q.ctypes.data, R.ctypes.data) == 0
    for i, w in enumerate(want):
        X, Y, ZZ, ZZZ = (_unpack(R[i:i + 1, 8 * j:8 * j + 8])[0] % P for j in range(4))
        if w is None:
            assert R[i, 32] == 1, (i, "expected the identity")
            continue
        assert R[i, 32] == 0, i
        assert ZZ and pow(ZZ, 3, P) == pow(ZZZ, 2, P), i
        assert (X * pow(ZZ, -1, P) % P, Y * pow(ZZZ, -1, P) % P) == w, (i, i % 4)


def test_coop_mul_norm_match_python_ints():
    """coop.h's cooperative product and WIDE reduction (one field element
    per 16-lane DPP row, ONE carry resolve each since round 6) on hardware
    against Python integers, over the edge-heavy operands of the per-lane
    tests plus values whose top limbs are all ones (the unresolved folds'
    largest digits and tail()'s rare second fold).  The digit bounds behind
    the single resolve are asserted by tests/test_coop_model.py."""
    rng = random.Random(31)
    a, b = _pairs(n=6000, seed=41)
    tops = [2**256 - 1 - rng.getrandbits(rng.choice([1, 4, 12, 33, 70])) for _ in range(4000)]
    a += tops
    b += [rng.choice(tops) for _ in tops]
    a = [x % 2**256 for x in a]
    b = [x % 2**256 for x in b]
    A, B = _pack(a), _pack(b)
    L = _lib()
    L.fc_coop_ops.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.fc_coop_ops.restype = ctypes.c_int
    want = {0: lambda x, y: x * y, 1: lambda x, y: x - y, 2: lambda x, y: x - 8 * y, 3: lambda x, y: 3 * x}
    for op, f in want.items():
        R = np.zeros_like(A)
        assert L.fc_coop_ops(op, len(a), A.ctypes.data, B.ctypes.data, R.ctypes.data) == 0
        r = _unpack(R)
        bad = [(op, hex(x), hex(y), hex(z)) for x, y, z in zip(a, b, r) if z >= 2**256 or (z - f(x, y)) % P]
        assert not bad, bad[:5]


def test_coop_xyzz_add_and_double():
    """The wave-cooperative XYZZ addition and doubling of k_small's cold
    path (coop.h add_xyzz / dbl_xyzz: one point per wave, the products of a
    level spread over the four DPP rows), against Python integers.  Both
    operands in random projective form; generic sums, P + P (the doubling
    branch), P + (-P) (the identity), the identity plus a point, and points
    with extreme coordinates.  The doubling's fourth product is beta X3
    (phi's x of the result)."""
    G = (0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
         0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8)
    beta = 0x7AE96A2B657C07106E64479EAC3434E99CF0497512F58995C1396C28719501EE
    rng = random.Random(29)

    def proj(pt, z):
        zz, zzz = z * z % P, z * z * z % P
        return [pt[0] * zz % P, pt[1] * zzz % P, zz, zzz, 0]

    accs, pts, want = [], [], []
    extreme = [_ec_mul(N - 1, G), _ec_mul(2, G), G]
    for i in range(192):
        a = extreme[i % 3] if i < 12 else _ec_mul(rng.randrange(1, N), G)
        kind = i % 4
        b = a if kind == 1 else ((a[0], P - a[1]) if kind == 2 else _ec_mul(rng.randrange(1, N), G))
        za = 1 if i % 16 == 0 else rng.randrange(1, P)
        zb = 1 if i % 8 == 0 else (P - 1 if i % 8 == 1 else rng.randrange(1, P))
        accs.append([0, 0, 0, 0, 1] if kind == 3 else proj(a, za))
        want.append(b if kind == 3 else _ec_add(a, b))
        pts.append((b, proj(b, zb)))
    A = np.zeros((len(accs), 33), np.uint32)
    B = np.zeros((len(pts), 33), np.uint32)
    for i, (acc, (_, pb)) in enumerate(zip(accs, pts)):
        for j in range(4):
            A[i, 8 * j:8 * j + 8] = _pack([acc[j]])[0]
            B[i, 8 * j:8 * j + 8] = _pack([pb[j]])[0]
        A[i, 32] = acc[4]
    R = np.zeros((len(accs), 74), np.uint32)
    L = _lib()
    L.fc_coop_xyzz.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.fc_coop_xyzz.restype = ctypes.c_int
    assert L.fc_coop_xyzz(len(accs), A.ctypes.data, B.ctypes.data, R.ctypes.data) == 0

    def affine(o):
        X, Y, ZZ, ZZZ = (_unpack(R[i:i + 1, o + 8 * j:o + 8 * j + 8])[0] % P for j in range(4))
        assert ZZ and pow(ZZ, 3, P) == pow(ZZZ, 2, P), i
        return X, ZZ, (X * pow(ZZ, -1, P) % P, Y * pow(ZZZ, -1, P) % P)

    for i, w in enumerate(want):
        if w is None:
            assert R[i, 32] == 1, (i, "expected the identity")
        else:
            assert R[i, 32] == 0, i
            assert affine(0)[2] == w, (i, i % 4)
        b = pts[i][0]
        X, ZZ, d = affine(33)
        assert d == _ec_add(b, b), i
        BX = _unpack(R[i:i + 1, 66:74])[0] % P
        assert BX == beta * X % P, i


@pytest.mark.parametrize("w,nwin", [(6, 22), (8, 16), (11, 12)], ids=["K12", "K8", "KC"])
def test_coop_base_chain_equals_per_lane(w, nwin):
    """The wave-cooperative base chain (coop.h: field elements in 16-lane DPP
    rows, the doubling's products spread over the rows, carry-lookahead over
    lane masks) equals the per-lane zipped chain (table_bases_one) mod p on
    every base of every key-table geometry, for random points and points
    with extreme limb patterns (x or y near 0 / p), and prints both chain
    latencies (one key, one wave)."""
    G = (0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
         0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8)
    rng = random.Random(w)
    pts = [_ec_mul(rng.randrange(1, N), G) for _ in range(60)]
    pts += [G, _ec_mul(2, G), _ec_mul(N - 1, G), _ec_mul(3, G)]
    xy = np.zeros((len(pts), 16), np.uint32)
    for i, (x, y) in enumerate(pts):
        xy[i, :8], xy[i, 8:] = _pack([x])[0], _pack([y])[0]
    L = _lib()
    L.fc_bases.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                           ctypes.POINTER(ctypes.c_float)]
    L.fc_bases.restype = ctypes.c_int
    outs, ms = [], []
    for coop in (0, 1):
        out = np.zeros((len(pts), nwin, 24), np.uint32)
        t = ctypes.c_float()
        assert L.fc_bases(coop, len(pts), xy.ctypes.data, out.ctypes.data, w, nwin, ctypes.byref(t)) == 0
        outs.append(out)
        ms.append(t.value)
    for i in range(len(pts)):
        for j in range(nwin):
            a = [_unpack(outs[0][i:i + 1, j, 8 * c:8 * c + 8])[0] % P for c in range(3)]
            b = [_unpack(outs[1][i:i + 1, j, 8 * c:8 * c + 8])[0] % P for c in range(3)]
            assert a == b, (i, j)
    # the chain's first base is the point itself; the last is 2^(w (nwin-1)) P
    X, Y, Z = [_unpack(outs[1][0:1, nwin - 1, 8 * c:8 * c + 8])[0] % P for c in range(3)]
    zi = pow(Z, -1, P)
    assert (X * zi * zi % P, Y * zi * zi * zi % P) == _ec_mul(2 ** (w * (nwin - 1)), pts[0])
    print(f"\nbase chain {w}x{nwin - 1} doublings, {len(pts)} keys: per-lane {ms[0]:.3f} ms, coop {ms[1]:.3f} ms")
