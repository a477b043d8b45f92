"""Host build of the device per-unit source (tests/emu) against the oracle.

The kernels' arithmetic (field.h, point.h, sha256.h, verify_core.h) is
compiled for the CPU and replayed with kernels.hip's index mapping; these
tests catch arithmetic and indexing bugs before any GPU run.  The GPU tests
(test_gpu.py) then check the real kernels bit for bit.
"""
import random

import numpy as np
import pytest

from babble_amd import synth
from oracle import coracle
from oracle import gosemantics as gs
from tests.emu import emu
from tests.helpers import golden_items_batch

P, N = gs.P, gs.N


def test_field_arithmetic_known_answers():
    rng = random.Random(3)
    edge = [0, 1, 2, P - 1, P, P + 1, 2**256 - 1, 2**256 - 2, 2**256 - P, 977, 2**32, 2**255, 2**32 + 977]
    vals = edge + [rng.getrandbits(256) for _ in range(200)]
    for a in vals:
        for b in rng.sample(vals, 6) + edge[:6]:
            assert emu.binop("emu_fe_mul", a, b) == a * b % P
            assert emu.binop("emu_fe_add", a, b) == (a + b) % P
            assert emu.binop("emu_fe_sub", a, b) == (a - b) % P
        assert emu.unop("emu_fe_sqr", a) == a * a % P
    for a in vals[:30]:
        if a % P:
            assert emu.unop("emu_fe_inv", a) == pow(a, -1, P)


def test_scalar_montgomery_and_inverse():
    rng = random.Random(4)
    R = 2**256
    for _ in range(100):
        a, b = rng.getrandbits(256), rng.randrange(N)  # a < R, b < N (the mont precondition)
        assert emu.binop("emu_sc_mont", a, b) == a * b * pow(R, -1, N) % N
    for s in [1, 2, N - 1, N - 2, (N + 1) // 2] + [rng.randrange(1, N) for _ in range(60)]:
        assert emu.unop("emu_sc_inverse", s) == pow(s, -1, N)


def test_divsteps_inversion():
    """modinv.h (variable-time Bernstein-Yang) against Python ints, both moduli,
    including weakly reduced field inputs in [p, 2^256) and sparse operands."""
    rng = random.Random(5)
    fe_vals = [1, 2, 3, P - 1, P - 2, P + 1, P + 2, 2**256 - 1, 2**255, 2**32 + 977, 2**128, 2**30, 2**30 - 1]
    fe_vals += [rng.getrandbits(256) for _ in range(3000)]
    fe_vals += [1 << rng.randrange(256) for _ in range(100)]
    fe_vals += [2**256 - 1 - (1 << rng.randrange(256)) for _ in range(100)]
    for a in fe_vals:
        if a % P:
            assert emu.unop("emu_fe_inv_var", a) == pow(a, -1, P), hex(a)
    sc_vals = [1, 2, 3, N - 1, N - 2, (N + 1) // 2, 2**128, 2**255] + [rng.randrange(1, N) for _ in range(3000)]
    sc_vals += [1 << rng.randrange(255) for _ in range(100)]
    for s in sc_vals:
        assert emu.unop("emu_sc_inverse_var", s) == pow(s, -1, N), hex(s)


LAMBDA = 0x5363AD4CC05C30E0A5261C028812645A122E22EA20816678DF02967C1B23BD72
BETA = 0x7AE96A2B657C07106E64479EAC3434E99CF0497512F58995C1396C28719501EE


def test_glv_constants_and_split():
    """lambda (mod N) and beta (mod p) are cube roots of one with
    lambda * G = (beta * Gx, Gy); the device split k = k1 + k2 lambda has
    |k1|, |k2| < 2^128."""
    import ctypes

    assert pow(LAMBDA, 3, N) == 1 and pow(BETA, 3, P) == 1
    assert gs.scalar_mult(LAMBDA, gs.G) == (BETA * gs.GX % P, gs.GY)
    L = emu.lib()
    L.emu_glv_split.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    rng = random.Random(8)
    ks = [0, 1, 2, N - 1, N - 2, (N - 1) // 2, (N + 1) // 2, LAMBDA, N - LAMBDA, 2**128, 2**128 - 1, 2**255]
    ks += [rng.randrange(N) for _ in range(3000)]
    for k in ks:
        kin = np.array([(k >> (32 * i)) & 0xFFFFFFFF for i in range(8)], np.uint32)
        out = np.zeros(9, np.uint32)
        L.emu_glv_split(kin.ctypes.data, out.ctypes.data)
        m1 = sum(int(out[i]) << (32 * i) for i in range(4))
        m2 = sum(int(out[4 + i]) << (32 * i) for i in range(4))
        k1 = -m1 if out[8] & 1 else m1
        k2 = -m2 if out[8] & 2 else m2
        assert (k1 + k2 * LAMBDA - k) % N == 0, hex(k)


# 5 / 6: K8 / K12 with the key part first (k_verify_qf, then k_verify_gf:
# the host entries' order), reported as modes 1 / 2
@pytest.mark.parametrize("mode", [2, 1, 0, 3, 5, 6])
def test_golden_items(mode):
    batch, expected, _ = golden_items_batch()
    h, st, bits, m = emu.verify_batch(batch.as_dict(), force_mode=mode)
    assert m == (mode - 4 if mode >= 5 else mode)
    assert np.array_equal(st, expected)


@pytest.mark.parametrize("mode", [2, 1, 0, 3, 5, 6])
def test_adversarial_mix(mode):
    b = synth.adversarial(2500, seed=21, n_creators=4, scale_per_million=dict(
        rflip=20000, sflip=20000, body=10000, highs=10000, range=8000, fmt=8000, key=12000))
    h, st, bits = coracle.verify_batch(b.as_dict())
    h2, st2, bits2, _ = emu.verify_batch(b.as_dict(), force_mode=mode)
    assert np.array_equal(h, h2)
    assert np.array_equal(st, st2)
    assert np.array_equal(bits, bits2)
    assert set(np.unique(st)) == {0, 1, 2, 3}


def test_c1_hashgraph_10k_events():
    """C1: 4 peers, 10k events in the InsertEvent play order; all ACCEPT."""
    b = synth.events(10_000, n_creators=4, seed=1)
    h2, st2, bits2, m = emu.verify_batch(b.as_dict())
    assert m == 2 and np.all(st2 == 1)
    for i in (0, 1, 5, 9999):
        assert h2[i].tobytes() == gs.SHA256(b.message(i))


def test_blocks_shared_messages():
    wb = synth.blocks(6, n_validators=20, seed=5)
    b = wb.batch
    # invalidate 5 % of signatures
    rng = np.random.default_rng(1)
    bad = rng.choice(b.n_items, size=b.n_items // 20, replace=False)
    b.s_be[bad, 31] ^= 1
    h, st, bits = coracle.verify_batch(b.as_dict())
    h2, st2, bits2, _ = emu.verify_batch(b.as_dict())
    assert np.array_equal(st, st2) and np.array_equal(h, h2)
    assert int((st2 == 0).sum()) == len(bad)


def test_empty_and_ragged():
    b = synth.events(67, n_creators=3, seed=8)
    h, st, bits = coracle.verify_batch(b.as_dict())
    h2, st2, bits2, _ = emu.verify_batch(b.as_dict())
    assert np.array_equal(st, st2) and len(bits2) == 2 and np.array_equal(bits, bits2)


def test_asan_ubsan_emulator(tmp_path):
    """Host-only AddressSanitizer + UBSan build of the device per-unit source
    (tests/emu/Makefile `asan`, emu_main.cpp) on the golden items plus an
    adversarial mix, in all three key-table modes, against the C oracle."""
    import subprocess

    subprocess.run(["make", "-s", "-C", emu._HERE, "asan"], check=True)
    exe = emu._HERE + "/_build/emu_asan"
    golden, _, _ = golden_items_batch()
    adv = synth.adversarial(700, seed=23, n_creators=3, scale_per_million=dict(
        rflip=20000, sflip=20000, body=10000, highs=10000, range=8000, fmt=8000, key=12000))
    for name, b in (("golden", golden), ("adv", adv)):
        path = str(tmp_path / f"{name}.bin")
        emu.dump_batch(path, b.as_dict())
        r = subprocess.run([exe, path, "4"], capture_output=True, text=True, timeout=600,
                           env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0", "PATH": "/usr/bin:/bin"})
        assert r.returncode == 0, r.stdout + r.stderr
        assert r.stdout.count("equal") == 4 and "MISMATCH" not in r.stdout, r.stdout
    # the product's host DAG hasher (hostdag.cpp + hostsha.cpp) under the
    # sanitizers on random wire batches in exactly-sized buffers
    for seed in (1, 2, 3):
        r = subprocess.run([exe, "dag", str(seed), "700"], capture_output=True, text=True, timeout=600,
                           env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0", "PATH": "/usr/bin:/bin"})
        assert r.returncode == 0, r.stdout + r.stderr
        assert r.stdout.count("equal") == 4 and "MISMATCH" not in r.stdout, r.stdout
