"""Debug: a process's first cold k_small batch with a BV_SMALL_DUMP library
(tools/build_variant.sh gpurun_var/dump.so -DBV_SMALL_DUMP=1): for every
item whose status differs from the oracle, each cold-path intermediate
against Python big-int values (development tool).  PROCS children."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("CHILD") is None:
    for p in range(int(os.environ.get("PROCS", "12"))):
        r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__)], env=dict(os.environ, CHILD="1"),
                           capture_output=True, text=True, timeout=120)
        out = [x for x in r.stdout.splitlines() if x.strip()]
        print(p, r.returncode, "\n   ".join(out[-14:]) if out else r.stderr[-400:], flush=True)
    sys.exit(0)
import hashlib  # noqa: E402

import numpy as np  # noqa: E402

from babble_amd import native  # noqa: E402
from babble_amd.batch import BatchBuilder  # noqa: E402
from oracle import coracle  # noqa: E402
from oracle import gosemantics as gs  # noqa: E402
from tests.test_bootstrap import make_db  # noqa: E402

native.LIB_PATH = os.path.abspath(os.environ.get("AB_LIB", "gpurun_var/dump.so"))
native._lib = None
from babble_amd.verifier import Verifier  # noqa: E402

dump_file = f"/tmp/bv_dump_{os.getpid()}.bin"
os.environ["BV_SMALL_DUMP_FILE"] = dump_file
evs = make_db(500)
bb = BatchBuilder()
for ev in evs:
    bb.add_item(bb.add_msg(ev.Body.Marshal()), bb.add_key(ev.Body.Creator or b""), ev.Signature)
p = bb.pack()
v = Verifier(0)
res = v.verify(p)
h, st, _ = coracle.verify_batch(p.as_dict())
bad = np.flatnonzero(res.status != st)
print(f"mismatches {bad.size} {bad[:6].tolist()}")
if bad.size:
    D = np.fromfile(dump_file, dtype=np.uint32).reshape(-1, 256)
    P, N = gs.P, gs.N
    BETA = 0x7AE96A2B657C07106E64479EAC3434E99CF0497512F58995C1396C28719501EE
    LAM = 0x5363AD4CC05C30E0A5261C028812645A122E22EA20816678DF02967C1B23BD72
    G = (gs.GX, gs.GY)
    Q = gs.Unmarshal(bytes(p.key_bytes[p.key_off[0]:p.key_off[1]]))

    def limbs(a):
        return sum(int(x) << (32 * k) for k, x in enumerate(a))

    def node(a):  # XYZZ node -> affine (None = identity)
        if a[32]:
            return None
        X, Y, ZZ, ZZZ = (limbs(a[8 * j:8 * j + 8]) % P for j in range(4))
        return (X * pow(ZZ, -1, P) % P, Y * pow(ZZZ, -1, P) % P)

    def neg(pt):
        return None if pt is None else (pt[0], (-pt[1]) % P)

    for i in bad[:3]:
        d = D[i]
        r = int.from_bytes(bytes(p.r_be[i]), "big")
        s = int.from_bytes(bytes(p.s_be[i]), "big")
        e = int.from_bytes(hashlib.sha256(bytes(p.msg_bytes[p.msg_off[i]:p.msg_off[i + 1]])).digest(), "big")
        w = pow(s, -1, N)
        u1, u2 = e * w % N, r * w % N
        R = 2 ** 256 % N
        print(f"item {i}: w ok {limbs(d[8:16]) % N == w * R % N}  u1 ok {limbs(d[0:8]) % N == u1}")
        k1, k2, signs, nb = limbs(d[49:53]), limbs(d[53:57]), int(d[57]), int(d[58])
        k1s = -k1 if signs & 1 else k1
        k2s = -k2 if signs & 2 else k2
        print(f"  glv ok {(k1s + k2s * LAM - u2) % N == 0}  nb {nb}  k1 bits {k1.bit_length()} k2 bits {k2.bit_length()}")
        gsum = node(d[16:49])
        print(f"  G sum ok {gsum == gs.scalar_mult(u1, G)}")
        phiQ = (BETA * Q[0] % P, Q[1])
        a2 = node(d[64:97])
        print(f"  acc2 (k2 phi(Q)) ok {a2 == gs.scalar_mult(k2s % N, phiQ)}")
        a1 = node(d[100:133])
        want1 = gs.point_add(gs.scalar_mult(u1, G), gs.scalar_mult(k1s % N, Q))
        print(f"  acc1 (u1 G + k1 Q) ok {a1 == want1}  g added at bit {int(d[140])}  "
              f"acc1 - u1G == k1Q {gs.point_add(a1, neg(gs.scalar_mult(u1, G))) == gs.scalar_mult(k1s % N, Q) if a1 else None}")
v.close()
