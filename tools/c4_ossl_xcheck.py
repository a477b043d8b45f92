"""C4 at 10^6 items: every WELL-FORMED item's GPU status against OpenSSL
libcrypto (oracle/openssl_ref.c, an independent ECDSA implementation), and
every item's status against the C oracle.  Run on the GPU box:

    python tools/c4_ossl_xcheck.py > profiles/r02_c4_1m_ossl_xcheck.log

Test infrastructure: pins the oracle's ECDSA math and the
device path on the whole adversarial 1M run, not only the golden items.
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from babble_amd import synth  # noqa: E402
from babble_amd.verifier import Verifier  # noqa: E402
from oracle import coracle  # noqa: E402


def main():
    t0 = time.time()
    b = synth.adversarial(1_000_000, seed=4)
    print(f"generated C4: {b.n_items} items, {b.n_keys} keys ({time.time() - t0:.1f}s)", flush=True)
    v = Verifier(0)
    res = v.verify(b)
    print(f"gpu: key_path {v.timing()['key_path']}, statuses {np.bincount(res.status, minlength=4).tolist()}",
          flush=True)
    t0 = time.time()
    o = coracle.ossl_verify_batch(b.as_dict())
    wf = o != coracle.OSSL_SKIP
    print(f"openssl: {int(wf.sum())} well-formed items verified in {time.time() - t0:.1f}s "
          f"({coracle.default_threads()} threads)", flush=True)
    diff = np.flatnonzero(res.status[wf] != o[wf])
    print(f"gpu vs openssl on well-formed items: {diff.size} differences "
          f"(accept {int((o[wf] == 1).sum())}, reject {int((o[wf] == 0).sum())})", flush=True)
    t0 = time.time()
    h, st, bits = coracle.verify_batch(b.as_dict())
    print(f"oracle: {time.time() - t0:.1f}s; gpu vs oracle: statuses equal {np.array_equal(st, res.status)}, "
          f"digests equal {np.array_equal(h, res.msg_hash)}, bits equal {np.array_equal(bits, res.accept_bits)}",
          flush=True)
    v.close()
    ok = diff.size == 0 and np.array_equal(st, res.status) and np.array_equal(h, res.msg_hash)
    print("PASS" if ok else "FAIL")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
