"""k_small phase clocks (BV_SMALL_STAMPS=1: the library prints workgroup 0's
s_memtime stamps per call to stderr) for 1 / 100 events, key cache warm and
cold, beside each call's host wall clock.  Stamps (clocks from the kernel's
first instruction): 1 SHA-256 of the item's message, 2 s^-1, 3 key decode,
4 digest of message b, 5 phase-1 barrier, 6 scalars (u1, u2, GLV), 7/8 the
two G halves, 9/10 the two Q halves, 11 phase-3 barrier, 12 the two pair
sums, 13 the decision.

    python tools/small_stamps.py > gpurun_out/small_stamps.log 2>&1
"""
import os
import sys
import time

os.environ["BV_SMALL_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from babble_amd import native, synth  # noqa: E402
from babble_amd.verifier import Verifier  # noqa: E402


def main():
    for n in (1, 100):
        b = synth.events(n, n_creators=min(4, n), seed=900 + n)
        for name, flags in (("warm", native.F_KEY_CACHE), ("cold", 0)):
            v = Verifier(0, flags=flags)
            if flags:
                v.register_keys([b.key(k) for k in range(b.n_keys)])
            for rep in range(4):
                t0 = time.perf_counter()
                res = v.verify(b)
                ms = (time.perf_counter() - t0) * 1e3
                t = v.timing()
                assert np.all(res.status == 1)
                print(f"{name} n={n} rep={rep} host_ms={ms:.4f} h2d={t['ms_h2d']:.4f} kernel={t['ms_total']:.4f} "
                      f"d2h={t['ms_d2h']:.4f} key_path={t['key_path']}", flush=True)
                sys.stderr.flush()
            v.close()


if __name__ == "__main__":
    main()
