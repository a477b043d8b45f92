"""FETCH_SIZE calibration summary (tools/gpu_gather_pmc.sh): per kernel of
tools/ubench_gather.hip, the algorithmic bytes it reads (its own log) over the
memory-side counters of the same dispatch (second repetition, warm):

  fetch_factor   = algorithmic bytes / (FETCH_SIZE KiB x 1024)
  bytes_per_req  = algorithmic bytes / TCC_EA0_RDREQ

The verify kernels' 64-B entry gathers use `gather64`'s factor
(bench.py GATHER_FETCH_FACTOR, pmc_summary.py)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def kernel(name):
    for k in ("k_stream", "k_gather<4>", "k_gather<8>"):
        if k in name:
            return {"k_stream": "stream", "k_gather<4>": "gather64", "k_gather<8>": "gather128"}[k]
    return None


def main(root):
    algo, ms = {}, defaultdict(list)
    for ln in open(os.path.join(root, "gather_time.log")):
        m = re.match(r"(\w+)\s+rep (\d) bytes (\d+) ms ([\d.]+)", ln)
        if m:
            algo[m.group(1)] = int(m.group(3))
            ms[m.group(1)].append(float(m.group(4)))
    cnt = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(root, "gpmc_*", "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        for row in csv.DictReader(open(path, newline="")):
            low = {k.lower(): v for k, v in row.items()}
            k = kernel(low.get("kernel_name", ""))
            if not k:
                continue
            per[(k, low.get("dispatch_id"), low.get("counter_name"))] += float(low["counter_value"])
        for (k, did, c), v in sorted(per.items(), key=lambda x: int(x[0][1] or 0)):
            cnt[k][c].append(v)
    out = {"source": "tools/ubench_gather.hip + tools/gpu_gather_pmc.sh (4 GiB table, past the 256 MiB "
                     "Infinity Cache; counters of the second, warm dispatch of each kernel)"}
    for k, b in algo.items():
        row = {"algorithmic_bytes": b, "ms": ms[k][-1], "gb_s": b / (ms[k][-1] * 1e6)}
        fs = cnt[k].get("FETCH_SIZE")
        if fs:
            row["fetch_size_bytes"] = fs[-1] * 1024
            row["fetch_factor"] = b / (fs[-1] * 1024)
        rq = cnt[k].get("TCC_EA0_RDREQ_sum")
        if rq:
            row["rdreq"] = rq[-1]
            row["bytes_per_rdreq"] = b / rq[-1]
        r32 = cnt[k].get("TCC_EA0_RDREQ_32B_sum")
        if r32:
            row["rdreq_32b"] = r32[-1]
        out[k] = row
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
