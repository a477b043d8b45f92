"""Per-variant, per-kernel averages of the counters of tools/gpu_pmc_ab.sh
(development tool): python tools/pmc_ab_summary.py gpurun_out"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1]
out = {}
for d in sorted(glob.glob(os.path.join(root, "pmcab_*"))):
    if not os.path.isdir(d):
        continue
    v = os.path.basename(d)[len("pmcab_"):]
    vals = defaultdict(lambda: defaultdict(float))
    dur = defaultdict(dict)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                low = {k.lower(): x for k, x in row.items()}
                name = low.get("kernel_name", "?").split("(")[0].replace("void ", "").strip()
                if "k_verify" not in name and "k_sha256" != name and "k_sinv" != name:
                    continue
                did = low.get("dispatch_id")
                try:
                    vals[name][(did, low.get("counter_name"))] += float(low.get("counter_value", "nan"))
                    dur[name][did] = (int(low["end_timestamp"]) - int(low["start_timestamp"])) * 1e-6
                except (KeyError, ValueError):
                    pass
    res = {}
    for name, cv in vals.items():
        per = defaultdict(list)
        for (did, c), x in cv.items():
            per[c].append(x)
        res[name] = {c: sum(xs) / len(xs) for c, xs in per.items()}
        res[name]["dispatches"] = len(dur[name])
        res[name]["ms_profiled_median"] = sorted(dur[name].values())[len(dur[name]) // 2]
    out[v] = res
json.dump(out, sys.stdout, indent=1)
