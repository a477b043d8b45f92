"""Copy one GPU evidence pass (tools/gpu_final.sh) from gpurun_out/ into the
tracked profiles/ files: bench line, rocprofv3 kernel stats, GPU test log,
PMC summary, and the verify-kernel traffic / instruction summary bench.py
reads (profiles/kverify_traffic.json)."""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
for src, dst in [("bench.json", f"{tag}_bench.json"), ("prof/run_kernel_stats.csv", f"{tag}_bench_kernel_stats.csv"),
                 ("pytest_gpu.log", f"{tag}_pytest_gpu.log"), ("bench_prof.json", f"{tag}_bench_under_rocprof.json"),
                 ("pmc_summary.json", f"{tag}_pmc_summary.json")]:
    shutil.copy(os.path.join(G, src), os.path.join(P, dst))
d = json.load(open(os.path.join(P, f"{tag}_pmc_summary.json")))
g = next(v for k, v in d.items() if k.startswith("k_verify_g"))
q = next(v for k, v in d.items() if k.startswith("k_verify_q"))
items = 1_000_000
out = {
    "source": f"profiles/{tag}_pmc_summary.json (tools/gpu_pmc.sh: separate rocprofv3 --pmc passes "
              "FETCH_SIZE / WRITE_SIZE / SQ_*, bench.py --events 1000000)",
    "kernels": "k_verify_g + k_verify_q<12,11> (throughput variants)",
    "items_per_launch": items,
    "hbm_bytes_per_launch": g["hbm_bytes"] + q["hbm_bytes"],
    "hbm_read_bytes_uncorrected": (g["counters"]["FETCH_SIZE"] + q["counters"]["FETCH_SIZE"]) * 1024,
    "algorithmic_table_bytes": items * (10 + 22) * 64,  # 10 G windows (26-bit) + 22 K12 windows
    "valu_wave_insts_per_launch": g["valu_wave_insts"] + q["valu_wave_insts"],
    "note": "hbm_bytes applies the guide's x2 FETCH_SIZE correction (calibrated for 16-B/lane streaming reads); "
            "the verify kernels read 64-B table entries by random gather, an uncalibrated width: uncorrected "
            "FETCH_SIZE equals the algorithmic table bytes (32 entries x 64 B per item).",
}
json.dump(out, open(os.path.join(P, "kverify_traffic.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
