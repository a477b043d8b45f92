"""Summarise rocprofv3 --pmc passes (tools/gpu_pmc.sh) per kernel.

    python tools/pmc_summary.py gpurun_out > summary.json

Reads every gpurun_out/pmc_*/**/*counter_collection.csv, averages each
counter per dispatch of each kernel, and derives:
  * hbm_read_bytes  = FETCH_SIZE (KiB) x 1024 x f, f per kernel from the
    calibration of the kernel's access pattern (profiles/r05_gather_calib.json,
    tools/ubench_gather.hip): 1.00 for the verify kernels, whose reads are
    random 64-B table entries (64 B per TCC_EA0_RDREQ: counted exactly), 2.00
    for the streaming kernels (16 B per lane, 128-B requests tallied at 64 B —
    MI355X_MICROARCH.md §HBM)
  * hbm_write_bytes = WRITE_SIZE (KiB) x 1024       (exact for wide stores)
  * valu_issue_util = (SQ_INSTS_VALU_INT64 x 5.39 + other SQ_INSTS_VALU x 3.03)
    / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): the fraction of SIMD cycles spent
    issuing VALU instructions, with the per-class issue costs measured on
    gfx950 (profiles/r01_ubench_ops.txt: v_mad_u64_u32 5.39 cycles per wave64
    instruction, 32-bit VALU 3.03).  On ROCm 7.2 / gfx950 SQ_ACTIVE_INST_VALU
    equals SQ_INSTS_VALU (an instruction count, not quad-cycles), so the
    gfx94x VALUBusy formula over-counts; this one is <= 1 up to noise.
  * valu_issue_util_mix = valu_issue_util x the kernel's static opcode-mix
    scale (tools/isa_mix.py): a diagnostic only — single-opcode costs do not
    add in mixed streams (the verify kernels read 1.12-1.13 on it)
  * valu_insts_per_s (wave instructions x 64 lanes / kernel time)
Writes nothing itself; bench.py reads profiles/kverify_traffic.json, which is
this script's output for k_verify_q copied into profiles/.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict

N_CU = 256
N_XCD = 8
CYC_MAD64, CYC_VALU32 = 5.39, 3.03  # profiles/r01_ubench_ops.txt


def short(name: str) -> str:
    n = name.split("(")[0]
    for tok in ("void ", "__global__ "):
        n = n.replace(tok, "")
    return n.strip()


def load(root: str):
    # per kernel -> counter -> list of (dispatch_id, value); also durations
    vals = defaultdict(lambda: defaultdict(dict))
    dur = defaultdict(dict)
    for path in glob.glob(os.path.join(root, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        pas = os.path.relpath(path, root).split(os.sep)[0]
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                low = {k.lower(): v for k, v in row.items()}
                k = short(low.get("kernel_name", "?"))
                did = (pas, low.get("dispatch_id") or low.get("correlation_id"))
                cname = low.get("counter_name")
                try:
                    v = float(low.get("counter_value", "nan"))
                except ValueError:
                    continue
                # per-dimension rows of one counter in one dispatch are summed
                vals[k][cname][did] = vals[k][cname].get(did, 0.0) + v
                try:
                    dur[k][did] = (int(low["end_timestamp"]) - int(low["start_timestamp"])) * 1e-9
                except (KeyError, ValueError):
                    pass
    return vals, dur


# FETCH_SIZE correction per kernel access pattern (profiles/r05_gather_calib.json):
# random 64-B gathers are counted exactly, 16-B/lane streams at half
GATHER_KERNELS = ("k_verify_g", "k_verify_q", "k_verify_gq", "k_verify_generic", "k_small")


def fetch_factor(kernel: str) -> float:
    return 1.0 if kernel.startswith(GATHER_KERNELS) else 2.0


def isa_scales() -> dict:
    """Per-kernel issue-cost scale of the static opcode mix over the
    two-class model (tools/isa_mix.py -> profiles/r05_isa_mix.json)."""
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r05_isa_mix.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return {}
    return {k: v["issue_scale"] for k, v in d.items() if isinstance(v, dict)}


def summarise(root: str) -> dict:
    vals, dur = load(root)
    scales = isa_scales()
    out = {}
    for k, counters in vals.items():
        avg = {c: sum(d.values()) / len(d) for c, d in counters.items() if d}
        n_disp = max(len(d) for d in counters.values())
        durs = list(dur[k].values())
        t = sum(durs) / len(durs) if durs else None
        e = {"dispatches_per_pass": n_disp, "counters": avg, "avg_duration_s_profiled": t}
        if "FETCH_SIZE" in avg:
            e["fetch_factor"] = fetch_factor(k)
            e["hbm_read_bytes"] = avg["FETCH_SIZE"] * 1024 * fetch_factor(k)
        if "WRITE_SIZE" in avg:
            e["hbm_write_bytes"] = avg["WRITE_SIZE"] * 1024
        if "hbm_read_bytes" in e and "hbm_write_bytes" in e:
            e["hbm_bytes"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
        if "SQ_INSTS_VALU" in avg and "SQ_INSTS_VALU_INT64" in avg and avg.get("GRBM_GUI_ACTIVE"):
            i64 = avg["SQ_INSTS_VALU_INT64"]
            cyc = i64 * CYC_MAD64 + (avg["SQ_INSTS_VALU"] - i64) * CYC_VALU32
            e["valu_issue_util"] = cyc / (N_CU * 4) / (avg["GRBM_GUI_ACTIVE"] / N_XCD)
            sc = next((v for name, v in scales.items() if k.startswith(name)), None)
            if sc is not None:  # with the kernel's measured opcode mix
                e["valu_issue_util_mix"] = e["valu_issue_util"] * sc
        if "SQ_INSTS_VALU" in avg and t:
            e["valu_wave_insts"] = avg["SQ_INSTS_VALU"]
            e["valu_lane_ops_per_s"] = avg["SQ_INSTS_VALU"] * 64 / t
        if "GRBM_GUI_ACTIVE" in avg and t:
            e["effective_clock_ghz"] = avg["GRBM_GUI_ACTIVE"] / N_XCD / t / 1e9
        out[k] = e
    return out


def kverify(summary: dict, items: int, source: str) -> dict:
    """The record bench.py reads (profiles/r02_kverify_pmc.json): PMC totals
    of k_verify_g + k_verify_q<12,11> per launch pair."""
    ks = [k for k in summary if k.startswith("k_verify_g") or k.startswith("k_verify_q<12")]
    tot = lambda f: sum(summary[k].get(f, 0.0) for k in ks)  # noqa: E731
    cnt = lambda c: sum(summary[k]["counters"].get(c, 0.0) for k in ks)  # noqa: E731
    # algorithmic bytes per item: 32 table entries of 64 B (10 G windows +
    # 22 K12 windows) plus the SoA streams the two kernels read and write
    # (r, w, digest, pre, item_key, item_msg, key status ~110 B; R_G 132 B
    # written by k_verify_g and read back by k_verify_q; u12 48 B read by
    # k_verify_q — k_glv_split writes it since round 6; status 1 B)
    table, stream = 32 * 64, 110 + 2 * 132 + 48 + 1
    return {"source": source, "kernels": ks, "items_per_launch": items,
            "hbm_bytes_per_launch": tot("hbm_bytes"), "hbm_read_bytes_uncorrected": cnt("FETCH_SIZE") * 1024,
            "fetch_factor": "1.00 (64-B gathers, profiles/r05_gather_calib.json)",
            "algorithmic_table_bytes": items * table,
            "algorithmic_bytes": items * (table + stream),
            "traffic_over_algorithmic": tot("hbm_bytes") / (items * (table + stream)),
            "valu_wave_insts": cnt("SQ_INSTS_VALU"), "valu_int64_wave_insts": cnt("SQ_INSTS_VALU_INT64"),
            "valu_issue_util": {k: summary[k].get("valu_issue_util") for k in ks}}


if __name__ == "__main__":
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    s = summarise(root)
    if len(sys.argv) > 3:  # <root> <items> <kverify-out.json>
        with open(sys.argv[3], "w") as f:
            json.dump(kverify(s, int(sys.argv[2]), f"{sys.argv[3]} <- tools/gpu_pmc.sh passes over bench.py "
                              f"--no-extras --events {sys.argv[2]}"), f, indent=1)
    print(json.dumps(s, indent=1, sort_keys=True))
