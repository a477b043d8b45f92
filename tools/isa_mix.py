"""Static VALU opcode mix of kernels in a gfx950 assembly listing, weighted
by the measured per-opcode issue costs (profiles/r03_ubench_ops.txt:
cycles per wave64 instruction at full occupancy), as a check on the PMC
summary's two-class issue model (v_mad_u64_u32 5.39 cycles, every other VALU
3.03).  A kernel whose mix is heavy in slower 32-bit ops (v_alignbit,
v_add3, v_perm: ~4.6-4.7 cycles) is busier than the two-class model says.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -x hip \\
        babble_amd/csrc/kernels.hip -o /tmp/kernels.s
    python tools/isa_mix.py /tmp/kernels.s k_sha256 k_verify_q k_verify_g > profiles/r05_isa_mix.json

The mix is static (each unrolled body counted once); for a kernel that is
one unrolled loop body (k_sha256's compression) it is the dynamic mix.
Inline-asm lines (the generated field arithmetic) carry no indent in the
listing and are counted too.

What it showed (round 5): the single-opcode costs do NOT add up in a mixed
stream.  Weighted by them, k_verify_g / k_verify_q would issue at 1.12-1.13
(impossible: the mads and carry ops overlap), k_sha256 at 0.89.  So the mix
model is a diagnostic, not a utilisation; the floor of k_sha256 was settled
by timing instead: the kernel runs within 2 % of the same compressions with
the words in registers (profiles/r05_ubench_sha_tp.txt).
"""
import json
import os
import re
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OPS_FILE = os.path.join(ROOT, "profiles", "r03_ubench_ops.txt")
DEFAULT = 3.03  # the two-class model's 32-bit VALU cost


def measured_costs():
    costs = {}
    for ln in open(OPS_FILE):
        m = re.match(r"(v_[a-z0-9_]+)\s+[\d.]+ ms\s+[\d.]+ T lane-ops/s\s+([\d.]+) cycles", ln)
        if m:
            costs[m.group(1)] = float(m.group(2))
    return costs


def cost_of(op, costs):
    base = re.sub(r"_e(32|64)$", "", op)
    for k in (op, base):
        if k in costs:
            return costs[k], True
    for k, v in costs.items():  # opcode family (v_addc_co_u32_e64 -> v_addc_co_u32)
        if re.sub(r"_e(32|64)$", "", k) == base:
            return v, True
    return DEFAULT, False


def kernel_body(asm, name):
    lines = asm.splitlines()
    for i, ln in enumerate(lines):
        if re.match(r"^_Z\d+" + re.escape(name) + r"[A-Za-z0-9_]*:", ln):
            body = []
            for x in lines[i + 1:]:
                body.append(x)
                if "s_endpgm" in x:
                    return body
    return None


def main():
    asm = open(sys.argv[1]).read()
    costs = measured_costs()
    out = {"source": f"{sys.argv[1]} (static mix) x {os.path.relpath(OPS_FILE, ROOT)} (per-opcode issue costs)"}
    for name in sys.argv[2:]:
        body = kernel_body(asm, name)
        if body is None:
            out[name] = None
            continue
        mix = Counter(m.group(1) for x in body if (m := re.match(r"^\s*(v_[a-z0-9_]+)", x)))  # (inline asm lines carry no indent)
        tot = sum(mix.values())
        weighted, unknown = 0.0, 0
        for op, c in mix.items():
            v, known = cost_of(op, costs)
            weighted += v * c
            unknown += 0 if known else c
        i64 = sum(c for op, c in mix.items() if op.startswith("v_mad_u64_u32"))
        two_class = (i64 * 5.39 + (tot - i64) * DEFAULT) / max(tot, 1)
        out[name] = {"valu_static": tot, "top": mix.most_common(12),
                     "cycles_per_valu_measured_mix": weighted / max(tot, 1),
                     "cycles_per_valu_two_class_model": two_class,
                     "issue_scale": (weighted / max(tot, 1)) / two_class,
                     "ops_without_a_measured_cost": unknown}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
