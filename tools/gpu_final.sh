# Round-end evidence: GPU parity tests, the full bench line (with the CPU
# baseline), the rocprofv3 kernel-trace summary and the PMC passes.
set -e
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_full.sh
bash tools/gpu_pmc.sh
