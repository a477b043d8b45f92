# PMC A/B of library builds (development tool): one rocprofv3 --pmc pass per
# variant in gpurun_var/*.so over tools/ab_steps.py (3 steps, one round), then
# per-kernel VALU / SALU instruction counts and cycles per dispatch.
#   bash tools/gpu_pmc_ab.sh      -> gpurun_out/pmcab_<variant>/, gpurun_out/pmcab.json
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for so in gpurun_var/*.so; do
  v=$(basename $so .so)
  AB_STEPS=3 AB_ROUNDS=1 timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_SALU \
    SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmcab_$v -o run --output-format csv -- \
    python3 tools/ab_steps.py $so > gpurun_out/pmcab_$v.log 2>&1 || { echo "PMC pass $v failed"; tail -20 gpurun_out/pmcab_$v.log; exit 1; }
  echo "pass $v ok"
done
python3 tools/pmc_ab_summary.py gpurun_out > gpurun_out/pmcab.json
cat gpurun_out/pmcab.json
