# PMC passes over the bench workload (one rocprofv3 --pmc run per counter
# group; never combined with tracing).  Output: gpurun_out/pmc_<pass>/...;
# summarised by tools/pmc_summary.py into profiles/.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
EV=${PMC_EVENTS:-1000000}
run_pass() {
  name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d gpurun_out/pmc_$name -o run --output-format csv -- \
    python3 bench.py --no-cpu --no-extras --inflight 1 --steps 2 --warmup 1 --events $EV > gpurun_out/pmc_$name.log 2>&1 \
    || { echo "PMC pass $name failed"; tail -20 gpurun_out/pmc_$name.log; exit 1; }
  echo "pass $name ok"
}
run_pass fetch FETCH_SIZE
run_pass write WRITE_SIZE
run_pass valu SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run_pass busy SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE
python3 tools/pmc_summary.py gpurun_out $EV gpurun_out/${ROUND:-r05}_kverify_pmc.json > gpurun_out/pmc_summary.json
cat gpurun_out/pmc_summary.json
