set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAILED; tail -30 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python -u tools/perf_quick.py ${PERF_N:-200000} > gpurun_out/perf.log 2>&1 || { echo PERF FAILED; tail -30 gpurun_out/perf.log; exit 1; }
cat gpurun_out/perf.log
