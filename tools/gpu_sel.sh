# GPU run of selected tests: bash tools/gpu_sel.sh <pytest args...>; then smoke.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/sel.log 2>&1 || { echo PYTEST FAILED; tail -60 gpurun_out/sel.log; exit 1; }
tail -15 gpurun_out/sel.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAILED; tail -30 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
