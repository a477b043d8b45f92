# GPU parity run: pytest -m gpu, then smoke().  Each step has its own limit;
# a failing step ends the script.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAILED; tail -30 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
