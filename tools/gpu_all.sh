# Full GPU evidence pass: pytest -m gpu, smoke, bench (all legs), C3 10^8 via the group API.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAILED; tail -30 gpurun_out/smoke.log; exit 1; }
grep smoke gpurun_out/smoke.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ -n "${C3:-}" ]; then
  timeout -k 10 600 python3 -u tools/c3_scale.py --workers 16 > gpurun_out/c3_1e8.log 2>&1 || { echo C3 FAILED; tail -20 gpurun_out/c3_1e8.log; exit 1; }
  tail -2 gpurun_out/c3_1e8.log
fi
