# Iteration pass: GPU parity tests + a bench line without the CPU leg.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err || { tail -30 gpurun_out/bench_iter.err; exit 1; }
cat gpurun_out/bench_iter.json
