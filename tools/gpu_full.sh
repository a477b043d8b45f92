# Full GPU pass: parity tests, bench line, rocprofv3 kernel-trace summary.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -4 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-extras --inflight 1 --steps 5 --warmup 2 > gpurun_out/bench_prof.json 2> gpurun_out/prof.err || { tail -30 gpurun_out/prof.err; exit 1; }
cat gpurun_out/bench_prof.json
find gpurun_out/prof -name '*stats*' | head
