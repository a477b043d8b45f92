# Full GPU pass: pytest -m gpu, smoke, default bench line, rocprofv3 kernel
# stats of the headline (one batch in flight), then optional extra steps
# ($FULL_EXTRA, a command).  Each step limited; a failing step ends the script.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "box $(hostname)"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAILED; tail -30 gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -30 gpurun_out/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench.json').read().strip().splitlines()[-1]); print('bench', round(d['value']/1e6,1), 'M/s', d['roofline']['frac'])"
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-extras --inflight 1 --steps 5 --warmup 2 > gpurun_out/bench_prof.json 2> gpurun_out/prof.err || { tail -30 gpurun_out/prof.err; exit 1; }
cp gpurun_out/prof/run_kernel_stats.csv gpurun_out/bench_kernel_stats.csv
rm -rf gpurun_out/prof
if [ -n "$FULL_EXTRA" ]; then eval "$FULL_EXTRA"; fi
