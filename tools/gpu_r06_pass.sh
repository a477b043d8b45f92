# Round 6 GPU pass: small-batch tests (k_small timing from its own clock
# writes, no launch events), small-batch latency, one short bench line.
# Each step has its own limit; a failing step ends the script.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout-method thread -m gpu"
timeout -k 10 600 $T --timeout 300 tests/test_gpu.py -k "small_batch" tests/test_cabi.py > gpurun_out/r06_small_tests.log 2>&1 || { echo SMALL FAILED; tail -40 gpurun_out/r06_small_tests.log; exit 1; }
tail -3 gpurun_out/r06_small_tests.log
timeout -k 10 300 python -u tools/small_lat.py 1 2 4 16 100 > gpurun_out/r06_small_lat_d.log 2>&1 || { echo LAT FAILED; tail -30 gpurun_out/r06_small_lat_d.log; exit 1; }
grep "small=1" gpurun_out/r06_small_lat_d.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r06_bench_d.json 2> gpurun_out/r06_bench_d.err || { echo BENCH FAILED; tail -30 gpurun_out/r06_bench_d.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r06_bench_d.json').read().splitlines()[-1]); print(round(d['value']/1e6,1), json.dumps(d['latency_ms']['1']), json.dumps(d['latency_ms']['100']), json.dumps(d['shim_path']['event_1']))"
