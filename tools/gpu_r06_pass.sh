# Round 6 GPU pass: small-batch (cold barrier phases, coop warm tree, VALU
# s^-1), events (device signature decode), C-shim, bootstrap and partial
# key-cache tests; small-batch latency; one short bench line.  Each step has
# its own limit; a failing step ends the script.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_field.py -k "coop" tests/test_gpu.py -k "coop or small_batch" tests/test_cabi.py tests/test_events.py > gpurun_out/r06_small_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r06_small_tests.log; exit 1; }
tail -30 gpurun_out/r06_small_tests.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_bootstrap.py tests/test_gpu_cache_group.py -k "bootstrap or partial" > gpurun_out/r06_boot.log 2>&1 || { echo BOOT FAILED; tail -40 gpurun_out/r06_boot.log; exit 1; }
tail -8 gpurun_out/r06_boot.log
BV_SMALL_STAMPS=1 timeout -k 10 200 python -u tools/small_lat.py 1 16 100 256 > gpurun_out/r06_small_lat.log 2>&1 || { echo LAT FAILED; tail -30 gpurun_out/r06_small_lat.log; exit 1; }
grep -v "^k_small" gpurun_out/r06_small_lat.log | tail -20
grep "stamps n=1 " gpurun_out/r06_small_lat.log | tail -4
timeout -k 10 600 python -u bench.py --steps 60 --warmup 10 > gpurun_out/r06_bench_b.json 2> gpurun_out/r06_bench_b.err || { echo BENCH FAILED; tail -30 gpurun_out/r06_bench_b.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r06_bench_b.json').read().splitlines()[-1]); print(d['value'], json.dumps(d.get('shim_path')), json.dumps(d['host_entry'].get('host_diag')), d['host_entry']['value'], json.dumps(d['latency_ms']['1']), json.dumps(d['roofline'].get('per_kernel')))"
