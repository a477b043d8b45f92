# Round 6 GPU pass: small-batch (cold barrier phases, coop warm tree, host
# item records), events (device signature decode), C-shim, bootstrap and
# partial key-cache tests; small-batch latency with and without host
# records; one short bench line with the host-entry stamps.  Each step has
# its own limit; a failing step ends the script.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout-method thread -m gpu"
timeout -k 10 500 $T --timeout 240 tests/test_gpu.py -k "small_batch" > gpurun_out/r06_small_tests.log 2>&1 || { echo SMALL FAILED; tail -40 gpurun_out/r06_small_tests.log; exit 1; }
tail -12 gpurun_out/r06_small_tests.log
timeout -k 10 500 $T --timeout 240 tests/test_cabi.py tests/test_events.py tests/test_gpu_field.py > gpurun_out/r06_cabi_events.log 2>&1 || { echo CABI/EVENTS FAILED; tail -40 gpurun_out/r06_cabi_events.log; exit 1; }
tail -6 gpurun_out/r06_cabi_events.log
timeout -k 10 400 $T --timeout 200 tests/test_bootstrap.py tests/test_gpu_cache_group.py -k "bootstrap or partial" > gpurun_out/r06_boot.log 2>&1 || { echo BOOT FAILED; tail -40 gpurun_out/r06_boot.log; exit 1; }
tail -4 gpurun_out/r06_boot.log
BV_SMALL_STAMPS=1 timeout -k 10 200 python -u tools/small_lat.py 1 2 4 16 100 > gpurun_out/r06_small_lat.log 2>&1 || { echo LAT FAILED; tail -30 gpurun_out/r06_small_lat.log; exit 1; }
grep -v "^k_small" gpurun_out/r06_small_lat.log | tail -20
grep "stamps n=1 " gpurun_out/r06_small_lat.log | tail -4
BV_HOST_SCALARS=0 timeout -k 10 200 python -u tools/small_lat.py 1 2 4 > gpurun_out/r06_small_lat_dev.log 2>&1 || { echo LAT0 FAILED; tail -30 gpurun_out/r06_small_lat_dev.log; exit 1; }
grep "small=1" gpurun_out/r06_small_lat_dev.log
BV_HOST_STAMPS=1 timeout -k 10 600 python -u bench.py --steps 60 --warmup 10 > gpurun_out/r06_bench_c.json 2> gpurun_out/r06_bench_c.err || { echo BENCH FAILED; tail -30 gpurun_out/r06_bench_c.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r06_bench_c.json').read().splitlines()[-1]); print(d['value'], json.dumps(d.get('shim_path')), d['host_entry']['value'], json.dumps(d['latency_ms']['1']), json.dumps(d['events_entry']['sync_dag_1000']['ms_median_sig_text']))"
grep "bv_host_launch" gpurun_out/r06_bench_c.err | tail -5
