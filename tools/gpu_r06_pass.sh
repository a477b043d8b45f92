# Round 6 GPU pass: small-batch tests (host item records; the warm record
# path decodes the key beside the leaf loads) and the small-batch latency
# with phase stamps.  Each step has its own limit; a failing step ends the
# script.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout-method thread -m gpu"
timeout -k 10 600 $T --timeout 300 tests/test_gpu.py -k "small_batch" tests/test_cabi.py > gpurun_out/r06_small_tests.log 2>&1 || { echo SMALL FAILED; tail -40 gpurun_out/r06_small_tests.log; exit 1; }
tail -3 gpurun_out/r06_small_tests.log
timeout -k 10 300 python -u tools/small_lat.py 1 4 16 100 > gpurun_out/r06_small_lat_e.log 2>&1 || { echo LAT FAILED; tail -30 gpurun_out/r06_small_lat_e.log; exit 1; }
grep "small=1" gpurun_out/r06_small_lat_e.log
BV_SMALL_STAMPS=1 timeout -k 10 300 python -u tools/small_lat.py 1 > gpurun_out/r06_small_stamps_e.log 2>&1 || { echo STAMPS FAILED; tail -30 gpurun_out/r06_small_stamps_e.log; exit 1; }
grep "stamps n=1 kernel_ms=0.0" gpurun_out/r06_small_stamps_e.log | tail -3
