# Round 6 GPU pass: small-batch tests (host item records: <= 4 items, or
# <= 16 when every key is cached) and the small-batch latency.  Each step has its own limit; a failing step ends the script.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout-method thread -m gpu"
timeout -k 10 600 $T --timeout 300 tests/test_gpu.py -k "small_batch" tests/test_cabi.py > gpurun_out/r06_small_tests.log 2>&1 || { echo SMALL FAILED; tail -40 gpurun_out/r06_small_tests.log; exit 1; }
tail -3 gpurun_out/r06_small_tests.log
for hs in 16; do
BV_HOST_SCALARS=$hs timeout -k 10 300 python -u tools/small_lat.py 1 4 16 64 100 128 256 > gpurun_out/r06_small_lat_hs$hs.log 2>&1 || { echo LAT FAILED; tail -30 gpurun_out/r06_small_lat_hs$hs.log; exit 1; }
echo "BV_HOST_SCALARS=$hs"; grep "small=1" gpurun_out/r06_small_lat_hs$hs.log
done
