# Round 6: the barrier-phased cold k_small path, the C shim harness and the
# partial key-cache tests on one GPU box; each step under its own limit.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_field.py -k "coop" tests/test_gpu.py -k "coop or small_batch" tests/test_cabi.py > gpurun_out/r06_small_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r06_small_tests.log; exit 1; }
tail -25 gpurun_out/r06_small_tests.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_bootstrap.py tests/test_gpu_cache_group.py -k "bootstrap or partial" > gpurun_out/r06_boot.log 2>&1 || { echo BOOT FAILED; tail -40 gpurun_out/r06_boot.log; exit 1; }
tail -8 gpurun_out/r06_boot.log
BV_SMALL_STAMPS=1 timeout -k 10 200 python -u tools/small_lat.py 1 16 100 256 > gpurun_out/r06_small_lat.log 2>&1 || { echo LAT FAILED; tail -30 gpurun_out/r06_small_lat.log; exit 1; }
grep -v "^k_small" gpurun_out/r06_small_lat.log | tail -20
grep "stamps n=1 " gpurun_out/r06_small_lat.log | tail -4
