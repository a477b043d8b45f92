# coop base chain in the product + coop NAF in k_small: parity + latency
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu.py tests/test_gpu_field.py tests/test_gpu_cache_group.py -k "small or coop or golden or key_cache or k12 or k8 or c4_adversarial_mix or generic or c5" > gpurun_out/sel.log 2>&1 || { echo PYTEST FAILED; tail -60 gpurun_out/sel.log; exit 1; }
grep -E "PASS|FAIL|base chain|passed|failed" gpurun_out/sel.log | tail -40
timeout -k 10 300 python -u tools/small_lat.py > gpurun_out/small_lat.log 2>&1 || { echo LAT FAILED; tail -30 gpurun_out/small_lat.log; exit 1; }
cat gpurun_out/small_lat.log
