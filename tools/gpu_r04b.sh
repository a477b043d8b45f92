# Round-4: small-batch kernel tests + latency table.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu.py tests/test_gpu_field.py tests/test_gpu_cache_group.py -k "small or xyzz or golden or key_cache_small" > gpurun_out/sel.log 2>&1 || { echo PYTEST FAILED; tail -60 gpurun_out/sel.log; exit 1; }
tail -15 gpurun_out/sel.log
timeout -k 10 300 python -u tools/small_lat.py > gpurun_out/small_lat.log 2>&1 || { echo LAT FAILED; tail -30 gpurun_out/small_lat.log; exit 1; }
cat gpurun_out/small_lat.log
