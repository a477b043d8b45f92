# Round 6 GPU pass: key-cache / group tests (partial mode off by default,
# on in its own tests), the events entry and host-entry key-part tests (the
# affine first key-table step in k_verify_qf), small batches.  Each step has
# its own limit; a failing step ends the script.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout-method thread -m gpu"
timeout -k 10 900 $T --timeout 400 tests/test_gpu_cache_group.py tests/test_events.py tests/test_sync.py tests/test_bootstrap.py > gpurun_out/r06_cache_events.log 2>&1 || { echo CACHE/EVENTS FAILED; tail -40 gpurun_out/r06_cache_events.log; exit 1; }
tail -3 gpurun_out/r06_cache_events.log
timeout -k 10 900 $T --timeout 400 tests/test_gpu.py -k "host_entry or key_part or c4 or small_batch" > gpurun_out/r06_test_gpu_sel.log 2>&1 || { echo TEST_GPU FAILED; tail -40 gpurun_out/r06_test_gpu_sel.log; exit 1; }
tail -3 gpurun_out/r06_test_gpu_sel.log
