# Round-4 check: key-cache / events / launcher GPU tests, smoke, DAG A/B.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_cache_group.py tests/test_events.py tests/test_gpu.py -k "key_cache or c5 or bench_gpus or native_library or events or host_entry_item_order" > gpurun_out/sel.log 2>&1 || { echo PYTEST FAILED; tail -60 gpurun_out/sel.log; exit 1; }
tail -25 gpurun_out/sel.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAILED; tail -30 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python -u tools/ab_dag.py > gpurun_out/ab_dag.log 2>&1 || { echo ABDAG FAILED; tail -30 gpurun_out/ab_dag.log; exit 1; }
cat gpurun_out/ab_dag.log
