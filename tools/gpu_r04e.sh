set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu.py -k "long_messages or host_entry" > gpurun_out/sel.log 2>&1 || { echo PYTEST FAILED; tail -40 gpurun_out/sel.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/sel.log | tail -6
bash tools/gpu_r04d.sh
