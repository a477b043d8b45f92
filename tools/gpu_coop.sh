# coop base chain: correctness vs per-lane + latency
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread -m gpu tests/test_gpu_field.py -k "coop or xyzz" > gpurun_out/coop.log 2>&1 || { echo PYTEST FAILED; tail -60 gpurun_out/coop.log; exit 1; }
grep -E "base chain|passed|failed" gpurun_out/coop.log
