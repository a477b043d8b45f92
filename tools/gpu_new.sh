# Targeted GPU tests (argument: pytest node ids / files).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_new.log 2>&1 || { echo PYTEST FAILED; tail -60 gpurun_out/pytest_new.log; exit 1; }
tail -15 gpurun_out/pytest_new.log
