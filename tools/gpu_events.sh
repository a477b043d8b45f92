# Events path check: GPU parity tests of bv_verify_events / core.sync, then
# the 1000-event SyncResponse latency with per-kernel device times.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_events.py tests/test_sync.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_events.log 2>&1 || { tail -40 gpurun_out/pytest_events.log; exit 1; }
tail -2 gpurun_out/pytest_events.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_events -o ev --output-format csv -- python3 -u tools/prof_events.py ${EV_N:-200000} > gpurun_out/prof_events.log 2>&1 || { tail -30 gpurun_out/prof_events.log; exit 1; }
grep -E "bulk|sync dag" gpurun_out/prof_events.log
find gpurun_out/prof_events -name "*kernel_stats.csv" | head -1 | xargs -I{} cut -c1-160 {} | head -20
