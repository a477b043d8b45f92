# Round evidence in one GPU call: bench (all legs), rocprofv3 kernel stats,
# PMC passes, C4 1M OpenSSL cross-check.  Every GPU step has its own limit;
# the first failure ends the script.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
bash tools/gpu_prof.sh > gpurun_out/prof.log 2>&1 || { echo PROF FAILED; tail -30 gpurun_out/prof.log; exit 1; }
tail -25 gpurun_out/prof.log
bash tools/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 || { echo PMC FAILED; tail -30 gpurun_out/pmc.log; exit 1; }
grep "pass" gpurun_out/pmc.log
if [ -z "${SKIP_XCHECK:-}" ]; then
  timeout -k 10 400 python3 -u tools/c4_ossl_xcheck.py > gpurun_out/c4_ossl_xcheck.log 2>&1 || { echo XCHECK FAILED; tail -20 gpurun_out/c4_ossl_xcheck.log; exit 1; }
  cat gpurun_out/c4_ossl_xcheck.log
fi
