# Round-2 closing evidence in one GPU call: the GPU parity suite, the bench
# line (all legs + CPU baseline), the headline-only rocprofv3 summary, the
# PMC passes, the C4 1M OpenSSL cross-check and the C3 10^8 bitmask run.
# Every GPU step has its own time limit; the first failure ends the script.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_full.sh > gpurun_out/full.log 2>&1 || { echo FULL FAILED; tail -40 gpurun_out/full.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
bash tools/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 || { echo PMC FAILED; tail -30 gpurun_out/pmc.log; exit 1; }
grep "pass" gpurun_out/pmc.log
timeout -k 10 400 python3 -u tools/c4_ossl_xcheck.py > gpurun_out/c4_ossl_xcheck.log 2>&1 || { echo XCHECK FAILED; tail -20 gpurun_out/c4_ossl_xcheck.log; exit 1; }
tail -3 gpurun_out/c4_ossl_xcheck.log
timeout -k 10 400 python3 -u tools/c3_scale.py > gpurun_out/c3_1e8.log 2>&1 || { echo C3 FAILED; tail -20 gpurun_out/c3_1e8.log; exit 1; }
tail -2 gpurun_out/c3_1e8.log
