# Round-3 GPU evidence, one step per argument (each GPU step has its own time
# limit; the first failure ends the script):
#   tests   pytest -m gpu (incl. C3 10^8 through bv_group)      -> gpurun_out/pytest_gpu.log
#   bench   bench.py, all legs, GPU_MAX_HW_QUEUES=4 (the box default) -> gpurun_out/bench_q4.json
#   ab      headline-only A/B at 4 vs 8 hardware queues, same box -> gpurun_out/ab_q{4,8}.json
#   prof    rocprofv3 --kernel-trace --stats of the headline      -> gpurun_out/prof/
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for step in "$@"; do
  case "$step" in
    quick)  # the GPU suite with C3 shortened to 2 chunks
      BV_C3_EVENTS=2000000 timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > gpurun_out/pytest_quick.log 2>&1 || { echo QUICK FAILED; tail -40 gpurun_out/pytest_quick.log; exit 1; }
      tail -3 gpurun_out/pytest_quick.log ;;
    abvar)  # same-box A/B of the library builds in gpurun_var/
      timeout -k 10 400 python3 -u tools/ab_steps.py gpurun_var/*.so > gpurun_out/ab_steps.log 2>&1 \
        || { echo ABVAR FAILED; tail -20 gpurun_out/ab_steps.log; exit 1; }
      tail -1 gpurun_out/ab_steps.log ;;
    tests)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
        > gpurun_out/pytest_gpu.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
      tail -3 gpurun_out/pytest_gpu.log ;;
    bench)
      GPU_MAX_HW_QUEUES=4 timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_q4.json 2> gpurun_out/bench_q4.err \
        || { echo BENCH FAILED; tail -30 gpurun_out/bench_q4.err; exit 1; }
      head -c 600 gpurun_out/bench_q4.json; echo ;;
    ab)
      for q in 4 8 4 8; do
        GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 -u bench.py --no-extras --no-cpu --steps 30 \
          >> gpurun_out/ab_q$q.json 2>> gpurun_out/ab_q$q.err || { echo AB FAILED; tail -20 gpurun_out/ab_q$q.err; exit 1; }
      done
      grep -ho '"value": [0-9.]*' gpurun_out/ab_q4.json gpurun_out/ab_q8.json ;;
    prof)
      GPU_MAX_HW_QUEUES=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
        python3 -u bench.py --no-extras --no-cpu --inflight 1 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err \
        || { echo PROF FAILED; tail -20 gpurun_out/prof.err; exit 1; }
      find gpurun_out/prof -name "*kernel_stats.csv" | head -3 ;;
    c4)
      timeout -k 10 300 python3 -u tools/c4_ossl_xcheck.py > gpurun_out/c4_ossl.log 2>&1 || { echo C4 FAILED; tail -20 gpurun_out/c4_ossl.log; exit 1; }
      tail -3 gpurun_out/c4_ossl.log ;;
    pmc)
      bash tools/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 || { echo PMC FAILED; tail -20 gpurun_out/pmc.log; exit 1; }
      cp gpurun_out/r03_kverify_pmc.json profiles/r03_kverify_pmc.json  # read by the bench steps after this one
      tail -5 gpurun_out/pmc.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
