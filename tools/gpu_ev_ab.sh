# events-entry A/Bs (tools/ab_ev_chunks.py specs in $EV_SPECS) and a rocprof
# timeline of the pinned bulk call per $EV_TL env spec; $EV_TESTS: a pytest
# -k filter run first (development tool)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "box $(hostname)"
export TMPDIR=/tmp
if [ -n "$EV_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$EV_TESTS" > gpurun_out/ev_tests.log 2>&1 || { tail -30 gpurun_out/ev_tests.log; exit 1; }
  tail -2 gpurun_out/ev_tests.log
fi
ROUNDS=${ROUNDS:-2} timeout -k 10 500 python -u tools/ab_ev_chunks.py $EV_SPECS > gpurun_out/ab_ev.log 2>&1 || { tail -30 gpurun_out/ab_ev.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_ev.log
i=0
for spec in $EV_TL; do
  rm -rf gpurun_out/evtl
  env $spec timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/evtl -o run --output-format csv -- python3 tools/events_prof.py 1000000 pinned > gpurun_out/evtl_$i.log 2>&1 || { tail -30 gpurun_out/evtl_$i.log; exit 1; }
  python3 tools/lat_timeline.py gpurun_out/evtl ${TL_N:-36} > gpurun_out/evtl_timeline_$i.txt
  i=$((i+1))
done
rm -rf gpurun_out/evtl
