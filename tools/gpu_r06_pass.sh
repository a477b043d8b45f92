# Round 6 GPU pass: tests/test_gpu.py and test_gpu_cache_group.py (k_glv_split
# on the device entry, the affine first G step, host item records, small batches, C4 at 10^6), then
# an A/B of the GLV split's placement on the headline (BV_GLV_SSTREAM) with
# the per-kernel spans.  Each step has its own limit; a failing step ends
# the script.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout-method thread -m gpu"
timeout -k 10 900 $T --timeout 400 tests/test_gpu.py tests/test_gpu_cache_group.py > gpurun_out/r06_test_gpu.log 2>&1 || { echo TEST_GPU FAILED; tail -40 gpurun_out/r06_test_gpu.log; exit 1; }
tail -4 gpurun_out/r06_test_gpu.log
for rep in 1 2; do for g in 0 1; do
BV_GLV_SSTREAM=$g timeout -k 10 400 python -u bench.py --steps 60 --warmup 10 --no-extras --no-cpu > gpurun_out/ab_glv_${g}_$rep.json 2> gpurun_out/ab_glv_${g}_$rep.err
python -c "import json; d=json.loads(open('gpurun_out/ab_glv_${g}_$rep.json').read().splitlines()[-1]); b=d['breakdown_ms']; print('glv_sstream=$g rep=$rep', round(d['value']/1e6,1), 'k_verify_g', round(b['k_verify_g'],3), 'k_verify_q', round(b['k_verify_q'],3), 'k_sinv', round(b['k_sinv'],3), 'device_total', round(b['device_total'],3))"
done; done
