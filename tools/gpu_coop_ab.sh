# coop.h A/B: one-wave chain latencies (HEAD's / the tree's header, same
# box), the coop field tests, the whole GPU suite, then small-batch latency
# of HEAD's library (gpurun_var/old.so) against the tree's.  Build first, here:
#   git show HEAD:babble_amd/csrc/coop.h > /tmp/coop_old.h
#   H="hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ibabble_amd/csrc"
#   $H -DCOOP_HEADER='"/tmp/coop_old.h"' -o gpurun_var/ubench_coop_old tools/ubench_coop_chain.hip
#   $H -o gpurun_var/ubench_coop_new tools/ubench_coop_chain.hip
#   BV_REV=HEAD bash tools/build_variant.sh gpurun_var/old.so
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/coop_ab.log
for r in 1 2; do
  timeout -k 10 60 ./gpurun_var/ubench_coop_old >> gpurun_out/coop_ab.log 2>&1
  timeout -k 10 60 ./gpurun_var/ubench_coop_new >> gpurun_out/coop_ab.log 2>&1
done
cat gpurun_out/coop_ab.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u tools/ab_small_lat_libs.py gpurun_var/old.so babble_amd/libbabbleverify.so > gpurun_out/coop_lat.log 2>&1 || { echo LAT FAILED; tail -30 gpurun_out/coop_lat.log; exit 1; }
cat gpurun_out/coop_lat.log
