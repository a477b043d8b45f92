# Kernel timelines of cold device-resident batches, two in flight (bench
# default), at the sizes in $TL_EVENTS.  Output gpurun_out/tl_<n>.txt.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for ev in ${TL_EVENTS:-125000 250000}; do
  rm -rf gpurun_out/tl_$ev
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl_$ev -o run --output-format csv -- python3 bench.py --no-cpu --no-extras --events $ev --steps 8 --warmup 3 > gpurun_out/tl_$ev.json 2> gpurun_out/tl.err || { tail -30 gpurun_out/tl.err; exit 1; }
  python3 tools/timeline.py gpurun_out/tl_$ev/run_kernel_trace.csv 6 > gpurun_out/tl_$ev.txt
  rm -rf gpurun_out/tl_$ev
done
