# GPU tests on the default (3-slot) library, then bench A/B of 2 vs 3 slots /
# batches in flight.  Every GPU step under its own limit.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -30 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
for v in 2 3 2 3; do
  cp gpurun_var/s$v.so babble_amd/libbabbleverify.so
  timeout -k 10 240 python3 -u bench.py --no-cpu --no-extras --steps 40 --inflight $v > gpurun_out/s$v.json 2> gpurun_out/s$v.err || { tail -20 gpurun_out/s$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s$v.json')); print('$v', round(d['value']/1e6,1), round(d['ms_per_step'],3))"
done
