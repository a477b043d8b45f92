# K12 build point-op variants (BV_K12_LAT) with two batches in flight, after
# the GPU tests.  Every GPU step under its own limit.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -30 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
for m in d 0 1 3 d 0 1 3; do
  if [ $m = d ]; then unset BV_K12_LAT; else export BV_K12_LAT=$m; fi
  timeout -k 10 240 python3 -u bench.py --no-cpu --no-extras --steps 40 > gpurun_out/k$m.json 2> gpurun_out/k$m.err || { tail -20 gpurun_out/k$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/k$m.json')); print('$m', round(d['value']/1e6,1), round(d['ms_per_step'],3))"
done
unset BV_K12_LAT
timeout -k 10 300 python3 -u bench.py --no-cpu > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b.json')); print('full', round(d['value']/1e6,1), 'warm', round(d['warm']['value']/1e6,1), d['latency_ms'])"
