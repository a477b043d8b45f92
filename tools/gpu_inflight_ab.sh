# A/B: one batch in flight vs two (alternating streams / work-buffer slots),
# after the GPU test suite.  Every GPU step under its own limit.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -30 gpurun_out/pt.log; exit 1; }
tail -2 gpurun_out/pt.log
for n in 1 2 1 2; do
  timeout -k 10 240 python3 -u bench.py --no-cpu --no-extras --inflight $n --steps 20 > gpurun_out/ab$n.json 2> gpurun_out/ab$n.err || { tail -20 gpurun_out/ab$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab$n.json')); print($n, round(d['value']/1e6,1), round(d['ms_per_step'],3))"
done
timeout -k 10 300 python3 -u bench.py --no-cpu > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b.json')); print('full', round(d['value']/1e6,1), d['ms_per_step'], 'warm', round(d['warm']['value']/1e6,1), 'host', round(d['host_entry']['value']/1e6,1) if 'host_entry' in d else None)"
