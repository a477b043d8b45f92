set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
timeout -k 10 300 python3 -u bench.py --no-cpu > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/b.json'))
print(round(d['value']/1e6,1), d['breakdown_ms']); print('warm', round(d['warm']['value']/1e6,1), d['warm']['breakdown_ms']); print(json.dumps(d['latency_ms'])); print('host', round(d['host_entry']['value']/1e6,1), json.dumps(d['host_entry']['host_breakdown_ms'])); print(json.dumps(d['events_entry']))"
