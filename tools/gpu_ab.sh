# Quick perf check: bench headline + extras (no CPU leg) and a rocprofv3
# kernel-trace summary of the headline.  Every GPU step under its own limit.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --no-cpu > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
cat gpurun_out/b.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_prof -o run --output-format csv -- python3 bench.py --no-cpu --no-extras --steps 5 --warmup 2 > gpurun_out/ab_prof.json 2> gpurun_out/ab_prof.err || { tail -20 gpurun_out/ab_prof.err; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/ab_prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f'{r["Name"][:60]:60s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:9.1f}')
PY
