# rocprofv3 kernel-trace summary of the bench (no CPU leg).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-extras --steps 5 --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench_prof.json 2> gpurun_out/prof.err || { tail -30 gpurun_out/prof.err; exit 1; }
cat gpurun_out/bench_prof.json
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/prof/run_kernel_stats.csv')))
for r in rows:
    print(f"{r['Name'].split('(')[0][:60]:60s} calls={r['Calls']:>4s} avg_us={float(r['AverageNs'])/1e3:9.1f}")
PY
