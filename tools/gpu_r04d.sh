# A/B: base chains per lane vs cooperative, headline (1M) and mid-size (250k)
# cold batches, alternating, plus rocprofv3 kernel stats of the headline.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for coop in 1 0; do
    for ev in 250000 1000000; do
      BV_COOP_BASES=$coop timeout -k 10 300 python -u bench.py --no-cpu --no-extras --events $ev --steps 20 --warmup 3 > gpurun_out/ab_${coop}_${ev}.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_${coop}_${ev}.json').read().strip().splitlines()[-1]); print('coop=$coop events=$ev', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms/step keyprep', round(d['breakdown_ms']['keyprep_stream'],3), 'ms')" | tee -a gpurun_out/ab_coop.log
    done
  done
done
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-extras --inflight 1 --steps 5 --warmup 2 > gpurun_out/bench_prof.json 2> gpurun_out/prof.err || { tail -30 gpurun_out/prof.err; exit 1; }
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/prof/run_kernel_stats.csv')))
for r in rows:
    print(f"{r['Name'].split('(')[0][:60]:60s} calls={r['Calls']:>4s} avg_us={float(r['AverageNs'])/1e3:9.1f}")
PY
