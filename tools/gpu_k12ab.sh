# A/B of the K12 table-build point-op variants (BV_K12_LAT bit 0: base
# chains zipped, bit 1: fills zipped) on the cold headline, same box.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for m in ${MASKS:-3 0 1 2 3 0}; do
  BV_K12_LAT=$m timeout -k 10 200 python3 -u bench.py --no-cpu --no-extras --steps 20 --warmup 3 > gpurun_out/k12ab_$m.json 2> gpurun_out/k12ab_$m.err || { tail -20 gpurun_out/k12ab_$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/k12ab_$m.json')); print('mask', '$m', round(d['value']/1e6,1), 'M/s', {k: round(v,3) for k,v in d['breakdown_ms'].items()})"
done
