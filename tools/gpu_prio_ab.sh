# Stream-priority variants (BV_KPRIO / BV_SPRIO builds) with two batches in
# flight, interleaved.  Every GPU step under its own limit.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cp babble_amd/libbabbleverify.so gpurun_out/keep.so
for v in d k0 s1 d k0 s1 d k0 s1; do
  cp gpurun_var/$v.so babble_amd/libbabbleverify.so
  timeout -k 10 240 python3 -u bench.py --no-cpu --no-extras --steps 40 > gpurun_out/p$v.json 2> gpurun_out/p$v.err || { tail -20 gpurun_out/p$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/p$v.json')); print('$v', round(d['value']/1e6,1), round(d['ms_per_step'],3))"
done
rm -f gpurun_out/keep.so
