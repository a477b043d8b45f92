# Kernel time of the SyncResponse DAG hashing per library build (development
# tool): one rocprofv3 --kernel-trace --stats pass per gpurun_var/stamps*.so
# over tools/chain_stamps.py (12 bv_verify_events calls of the 1000-event,
# 250-level DAG), then k_ev_hash_chain's total time per call.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for so in gpurun_var/stamps*.so; do
  v=$(basename $so .so)
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/chainprof_$v -o run --output-format csv -- \
    python3 tools/chain_stamps.py $so > gpurun_out/chainprof_$v.log 2>&1 || { echo "pass $v failed"; tail -20 gpurun_out/chainprof_$v.log; exit 1; }
  python3 - gpurun_out/chainprof_$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "ev_hash_chain" in r["Name"] or "k_ev_mid" in r["Name"] or "k_ev_hash" == r["Name"].split("(")[0]:
        n = int(r["Calls"]); tot = float(r["TotalDurationNs"])
        print(sys.argv[1].split("chainprof_")[1], r["Name"][:40], "calls", n, "avg us %.1f" % (tot / n / 1e3), "per call-of-12 us %.1f" % (tot / 12 / 1e3))
PY
done
