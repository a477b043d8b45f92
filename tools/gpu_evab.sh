# A/B of bv_verify_events staging chunk size (BV_EV_CHUNK_MB; 0 = one chunk)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for c in ${CHUNKS:-0 16 8 32 0 16}; do
  echo "chunk_mb=$c"
  BV_EV_CHUNK_MB=$c timeout -k 10 200 python3 -u tools/prof_events.py 1000000 > gpurun_out/evab_$c.log 2>&1 || { tail -20 gpurun_out/evab_$c.log; exit 1; }
  grep bulk gpurun_out/evab_$c.log | tail -3
done
