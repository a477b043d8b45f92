# Development A/B runner: the library variants in gpurun_var/ (tools/ab_steps.py)
# and the SyncResponse chain stamps of gpurun_var/stamps*.so (tools/chain_stamps.py).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
if ls gpurun_var/stamps*.so > /dev/null 2>&1; then
  for rep in 1 2; do
    timeout -k 10 200 python3 -u tools/chain_stamps.py gpurun_var/stamps*.so >> gpurun_out/stamps.log 2>&1 || { tail -20 gpurun_out/stamps.log; exit 1; }
  done
  grep -v amdgpu gpurun_out/stamps.log
fi
mkdir -p /tmp/abv && for f in gpurun_var/*.so; do case "$f" in *stamps*) ;; *) cp "$f" /tmp/abv/ ;; esac; done
ls /tmp/abv/*.so > /dev/null 2>&1 || exit 0
timeout -k 10 500 python3 -u tools/ab_steps.py /tmp/abv/*.so > gpurun_out/ab_steps.log 2>&1 || { tail -20 gpurun_out/ab_steps.log; exit 1; }
tail -1 gpurun_out/ab_steps.log
if [ -n "$AB_LATENCY" ]; then
  timeout -k 10 300 python3 -u tools/ab_latency.py /tmp/abv/*.so > gpurun_out/ab_latency.log 2>&1 || { tail -20 gpurun_out/ab_latency.log; exit 1; }
  cat gpurun_out/ab_latency.log | grep -v amdgpu
fi
