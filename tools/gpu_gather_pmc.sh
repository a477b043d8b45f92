#!/bin/bash
# FETCH_SIZE calibration for 64-B table gathers (tools/ubench_gather.hip):
# HIP-event timings, then one rocprofv3 --pmc pass per counter group (never
# combined with tracing); tools/gather_calib.py divides algorithmic bytes by
# the counters per kernel.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/ubench_gather > gpurun_out/gather_time.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/gpmc_fetch -o run --output-format csv -- \
  ./tools/ubench_gather > gpurun_out/gpmc_fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d gpurun_out/gpmc_req -o run \
  --output-format csv -- ./tools/ubench_gather > gpurun_out/gpmc_req.log 2>&1
python3 tools/gather_calib.py gpurun_out > gpurun_out/gather_calib.json
cat gpurun_out/gather_calib.json
