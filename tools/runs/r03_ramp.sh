#!/bin/bash
# (Evidence only: the ramp was removed after this run -- RRTE_GATHER_RAMP no longer exists.)
# Emulated N=8 rank-0 batched frame (RRTE_EMULATE_RANK=8:0, RRTE_BENCH_GATHER=1) with the batch ramp
# (RRTE_GATHER_RAMP) and the high-priority comm stream (RRTE_COMM_PRIORITY) on and off, interleaved
# rounds at the driver's 20 steps and at 200; then the gather and comm test files.
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/r03_ramp.txt
: > $OUT
for r in 1 2; do
  for v in "RRTE_GATHER_RAMP=0 RRTE_COMM_PRIORITY=0" "RRTE_GATHER_RAMP=1 RRTE_COMM_PRIORITY=0" \
           "RRTE_GATHER_RAMP=0 RRTE_COMM_PRIORITY=1" "RRTE_GATHER_RAMP=1 RRTE_COMM_PRIORITY=1"; do
    for st in 20 200; do
      env $v RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=8:0 timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps $st > gpurun_out/rp.log 2>&1 || { tail -5 gpurun_out/rp.log; exit 1; }
      tail -1 gpurun_out/rp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'"$v"' N=8:0 steps='$st'", d["ms_per_step"], "enqueue", d.get("host_enqueue_ms_per_step"))' | tee -a $OUT
    done
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_gather.py tests/test_gpu_comm.py tests/test_gpu_tile_order.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_ramp_tests.log 2>&1; tail -2 gpurun_out/r03_ramp_tests.log
