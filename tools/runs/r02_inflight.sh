#!/bin/bash
# Frames-in-flight x hardware-queue sweep of the default bench at the driver's 20 steps and at 200,
# one GPU and one emulated rank of 8 (RRTE_EMULATE_RANK=8:0: rank 0's bands, no gather).
set -o pipefail
mkdir -p gpurun_out
b() { timeout -k 10 100 python -u bench.py --no-cpu --no-stock "$@" 2>/dev/null | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["steps"], round(d["value"]), d["ms_per_step"], d["roofline"]["avg_launch_ms"])'; }
for q in 4 32; do for f in 2 4 8 12; do
  echo -n "q=$q inflight=$f 1gpu: "; GPU_MAX_HW_QUEUES=$q b --steps 20 --inflight $f
  echo -n "q=$q inflight=$f rank0/8: "; GPU_MAX_HW_QUEUES=$q RRTE_EMULATE_RANK=8:0 b --steps 20 --inflight $f
done; done
