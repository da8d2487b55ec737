#!/bin/bash
# Frames in flight re-swept with the hot-first tile order: headline at the driver's 20 steps and at 200
# for F in ${FS:-2 3 4 6}, interleaved rounds; host enqueue time per frame alongside.
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/r03_fsweep.txt
: > $OUT
for r in 1 2; do
  for f in ${FS:-2 3 4 6}; do
    for st in 20 200; do
      timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps $st --inflight $f > gpurun_out/fs.log 2>&1 || { tail -5 gpurun_out/fs.log; exit 1; }
      tail -1 gpurun_out/fs.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("F='$f' steps='$st'", d["ms_per_step"], "enqueue", d.get("host_enqueue_ms_per_step"), "latency", d["frame_latency_ms"])' | tee -a $OUT
    done
  done
done
