#!/bin/bash
# A/B of the hot-first tile order and split hot tiles, interleaved rounds: image order
# (RRTE_TILE_ORDER=0), hot order (the default), hot order with split tiles (RRTE_TILE_SPLIT=1;
# RRTE_SPLIT_FRAC sets the threshold): headline at 200 and 20 steps (ms/frame, lone launch, frame latency) and the emulated
# N=8 rank-0 batched frame (EMU_STEPS, default 20).  usage: bash tools/r03_order.sh [rounds]
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/r03_order.txt
: > $OUT
R=${1:-2}
for r in $(seq $R); do
  for v in ${VARIANTS:-"RRTE_TILE_ORDER=0" "RRTE_TILE_ORDER=1" "RRTE_TILE_SPLIT=1"}; do
    for st in 200 20; do
      env $v timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps $st > gpurun_out/ord.log 2>&1 || { tail -5 gpurun_out/ord.log; exit 1; }
      tail -1 gpurun_out/ord.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v' steps='$st'", d["ms_per_step"], "launch", d["roofline"]["avg_launch_ms"], "latency", d["frame_latency_ms"])' | tee -a $OUT
    done
    for st in ${EMU_STEPS:-20}; do
      env $v RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=8:0 timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps $st > gpurun_out/ord.log 2>&1 || { tail -5 gpurun_out/ord.log; exit 1; }
      tail -1 gpurun_out/ord.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v' N=8:0 batched steps='$st'", d["ms_per_step"])' | tee -a $OUT
    done
  done
done
