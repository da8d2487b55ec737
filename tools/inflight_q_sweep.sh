#!/bin/bash
# Frames in flight x hardware queues, interleaved rounds: one GPU (N=1) and rank 0 of N=8 emulated
# (RRTE_EMULATE_RANK=8:0).  usage: tools/inflight_q_sweep.sh <outfile>
set -o pipefail
OUT=${1:?outfile}
for round in 1 2 3; do
  for fq in "8 16" "16 32" "12 32"; do
    set -- $fq
    for emu in "" "8:0"; do
      r=$(GPU_MAX_HW_QUEUES=$2 RRTE_EMULATE_RANK=$emu timeout -k 10 120 python bench.py --no-cpu --no-stock --inflight $1 --steps 600 2>/dev/null |
          python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])') || exit 1
      echo "round$round F=$1 Q=$2 emu=[$emu] $r" | tee -a "$OUT"
    done
  done
done
