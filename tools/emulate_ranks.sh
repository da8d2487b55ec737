#!/bin/bash
# Per-rank frame time of an N-GPU row-band split, emulated on one GPU (RRTE_EMULATE_RANK=N:0
# renders exactly rank 0's bands; no gather).  ms_per_step only (the ray count is the full frame's).
SCENE=${1:-sdf-showcase}; shift
for n in 1 2 4 8; do for f in ${FRAMES:-1 4}; do
  if [ $n = 1 ]; then E=""; else E="$n:0"; fi
  r=$(RRTE_EMULATE_RANK=$E timeout -k 10 120 python bench.py --no-cpu --no-stock --scene $SCENE --inflight $f --steps 200 "$@" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"])')
  echo "$SCENE N=$n F=$f $r"
done; done
