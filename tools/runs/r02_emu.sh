#!/bin/bash
# Rank 0's per-frame render time for N = 1/2/4/8 (RRTE_EMULATE_RANK, no gather), 4 frames in flight,
# at the driver's 20 steps and at 200, after the 64-thread workgroups.
set -o pipefail
for st in 20 200; do for n in 1 2 4 8; do
  if [ $n = 1 ]; then E=""; else E="$n:0"; fi
  r=$(RRTE_EMULATE_RANK=$E timeout -k 10 120 python bench.py --no-cpu --no-stock --steps $st --warmup 5 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"])') || exit 1
  echo "steps=$st N=$n $r"
done; done
