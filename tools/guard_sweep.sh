#!/bin/bash
# Deformation-stress 4K frame time with the CSG early-outs off / default / every operand.
# usage: tools/guard_sweep.sh [scene] [width] [height]
SCENE=${1:-deformation-stress}; W=${2:-3840}; H=${3:-2160}
for g in 0 2 1; do
  echo "RRTE_CSG_GUARDS=$g $SCENE ${W}x${H}: $(RRTE_CSG_GUARDS=$g timeout -k 10 200 python bench.py --scene $SCENE --width $W --height $H --no-cpu --no-stock --steps 6 --warmup 2 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("ms/frame", d["ms_per_step"], "launch_ms", d["roofline"]["avg_launch_ms"], "Mray/s", d["value"])')" || exit 1
done
