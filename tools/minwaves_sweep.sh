#!/bin/bash
# Scene-specialised kernel under several register budgets (RRTE_JIT_MIN_WAVES, diagnostics only):
# ms/frame (8 in flight) and per-launch ms, interleaved rounds.  usage: tools/minwaves_sweep.sh <out> [bench args]
set -o pipefail
OUT=${1:?outfile}; shift
for round in 1 2; do
  for w in "" 5 6; do
    r=$(RRTE_JIT_MIN_WAVES=$w timeout -k 10 200 python bench.py --no-cpu --no-stock "$@" |
        python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"])') || exit 1
    echo "round$round waves=[$w] $* : $r" | tee -a "$OUT"
  done
done
