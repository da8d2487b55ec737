#!/bin/bash
# Headline bench under several hiprtc option sets for the scene-specialised kernel
# (RRTE_JIT_EXTRA_OPTS, diagnostics only), interleaved rounds; results appended to $1.
# usage: bash tools/jitopt_sweep.sh <outfile> [bench args...]
set -o pipefail
OUT=${1:?outfile}; shift
OPTS=("" "-mllvm -amdgpu-sched-strategy=max-ilp" "-mllvm -amdgpu-sched-strategy=iterative-ilp"
      "-mllvm -amdgpu-sched-strategy=max-memory-clause" "-O2")
for round in 1 2; do
  for o in "${OPTS[@]}"; do
    r=$(RRTE_JIT_EXTRA_OPTS="$o" timeout -k 10 150 python bench.py --no-cpu --no-stock --steps 40 "$@" |
        python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["jit_compile_ms"])') || exit 1
    echo "round$round [$o] $r" | tee -a "$OUT"
  done
done
