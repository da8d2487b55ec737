#!/bin/bash
# Timing experiments on the scene-specialised kernel: correctly rounded sqrt/div vs hardware
# approximations (RRTE_JIT_EXTRA_OPTS; parity-breaking, timing only) and the RRTE_DEBUG splits.
# usage: tools/ablate_math.sh <outfile> [bench args...]
OUT=$1; shift
ARGS=("$@")
run() {  # label, VAR=value...
  local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --no-cpu --no-stock --steps 60 --warmup 5 "${ARGS[@]}" \
      | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"])') || return 1
  echo "$label $r" >> $OUT
}
for round in 1 2; do
  run base X=1 || exit 1
  run fast_sqrt RRTE_JIT_EXTRA_OPTS=-DRRTE_ABLATE_FAST_SQRT || exit 1
  run fast_div_sqrt "RRTE_JIT_EXTRA_OPTS=-DRRTE_ABLATE_FAST_SQRT -fno-hip-fp32-correctly-rounded-divide-sqrt" || exit 1
  run no_shadow RRTE_DEBUG=1 || exit 1
  run primary_only RRTE_DEBUG=2 || exit 1
done
