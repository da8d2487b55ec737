#!/bin/bash
# Headline A/B of LLVM machine-scheduler strategies for the scene-specialised kernel (hiprtc option
# -mllvm -amdgpu-sched-strategy=S via RRTE_JIT_EXTRA_OPTS; "default" = none).  Two interleaved rounds,
# 20 and 200 timed steps, the bench's own verification printed beside each (scheduling cannot change
# the IEEE operations: same bits expected).  S:W also sets RRTE_JIT_MIN_WAVES=W (the kernel's wave budget).
# usage: bash tools/sched_ab.sh default iterative-ilp max-ilp:8 ...
set -o pipefail
for round in 1 2; do
  for s in "$@"; do
    st=${s%%:*}; w=${s#*:}; [ "$w" = "$s" ] && w=""
    if [ -n "$w" ]; then export RRTE_JIT_MIN_WAVES=$w; else unset RRTE_JIT_MIN_WAVES; fi
    if [ "$st" = default ]; then unset RRTE_JIT_EXTRA_OPTS; else export RRTE_JIT_EXTRA_OPTS="-mllvm -amdgpu-sched-strategy=$st"; fi
    for steps in 20 200; do
      r=$(timeout -k 10 200 python bench.py --steps $steps --warmup 5 --no-legs --no-stock --no-cpu --no-boundary \
          | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["verified"]["u8_max_diff"], d["verified"]["shadow_rays_match"])') || exit 1
      echo "r$round [$s] steps=$steps ms_per_step/avg_launch/u8/shadow_ok = $r"
    done
  done
done
