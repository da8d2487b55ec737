#!/bin/bash
# Headline A/B of extra hiprtc options for the scene-specialised kernel (RRTE_JIT_EXTRA_OPTS, appended
# after the fixed ones, so "-O3" overrides the default -O1; "" = the defaults).  Two interleaved rounds,
# 20 and 200 timed steps, with the bench's launch time and its own verification beside each; then one
# 4K deformation-stress frame time per variant (the JIT options apply to every scene).
# usage: bash tools/opt_ab.sh "" "-O2" "-O3" ...
set -o pipefail
for round in 1 2; do
  for o in "$@"; do
    export RRTE_JIT_EXTRA_OPTS="$o"
    for steps in 20 200; do
      r=$(timeout -k 10 200 python bench.py --steps $steps --warmup 5 --no-legs --no-stock --no-cpu --no-boundary \
          | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["verified"]["u8_max_diff"], d["verified"]["shadow_rays_match"])') || exit 1
      echo "r$round [$o] steps=$steps ms_per_step/avg_launch/u8/shadow_ok = $r"
    done
  done
done
for o in "$@"; do
  export RRTE_JIT_EXTRA_OPTS="$o"
  r=$(timeout -k 10 200 python bench.py --no-cpu --no-stock --no-legs --no-boundary --scene deformation-stress --width 3840 --height 2160 --steps 10 --warmup 3 \
      | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d["verified"]["u8_max_diff"])') || exit 1
  echo "[$o] stress 4K ms_per_step/u8 = $r"
done
