#!/bin/bash
# Headline A/B of environment variants (two interleaved rounds, 20 and 200 timed steps, no legs):
# one summary line per run.  usage: bash tools/policy_ab.sh "" "RRTE_GUARD_POLICY=2" ...
set -o pipefail
for round in 1 2; do
  for v in "$@"; do
    for steps in 20 200; do
      r=$(env $v timeout -k 10 200 python bench.py --steps $steps --warmup 5 --no-legs --no-stock --no-cpu --no-boundary \
          | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["frame_latency_ms"], d["verified"]["u8_max_diff"], d["verified"]["shadow_rays_match"])') || exit 1
      echo "r$round [$v] steps=$steps ms_per_step/avg_launch/latency/u8/shadow_ok = $r"
    done
  done
done
