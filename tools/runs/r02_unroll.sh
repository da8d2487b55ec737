#!/bin/bash
# Unroll factor of the sphere-tracing loop (-DRRTE_EXP_MARCH_UNROLL via the hiprtc options), headline
# and 4K deformation stress, two rounds.
set -o pipefail
b() { timeout -k 10 150 python -u bench.py --no-cpu --no-stock "$@" 2>/dev/null | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"])'; }
for rep in 1 2; do for u in 1 2 4; do
  echo -n "unroll=$u sdf: "; RRTE_JIT_EXTRA_OPTS="-DRRTE_EXP_MARCH_UNROLL=$u" b || exit 1
  echo -n "unroll=$u stress: "; RRTE_JIT_EXTRA_OPTS="-DRRTE_EXP_MARCH_UNROLL=$u" b --scene deformation-stress --width 3840 --height 2160 --steps 10 --warmup 3 || exit 1
done; done
