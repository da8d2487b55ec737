#!/bin/bash
# How much of the shadow phase is rays marching the object they start on: RRTE_DEBUG=64 skips that
# object in the any-hit search (timing only, wrong images), against the full frame and no shadows.
set -o pipefail
b() { timeout -k 10 100 python -u bench.py --no-cpu --no-stock "$@" 2>/dev/null | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"])'; }
for rep in 1 2; do for d in 0 64 1; do echo -n "debug=$d: "; RRTE_DEBUG=$d b || exit 1; done; done
for d in 0 64; do echo -n "stress debug=$d: "; RRTE_DEBUG=$d b --scene deformation-stress --width 3840 --height 2160 --steps 10 --warmup 3 || exit 1; done
