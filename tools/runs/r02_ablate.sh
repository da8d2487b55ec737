#!/bin/bash
# Where the headline frame's time goes (RRTE_DEBUG ablations, diagnostics only): primary visibility only
# (2), + attributes and shading without shadow tests (1), full frame (0); bench default 200 steps.
set -o pipefail
b() { timeout -k 10 100 python -u bench.py --no-cpu --no-stock "$@" 2>/dev/null | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"])'; }
for rep in 1 2; do for d in 2 1 0; do echo -n "debug=$d: "; RRTE_DEBUG=$d b; done; done
