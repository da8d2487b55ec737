#!/bin/bash
# Cost of the shadow-ray culling machinery: RRTE_DEBUG=1 (no shadow tests) and the full frame, with
# culling on (default) and off (RRTE_CULL=0), headline bench, two rounds.
set -o pipefail
b() { timeout -k 10 100 python -u bench.py --no-cpu --no-stock "$@" 2>/dev/null | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"])'; }
for rep in 1 2; do for d in 1 0; do for c in 1 0; do echo -n "debug=$d cull=$c: "; RRTE_CULL=$c RRTE_DEBUG=$d b || exit 1; done; done; done
