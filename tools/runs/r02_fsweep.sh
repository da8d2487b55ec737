#!/bin/bash
# Frames in flight at the driver's 20 steps (and 200), 32 hardware queues, interleaved repetitions.
set -o pipefail
b() { timeout -k 10 100 python -u bench.py --no-cpu --no-stock "$@" 2>/dev/null | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["steps"], d["value"], d["ms_per_step"])'; }
for rep in 1 2 3; do for f in 2 3 4 6 8; do echo -n "F=$f: "; b --steps 20 --inflight $f; done; done
for f in 3 4 6; do echo -n "F=$f: "; b --steps 200 --inflight $f; done
