#!/bin/bash
# Frames in flight at the driver's 20 steps: F in {3,4,5,6,8}, three interleaved rounds.
set -o pipefail
for r in 1 2 3; do for f in 3 4 5 6 8; do
  x=$(timeout -k 10 120 python bench.py --no-cpu --no-stock --inflight $f --steps 20 --warmup 5 | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])') || exit 1
  echo "F=$f $x"
done; done
