#!/bin/bash
# The reference's stock config (REFCOMPAT spp 4, depth 50, random) on its scene-specialised kernel at
# the JIT's register budgets (RRTE_JIT_MIN_WAVES: 8 = the default for runtime sample / bounce loops,
# 0 = the compiler's choice), two rounds.
set -o pipefail
for k in 1 2; do
  for w in 8 0 6; do
    RRTE_JIT_MIN_WAVES=$w timeout -k 10 300 python bench.py --no-cpu --no-boundary --steps 5 --warmup 2 > /tmp/sw.json || exit 1
    python3 -c "import json; d=json.loads(open('/tmp/sw.json').read().strip().splitlines()[-1]); s=d['stock_config']; print('r$k min_waves=$w stock', s['ms_per_frame'], 'ms', s['value'], s['unit'])"
  done
done
