#!/bin/bash
# Time bench variants: full, no shadow-ray tests (RRTE_DEBUG=1), primary visibility only (=2),
# plus the analytic literal scene.  usage: tools/ablate.sh <outfile>
OUT=$1
for v in 0 1 2; do
  echo "RRTE_DEBUG=$v $(RRTE_DEBUG=$v timeout -k 10 120 python bench.py --no-cpu --steps 20 --warmup 3 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $OUT
done
echo "literal $(timeout -k 10 120 python bench.py --no-cpu --steps 20 --warmup 3 --scene sdf-showcase-literal | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $OUT
echo "advanced $(timeout -k 10 120 python bench.py --no-cpu --steps 20 --warmup 3 --scene advanced-demo | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $OUT
