#!/bin/bash
# every rrte_amd/lib/variants/*.so on the given scenes, sequential kernels (F=1) and 8 in flight, 2 rounds
OUT=$1; shift
for round in 1 2; do for sc in "$@"; do for v in rrte_amd/lib/variants/*.so; do
  r=$(RRTE_HIP_LIB=$v timeout -k 10 120 python bench.py --no-cpu --no-stock --scene $sc --steps 60 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"])')
  echo "round$round $sc $(basename $v) $r" >> $OUT
done; done; done
