#!/bin/bash
# Bench every rrte_amd/lib/variants/*.so (RRTE_HIP_LIB override), interleaved rounds.
OUT=$1; shift
for round in 1 2; do
for v in rrte_amd/lib/variants/*.so; do
  r=$(RRTE_HIP_LIB=$v timeout -k 10 120 python bench.py --no-cpu --steps 30 --warmup 5 "$@" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')
  echo "round$round $(basename $v) $r" >> $OUT
done; done
