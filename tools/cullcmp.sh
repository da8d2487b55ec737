#!/bin/bash
# culling on/off A/B (RRTE_CULL), generic and specialised kernels, on the BASELINE scenes
OUT=$1
for scene in sdf-showcase advanced-demo deformation-stress; do
  for j in off on; do
    for c in 0 1; do
      r=$(RRTE_CULL=$c timeout -k 10 200 python bench.py --no-cpu --steps 30 --warmup 5 --jit $j --scene $scene | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["roofline"]["kernel"])')
      echo "$scene jit=$j cull=$c $r" >> $OUT
    done
  done
done
