#!/bin/bash
# generic vs scene-specialised kernel, interleaved rounds, on the BASELINE scenes
OUT=$1
for round in 1 2; do
  for scene in sdf-showcase advanced-demo sdf-showcase-literal; do
    for j in off on; do
      r=$(timeout -k 10 200 python bench.py --no-cpu --steps 30 --warmup 5 --jit $j --scene $scene | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["roofline"]["kernel"], d["roofline"]["jit_compile_ms"])')
      echo "round$round $scene jit=$j $r" >> $OUT
    done
  done
done
