#!/bin/bash
# ms/frame of emulated rank 0 for N in {1,2,4,8} vs frames in flight (F) and HW queues (Q)
for n in 1 2 4 8; do for q in 8 16; do for f in 4 8 12; do
  if [ $n = 1 ]; then E=""; else E="$n:0"; fi
  r=$(GPU_MAX_HW_QUEUES=$q RRTE_EMULATE_RANK=$E timeout -k 10 120 python bench.py --no-cpu --no-stock --inflight $f --steps 200 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')
  echo "N=$n Q=$q F=$f $r"
done; done; done
