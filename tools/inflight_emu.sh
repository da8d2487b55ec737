#!/bin/bash
# emulated rank-0 frame time of an N=8 split vs frames in flight and HW queue count
for q in 4 8 16; do for f in 4 8 16; do
  r=$(GPU_MAX_HW_QUEUES=$q RRTE_EMULATE_RANK=8:0 timeout -k 10 120 python bench.py --no-cpu --no-stock --inflight $f --steps 200 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')
  echo "queues=$q F=$f emu8 $r"
done; done
for q in 4 8; do for f in 4 8; do
  r=$(GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --no-cpu --no-stock --inflight $f --steps 100 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')
  echo "queues=$q F=$f N=1 $r"
done; done
