#!/bin/bash
# every rrte_amd/lib/variants/*.so at N=1 (F=1, F=4) and emulated N=8 rank 0 (F=4), 2 rounds
OUT=$1; shift
for round in 1 2; do for v in rrte_amd/lib/variants/*.so; do
  for cfg in "1:" "4:" "4:8:0"; do f=${cfg%%:*}; e=${cfg#*:}
    r=$(RRTE_EMULATE_RANK=$e RRTE_HIP_LIB=$v timeout -k 10 120 python bench.py --no-cpu --no-stock --inflight $f --steps 100 "$@" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"])')
    echo "round$round $(basename $v) F=$f emu=$e $r" >> $OUT
  done
done; done
