#!/bin/bash
# Emulated N=8 rank frame (root 0 and peer 1) at 20 and 200 steps per gather batch size (--inflight)
# and slab ring size (RRTE_BATCH_SLABS), with the sky band partition on/off (RRTE_BAND_SKY).
set -o pipefail
for sky in ${SKY:-1 0}; do for b in ${BATCHES:-2 4 8}; do for sl in ${SLABS:-3 6}; do for rk in 0 1; do
  line=""
  for steps in 20 200; do
    r=$(RRTE_BAND_SKY=$sky RRTE_BATCH_SLABS=$sl RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=8:$rk timeout -k 10 120 python bench.py --no-cpu --no-stock --steps $steps --inflight $b | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d["host_enqueue_ms_per_step"])') || exit 1
    line="$line steps$steps=$r"
  done
  echo "sky=$sky batch=$b slabs=$sl rank=$rk $line"
done; done; done; done
