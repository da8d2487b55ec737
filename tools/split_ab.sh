#!/bin/bash
# Emulated N-GPU rank frames with the batch launch's tile-list head split onto a high-priority stream
# (RRTE_SPLIT_HEAD per mille) against no split: N in $NS (default "8 4"), ranks $RANKS (default "0 1"),
# SPLITS (default "0 100 250"), 20 and 200 steps, ROUNDS (default 1).
set -o pipefail
for k in $(seq 1 ${ROUNDS:-1}); do
for steps in ${STEPS_LIST:-20 200}; do
  for sp in ${SPLITS:-0 100 250}; do
    for n in ${NS:-8 4}; do
      for rk in ${RANKS:-0 1}; do
        r=$(RRTE_SPLIT_HEAD=$sp RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=$n:$rk timeout -k 10 120 python bench.py --no-cpu --no-stock --no-boundary --steps $steps | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"])') || exit 1
        echo "r$k steps=$steps split=$sp N=$n rank$rk ms_per_step=$r"
      done
    done
  done
done
done
