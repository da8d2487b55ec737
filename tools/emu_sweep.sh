#!/bin/bash
# Emulated per-rank frame of the N-GPU batched-gather bench path on one GPU (RRTE_EMULATE_RANK=N:0,
# RRTE_BENCH_GATHER=1: rank 0's bands, multi-frame launches, the gather through a 1-rank communicator,
# the root's composition; no xGMI) for N in $NS (default 2 4 8) at STEPS in $STEPS_LIST (default 20 200),
# plus the plain one-GPU headline; ranks in $RANKS (default 0); $BENCH_ARGS pass to bench.py.  Extra env (A/B switches) passes through.  Prints ms_per_step.
set -o pipefail
for steps in ${STEPS_LIST:-20 200}; do
  r=$(timeout -k 10 120 python bench.py --no-cpu --no-stock ${BENCH_ARGS:-} --steps $steps | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"])') || exit 1
  echo "N=1 steps=$steps ms_per_step=$r"
  for n in ${NS:-2 4 8}; do
    for rk in ${RANKS:-0}; do
      r=$(RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=$n:$rk timeout -k 10 120 python bench.py --no-cpu --no-stock ${BENCH_ARGS:-} --steps $steps | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"])') || exit 1
      echo "N=$n steps=$steps rank$rk ms_per_step=$r"
    done
  done
done
