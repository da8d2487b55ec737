#!/bin/bash
# Emulated N-GPU rank frames (RRTE_EMULATE_RANK=N:R, RRTE_BENCH_GATHER=1; no xGMI) per launch policy:
# "batch" = multi-frame launches at the batch's close (default), "frame" = RRTE_BATCH_LAUNCH=0 (each
# frame launched at its call, 4 caller streams).  NS (default "8 4 2"), RANKS (default "0 1"), STEPS_LIST (default
# "20 200"), ROUNDS (default 1); BENCH_ARGS pass to bench.py.  Prints ms_per_step per case.
set -o pipefail
for k in $(seq 1 ${ROUNDS:-1}); do
for steps in ${STEPS_LIST:-20 200}; do
  for pol in ${POLICIES:-batch frame}; do
    env_pol=""; arg_pol=""; [ $pol = frame ] && { env_pol="RRTE_BATCH_LAUNCH=0"; arg_pol="--streams 4"; }
    for n in ${NS:-8 4 2}; do
      for rk in ${RANKS:-0 1}; do
        r=$(env $env_pol RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=$n:$rk timeout -k 10 120 python bench.py --no-cpu --no-stock ${BENCH_ARGS:-} $arg_pol --steps $steps | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d.get("host_enqueue_ms_per_step"))') || exit 1
        echo "r$k steps=$steps $pol N=$n rank$rk ms_per_step/host_enqueue=$r"
      done
    done
  done
done
done
