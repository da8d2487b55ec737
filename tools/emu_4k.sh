#!/bin/bash
# BASELINE configs[3] (sdf-showcase 3840x2160 over 2/4/8 GPUs) and configs[4] (deformation
# stress 3840x2160, 8 GPUs) as emulated rank frames on one GPU (RRTE_EMULATE_RANK=N:R, the exact bands of
# rank R, batched multi-frame launches, the exchange through a 1-rank communicator -- no xGMI), next to
# the one-GPU frame of the same workload; 20 and 200 timed steps.  One line per case.
set -o pipefail
W="--width 3840 --height 2160 --no-cpu --no-stock --no-boundary --no-legs"
for scene in ${SCENES:-sdf-showcase deformation-stress}; do
  for steps in ${STEPS_LIST:-20 200}; do
    [ $scene = deformation-stress ] && [ $steps = 200 ] && steps=60
    r=$(timeout -k 10 180 python bench.py --scene $scene $W --steps $steps | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"])') || exit 1
    echo "$scene steps=$steps N=1 ms_per_step=$r"
    for n in ${NS:-2 4 8}; do
      for rk in $(seq 0 $((n - 1))); do
        [ $n = 8 ] && [ $rk -gt 2 ] && [ $rk -lt 7 ] && continue  # (root, two peers and the last)
        r=$(RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=$n:$rk timeout -k 10 180 python bench.py --scene $scene $W --steps $steps | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"])') || exit 1
        echo "$scene steps=$steps N=$n rank$rk ms_per_step=$r"
      done
    done
  done
done
