#!/bin/bash
# A/B two builds of librrte_hip.so on the GPU box, interleaved rounds (headline + 4K stress).
# usage: bash tools/ab_lib.sh <libA.so> <libB.so>   (build B in-tree, copy the other build to A)
set -o pipefail
A=${1:?libA}; B=${2:?libB}
mkdir -p gpurun_out
for r in 1 2; do for v in A B; do
  if [ $v = A ]; then L=$A; else L=$B; fi
  RRTE_HIP_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu --no-stock > gpurun_out/ab_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/ab_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v' sdf", d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])' | tee -a gpurun_out/ab.txt
  RRTE_HIP_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu --no-stock --scene deformation-stress --width 3840 --height 2160 --steps 10 --warmup 3 > gpurun_out/ab_s$v.log 2>&1 || exit 1
  tail -1 gpurun_out/ab_s$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v' stress", d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])' | tee -a gpurun_out/ab.txt
done; done
