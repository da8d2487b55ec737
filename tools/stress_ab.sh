#!/bin/bash
# A/B of the deformation-stress frame (4K, scene-specialised and generic kernels) over environment
# variants, two interleaved rounds; one JSON line per run into gpurun_out/stress_ab.log.
# usage: bash tools/stress_ab.sh "ENV_A" "ENV_B" ...   ("" = default)
set -o pipefail
mkdir -p gpurun_out
LOG=gpurun_out/stress_ab_runs.log
for round in 1 2; do
  for v in "$@"; do
    for k in ${KINDS:-on off}; do
      sz="--width 3840 --height 2160"; [ $k = off ] && sz="--width 960 --height 540"
      env $v timeout -k 10 120 python tools/leg_time.py --scene deformation-stress $sz --jit $k >> $LOG 2>&1 || { echo "FAILED: $v $k" >> $LOG; exit 1; }
    done
  done
done
grep '^{' $LOG || true
