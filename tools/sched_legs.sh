#!/bin/bash
# Scheduler-strategy variants (as tools/sched_ab.sh: S or S:W) on the other BASELINE workloads, two
# interleaved rounds, tools/leg_time.py (ms per frame, lone launch, frame hash).
# usage: bash tools/sched_legs.sh default max-ilp:8 ...
set -o pipefail
VARIANTS=("$@")
LEGS=("advanced-demo 1920 1080 lambert_shadow 0" "deformation-stress 3840 2160 lambert_shadow 12"
      "sdf-showcase 3840 2160 lambert_shadow 0" "basic-demo 640 480 refcompat 0")
for round in 1 2; do
  for s in "${VARIANTS[@]}"; do
    st=${s%%:*}; w=${s#*:}; [ "$w" = "$s" ] && w=""
    if [ -n "$w" ]; then export RRTE_JIT_MIN_WAVES=$w; else unset RRTE_JIT_MIN_WAVES; fi
    if [ "$st" = default ]; then unset RRTE_JIT_EXTRA_OPTS; else export RRTE_JIT_EXTRA_OPTS="-mllvm -amdgpu-sched-strategy=$st"; fi
    for leg in "${LEGS[@]}"; do
      read -r scene wd ht mode fr <<< "$leg"
      a=$(timeout -k 10 300 python tools/leg_time.py --scene $scene --width $wd --height $ht --mode $mode --frames $fr 2>/dev/null | tail -1) || exit 1
      echo "r$round [$s] $a"
    done
  done
done
