set -o pipefail
for round in 1 2; do
  for s in default iterative-ilp; do
    if [ "$s" = default ]; then unset RRTE_JIT_EXTRA_OPTS; else export RRTE_JIT_EXTRA_OPTS="-mllvm -amdgpu-sched-strategy=$s"; fi
    a=$(timeout -k 10 200 python tools/leg_time.py --scene advanced-demo --width 1920 --height 1080 2>/dev/null | tail -1) || exit 1
    echo "r$round [$s] advanced-demo $a"
    b=$(timeout -k 10 300 python tools/leg_time.py --scene deformation-stress --width 3840 --height 2160 --frames 12 2>/dev/null | tail -1) || exit 1
    echo "r$round [$s] stress4k $b"
    c=$(timeout -k 10 200 python tools/leg_time.py --scene sdf-showcase --width 3840 --height 2160 2>/dev/null | tail -1) || exit 1
    echo "r$round [$s] showcase4k $c"
  done
done
