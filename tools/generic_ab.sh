#!/bin/bash
# Generic-kernel A/B on the headline workload (bench.py --jit off: every frame on rrte::ray_kernel):
# per variant and round, ms per frame at 100 steps.  Variants are environment assignments, e.g.
#   tools/generic_ab.sh 2 "feat|" "all|RRTE_GENERIC_ALL=1" "mw5|RRTE_HIP_LIB=rrte_amd/lib/ab/librrte_hip_mw5.so"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ROUNDS=${1:?rounds}; shift
OUT=$R/gpurun_out/generic_ab; mkdir -p $OUT
for k in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    name=${spec%%|*}; envs=${spec#*|}
    ( cd $R && env $envs timeout -k 10 240 python3 bench.py --jit off --no-cpu --no-stock --steps 100 --warmup 3 \
        ${GENERIC_AB_ARGS:-} > $OUT/${name}_r$k.log 2>&1 ) || { tail $OUT/${name}_r$k.log; echo "failed: $name"; exit 1; }
    python3 - "$OUT/${name}_r$k.log" "$name" "$k" <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"{sys.argv[2]:>8} r{sys.argv[3]}  {j['ms_per_step']:.4f} ms/frame  launch {j['roofline']['avg_launch_ms']:.4f} ms  "
      f"verified {j.get('verified', {}).get('u8_max_diff')}", flush=True)
PY
  done
done
