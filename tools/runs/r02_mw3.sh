#!/bin/bash
# RRTE_JIT_MIN_WAVES 6 vs 8 for the looped (stock config) and deformer (4K stress) specialisations,
# three interleaved rounds.
set -o pipefail
mkdir -p gpurun_out/mw3
b() { tag=$1; shift; timeout -k 10 150 python -u bench.py --no-cpu --no-stock "$@" > gpurun_out/mw3/$tag.log 2>&1 || { echo "FAIL $tag"; exit 1; }; tail -1 gpurun_out/mw3/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"; }
for r in 1 2 3; do for mw in 6 8; do
  RRTE_JIT_MIN_WAVES=$mw b stock_mw$mw --mode refcompat --spp 4 --max-depth 50 --random --steps 40 --warmup 3 || exit 1
  RRTE_JIT_MIN_WAVES=$mw b stress_mw$mw --scene deformation-stress --width 3840 --height 2160 --steps 10 --warmup 3 || exit 1
done; done
