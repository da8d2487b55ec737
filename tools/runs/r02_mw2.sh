#!/bin/bash
# Register budget of the looped / deformer specialisations after the 64-thread workgroups:
# RRTE_JIT_MIN_WAVES in {0 (compiler), 4, 6, 8} on the stock config and the 4K stress scene; then
# the other BASELINE configs at the default.
set -o pipefail
mkdir -p gpurun_out/mw2
b() { tag=$1; shift; timeout -k 10 150 python -u bench.py --no-cpu --no-stock "$@" > gpurun_out/mw2/$tag.log 2>&1 || { echo "FAIL $tag"; exit 1; }; tail -1 gpurun_out/mw2/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('frame_latency_ms'))"; }
for mw in 6 0 4 8; do
  RRTE_JIT_MIN_WAVES=$mw b stock_mw$mw --mode refcompat --spp 4 --max-depth 50 --random --steps 20 --warmup 3 || exit 1
  RRTE_JIT_MIN_WAVES=$mw b stress_mw$mw --scene deformation-stress --width 3840 --height 2160 --steps 10 --warmup 3 || exit 1
done
b basic --scene basic-demo --width 640 --height 480 --mode refcompat || exit 1
b adv --scene advanced-demo || exit 1
b literal --scene sdf-showcase-literal || exit 1
b mesh --scene mesh-demo || exit 1
b sdf4k --scene sdf-showcase --width 3840 --height 2160 --steps 50 || exit 1
