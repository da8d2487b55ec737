#!/bin/bash
# Camera-ray tile culling for the path-regeneration (stock config) loop: parity of the stochastic /
# multi-bounce cases and tile culling, then stock-config A/B vs HEAD, three interleaved rounds.
set -o pipefail
mkdir -p gpurun_out/sc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "stochastic or stock or tile_culling or refcompat or golden or path_loop" > gpurun_out/sc/parity.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/sc/parity.log; exit 1; }
tail -1 gpurun_out/sc/parity.log
b() { tag=$1; lib=$2; shift; shift; RRTE_HIP_LIB=$lib timeout -k 10 150 python -u bench.py --no-cpu --no-stock "$@" > gpurun_out/sc/$tag.log 2>&1 || { echo "FAIL $tag"; exit 1; }; tail -1 gpurun_out/sc/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"; }
for r in 1 2 3; do
  b stockA ab/libA.so --mode refcompat --spp 4 --max-depth 50 --random --steps 40 --warmup 3 || exit 1
  b stockB rrte_amd/lib/librrte_hip.so --mode refcompat --spp 4 --max-depth 50 --random --steps 40 --warmup 3 || exit 1
done
