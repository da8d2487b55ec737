#!/bin/bash
# Split (two-cluster) shadow-culling bound: culling exactness and parity subset, then headline with
# RRTE_SPLIT_CULL=0 / radius 0.5 (default) / 0.2 / 1.0 through RRTE_JIT_EXTRA_OPTS, two rounds.
set -o pipefail
mkdir -p gpurun_out/split
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "culling or specialised or 1080p or convex or extra" > gpurun_out/split/parity.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/split/parity.log; exit 1; }
tail -1 gpurun_out/split/parity.log
RRTE_JIT_EXTRA_OPTS="-DRRTE_SPLIT_CULL_R=0.0f" timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "culling or sdf-showcase or 1080p or convex" > gpurun_out/split/parity0.log 2>&1 || { echo PARITY0 FAILED; tail -30 gpurun_out/split/parity0.log; exit 1; }
tail -1 gpurun_out/split/parity0.log
b() { tag=$1; opt=$2; shift; shift; RRTE_JIT_EXTRA_OPTS="$opt" timeout -k 10 150 python -u bench.py --no-cpu --no-stock "$@" > gpurun_out/split/$tag.log 2>&1 || { echo "FAIL $tag"; exit 1; }; tail -1 gpurun_out/split/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"; }
for r in 1 2; do
  b off "-DRRTE_SPLIT_CULL=0" || exit 1
  b r05 "" || exit 1
  b r02 "-DRRTE_SPLIT_CULL_R=0.2f" || exit 1
  b r10 "-DRRTE_SPLIT_CULL_R=1.0f" || exit 1
done
