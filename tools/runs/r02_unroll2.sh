#!/bin/bash
# March-loop unroll 1 vs 2 after the 64-thread workgroups (RRTE_JIT_EXTRA_OPTS=-DRRTE_MARCH_UNROLL=2):
# parity subset, then default and 20-step headline, two interleaved rounds.
set -o pipefail
mkdir -p gpurun_out/unr
RRTE_JIT_EXTRA_OPTS="-DRRTE_MARCH_UNROLL=2" timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "specialised or 1080p or convex" > gpurun_out/unr/parity.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/unr/parity.log; exit 1; }
tail -1 gpurun_out/unr/parity.log
b() { tag=$1; opt=$2; shift; shift; RRTE_JIT_EXTRA_OPTS="$opt" timeout -k 10 150 python -u bench.py --no-cpu --no-stock "$@" > gpurun_out/unr/$tag.log 2>&1 || { echo "FAIL $tag"; exit 1; }; tail -1 gpurun_out/unr/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['frame_latency_ms'])"; }
for r in 1 2; do
  b u1 "" || exit 1; b u2 "-DRRTE_MARCH_UNROLL=2" || exit 1
  b u1_20 "" --steps 20 --warmup 5 || exit 1; b u2_20 "-DRRTE_MARCH_UNROLL=2" --steps 20 --warmup 5 || exit 1
done
