#!/bin/bash
# A/B of scene-specialised kernel build options (RRTE_JIT_EXTRA_OPTS), interleaved rounds: headline
# (200 and 20 steps) and the 4K deformation stress.  Then the parity subset under the LAST variant.
# usage: bash tools/jit_ab.sh "<opts A>" "<opts B>" ...   ("" = defaults)
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/r03_ab.txt
: > $OUT
for r in 1 2; do
  k=0
  for o in "$@"; do
    for st in 200 20; do
      RRTE_JIT_EXTRA_OPTS="$o" timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps $st > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
      tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'"v$k [$o] steps=$st"'", d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["frame_latency_ms"])' | tee -a $OUT
    done
    RRTE_JIT_EXTRA_OPTS="$o" timeout -k 10 200 python -u bench.py --no-cpu --no-stock --scene deformation-stress --width 3840 --height 2160 --steps 10 --warmup 3 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'"v$k [$o] stress"'", d["ms_per_step"])' | tee -a $OUT
    k=$((k+1))
  done
done
last="${@: -1}"
RRTE_JIT_EXTRA_OPTS="$last" timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sdf_guards.py -x -q --timeout 300 --timeout-method thread -k "jit or scene_specialised or golden or secant or 160x90" > gpurun_out/r03_ab_parity.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/r03_ab_parity.log; exit 1; }
tail -2 gpurun_out/r03_ab_parity.log
