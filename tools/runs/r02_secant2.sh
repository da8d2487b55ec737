#!/bin/bash
# Secant early miss: new exactness tests, then A/B/C of RRTE_SECANT_EXIT 0 / 1 / 2 (off, any-hit
# marches, closest-hit marches too) on the headline, two interleaved rounds.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "convex or extra_scenes" > gpurun_out/secant2_parity.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/secant2_parity.log; exit 1; }
tail -1 gpurun_out/secant2_parity.log
RRTE_JIT_EXTRA_OPTS="-DRRTE_SECANT_EXIT=2" timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "specialised or jit_on or JIT_ON or 1080p or convex or extra" > gpurun_out/secant2_parity2.log 2>&1 || { echo PARITY2 FAILED; tail -30 gpurun_out/secant2_parity2.log; exit 1; }
tail -1 gpurun_out/secant2_parity2.log
for r in 1 2; do for v in 0 1 2; do
  RRTE_JIT_EXTRA_OPTS="-DRRTE_SECANT_EXIT=$v" timeout -k 10 200 python -u bench.py --no-cpu --no-stock > gpurun_out/sec2_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/sec2_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v' sdf", d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])' | tee -a gpurun_out/sec2.txt
done; done
