#!/bin/bash
# Convex secant early miss for any-hit SDF marches: parity suite, then headline A/B in one library
# (A: RRTE_JIT_EXTRA_OPTS=-DRRTE_SECANT_EXIT=0, B: default), two interleaved rounds.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sdf_guards.py -x -q --timeout 200 --timeout-method thread > gpurun_out/secant_parity.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/secant_parity.log; exit 1; }
tail -1 gpurun_out/secant_parity.log
for r in 1 2; do for v in A B; do
  if [ $v = A ]; then X="-DRRTE_SECANT_EXIT=0"; else X=""; fi
  RRTE_JIT_EXTRA_OPTS="$X" timeout -k 10 200 python -u bench.py --no-cpu --no-stock > gpurun_out/sec_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/sec_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v' sdf", d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])' | tee -a gpurun_out/sec.txt
done; done
