#!/bin/bash
# Uniform-branch guard fallbacks (-DRRTE_GUARD_UNIFORM=1): first the specialised-kernel parity subset under
# that build (short time limit: the variant resembles the round-2 one that faulted once), then the
# interleaved A/B of tools/r03_ab.sh.
set -o pipefail
mkdir -p gpurun_out
RRTE_JIT_EXTRA_OPTS="-DRRTE_GUARD_UNIFORM=1" timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_sdf_guards.py -k "specialised or secant or guard" > gpurun_out/r03_gu_parity.log 2>&1 \
  || { tail -30 gpurun_out/r03_gu_parity.log; echo PARITY FAILED; exit 1; }
tail -2 gpurun_out/r03_gu_parity.log
bash tools/r03_ab.sh "" "-DRRTE_GUARD_UNIFORM=1"
