#!/bin/bash
# Vectorised de-interleave: gather tests, then the 1-rank proxy decomposition at batch 8.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gather.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mf4_tests.log 2>&1 || { echo GATHER TESTS FAILED; tail -30 gpurun_out/mf4_tests.log; exit 1; }
tail -1 gpurun_out/mf4_tests.log
for B in 8 16; do for S in 0 1 2 3; do
  RRTE_DIAG_SKIP=$S timeout -k 10 200 python -u tools/gather_variants.py 1920 136 16 400 $B > gpurun_out/mf4_${B}_$S.log 2>&1 || { tail -20 gpurun_out/mf4_${B}_$S.log; exit 1; }
  echo "B=$B skip=$S: $(grep -E "1 stream" gpurun_out/mf4_${B}_$S.log | tail -2 | awk '{print $(NF-1)}' | tr '\n' ' ')"
done; done
