#!/bin/bash
# Where the batched gather's cost goes in the 1-rank proxy: skip the gather (1), the de-interleave (2), both (3).
set -o pipefail
mkdir -p gpurun_out
for B in 8 16; do for S in 0 1 2 3; do
  RRTE_DIAG_SKIP=$S timeout -k 10 200 python -u tools/gather_variants.py 1920 136 16 400 $B > gpurun_out/mf3_$B_$S.log 2>&1 || { tail -20 gpurun_out/mf3_$B_$S.log; exit 1; }
  echo "B=$B skip=$S: $(grep -E "1 stream" gpurun_out/mf3_$B_$S.log | tail -2 | awk '{print $(NF-1)}' | tr '\n' ' ')"
done; done
