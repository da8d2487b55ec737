#!/bin/bash
# Multi-frame batched launches: gather proxy at batch 4/8/16, and with the gather skipped (diagnostic).
set -o pipefail
mkdir -p gpurun_out
for B in 4 8 16; do
  timeout -k 10 200 python -u tools/gather_variants.py 1920 136 16 400 $B > gpurun_out/mf2_gv$B.log 2>&1 || { tail -20 gpurun_out/mf2_gv$B.log; exit 1; }
  grep -E "batch|plain" gpurun_out/mf2_gv$B.log | tail -4
done
RRTE_DIAG_SKIP=3 timeout -k 10 200 python -u tools/gather_variants.py 1920 136 16 400 8 > gpurun_out/mf2_skip.log 2>&1 || { tail -20 gpurun_out/mf2_skip.log; exit 1; }
echo "skip gather+deinterleave:"; grep -E "batch" gpurun_out/mf2_skip.log | tail -3
