#!/bin/bash
# Batched gather proxy (1920x136 frames, one caller stream): HEAD's one-launch-per-batch design (old)
# against chunked launches over rotating render streams with RRTE_LAUNCH_FRAMES = B (new).
set -o pipefail
mkdir -p gpurun_out
for B in 4 8 16; do for N in 20 400; do for v in old new; do
  if [ $v = old ]; then L=ab/libOld.so; else L=rrte_amd/lib/librrte_hip.so; fi
  GV_REPS=3 RRTE_HIP_LIB=$L RRTE_LAUNCH_FRAMES=$((B < 8 ? B : 8)) timeout -k 10 200 python -u tools/gather_variants.py 1920 136 16 $N $B > gpurun_out/mf6_${v}_${B}_$N.log 2>&1 || { tail -20 gpurun_out/mf6_${v}_${B}_$N.log; exit 1; }
  echo "$v B=$B frames=$N: $(grep -E "1 stream" gpurun_out/mf6_${v}_${B}_$N.log | awk '{print $(NF-1)}' | tr '\n' ' ')"
done; done; done
