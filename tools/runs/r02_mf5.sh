#!/bin/bash
# Chunked multi-frame launches: gather tests; rehearsal bench (20 / 200 steps) per RRTE_LAUNCH_FRAMES;
# the 1920x136 proxy at 20 frames (the driver's step count) and 400.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_gather.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mf5_tests.log 2>&1 || { echo GATHER TESTS FAILED; tail -30 gpurun_out/mf5_tests.log; exit 1; }
tail -1 gpurun_out/mf5_tests.log
for LF in 2 4 8; do for st in 20 200; do
  RRTE_LAUNCH_FRAMES=$LF RRTE_BENCH_GATHER=1 timeout -k 10 300 python -u bench.py --steps $st --warmup 5 --no-cpu --no-stock > gpurun_out/mf5_reh_${LF}_$st.log 2>&1 || { tail -20 gpurun_out/mf5_reh_${LF}_$st.log; exit 1; }
  tail -1 gpurun_out/mf5_reh_${LF}_$st.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("rehearsal LF='$LF'", d["steps"], d["value"], d["ms_per_step"])'
done; done
for LF in 2 4 8; do for N in 20 400; do
  GV_REPS=3 RRTE_LAUNCH_FRAMES=$LF timeout -k 10 200 python -u tools/gather_variants.py 1920 136 16 $N 16 > gpurun_out/mf5_gv_${LF}_$N.log 2>&1 || { tail -20 gpurun_out/mf5_gv_${LF}_$N.log; exit 1; }
  echo "proxy LF=$LF frames=$N: $(grep -E "1 stream" gpurun_out/mf5_gv_${LF}_$N.log | awk '{print $(NF-1)}' | tr '\n' ' ')"
done; done
