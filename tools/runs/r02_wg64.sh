#!/bin/bash
# 64-thread workgroups (one 8x8 tile per workgroup) for the specialised kernels: parity subset with
# RRTE_WG64=1, then headline and 4K stress A/B (RRTE_WG64 0 / 1), two interleaved rounds.
set -o pipefail
mkdir -p gpurun_out
RRTE_WG64=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "specialised or 1080p or convex or extra or culling or motion" > gpurun_out/wg64_parity.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/wg64_parity.log; exit 1; }
tail -1 gpurun_out/wg64_parity.log
for r in 1 2; do for v in 0 1; do
  RRTE_WG64=$v timeout -k 10 200 python -u bench.py --no-cpu --no-stock > gpurun_out/wg_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/wg_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v' sdf", d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])' | tee -a gpurun_out/wg.txt
  RRTE_WG64=$v timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps 20 --warmup 5 > gpurun_out/wg20_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/wg20_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v' sdf20", d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])' | tee -a gpurun_out/wg.txt
  RRTE_WG64=$v timeout -k 10 200 python -u bench.py --no-cpu --no-stock --scene deformation-stress --width 3840 --height 2160 --steps 10 --warmup 3 > gpurun_out/wgs_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/wgs_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v' stress", d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])' | tee -a gpurun_out/wg.txt
done; done
