#!/bin/bash
# Hot list (1024 slowest tiles first) vs whole-frame LPT order (RRTE_TILE_ORDER=3), each without and
# with split tiles: headline at 200 and 20 steps, lone-frame latency, emulated N=8 rank frame at 20
# steps; two interleaved rounds.  Then the split critical-path probe under LPT + split.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tile_order.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lpt_tests.log 2>&1; tail -1 gpurun_out/lpt_tests.log
for r in 1 2; do
  for v in ${VARIANTS:-"RRTE_TILE_ORDER=1:RRTE_TILE_SPLIT=0" "RRTE_TILE_ORDER=1:RRTE_TILE_SPLIT=1" "RRTE_TILE_ORDER=3:RRTE_TILE_SPLIT=0" "RRTE_TILE_ORDER=3:RRTE_TILE_SPLIT=1"}; do
    e="${v//:/ }"
    for st in 200 20; do
      env $e timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps $st > gpurun_out/lp.log 2>&1 || { tail -5 gpurun_out/lp.log; exit 1; }
      tail -1 gpurun_out/lp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'"$v"' steps='$st'", d["ms_per_step"], "lat", d["frame_latency_ms"], "slots", d["tile_order"]["hot_slots"])'
    done
    env $e RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=8:0 timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps 20 > gpurun_out/lp.log 2>&1 || { tail -5 gpurun_out/lp.log; exit 1; }
    tail -1 gpurun_out/lp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'"$v"' N=8:0 steps=20", d["ms_per_step"])'
  done
done
RRTE_TILE_ORDER=3 RRTE_TILE_SPLIT=1 timeout -k 10 200 python -u tools/split_tiles.py 2>&1 | grep -v amdgpu.ids | tail -12
