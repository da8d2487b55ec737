#!/bin/bash
# Where does the split tiles' stream cost come from?  LPT order without and with split tiles, and with
# split tiles minus their fences (RRTE_DEBUG=1024) and minus the exchange areas' events
# (RRTE_SPLIT_NOEVENT=1) -- both timing only: headline at 20 steps and the lone-frame latency, two rounds.
set -o pipefail
for r in 1 2; do
  for v in "RRTE_TILE_SPLIT=0" "RRTE_TILE_SPLIT=1" "RRTE_TILE_SPLIT=1:RRTE_DEBUG=1024" "RRTE_TILE_SPLIT=1:RRTE_SPLIT_NOEVENT=1" "RRTE_TILE_SPLIT=1:RRTE_DEBUG=1024:RRTE_SPLIT_NOEVENT=1"; do
    e="${v//:/ }"
    env $e timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps 20 > gpurun_out/sc.log 2>&1 || { tail -5 gpurun_out/sc.log; exit 1; }
    tail -1 gpurun_out/sc.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'"$v"' steps=20", d["ms_per_step"], "lat", d["frame_latency_ms"], "enq", d["host_enqueue_ms_per_step"])'
  done
done
