#!/bin/bash
# Secondary numbers (kernel kinds, stock config, boundary, 20-step headline, per-launch times) for
# image order, hot order at default wave priority, hot order with raised priority; two rounds.
for r in 1 2; do for v in "RRTE_TILE_ORDER=0" "RRTE_HOT_PRIO=0" "RRTE_HOT_PRIO=1"; do
  env $v timeout -k 10 300 python -u bench.py --no-cpu --steps 20 > gpurun_out/kd.log 2>&1 || exit 1
  tail -1 gpurun_out/kd.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel_kinds"]; r=d["roofline"]; print("'$v'", d["ms_per_step"], "kinds", k["generic"]["ms_per_frame"], k["topology"]["ms_per_frame"], k["full"]["ms_per_frame"], "stock", d["stock_config"]["ms_per_frame"], "bnd", d["boundary"]["ms_per_frame_reused_buffer"], "lat", d["frame_latency_ms"], "launch", r["avg_launch_ms"], "first3", r["launch_ms_each"][:3])'
done; done
