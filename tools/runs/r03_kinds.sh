#!/bin/bash
# Secondary numbers (kernel kinds, stock config, boundary) with the tile order off / on, two rounds.
for r in 1 2; do for o in 0 1; do
  RRTE_TILE_ORDER=$o timeout -k 10 300 python -u bench.py --no-cpu --steps 20 > gpurun_out/kd.log 2>&1 || exit 1
  tail -1 gpurun_out/kd.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel_kinds"]; print("order='$o'", d["ms_per_step"], "kinds", k["generic"]["ms_per_frame"], k["topology"]["ms_per_frame"], k["full"]["ms_per_frame"], "stock", d["stock_config"]["ms_per_frame"], "bnd", d["boundary"]["ms_per_frame_reused_buffer"], "launch", d["roofline"]["avg_launch_ms"])'
done; done
