#!/bin/bash
# Round-2 probe: default bench at the driver's step count and at 200 steps, plus per-wave timing of
# one frame (tools/wave_times.py).  Outputs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-stock > gpurun_out/b20.log 2>&1 || { tail -20 gpurun_out/b20.log; exit 1; }
timeout -k 10 200 python -u bench.py --steps 200 --warmup 5 --no-cpu --no-stock > gpurun_out/b200.log 2>&1 || { tail -20 gpurun_out/b200.log; exit 1; }
for f in b20 b200; do tail -1 gpurun_out/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["frame_latency_ms"])' $f; done
RRTE_DEBUG=16 timeout -k 10 120 python -u tools/wave_times.py sdf-showcase 1920 1080 > gpurun_out/wt.log 2>&1 || { tail -20 gpurun_out/wt.log; exit 1; }
cat gpurun_out/wt.log
