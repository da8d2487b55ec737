#!/bin/bash
# Round-3 baseline on a fresh box: the driver's bench line (20 steps), the default, and the tail analysis.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03_base_b20.log 2>&1 || exit 1
tail -1 gpurun_out/r03_base_b20.log | cut -c1-600
timeout -k 10 200 python -u bench.py --no-cpu --no-stock > gpurun_out/r03_base_b200.log 2>&1 || exit 1
tail -1 gpurun_out/r03_base_b200.log | cut -c1-400
timeout -k 10 300 python -u tools/tail.py sdf-showcase 1920 1080 6 2>&1 | tee gpurun_out/r03_base_tail.log || exit 1
