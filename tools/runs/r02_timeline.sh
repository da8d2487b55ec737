#!/bin/bash
# Kernel timeline of the driver's bench (20 steps, 5 warm-up) on one GPU.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/tl
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --no-cpu --no-stock --steps 20 --warmup 5 > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
F=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
cp $F $OUT/kernel_trace.csv
python3 $R/tools/timeline.py $OUT/kernel_trace.csv 25 20
