#!/bin/bash
# Host API + kernel timeline of the driver's bench (20 steps, 5 warm-up) on one GPU (no counters).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/tl2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --no-cpu --no-stock --steps 20 --warmup 5 > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
for f in $(find $OUT/trace -name "*.csv"); do cp $f $OUT/; done
ls $OUT
tail -1 $OUT/trace.log | cut -c1-300
