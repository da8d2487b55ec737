#!/bin/bash
# Kernel trace + PMC passes of bench.py on one GPU; outputs under gpurun_out/prof_<tag>/.
# The trace pass runs frames one at a time (--inflight 1): overlapping in-flight launches inflate
# rocprof per-kernel durations, so only a serialized trace is comparable to bench avg_launch_ms.
# usage: tools/prof_gpu.sh <tag> [bench args...]
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --no-cpu --no-stock --inflight 1 "$@" > $OUT/trace.log 2>&1 || exit 1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES" \
           "SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "VALUUtilization VALUBusy OccupancyPercent"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python3 $R/bench.py --no-cpu --no-stock "$@" > $OUT/pmc$i.log 2>&1 || echo "pmc pass $i failed" >> $OUT/errors.log
done
echo done > $OUT/done
