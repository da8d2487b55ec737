#!/bin/bash
# Profiles of the headline on one GPU, outputs under gpurun_out/prof_<tag>/:
#  trace/  rocprofv3 --kernel-trace --stats of frames launched one after another (--inflight 1): the
#          per-launch kernel duration bench.py's roofline.avg_launch_ms is compared with;
#  tl/     the kernel trace of the driver's configuration (20 timed steps, 5 warm-up, 4 in flight):
#          per-frame spans and overlap (tools/timeline2.py);
#  pmcN/   one --pmc pass per counter group (never combined with tracing domains).
# GPU_MAX_HW_QUEUES is exported here: under rocprofv3 HIP starts before bench.py sets it.
# usage: tools/prof.sh TAG ["BENCH ARGS"]   (e.g. "--scene advanced-demo", or "--scene deformation-stress
#        --width 3840 --height 2160": the profile of that workload; default the headline)
set -o pipefail
TAG=${1:?tag}
XA=${2:-}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export GPU_MAX_HW_QUEUES=32
( cd $R && python3 -c "from rrte_amd import abi; print(abi.build_id())" ) > $OUT/build_id.txt || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --no-cpu --no-stock --no-boundary --no-legs --inflight 1 --steps 20 $XA > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/tl -o run -- python3 $R/bench.py --no-cpu --no-stock --no-boundary --no-legs --steps 20 --warmup 5 $XA > $OUT/tl.log 2>&1 || { tail $OUT/tl.log; exit 1; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES" \
           "SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "VALUUtilization VALUBusy OccupancyPercent"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python3 $R/bench.py --no-cpu --no-stock --no-boundary --no-legs --steps 20 $XA > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed" >> $OUT/errors.log; exit 1; }
done
echo done > $OUT/done
