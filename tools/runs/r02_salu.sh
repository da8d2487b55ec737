#!/bin/bash
# Is the scalar unit a co-bottleneck?  List the SQ counters, then scalar / vector issue-cycle counters
# on the headline frame (one PMC pass each; counters the box does not list are dropped).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/salu
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/salu/counters.txt 2>&1 || true
grep -oE "(SQ|GRBM)_[A-Z0-9_]+" $R/gpurun_out/salu/counters.txt | sort -u > $R/gpurun_out/salu/names.txt || true
i=0
for grp in "SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE SQ_INSTS_SALU" "SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_BUSY_CU_CYCLES SQ_INSTS_VALU" "SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_WAVE_CYCLES SQ_INSTS_SMEM"; do
  i=$((i+1))
  sel=""
  for c in $grp; do grep -qx "$c" $R/gpurun_out/salu/names.txt && sel="$sel $c"; done
  echo "pass $i:$sel"
  [ -z "$sel" ] && continue
  timeout -s KILL 90 rocprofv3 --pmc $sel --output-format csv -d $R/gpurun_out/salu/p$i -o run -- python3 $R/bench.py --no-cpu --no-stock --steps 30 > $R/gpurun_out/salu/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
