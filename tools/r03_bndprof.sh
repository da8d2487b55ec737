#!/bin/bash
# Kernel trace of the blocking entry point: 10 frames plain (RRTE_BOUNDARY_PIPE=0), then 10 pipelined
# with each band release (1, 2): render / band-copy kernel durations and their overlap.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/bndprof
cd /tmp && export TMPDIR=/tmp
for v in "0 2" "1 1" "1 2"; do set -- $v
  RRTE_BOUNDARY_PIPE=$1 RRTE_BAND_RELEASE=$2 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/bndprof/p$1r$2 -o run -- python3 $R/tools/bnd_loop.py > $R/gpurun_out/bndprof/p$1r$2.log 2>&1 || { tail $R/gpurun_out/bndprof/p$1r$2.log; exit 1; }
  grep "ms per frame" $R/gpurun_out/bndprof/p$1r$2.log
done
for v in "0 2" "1 1" "1 2"; do set -- $v
  RRTE_BOUNDARY_PIPE=$1 RRTE_BAND_RELEASE=$2 timeout -k 10 60 python3 $R/tools/bnd_loop.py 2>&1 | grep "ms per frame" | sed "s/^/untraced pipe=$1 release=$2 /"
done
