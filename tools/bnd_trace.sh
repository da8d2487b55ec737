#!/bin/bash
# Kernel + memory-copy trace of the blocking drop-in path (tools/bnd_loop.py: 3 warm-up + 10 frames)
# for each RRTE_BND_CHUNKS given, under GPU_MAX_HW_QUEUES=32 (as bench.py runs it).  Outputs
# gpurun_out/bnd_trace_<chunks>/ (csv) and a per-frame summary (tools/bnd_timeline.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
export GPU_MAX_HW_QUEUES=32
cd /tmp && export TMPDIR=/tmp
for ch in "$@"; do
  OUT=$R/gpurun_out/bnd_trace_$ch
  mkdir -p $OUT
  RRTE_BND_CHUNKS=$ch timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT -o run \
    -- python3 $R/tools/bnd_loop.py > $OUT/run.log 2>&1 || { tail $OUT/run.log; exit 1; }
  tail -1 $OUT/run.log
  python3 $R/tools/bnd_timeline.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
done
