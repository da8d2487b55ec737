#!/bin/bash
# Serialized lone launches (--inflight 1) under rocprofv3 --kernel-trace --stats: hot order without
# splits, with split tiles (agent-scope fences), and split tiles without fences (RRTE_DEBUG bit 10,
# timing only); plus the split threshold at 0.5.  Per-kernel average from the stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
export GPU_MAX_HW_QUEUES=32
cd /tmp && export TMPDIR=/tmp
for v in "RRTE_TILE_SPLIT=0" "RRTE_TILE_SPLIT=1" "RRTE_TILE_SPLIT=1 RRTE_DEBUG=1024" "RRTE_TILE_SPLIT=1 RRTE_SPLIT_FRAC=0.5"; do
  rm -rf $R/gpurun_out/sp; mkdir -p $R/gpurun_out/sp
  env $v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/sp -o run -- python3 $R/bench.py --no-cpu --no-stock --inflight 1 --steps 20 > $R/gpurun_out/sp/log 2>&1 || { tail $R/gpurun_out/sp/log; exit 1; }
  python3 - "$v" $R/gpurun_out/sp/run_kernel_trace.csv <<'PY'
import csv, sys, statistics
rows = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "rrte_jit_kernel" in r["Kernel_Name"]]
print(sys.argv[1], "launches", len(d), "median of last 40 %.1f us, min %.1f" % (statistics.median(d[-40:]), min(d[-40:])))
PY
done
