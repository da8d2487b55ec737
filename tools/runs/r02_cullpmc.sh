#!/bin/bash
# The query test, then instruction counts of the culling pre-pass: RRTE_DEBUG=1 (no shadow tests)
# with culling on / off, one PMC pass each, plus their frame times.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/cullpmc
timeout -k 10 300 python -u -m pytest tests/test_gpu_gather.py -x -q -k query --timeout 120 --timeout-method thread > $R/gpurun_out/cullpmc/query.log 2>&1 || { tail -30 $R/gpurun_out/cullpmc/query.log; exit 1; }
tail -1 $R/gpurun_out/cullpmc/query.log
cd /tmp && export TMPDIR=/tmp
for c in 1 0; do
  RRTE_DEBUG=1 RRTE_CULL=$c timeout -k 10 120 python3 $R/bench.py --no-cpu --no-stock --steps 100 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("cull='$c'", d["ms_per_step"], d["roofline"]["avg_launch_ms"])'
  RRTE_DEBUG=1 RRTE_CULL=$c timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/cullpmc/c$c -o run -- python3 $R/bench.py --no-cpu --no-stock --steps 50 > $R/gpurun_out/cullpmc/c$c.log 2>&1 || exit 1
done
