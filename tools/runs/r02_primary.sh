#!/bin/bash
# Primary phase split (timing diagnostics): closest-hit search alone (RRTE_DEBUG=130), + hit attributes
# (2), + shading and culling (1), full frame (0); one PMC pass of VALU/SALU for 130.
set -o pipefail
R=$GRAFT_REPO_ROOT
b() { timeout -k 10 100 python -u bench.py --no-cpu --no-stock "$@" 2>/dev/null | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"])'; }
for rep in 1 2; do for d in 130 2 1 0; do echo -n "debug=$d: "; RRTE_DEBUG=$d b || exit 1; done; done
mkdir -p $R/gpurun_out/primpmc && cd /tmp && export TMPDIR=/tmp
RRTE_DEBUG=130 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/primpmc/d130 -o run -- python3 $R/bench.py --no-cpu --no-stock --steps 50 > $R/gpurun_out/primpmc/d130.log 2>&1 || exit 1
