#!/bin/bash
# VALU / SALU instructions per frame by phase: RRTE_DEBUG=2 (primary + attributes), 1 (+ shading and
# the culling pre-pass, no shadow tests), 0 (full frame); one PMC pass each, plus frame times.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/phasepmc
cd /tmp && export TMPDIR=/tmp
for d in 2 1 0; do
  RRTE_DEBUG=$d timeout -k 10 120 python3 $R/bench.py --no-cpu --no-stock --steps 100 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("debug='$d'", d["ms_per_step"], d["roofline"]["avg_launch_ms"])'
  RRTE_DEBUG=$d timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/phasepmc/d$d -o run -- python3 $R/bench.py --no-cpu --no-stock --steps 50 > $R/gpurun_out/phasepmc/d$d.log 2>&1 || exit 1
done
