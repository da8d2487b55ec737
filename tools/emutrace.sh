#!/bin/bash
# Kernel trace of the emulated N=8 rank-0 batched path at the driver's 20 steps (RRTE_EMULATE_RANK=$N:$RK,
# RRTE_BENCH_GATHER=1): per-kernel totals, busy union and idle gaps of the timed window
# (tools/trace_window.py), plus the host-side section profile (RRTE_HOST_PROFILE=1).
set -o pipefail
R=$GRAFT_REPO_ROOT
STEPS=${1:-20}; N=${2:-8}; RK=${3:-0}
OUT=$R/gpurun_out/emutrace_${N}_${RK}_$STEPS
rm -rf $OUT; mkdir -p $OUT
export GPU_MAX_HW_QUEUES=32  # (under rocprofv3 HIP starts before bench.py could set it)
cd /tmp && export TMPDIR=/tmp
RRTE_HOST_PROFILE=1 RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=$N:$RK timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 $R/bench.py --no-cpu --no-stock --steps $STEPS > $OUT/run.log 2>&1 || { tail $OUT/run.log; exit 1; }
tail -1 $OUT/run.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms_per_step', d['ms_per_step'], 'host_enqueue_ms_per_step', d['host_enqueue_ms_per_step'])"
grep "rrte host profile" $OUT/run.log | tail -2
python3 $R/tools/trace_window.py $(ls $OUT/*kernel_trace.csv | head -1) 3 $STEPS $OUT/window.md "emulated N=$N rank 0, batched gathers, $STEPS frames"
python3 - $(ls $OUT/*kernel_trace.csv | head -1) <<'PY'
# timeline of the last 40 kernels: start/end relative to the first multi-frame launch of the window
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ray = [i for i, r in enumerate(rows) if ("rrte_jit_kernel" in r["Kernel_Name"] or "ray_kernel" in r["Kernel_Name"]) and int(r.get("Grid_Size_Y") or 1) > 1]
first = ray[-3]
t0 = int(rows[first]["Start_Timestamp"])
for r in rows[first:first + 40]:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{s:9.1f} {e:9.1f} {e - s:8.1f}  q{r.get('Queue_Id', '?'):>3}  {r['Kernel_Name'][:70]}")
PY
