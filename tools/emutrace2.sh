#!/bin/bash
# Host + device timeline of the emulated rank path (RRTE_EMULATE_RANK=$N:$RK, RRTE_BENCH_GATHER=1) at STEPS
# timed frames: rocprofv3 --kernel-trace --hip-runtime-trace (no counters), then tools/emu_timeline.py over
# the timed window's multi-frame launches.  usage: tools/emutrace2.sh STEPS N RK [extra bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT
STEPS=${1:-20}; N=${2:-8}; RK=${3:-0}; shift 3
OUT=$R/gpurun_out/emutrace2_${N}_${RK}_$STEPS
rm -rf $OUT; mkdir -p $OUT
export GPU_MAX_HW_QUEUES=32  # (under rocprofv3 HIP starts before bench.py could set it)
cd /tmp && export TMPDIR=/tmp
RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=$N:$RK timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $OUT -o run -- python3 $R/bench.py --no-cpu --no-stock --steps $STEPS "$@" > $OUT/run.log 2>&1 || { tail $OUT/run.log; exit 1; }
tail -1 $OUT/run.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms_per_step', d['ms_per_step'], 'host_enqueue_ms_per_step', d['host_enqueue_ms_per_step'])"
NB=$(( (STEPS + 7) / 8 ))
python3 $R/tools/emu_timeline.py $OUT $NB > $OUT/timeline.txt && tail -3 $OUT/timeline.txt
