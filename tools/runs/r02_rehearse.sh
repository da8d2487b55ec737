#!/bin/bash
# bench.py's N>1 frame path rehearsed on one GPU (RRTE_BENCH_GATHER=1), then the headline bench.
set -o pipefail
mkdir -p gpurun_out
for st in 20 200; do
  RRTE_BENCH_GATHER=1 timeout -k 10 300 python -u bench.py --steps $st --warmup 5 --no-cpu --no-stock > gpurun_out/reh_$st.log 2>&1 || { tail -20 gpurun_out/reh_$st.log; exit 1; }
  tail -1 gpurun_out/reh_$st.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("rehearsal", d["steps"], d["value"], d["ms_per_step"], d["config"]["workload"])'
done
timeout -k 10 300 python -u bench.py --no-cpu --no-stock > gpurun_out/reh_head.log 2>&1 || { tail -20 gpurun_out/reh_head.log; exit 1; }
tail -1 gpurun_out/reh_head.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("headline", d["steps"], d["value"], d["ms_per_step"])'
