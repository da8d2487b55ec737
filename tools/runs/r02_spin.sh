#!/bin/bash
# Closing the timed region by polling (RRTE_BENCH_SPIN=1, default) vs the blocking sync alone, at the
# driver's 20 steps (3 interleaved rounds) and the default step count; then the N>1 rehearsal.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do for sp in 0 1; do
  RRTE_BENCH_SPIN=$sp timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-stock > gpurun_out/spin_$sp.log 2>&1 || { tail -20 gpurun_out/spin_$sp.log; exit 1; }
  tail -1 gpurun_out/spin_$sp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("spin='$sp'", d["steps"], d["value"], d["ms_per_step"])'
done; done
timeout -k 10 200 python -u bench.py --no-cpu --no-stock > gpurun_out/spin_def.log 2>&1 || { tail -20 gpurun_out/spin_def.log; exit 1; }
tail -1 gpurun_out/spin_def.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("default", d["steps"], d["value"], d["ms_per_step"])'
for st in 20 200; do
  RRTE_BENCH_GATHER=1 timeout -k 10 300 python -u bench.py --steps $st --warmup 5 --no-cpu --no-stock > gpurun_out/spin_reh_$st.log 2>&1 || { tail -20 gpurun_out/spin_reh_$st.log; exit 1; }
  tail -1 gpurun_out/spin_reh_$st.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("rehearsal", d["steps"], d["value"], d["ms_per_step"])'
done
