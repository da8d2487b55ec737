#!/bin/bash
# Host enqueue time per frame against the frame time: plain headline and the emulated N=8 rank-0 batched
# path (200 and 20 steps), with the library's host section profile for the emulated run.
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/r03_host.txt
: > $OUT
for st in 200 20; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps $st > gpurun_out/h.log 2>&1 || { tail -5 gpurun_out/h.log; exit 1; }
  tail -1 gpurun_out/h.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("headline steps='$st'", d["ms_per_step"], "enqueue", d["host_enqueue_ms_per_step"])' | tee -a $OUT
  RRTE_HOST_PROFILE=1 RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=8:0 timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps $st > gpurun_out/h.log 2> gpurun_out/h_err_$st.log || { tail -5 gpurun_out/h_err_$st.log; exit 1; }
  tail -1 gpurun_out/h.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("N=8:0 steps='$st'", d["ms_per_step"], "enqueue", d["host_enqueue_ms_per_step"])' | tee -a $OUT
done
