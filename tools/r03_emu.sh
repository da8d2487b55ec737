#!/bin/bash
# Per-rank frame time of an emulated N=8 job on one GPU (RRTE_EMULATE_RANK=8:0: rank 0's bands, the
# batched gather path through a 1-rank communicator laid out as rank 0 of 8, de-interleave of the full
# frame; no xGMI) for the kernel variants given, at the driver's 20 steps and at 200; then the
# blocking drop-in boundary with and without the pipelined host copy.
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/r03_emu.txt
: > $OUT
for r in 1 2; do for o in "$@"; do for st in 20 200; do
  RRTE_JIT_EXTRA_OPTS="$o" RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=8:0 timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps $st > gpurun_out/emu.log 2>&1 || { tail -5 gpurun_out/emu.log; exit 1; }
  tail -1 gpurun_out/emu.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'"[$o] N=8:0 batched steps=$st"'", d["ms_per_step"], d["config"]["frames_in_flight"])' | tee -a $OUT
done; done; done
for pipe in 0 1; do
  RRTE_BOUNDARY_PIPE=$pipe timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps 20 > gpurun_out/bnd.log 2>&1 || { tail -5 gpurun_out/bnd.log; exit 1; }
  tail -1 gpurun_out/bnd.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("boundary pipe='$pipe'", d["boundary"])' | tee -a $OUT
done
