#!/bin/bash
# Batch slab ring size (RRTE_BATCH_SLABS 3 / 4 / 6) for the emulated N=8 rank-0 frame at 20 and 200 steps,
# two interleaved rounds; then the same for the 1-rank gather rehearsal of the full frame (N=1 path).
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/r03_slabs.txt
: > $OUT
for r in 1 2; do for ns in 3 4 6; do for st in 20 200; do
  RRTE_BATCH_SLABS=$ns RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=8:0 timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps $st > gpurun_out/emu.log 2>&1 || { tail -5 gpurun_out/emu.log; exit 1; }
  tail -1 gpurun_out/emu.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("slabs='$ns' N=8:0 steps='$st'", d["ms_per_step"])' | tee -a $OUT
done; done; done
for ns in 3 6; do
  RRTE_BATCH_SLABS=$ns RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=2:0 timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps 20 > gpurun_out/emu.log 2>&1 || { tail -5 gpurun_out/emu.log; exit 1; }
  tail -1 gpurun_out/emu.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("slabs='$ns' N=2:0 steps=20", d["ms_per_step"])' | tee -a $OUT
  RRTE_BATCH_SLABS=$ns RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=4:0 timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps 20 > gpurun_out/emu.log 2>&1 || { tail -5 gpurun_out/emu.log; exit 1; }
  tail -1 gpurun_out/emu.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("slabs='$ns' N=4:0 steps=20", d["ms_per_step"])' | tee -a $OUT
done
