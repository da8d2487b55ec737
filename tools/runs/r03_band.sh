#!/bin/bash
# Emulated N=8 rank-0 batched frame (RRTE_EMULATE_RANK=8:0, RRTE_BENCH_GATHER=1): 8- vs 16-row bands
# (rank 0 renders 136 vs 144 of the 1080 rows) and gather batches of 4 vs 8 frames, at the driver's 20
# steps and at 200; two interleaved rounds.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for band in 16 8; do for f in 8 4; do for st in 20 200; do
  RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=8:0 timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps $st --band-rows $band --inflight $f > gpurun_out/bd.log 2>&1 || { tail -5 gpurun_out/bd.log; exit 1; }
  tail -1 gpurun_out/bd.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("band='$band' batch='$f' steps='$st'", d["ms_per_step"], "enqueue", d.get("host_enqueue_ms_per_step"))'
done; done; done; done
