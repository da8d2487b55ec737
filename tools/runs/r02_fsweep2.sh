#!/bin/bash
# Frames in flight after the 64-thread workgroups: F in {2,3,4,6,8} at 20 and 200 steps, two rounds.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for st in 20 200; do for f in 2 3 4 6 8; do
  timeout -k 10 120 python -u bench.py --no-cpu --no-stock --inflight $f --steps $st --warmup 5 > gpurun_out/fs_$f.log 2>&1 || exit 1
  tail -1 gpurun_out/fs_$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("F='$f' steps='$st'", d["value"], d["ms_per_step"])' | tee -a gpurun_out/fs.txt
done; done; done
