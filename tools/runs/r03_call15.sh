#!/bin/bash
# Ring of 6 batch slabs (all allocated at the first batch): gather / comm tests, then the emulated N=8
# rank-0 frame at 200 and 20 steps (two rounds) and the plain headline at 20 steps as a control.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_gather.py tests/test_gpu_comm.py > gpurun_out/r03_slab_tests.log 2>&1 \
  || { tail -40 gpurun_out/r03_slab_tests.log; echo TESTS FAILED; exit 1; }
tail -2 gpurun_out/r03_slab_tests.log
OUT=gpurun_out/r03_slab.txt
: > $OUT
for r in 1 2; do for st in 200 20; do
  RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=8:0 timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps $st > gpurun_out/emu.log 2>&1 || { tail -5 gpurun_out/emu.log; exit 1; }
  tail -1 gpurun_out/emu.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("slabs6 N=8:0 steps='$st'", d["ms_per_step"])' | tee -a $OUT
done; done
timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps 20 > gpurun_out/emu.log 2>&1 || { tail -5 gpurun_out/emu.log; exit 1; }
tail -1 gpurun_out/emu.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("headline steps=20", d["ms_per_step"])' | tee -a $OUT
