#!/bin/bash
# In-place root share of batched gathers: the gather / comm / 4K / boundary tests, then the emulated
# N=8 rank-0 frame (RRTE_EMULATE_RANK=8:0, batches of 8, 1-rank communicator) with in-place off / on,
# two interleaved rounds at 200 and 20 steps.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_gather.py tests/test_gpu_comm.py tests/test_gpu_boundary.py tests/test_gpu_4k.py > gpurun_out/r03_inplace_tests.log 2>&1 \
  || { tail -40 gpurun_out/r03_inplace_tests.log; echo TESTS FAILED; exit 1; }
tail -2 gpurun_out/r03_inplace_tests.log
OUT=gpurun_out/r03_inplace.txt
: > $OUT
for r in 1 2; do for ip in 0 1; do for st in 200 20; do
  RRTE_GATHER_INPLACE=$ip RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=8:0 timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps $st > gpurun_out/emu.log 2>&1 || { tail -5 gpurun_out/emu.log; exit 1; }
  tail -1 gpurun_out/emu.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("inplace='$ip' N=8:0 steps='$st'", d["ms_per_step"])' | tee -a $OUT
done; done; done
RRTE_BENCH_GATHER=1 timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps 200 > gpurun_out/emu.log 2>&1 || { tail -5 gpurun_out/emu.log; exit 1; }
tail -1 gpurun_out/emu.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("rehearsal N=1 gather path steps=200", d["ms_per_step"])' | tee -a $OUT
