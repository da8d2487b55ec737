#!/bin/bash
# What serialises the emulated N=8 rank-0 batch renders?  RRTE_DIAG_SKIP (timing diagnostics, results
# wrong): 1 no ncclGather, 2 no de-interleave, 3 neither; 200 steps each, then a kernel trace of skip=1.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
OUT=$R/gpurun_out/r03_skip.txt
: > $OUT
for sk in 0 1 2 3; do
  RRTE_DIAG_SKIP=$sk RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=8:0 timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps 200 > gpurun_out/s.log 2>&1 || { tail -5 gpurun_out/s.log; exit 1; }
  tail -1 gpurun_out/s.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("skip='$sk' N=8:0 steps=200", d["ms_per_step"])' | tee -a $OUT
done
rm -rf $R/gpurun_out/emutrace3; mkdir -p $R/gpurun_out/emutrace3
cd /tmp && export TMPDIR=/tmp
RRTE_DIAG_SKIP=1 RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=8:0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/emutrace3 -o run -- python3 $R/bench.py --no-cpu --no-stock --steps 200 > $R/gpurun_out/emutrace3/run.log 2>&1 || { tail $R/gpurun_out/emutrace3/run.log; exit 1; }
echo traced
