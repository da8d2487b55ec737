#!/bin/bash
# Kernel trace of the emulated N=8 rank-0 batched path (in-place root share), 200 frames.
set -o pipefail
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/emutrace2; mkdir -p $R/gpurun_out/emutrace2
cd /tmp && export TMPDIR=/tmp
RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=8:0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/emutrace2 -o run -- python3 $R/bench.py --no-cpu --no-stock --steps 200 > $R/gpurun_out/emutrace2/run.log 2>&1 || { tail $R/gpurun_out/emutrace2/run.log; exit 1; }
python3 $R/tools/trace_window.py $R/gpurun_out/emutrace2/run_kernel_trace.csv 25 200 $R/gpurun_out/emutrace2/window.md "emulated N=8 rank 0, in-place batched gathers, 200 frames"
