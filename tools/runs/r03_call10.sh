#!/bin/bash
# Blocking entry point with the page pre-touch: its tests, then interleaved boundary timings with the
# pre-touch off / on; then a kernel trace of the emulated N=8 rank-0 batched path (200 frames).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_boundary.py > gpurun_out/r03_bnd_tests.log 2>&1 \
  || { tail -40 gpurun_out/r03_bnd_tests.log; echo TESTS FAILED; exit 1; }
tail -2 gpurun_out/r03_bnd_tests.log
: > gpurun_out/r03_bnd.txt
for r in 1 2; do for pf in 0 1; do
  RRTE_BOUNDARY_PREFAULT=$pf timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps 20 > gpurun_out/bnd.log 2>&1 || { tail -5 gpurun_out/bnd.log; exit 1; }
  tail -1 gpurun_out/bnd.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); b=d["boundary"]; print("prefault='$pf'", b["ms_per_frame_reused_buffer"], b["ms_per_frame_fresh_buffer"], "headline", d["ms_per_step"], d["roofline"]["avg_launch_ms"])' | tee -a gpurun_out/r03_bnd.txt
done; done
mkdir -p $R/gpurun_out/emutrace
cd /tmp && export TMPDIR=/tmp
RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=8:0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/emutrace -o run -- python3 $R/bench.py --no-cpu --no-stock --steps 200 > $R/gpurun_out/emutrace/run.log 2>&1 || { tail $R/gpurun_out/emutrace/run.log; exit 1; }
tail -1 $R/gpurun_out/emutrace/run.log | cut -c1-300
python3 $R/tools/trace_window.py $R/gpurun_out/emutrace/run_kernel_trace.csv 25 200 $R/gpurun_out/emutrace/window.md "emulated N=8 rank 0, batched gathers, 200 frames"
