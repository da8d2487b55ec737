#!/bin/bash
# Band-signalled pipelined copy of the blocking entry point: its tests, the parity subset that goes
# through rrte_hip_render, then three interleaved rounds of the bench's boundary line, pipe off / on.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_boundary.py \
  tests/test_gpu_parity.py -k "boundary or pipelined or golden or persist or specialised" > gpurun_out/r03_bnd_tests.log 2>&1 \
  || { tail -40 gpurun_out/r03_bnd_tests.log; echo TESTS FAILED; exit 1; }
tail -3 gpurun_out/r03_bnd_tests.log
: > gpurun_out/r03_bnd.txt
for r in 1 2 3; do for pipe in 0 1; do
  RRTE_BOUNDARY_PIPE=$pipe timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps 20 > gpurun_out/bnd.log 2>&1 || { tail -5 gpurun_out/bnd.log; exit 1; }
  tail -1 gpurun_out/bnd.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); b=d["boundary"]; print("pipe='$pipe'", b["ms_per_frame_reused_buffer"], b["ms_per_frame_fresh_buffer"], "headline", d["ms_per_step"], d["roofline"]["avg_launch_ms"])' | tee -a gpurun_out/r03_bnd.txt
done; done
