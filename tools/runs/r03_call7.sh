#!/bin/bash
# Band release variants of the pipelined blocking copy (RRTE_BAND_RELEASE 0/1/2) against the plain
# path: boundary tests under the default (2), then interleaved boundary timings; then the deferred
# guard A/B of the headline (tools/r03_ab.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_boundary.py > gpurun_out/r03_bnd_tests.log 2>&1 \
  || { tail -40 gpurun_out/r03_bnd_tests.log; echo TESTS FAILED; exit 1; }
tail -2 gpurun_out/r03_bnd_tests.log
: > gpurun_out/r03_bnd.txt
for r in 1 2; do for v in "0 0" "1 0" "1 1" "1 2"; do set -- $v
  RRTE_BOUNDARY_PIPE=$1 RRTE_BAND_RELEASE=$2 timeout -k 10 200 python -u bench.py --no-cpu --no-stock --steps 20 > gpurun_out/bnd.log 2>&1 || { tail -5 gpurun_out/bnd.log; exit 1; }
  tail -1 gpurun_out/bnd.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); b=d["boundary"]; print("pipe='$1' release='$2'", b["ms_per_frame_reused_buffer"], b["ms_per_frame_fresh_buffer"], "headline", d["ms_per_step"], d["roofline"]["avg_launch_ms"])' | tee -a gpurun_out/r03_bnd.txt
done; done
bash tools/r03_ab.sh "" "-DRRTE_DEFER_GUARDS=1"
