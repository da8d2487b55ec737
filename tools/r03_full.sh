#!/bin/bash
# The whole GPU suite, smoke, then the round-3 profiles of the current kernel (tools/r03_prof.sh <tag>).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_full_tests.log 2>&1 \
  || { tail -40 gpurun_out/r03_full_tests.log; echo TESTS FAILED; exit 1; }
tail -2 gpurun_out/r03_full_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || { tail gpurun_out/r03_smoke.log; exit 1; }
tail -2 gpurun_out/r03_smoke.log
bash tools/r03_prof.sh "$1"
