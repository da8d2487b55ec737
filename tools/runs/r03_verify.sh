#!/bin/bash
# Round-3 checks of the new GPU tests (comm semantics + failure detection, 4K parity and rank shares,
# batched gathers after the synchronize change, the persistent JIT cache) and the D2H design probe.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 90 ./tools/micro/d2h > gpurun_out/d2h.txt 2>&1 || { echo D2H PROBE FAILED; tail gpurun_out/d2h.txt; }
export RRTE_JIT_CACHE_DIR=$PWD/gpurun_out/jitcache
timeout -k 10 900 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_gather.py tests/test_gpu_4k.py \
  "tests/test_gpu_parity.py::test_jit_code_objects_persist_across_contexts" -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03_verify.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r03_verify.log; exit 1; }
tail -3 gpurun_out/r03_verify.log
cat gpurun_out/d2h.txt
