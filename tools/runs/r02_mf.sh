#!/bin/bash
# Multi-frame batched launches: gather tests, the 1-GPU gather proxy, headline A/B against HEAD.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gather.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mf_tests.log 2>&1 || { echo GATHER TESTS FAILED; tail -30 gpurun_out/mf_tests.log; exit 1; }
tail -1 gpurun_out/mf_tests.log
timeout -k 10 200 python -u tools/gather_variants.py 1920 136 8 200 8 > gpurun_out/mf_gv.log 2>&1 || { tail -20 gpurun_out/mf_gv.log; exit 1; }
cat gpurun_out/mf_gv.log
bash tools/ab_lib.sh ab/libA.so rrte_amd/lib/librrte_hip.so
