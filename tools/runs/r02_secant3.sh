#!/bin/bash
# Secant error bound with the leaves' scale and 2^-17: exactness tests, headline A/B vs the 2^-16 build.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sdf_guards.py -x -q --timeout 200 --timeout-method thread > gpurun_out/secant3_parity.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/secant3_parity.log; exit 1; }
tail -1 gpurun_out/secant3_parity.log
bash tools/ab_lib.sh ab/libA.so rrte_amd/lib/librrte_hip.so
