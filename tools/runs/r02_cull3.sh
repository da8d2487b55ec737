#!/bin/bash
# Culling pre-pass variant: parity suite, headline A/B vs HEAD.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sdf_guards.py tests/test_gpu_mesh.py -x -q --timeout 200 --timeout-method thread > gpurun_out/cull3_parity.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/cull3_parity.log; exit 1; }
tail -1 gpurun_out/cull3_parity.log
bash tools/ab_lib.sh ab/libA.so rrte_amd/lib/librrte_hip.so
