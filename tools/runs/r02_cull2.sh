#!/bin/bash
# DPP wave reductions + cheaper shadow culling: parity suite, then headline A/B against HEAD.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sdf_guards.py -x -q --timeout 200 --timeout-method thread > gpurun_out/cull2_parity.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/cull2_parity.log; exit 1; }
tail -1 gpurun_out/cull2_parity.log
bash tools/ab_lib.sh ab/libA.so rrte_amd/lib/librrte_hip.so
