#!/bin/bash
# sqrt_rn from one v_rsq_f32 (M3): exhaustive bit check, parity suite, headline A/B against HEAD.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fpexact.py -x -q --timeout 250 --timeout-method thread > gpurun_out/sqrt3_fp.log 2>&1 || { echo FPEXACT FAILED; tail -30 gpurun_out/sqrt3_fp.log; exit 1; }
tail -1 gpurun_out/sqrt3_fp.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sdf_guards.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sqrt3_parity.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/sqrt3_parity.log; exit 1; }
tail -1 gpurun_out/sqrt3_parity.log
bash tools/ab_lib.sh ab/libA.so rrte_amd/lib/librrte_hip.so
