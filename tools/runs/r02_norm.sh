#!/bin/bash
# normalize from one v_rsq_f32 (sqrt_rcp_rn): exhaustive bit check, parity suite, headline A/B vs HEAD.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fpexact.py -x -q --timeout 250 --timeout-method thread > gpurun_out/norm_fp.log 2>&1 || { echo FPEXACT FAILED; tail -30 gpurun_out/norm_fp.log; exit 1; }
tail -1 gpurun_out/norm_fp.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sdf_guards.py tests/test_gpu_mesh.py -x -q --timeout 200 --timeout-method thread > gpurun_out/norm_parity.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/norm_parity.log; exit 1; }
tail -1 gpurun_out/norm_parity.log
bash tools/ab_lib.sh ab/libA.so rrte_amd/lib/librrte_hip.so
