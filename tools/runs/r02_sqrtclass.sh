#!/bin/bash
# sqrt_rn guard as one v_cmp_class (every x but a positive normal takes the full sequence): the
# exhaustive 2^32 check of the shipped sqrt_rn, parity subset, headline A/B vs HEAD.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fpexact.py -x -q --timeout 250 --timeout-method thread -k "sqrt or rcp or detects" > gpurun_out/sqc_fp.log 2>&1 || { echo FPEXACT FAILED; tail -30 gpurun_out/sqc_fp.log; exit 1; }
tail -1 gpurun_out/sqc_fp.log
bash tools/runs/r02_ab2.sh ab/libA.so rrte_amd/lib/librrte_hip.so "specialised or 1080p or convex or extra or golden or baseline"
