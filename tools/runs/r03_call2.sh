#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/micro/exec_half > gpurun_out/exec_half2.txt 2>&1 || { echo EXEC PROBE FAILED; exit 1; }
bash tools/runs/r03_verify.sh
