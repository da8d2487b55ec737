#!/bin/bash
# EXEC half-wave microbenchmark, then the r03_ab.sh A/B of the given JIT option sets.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/micro/exec_half | tee gpurun_out/exec_half.txt || exit 1
bash tools/r03_ab.sh "$@"
