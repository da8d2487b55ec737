#!/bin/bash
# A/B of two library builds on the headline (three interleaved rounds) and advanced-demo (two),
# after a parity subset.  usage: tools/runs/r02_ab2.sh <libA.so> <libB.so> <pytest -k expr>
set -o pipefail
A=${1:?libA}; B=${2:?libB}; K=${3:?k}
mkdir -p gpurun_out/ab2
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sdf_guards.py -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/ab2/parity.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/ab2/parity.log; exit 1; }
tail -1 gpurun_out/ab2/parity.log
b() { tag=$1; lib=$2; shift; shift; RRTE_HIP_LIB=$lib timeout -k 10 150 python -u bench.py --no-cpu --no-stock "$@" > gpurun_out/ab2/$tag.log 2>&1 || { echo "FAIL $tag"; exit 1; }; tail -1 gpurun_out/ab2/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"; }
for r in 1 2 3; do b sdfA $A || exit 1; b sdfB $B || exit 1; done
for r in 1 2; do b advA $A --scene advanced-demo || exit 1; b advB $B --scene advanced-demo || exit 1; done
