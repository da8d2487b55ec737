#!/bin/bash
# Topology kernels on the GPU: their parity tests, the JIT/gather/comm suites they touch, one bench line
# with the kernel-kind secondary numbers, then the emulated-rank / boundary measurements.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_topology.py \
  tests/test_gpu_parity.py -k "topology or animation or specialised or persist or full_1080p" > gpurun_out/r03_topo_tests.log 2>&1 \
  || { tail -40 gpurun_out/r03_topo_tests.log; echo TESTS FAILED; exit 1; }
tail -3 gpurun_out/r03_topo_tests.log
timeout -k 10 240 python -u bench.py --no-cpu --steps 20 > gpurun_out/r03_topo_bench.log 2>&1 || { tail -20 gpurun_out/r03_topo_bench.log; exit 1; }
tail -1 gpurun_out/r03_topo_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], json.dumps(d.get("kernel_kinds")), json.dumps(d.get("boundary")))'
bash tools/r03_emu.sh "" "-DRRTE_MARCH_PRED=1"
