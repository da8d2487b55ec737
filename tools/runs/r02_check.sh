#!/bin/bash
# Round check on one GPU: the whole GPU test suite, smoke(), and the bench at the driver's 20 steps
# and at the default step count.  Outputs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gputests.log; exit 1; }
tail -2 gpurun_out/gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids || exit 1
for st in 20 200; do
  timeout -k 10 300 python -u bench.py --steps $st --warmup 5 > gpurun_out/bench_$st.log 2>&1 || { tail -20 gpurun_out/bench_$st.log; exit 1; }
  tail -1 gpurun_out/bench_$st.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["steps"], d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d.get("cpu_baseline", {}).get("value"))'
done
