#!/bin/bash
# Full check of HEAD on one GPU: GPU suite, smoke, default and 20-step bench, trace + PMC profile.
# usage: tools/runs/r02_head.sh <tag>
set -o pipefail
TAG=${1:-head}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gputests.log 2>&1 || { echo GPU TESTS FAILED; tail -30 gpurun_out/${TAG}_gputests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench_default.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/${TAG}_bench_default.log; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_20steps.log 2>&1 || { echo BENCH20 FAILED; tail -20 gpurun_out/${TAG}_bench_20steps.log; exit 1; }
python - <<EOF
import json
for f in ("default", "20steps"):
    line = [l for l in open("gpurun_out/${TAG}_bench_%s.log" % f) if l.startswith("{")][-1]
    d = json.loads(line)
    print(f, d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["cpu_baseline"]["gpu_over_cpu"] if d.get("cpu_baseline") else None)
EOF
bash tools/prof_gpu.sh $TAG
