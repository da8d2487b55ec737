set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gputests.log; exit 1; }
tail -2 gpurun_out/gputests.log
timeout -k 10 200 python -u bench.py --no-cpu --no-stock > gpurun_out/b_sdf.log 2>&1 && tail -1 gpurun_out/b_sdf.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("sdf", d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])'
timeout -k 10 200 python -u bench.py --no-cpu --no-stock --scene deformation-stress --width 3840 --height 2160 --steps 10 --warmup 3 > gpurun_out/b_stress.log 2>&1 && tail -1 gpurun_out/b_stress.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("stress", d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])'
