mkdir -p gpurun_out
b() { timeout -k 10 100 python -u bench.py --no-cpu --no-stock "$@" 2>/dev/null | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["steps"], d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])'; }
echo q4; b --steps 20; b --steps 20; b --steps 20 --inflight 4; b --steps 20 --inflight 24
echo q32; export GPU_MAX_HW_QUEUES=32; b --steps 20; b --steps 20; b --steps 20 --inflight 24; b --steps 200
