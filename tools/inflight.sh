for sc in sdf-showcase advanced-demo; do for f in 1 2 3 4; do
  timeout -k 10 120 python bench.py --no-cpu --no-stock --scene $sc --inflight $f --steps 100 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$sc', 'F=$f', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['frame_latency_ms'])"
done; done
for wh in "960 540" "480 270"; do set -- $wh; for f in 1 4; do
  timeout -k 10 120 python bench.py --no-cpu --no-stock --width $1 --height $2 --inflight $f --steps 200 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', 'F=$f', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['frame_latency_ms'])"
done; done
