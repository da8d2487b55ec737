set -o pipefail
mkdir -p gpurun_out/cfgs
run() { tag=$1; shift; timeout -k 10 200 python -u bench.py --no-stock --steps 10 --warmup 3 "$@" > gpurun_out/cfgs/$tag.log 2>&1 || { echo "FAIL $tag"; exit 1; }; tail -1 gpurun_out/cfgs/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('frame_latency_ms'), d['cpu_baseline']['value'] if d.get('cpu_baseline') else None)"; }
run basic --scene basic-demo --width 640 --height 480 --mode refcompat
run adv --scene advanced-demo
run sdf4k --scene sdf-showcase --width 3840 --height 2160
run stress4k --scene deformation-stress --width 3840 --height 2160 --cpu-seconds 20
