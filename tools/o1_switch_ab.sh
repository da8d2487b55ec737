set -o pipefail
for k in 1 2; do
  for v in "base||" "pair|-DRRTE_MARCH_PAIR=1|" "uniform||1"; do
    name=${v%%|*}; rest=${v#*|}; opts=${rest%%|*}; gp=${rest#*|}
    for steps in 200 20; do
      RRTE_JIT_EXTRA_OPTS="$opts" RRTE_GUARD_POLICY=${gp:-0} timeout -k 10 200 python bench.py --no-cpu --no-boundary --no-stock --steps $steps > /tmp/ab3.json || exit 1
      python3 -c "import json; d=json.loads(open('/tmp/ab3.json').read().strip().splitlines()[-1]); print('r$k $name steps=$steps', d['ms_per_step'], 'launch', d['roofline']['avg_launch_ms'], 'u8diff', d['verified']['u8_max_diff'])"
    done
  done
done
