#!/bin/bash
# hiprtc optimisation settings of the scene-specialised kernel (RRTE_JIT_EXTRA_OPTS, appended to the
# fixed options): per setting and round, the headline at 200 and 20 steps (ms per frame), the lone
# launch and the compile time.  usage: tools/jit_opt_ab.sh ROUNDS "opts1" "opts2" ...
set -o pipefail
ROUNDS=${1:?rounds}; shift
for k in $(seq 1 $ROUNDS); do
  for o in "$@"; do
    for steps in 200 20; do
      RRTE_JIT_EXTRA_OPTS="$o" timeout -k 10 200 python bench.py --no-cpu --no-boundary --no-stock --steps $steps > /tmp/joa.json || exit 1
      python3 -c "import json; d=json.loads(open('/tmp/joa.json').read().strip().splitlines()[-1]); print('r$k [$o] steps=$steps', d['ms_per_step'], 'launch', d['roofline']['avg_launch_ms'], 'compile_ms', d['roofline'].get('jit_compile_ms'), 'u8diff', d['verified']['u8_max_diff'])"
    done
  done
done
