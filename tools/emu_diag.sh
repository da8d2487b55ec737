#!/bin/bash
# Where the emulated N-GPU rank-0 frame goes (N=${N:-8}): the batched gather path as the bench runs it,
# without the root's expansion (RRTE_DIAG_SKIP=2: wrong frames, timing only), and the rank's render
# alone without any gather path (per-frame launches, 4 and 8 frames in flight), at 20 and 200 steps.
set -o pipefail
N=${N:-8}
one() {  # label, env..., -- bench args
  local label=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  r=$(env "${envs[@]}" timeout -k 10 120 python bench.py --no-cpu --no-stock "$@" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"])') || exit 1
  echo "$label $* -> $r"
}
for steps in 20 200; do
  one "gather" RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=$N:0 -- --steps $steps
  one "gather-no-expand" RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=$N:0 RRTE_DIAG_SKIP=2 -- --steps $steps
  one "render-only-F4" RRTE_EMULATE_RANK=$N:0 -- --steps $steps --inflight 4
  one "render-only-F8" RRTE_EMULATE_RANK=$N:0 -- --steps $steps --inflight 8
  one "gather-peer1" RRTE_BENCH_GATHER=1 RRTE_EMULATE_RANK=$N:1 -- --steps $steps
done
