#!/bin/bash
# Where the frame goes (RRTE_DEBUG 2 = primary only, 1 = no shadow tests) and the object order of the
# closest-hit / any-hit searches (-DRRTE_EXP_PRIM_ORDER bit 0 / bit 1 = reversed), headline bench;
# then the parity suite with both searches reversed (the order must not change any result).
set -o pipefail
mkdir -p gpurun_out
b() { timeout -k 10 100 python -u bench.py --no-cpu --no-stock "$@" 2>/dev/null | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["config"]["shadow_rays_per_frame"])'; }
for d in 2 1; do echo -n "debug=$d: "; RRTE_DEBUG=$d b || exit 1; done
for rep in 1 2; do for o in 0 1 2 3; do echo -n "order=$o: "; RRTE_JIT_EXTRA_OPTS="-DRRTE_EXP_PRIM_ORDER=$o" b || exit 1; done; done
RRTE_JIT_EXTRA_OPTS="-DRRTE_EXP_PRIM_ORDER=3" timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sdf_guards.py -x -q --timeout 200 --timeout-method thread > gpurun_out/order_parity.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/order_parity.log; exit 1; }
tail -1 gpurun_out/order_parity.log
