#!/bin/bash
# One parameterised GPU harness (run on the GPU box through gpurun; every step under its own time
# limit, outputs under gpurun_out/).  Steps run in the order given and stop at the first failure:
#   suite [PYTEST_K]      the -m gpu suite (optionally -k PYTEST_K)            -> gpurun_out/suite.log
#   smoke                 __graft_entry__.smoke()                              -> gpurun_out/smoke.log
#   bench NAME "ARGS"     python bench.py ARGS (one JSON line)                 -> gpurun_out/bench_NAME.log
#   prof TAG "ARGS"       kernel trace + stats, the 20-step timeline, the PMC passes (tools/prof.sh) of
#                         bench.py ARGS ("" = the headline)
#   run NAME SECS "CMD"   any other command (a tool script), time-limited      -> gpurun_out/NAME.log
# e.g.  gpurun --timeout 900 -- 'bash tools/gpu.sh suite smoke bench b20 "--steps 20 --warmup 5"'
set -o pipefail
mkdir -p gpurun_out
while [ $# -gt 0 ]; do
  step=$1; shift
  case $step in
    suite)
      k=()
      if [ $# -gt 0 ] && [[ "$1" != suite && "$1" != smoke && "$1" != bench && "$1" != prof && "$1" != run ]]; then k=(-k "$1"); shift; fi
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" \
        > gpurun_out/suite.log 2>&1 || { tail -40 gpurun_out/suite.log; echo "SUITE FAILED"; exit 1; }
      tail -2 gpurun_out/suite.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
        || { tail gpurun_out/smoke.log; echo "SMOKE FAILED"; exit 1; }
      tail -2 gpurun_out/smoke.log ;;
    bench)
      name=$1; args=$2; shift 2
      timeout -k 10 400 python -u bench.py $args > gpurun_out/bench_$name.log 2>&1 \
        || { tail -20 gpurun_out/bench_$name.log; echo "BENCH FAILED"; exit 1; }
      tail -1 gpurun_out/bench_$name.log | python3 tools/bench_summary.py ;;
    prof)
      tag=$1; pargs=$2; shift 2
      bash tools/prof.sh "$tag" "$pargs" || { echo "PROF FAILED"; exit 1; } ;;
    run)
      name=$1; secs=$2; cmd=$3; shift 3
      timeout -k 10 "$secs" bash -c "$cmd" > gpurun_out/$name.log 2>&1 || { tail -30 gpurun_out/$name.log; echo "RUN $name FAILED"; exit 1; }
      tail -5 gpurun_out/$name.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
