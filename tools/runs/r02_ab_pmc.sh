#!/bin/bash
# Headline A/B of two library builds (three interleaved rounds, default and 20 steps) plus one PMC
# pass each of VALU / SALU instruction counts.  usage: tools/runs/r02_ab_pmc.sh <libA.so> <libB.so> [parity-k]
set -o pipefail
A=${1:?libA}; B=${2:?libB}; K=${3:-}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/abp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sdf_guards.py -x -q --timeout 200 --timeout-method thread -k "$K" > $R/gpurun_out/abp/parity.log 2>&1 || { echo PARITY FAILED; tail -30 $R/gpurun_out/abp/parity.log; exit 1; }
  tail -1 $R/gpurun_out/abp/parity.log
fi
for r in 1 2 3; do for v in A B; do
  if [ $v = A ]; then L=$A; else L=$B; fi
  RRTE_HIP_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu --no-stock > $R/gpurun_out/abp/$v.log 2>&1 || exit 1
  tail -1 $R/gpurun_out/abp/$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v' sdf", d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])'
done; done
for v in A B; do
  if [ $v = A ]; then L=$A; else L=$B; fi
  RRTE_HIP_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu --no-stock --mode refcompat --spp 4 --max-depth 50 --random --steps 40 --warmup 3 > $R/gpurun_out/abp/s$v.log 2>&1 || exit 1
  tail -1 $R/gpurun_out/abp/s$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v' stock", d["value"], d["ms_per_step"])'
done
cd /tmp && export TMPDIR=/tmp
for v in A B; do
  if [ $v = A ]; then L=$A; else L=$R/$B; fi
  case $L in /*) ;; *) L=$R/$L;; esac
  RRTE_HIP_LIB=$L timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH --output-format csv -d $R/gpurun_out/abp/pmc$v -o run -- python3 $R/bench.py --no-cpu --no-stock --steps 20 > $R/gpurun_out/abp/pmc$v.log 2>&1 || exit 1
  python3 - <<PY
import csv,collections
c=collections.defaultdict(list)
for r in csv.DictReader(open('$R/gpurun_out/abp/pmc$v/run_counter_collection.csv')):
    if 'rrte_jit' in r['Kernel_Name']: c[r['Counter_Name']].append(float(r['Counter_Value']))
print('$v pmc', {k: round(sum(x)/len(x)/1e6,2) for k,x in c.items()})
PY
done
