#!/bin/bash
# Timing-only ablation: the correctly-rounded helpers' out-of-range fallback branches removed
# (-DRRTE_ABLATE_NO_GUARDS; real scenes never take them, so images are unchanged): how much of the
# frame the guards' EXEC bookkeeping costs.  Three interleaved rounds + VALU/SALU PMC per variant.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/gabl
b() { tag=$1; opt=$2; RRTE_JIT_EXTRA_OPTS="$opt" timeout -k 10 150 python -u bench.py --no-cpu --no-stock > gpurun_out/gabl/$tag.log 2>&1 || { echo "FAIL $tag"; exit 1; }; tail -1 gpurun_out/gabl/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"; }
for r in 1 2 3; do b base "" || exit 1; b noguard "-DRRTE_ABLATE_NO_GUARDS" || exit 1; done
cd /tmp && export TMPDIR=/tmp
for v in base noguard; do
  if [ $v = base ]; then X=""; else X="-DRRTE_ABLATE_NO_GUARDS"; fi
  RRTE_JIT_EXTRA_OPTS="$X" timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH --output-format csv -d $R/gpurun_out/gabl/pmc_$v -o run -- python3 $R/bench.py --no-cpu --no-stock --steps 20 > $R/gpurun_out/gabl/pmc_$v.log 2>&1 || exit 1
  python3 - <<PY
import csv,collections
c=collections.defaultdict(list)
for r in csv.DictReader(open('$R/gpurun_out/gabl/pmc_$v/run_counter_collection.csv')):
    if 'rrte_jit' in r['Kernel_Name']: c[r['Counter_Name']].append(float(r['Counter_Value']))
print('$v pmc', {k: round(sum(x)/len(x)/1e6,2) for k,x in c.items()})
PY
done
