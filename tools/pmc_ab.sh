#!/bin/bash
# Interleaved A/B of headline variants: per variant and round, the frame time (bench.py, 200 and 20
# steps) and one PMC pass of per-dispatch instruction counts of the ray kernel.
# usage: tools/pmc_ab.sh ROUNDS "name|ENV=V ENV2=W" ["name2|..."] ...
#   e.g. tools/pmc_ab.sh 2 "base|" "noguard|RRTE_JIT_EXTRA_OPTS=-DRRTE_ABLATE_NO_GUARDS" "primary|RRTE_DEBUG=2"
# Device-code variants go through RRTE_JIT_EXTRA_OPTS (the scene-specialised kernel is compiled at run
# time; the disk-cache key includes the options).  Output: gpurun_out/pmc_ab/<name>_r<k>/ and a table
# on stdout.  Every step has its own time limit; the first failure ends the run.  PMC_COUNTERS replaces
# the counter set (one pass; e.g. "FETCH_SIZE" or "WRITE_SIZE" -- the block limits of rocprofv3 apply).
# A variant's BENCH_ARGS=... (no spaces: e.g. BENCH_ARGS=--jit=off) passes to bench.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ROUNDS=${1:?rounds}; shift
OUT=$R/gpurun_out/${PMC_AB_OUT:-pmc_ab}
mkdir -p $OUT
export GPU_MAX_HW_QUEUES=32  # (under rocprofv3 HIP starts before bench.py could set it)
cd /tmp && export TMPDIR=/tmp
COUNTERS=${PMC_COUNTERS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES"}
for k in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    name=${spec%%|*}; envs=${spec#*|}
    bargs=$(echo "$envs" | tr ' ' '\n' | sed -n 's/^BENCH_ARGS=//p')
    d=$OUT/${name}_r$k; mkdir -p $d
    for steps in 200 20; do
      env $envs timeout -k 10 180 python3 $R/bench.py --no-cpu --no-stock --no-boundary $bargs --steps $steps > $d/bench$steps.log 2>&1 \
        || { tail $d/bench$steps.log; echo "bench failed: $name"; exit 1; }
    done
    # (the program itself right after --: env assignments are exported before rocprofv3 starts)
    ( [ -n "$envs" ] && export $envs; timeout -s KILL 120 rocprofv3 --pmc $COUNTERS --output-format csv -d $d/pmc -o run -- python3 $R/bench.py --no-cpu --no-stock --no-boundary $bargs --steps 20 > $d/pmc.log 2>&1 ) \
      || { tail $d/pmc.log; echo "pmc failed: $name"; exit 1; }
    python3 - "$d" "$name" "$k" <<'PY'
import csv, json, sys, collections
from pathlib import Path
d, name, k = Path(sys.argv[1]), sys.argv[2], sys.argv[3]
def ms(f):
    line = [l for l in open(f) if l.startswith("{")][-1]
    j = json.loads(line)
    return j["ms_per_step"], j["roofline"]["avg_launch_ms"], j.get("verified", {}).get("u8_max_diff")
m200, lone, vd = ms(d / "bench200.log")
m20, _, _ = ms(d / "bench20.log")
acc = collections.defaultdict(list)
for f in d.glob("pmc/**/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "rrte_jit_kernel" in r["Kernel_Name"] or "ray_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
c = {n: sum(v) / len(v) for n, v in acc.items()}
res = {"name": name, "round": int(k), "ms200": m200, "ms20": m20, "launch_ms": lone, "u8_max_diff": vd,
       "VALU_M": c.get("SQ_INSTS_VALU", 0) / 1e6, "SALU_M": c.get("SQ_INSTS_SALU", 0) / 1e6,
       "SMEM_M": c.get("SQ_INSTS_SMEM", 0) / 1e6, "VMEM_RD_M": c.get("SQ_INSTS_VMEM_RD", 0) / 1e6,
       "waves": c.get("SQ_WAVES", 0), "dispatches": max((len(v) for v in acc.values()), default=0),
       "counters": c}
json.dump(res, open(d / "summary.json", "w"))
print(f"{name:>14} r{k}  200st {m200:.4f}  20st {m20:.4f}  launch {lone:.4f}  VALU {res['VALU_M']:.2f}M  "
      f"SALU {res['SALU_M']:.2f}M  SMEM {res['SMEM_M']:.2f}M  VMEM_RD {res['VMEM_RD_M']:.3f}M  u8diff {vd}"
      + "".join(f"  {n} {v:.1f}" for n, v in c.items() if not n.startswith("SQ_")), flush=True)
PY
  done
done
