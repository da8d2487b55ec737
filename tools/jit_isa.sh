#!/bin/bash
# Compile the scene-specialised kernel of <scene> offline (hipcc, as hiprtc would) with extra flags and
# report resources plus static instruction counts: VALU, SALU, EXEC writes, and per-loop body sizes.
# usage: tools/jit_isa.sh <scene> <out.s> [extra hipcc flags...]
SCENE=${1:-sdf-showcase}; OUT=${2:-/tmp/jit.s}; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
RRTE_JIT_DUMP=$T/jit.hip python -c "
import sys; sys.path.insert(0, '$R')
from rrte_amd import abi, scenes, LoweredScene
lib = abi.load(); o,l,c,cfg = scenes.SCENES['$SCENE'](64,36); sc = LoweredScene(o,l,c)
lib.rrte_hip_jit_check(sc.ref(), 1, None, 0)" || exit 1
mkdir -p $T/inc && cp $R/include/rrte_hip.h $T/inc/ && cp $R/rrte_amd/csrc/device_scene.hpp $R/rrte_amd/csrc/ray_kernels.hpp $T/
sed -i "s#../../include/rrte_hip.h#$T/inc/rrte_hip.h#" $T/device_scene.hpp
sed -i 's/^typedef __hip_internal.*$//' $T/jit.hip && sed -i '1i #include <hip/hip_runtime.h>' $T/jit.hip
# (the JIT's own options, jit.hip rtc_options: -O1, no contraction, the max-ILP scheduler)
cd $T && /opt/rocm/bin/hipcc -std=c++17 -O1 --offload-arch=gfx950 -ffp-contract=off -mllvm -amdgpu-sched-strategy=max-ilp --cuda-device-only -S -o $OUT \
   -Rpass-analysis=kernel-resource-usage "$@" jit.hip 2>&1 | grep -E "(VGPRs:|SGPRs:|Scratch|Occupancy)" | sed 's/.*remark: *//' | tr '\n' ' '
echo
python3 - "$OUT" <<'PY'
import re, sys
lines = [l.strip() for l in open(sys.argv[1]) if l.strip() and not l.strip().startswith(('.', ';'))]
v = sum(1 for l in lines if l.startswith('v_')); s = sum(1 for l in lines if l.startswith('s_') and not l.startswith(('s_waitcnt', 's_nop')))
ex = sum(1 for l in lines if re.match(r's_\w+ exec', l) or 'saveexec' in l)
print(f"static: VALU {v}  SALU {s}  exec-writes {ex}")
PY
