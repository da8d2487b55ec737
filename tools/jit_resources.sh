#!/bin/bash
# Dump the scene-specialised kernel source for a scene and report its resource usage (hipcc).
# usage: tools/jit_resources.sh <scene> [mode]
SCENE=${1:-sdf-showcase}; MODE=${2:-1}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
RRTE_JIT_DUMP=$T/jit.hip python -c "
import sys; sys.path.insert(0, '$R')
from rrte_amd import abi, scenes, LoweredScene
lib = abi.load(); o,l,c,cfg = scenes.SCENES['$SCENE'](64,36); sc = LoweredScene(o,l,c)
print('jit_check', lib.rrte_hip_jit_check(sc.ref(), $MODE, None, 0))" || exit 1
mkdir -p $T/inc && cp $R/include/rrte_hip.h $T/inc/ && cp $R/rrte_amd/csrc/device_scene.hpp $R/rrte_amd/csrc/ray_kernels.hpp $T/
sed -i "s#../../include/rrte_hip.h#$T/inc/rrte_hip.h#" $T/device_scene.hpp
sed -i 's/^typedef __hip_internal.*$//' $T/jit.hip && sed -i '1i #include <hip/hip_runtime.h>' $T/jit.hip
cd $T && /opt/rocm/bin/hipcc -std=c++17 -O3 --offload-arch=gfx950 -ffp-contract=off --cuda-device-only -S -o $T/jit.s \
   -Rpass-analysis=kernel-resource-usage jit.hip 2>&1 | grep -E "warning: loop|jit.hip.*(VGPRs:|SGPRs:|Scratch|Occupancy|LDS|Spill)|hipcc" | sort | uniq -c
echo "isa: $T/jit.s ($(grep -c '^\s*v_' $T/jit.s) VALU lines)"
