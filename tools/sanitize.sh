#!/bin/bash
# Host-only code under ASan + UBSan (clang's runtime, ROCm LLVM): the CPU oracle, the C++ mirror,
# and the host parts of librrte_hip (validation, lowering, BVH builder, CSG-guard analysis, JIT
# source generation + hiprtc).  Device code is compiled without instrumentation (-Xarch_host).
# Builds build/sanitize/sanitize_driver and runs it; tests/test_sanitize.py drives this script.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
B=$R/build/sanitize
mkdir -p $B
CLANG=/opt/rocm/llvm/bin/clang
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1"
HSAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined -Xarch_host -fno-omit-frame-pointer"
cd $R/rrte_amd/csrc
make -s jit_headers.inc
for f in rrte_hip jit bvh sdf_guard scene_io; do
  [ $B/$f.o -nt $f.hip ] && [ $B/$f.o -nt ray_kernels.hpp ] && [ $B/$f.o -nt device_scene.hpp ] && continue
  /opt/rocm/bin/hipcc -std=c++17 -O1 -g --offload-arch=gfx950 -ffp-contract=off -fPIC $HSAN -I/opt/rocm/include -c $f.hip -o $B/$f.o &
done
$CLANG -std=c11 $SAN -ffp-contract=off -pthread -c $R/oracle/rrte_oracle.c -o $B/rrte_oracle.o &
for f in rrte_renderer examples; do
  $CLANG++ -std=c++17 $SAN -ffp-contract=off -I$R/include -c $R/rrte_amd/cpp/$f.cpp -o $B/$f.o &
done
$CLANG++ -std=c++17 $SAN -I$R/include -c $R/tests/cpp/sanitize_driver.cpp -o $B/sanitize_driver.o &
wait
$CLANG++ $SAN -o $B/sanitize_driver $B/sanitize_driver.o $B/rrte_renderer.o $B/examples.o $B/rrte_oracle.o \
  $B/rrte_hip.o $B/jit.o $B/bvh.o $B/sdf_guard.o $B/scene_io.o -L/opt/rocm/lib -lamdhip64 -lrccl -lhiprtc -pthread -lm \
  -Wl,-rpath,/opt/rocm/lib
# leaks inside the ROCm runtime / comgr (not ours) are suppressed by library; ours are reported
cat > $B/lsan.supp <<'SUPP'
leak:libamdhip64
leak:libamd_comgr
leak:libhiprtc
leak:librccl
leak:libhsa-runtime64
SUPP
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 LSAN_OPTIONS=suppressions=$B/lsan.supp UBSAN_OPTIONS=print_stacktrace=1 \
  $B/sanitize_driver
