#!/bin/bash
# Host code on several threads under ThreadSanitizer (clang's runtime, ROCm LLVM): the CPU oracle's
# thread pool, the C++ mirror, and the host parts of librrte_hip that a context runs on its worker
# threads (JIT source generation + hiprtc, tile-order planning, SceneIR dump / load, cache keys).
# Device code is compiled without instrumentation (-Xarch_host).  Builds build/tsan/tsan_driver and
# runs it; tests/test_sanitize.py drives this script.
# `tools/tsan.sh gpu-build` instead links tests/cpp/tsan_gpu_driver.cpp (the contexts' own worker threads
# beside two rendering threads; needs a GPU) to rrte_amd/lib/tsan_gpu_driver, which travels to the GPU
# box, and `tools/tsan.sh gpu-run` runs it there.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
B=$R/build/tsan
mkdir -p $B
CLANG=/opt/rocm/llvm/bin/clang
SAN="-fsanitize=thread -fno-omit-frame-pointer -g -O1"
HSAN="-Xarch_host -fsanitize=thread -Xarch_host -fno-omit-frame-pointer"
if [ "${1:-}" = gpu-run ]; then
  # The ROCm runtime libraries are not instrumented: their own threads synchronise through atomics TSan
  # cannot see, so allocations they make and free on their threads read as races (the first run
  # reported exactly that, an operator new / delete pair inside libhsa-runtime64 during context
  # creation: profiles/r06_tsan_gpu_unsuppressed.log).  Their interceptor calls are ignored and
  # reports with a runtime frame in an access stack suppressed; a race between two of our own
  # accesses is still reported.
  SUPP=$(mktemp)
  printf '%s\n' called_from_lib:libhsa-runtime64.so.1 called_from_lib:libamdhip64.so.7 called_from_lib:libhiprtc.so.7 \
    called_from_lib:libamd_comgr.so.3 called_from_lib:librccl.so.1 race:libhsa-runtime64.so race:libamdhip64.so \
    race:libhiprtc.so race:libamd_comgr.so race:librccl.so > $SUPP
  RRTE_JIT_CACHE=0 RRTE_TEST_RECYCLE=1 TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1 suppressions=$SUPP" \
    timeout -k 10 300 $R/rrte_amd/lib/tsan_gpu_driver "${2:-160}"
  exit $?
fi
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
$CLANG++ -std=c++17 $SAN -I$R/include -c $R/tests/cpp/tsan_driver.cpp -o $B/tsan_driver.o &
$CLANG++ -std=c++17 $SAN -I$R/include -c $R/tests/cpp/tsan_gpu_driver.cpp -o $B/tsan_gpu_driver.o &
wait
if [ "${1:-}" = gpu-build ]; then
  $CLANG++ $SAN -o $R/rrte_amd/lib/tsan_gpu_driver $B/tsan_gpu_driver.o $B/rrte_renderer.o $B/examples.o \
    $B/rrte_hip.o $B/jit.o $B/bvh.o $B/sdf_guard.o $B/scene_io.o -L/opt/rocm/lib -lamdhip64 -lrccl -lhiprtc -pthread -lm \
    -Wl,-rpath,/opt/rocm/lib
  exit 0
fi
$CLANG++ $SAN -o $B/tsan_driver $B/tsan_driver.o $B/rrte_renderer.o $B/examples.o $B/rrte_oracle.o \
  $B/rrte_hip.o $B/jit.o $B/bvh.o $B/sdf_guard.o $B/scene_io.o -L/opt/rocm/lib -lamdhip64 -lrccl -lhiprtc -pthread -lm \
  -Wl,-rpath,/opt/rocm/lib
# halt_on_error: the first race ends the run with TSan's report and a non-zero status
TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" $B/tsan_driver
