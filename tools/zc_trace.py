"""Blocking drop-in frames (rrte_hip_render) for a kernel trace: 30 frames into a reused pageable buffer,
then 30 into the same buffer registered with rrte_hip_host_register (the kernel stores the frame over
PCIe).  Prints the host ms per frame of each; run under `rocprofv3 --kernel-trace --stats` to see the
launches' own durations (the zero-copy launches are the 32x2-tile grid).
usage: python tools/zc_trace.py [scene]"""
import ctypes as C
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from rrte_amd import LoweredScene, abi, scenes  # noqa: E402
from rrte_amd.renderer import Context  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "sdf-showcase"
objs, lights, cam, cfg = scenes.SCENES[name](1920, 1080, mode="lambert_shadow")
sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
ctx = Context(0, jit=abi.JIT_ON)
lib = ctx.lib
buf = np.zeros(1920 * 1080 * 4, dtype=np.uint8)
ptr = buf.ctypes.data_as(C.POINTER(C.c_uint8))
frames = {}
for label, reg in (("reused", False), ("registered", True)):
    if reg:
        ctx.check(lib.rrte_hip_host_register(ctx.h, buf.ctypes.data, buf.nbytes))
        buf[:] = 0  # (so the comparison below shows the zero-copy frames' own bytes)
    for _ in range(5):
        ctx.check(lib.rrte_hip_render(ctx.h, sc.ref(), C.byref(prm), ptr))
    t = time.perf_counter()
    for _ in range(30):
        ctx.check(lib.rrte_hip_render(ctx.h, sc.ref(), C.byref(prm), ptr))
    print(f"{label}: {(time.perf_counter() - t) / 30 * 1e3:.4f} ms per frame", flush=True)
    frames[label] = buf.copy()
print("registered frame equals the copy path's:", bool(np.array_equal(frames["reused"], frames["registered"])))
ctx.check(lib.rrte_hip_host_unregister(ctx.h, buf.ctypes.data))
# page-locked by the allocator instead (hipHostMalloc, as torch's pinned memory is): zero copy as well
import torch  # noqa: E402
pin = torch.zeros(1920 * 1080 * 4, dtype=torch.uint8, pin_memory=True)
pptr = C.cast(C.c_void_p(pin.data_ptr()), C.POINTER(C.c_uint8))
for _ in range(5):
    ctx.check(lib.rrte_hip_render(ctx.h, sc.ref(), C.byref(prm), pptr))
t = time.perf_counter()
for _ in range(30):
    ctx.check(lib.rrte_hip_render(ctx.h, sc.ref(), C.byref(prm), pptr))
print(f"hostmalloc: {(time.perf_counter() - t) / 30 * 1e3:.4f} ms per frame", flush=True)
print("hostmalloc frame equals the copy path's:", bool(np.array_equal(frames["reused"], pin.numpy())))
ctx.close()
