"""10 blocking rrte_hip_render frames of the headline workload after 3 warm-up frames (trace target)."""
import ctypes as C
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from rrte_amd import LoweredScene, abi, scenes  # noqa: E402
from rrte_amd.renderer import Context  # noqa: E402

objs, lights, cam, cfg = scenes.sdf_showcase(1920, 1080)
sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
ctx = Context(0, jit=abi.JIT_ON)
buf = np.zeros(1920 * 1080 * 4, np.uint8)
p = buf.ctypes.data_as(C.POINTER(C.c_uint8))
for _ in range(3):
    ctx.check(ctx.lib.rrte_hip_render(ctx.h, sc.ref(), C.byref(prm), p))
t = []
for _ in range(10):
    a = time.perf_counter()
    ctx.check(ctx.lib.rrte_hip_render(ctx.h, sc.ref(), C.byref(prm), p))
    t.append(time.perf_counter() - a)
print("ms per frame", [round(x * 1e3, 3) for x in t])
