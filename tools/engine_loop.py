"""Engine::render_frame's loop (Raytracer.render_into: one reused buffer, pinned once) timed per JIT policy,
beside the raw C-ABI blocking call into a registered buffer.  usage: python tools/engine_loop.py"""
import ctypes as C
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402

from rrte_amd import LoweredScene, Raytracer, abi, scenes  # noqa: E402

objs, lights, cam, cfg = scenes.sdf_showcase(1920, 1080)
for name, jit in (("on", abi.JIT_ON), ("auto", abi.JIT_AUTO), ("off", abi.JIT_OFF)):
    rt = Raytracer(cfg, device=0, jit=jit)
    buf = np.zeros(1920 * 1080 * 4, np.uint8)
    for _ in range(60):
        rt.render_into(objs, lights, [], cam, buf)
    sc = LoweredScene(objs, lights, cam)
    prm = cfg.lower()
    n = 40
    a = time.perf_counter()
    for _ in range(n):
        rt.render_into(objs, lights, [], cam, buf)
    t_mirror = (time.perf_counter() - a) / n * 1e3
    ctx = rt.ctx
    a = time.perf_counter()
    for _ in range(n):
        ctx.check(ctx.lib.rrte_hip_render(ctx.h, sc.ref(), C.byref(prm), buf.ctypes.data))
    t_abi = (time.perf_counter() - a) / n * 1e3
    st = rt.stats()
    print(f"jit={name}: mirror render_into {t_mirror:.4f} ms/frame, C-ABI same buffer {t_abi:.4f} ms/frame, "
          f"jit_active {st.jit_active}, kernel_ms {st.kernel_ms:.4f}, pinned {rt._pinned is not None}", flush=True)
    ctx.close()
