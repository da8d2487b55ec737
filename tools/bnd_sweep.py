"""The blocking drop-in entry point (rrte_hip_render into a host RGBA8 buffer) per row-chunk count
(RRTE_BND_CHUNKS) and host-buffer kind: median ms per 1080p sdf-showcase frame after warm-up.
usage: python tools/bnd_sweep.py [chunks ...]"""
import ctypes as C
import os
import statistics
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from rrte_amd import LoweredScene, abi, scenes  # noqa: E402
from rrte_amd.renderer import Context  # noqa: E402

import torch  # noqa: E402

objs, lights, cam, cfg = scenes.sdf_showcase(1920, 1080)
sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
n = 1920 * 1080 * 4
for chunks in (sys.argv[1:] or ["1", "2", "3", "4", "6", "8"]):
    os.environ["RRTE_BND_CHUNKS"] = chunks
    ctx = Context(0, jit=abi.JIT_ON)
    res = {}
    for kind in ("pageable", "pinned", "fresh"):
        pinned = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        page = np.zeros(n, np.uint8)
        def ptr():
            if kind == "pinned":
                return C.cast(C.c_void_p(pinned.data_ptr()), C.POINTER(C.c_uint8))
            b = np.zeros(n, np.uint8) if kind == "fresh" else page
            ptr.keep = b
            return b.ctypes.data_as(C.POINTER(C.c_uint8))
        for _ in range(40):
            ctx.check(ctx.lib.rrte_hip_render(ctx.h, sc.ref(), C.byref(prm), ptr()))
        t = []
        for _ in range(30):
            a = time.perf_counter()
            ctx.check(ctx.lib.rrte_hip_render(ctx.h, sc.ref(), C.byref(prm), ptr()))
            t.append(time.perf_counter() - a)
        res[kind] = round(statistics.median(t) * 1e3, 4)
    st = ctx.stats()
    print(f"chunks {chunks}: {res}  kernel_ms {st.kernel_ms:.4f} hot {st.hot_tiles}", flush=True)
    ctx.close()
