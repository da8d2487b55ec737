"""Per-wave stamps (RRTE_DEBUG=16) of lone 1080p sdf-showcase frames under the hot-first tile order,
split tiles (RRTE_TILE_SPLIT=1) or not: each part of a split tile stamps its own slot.  Prints the
span and the slowest tiles with every part's start and duration -- diagnostic for the split's
critical path.  usage: RRTE_TILE_SPLIT=0|1 python tools/split_tiles.py"""
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from rrte_amd import LoweredScene, abi, scenes  # noqa: E402
from rrte_amd.renderer import Context  # noqa: E402
import torch  # noqa: E402

W, H = 1920, 1080
objs, lights, cam, cfg = scenes.sdf_showcase(W, H)
sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
os.environ["RRTE_DEBUG"] = "16"
ctx = Context(0, jit=abi.JIT_ON)
gx, gy = (W + 7) // 8, (H + 7) // 8
n = gx * gy
rgba = torch.empty(W * H, dtype=torch.int32, device="cuda")
f32 = torch.zeros(W * H * 4 + 4096, dtype=torch.float32, device="cuda")
torch.cuda.synchronize()
for rep in range(6):
    f32.zero_()
    torch.cuda.synchronize()
    ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(prm), rgba.data_ptr(), f32.data_ptr(), None))
    torch.cuda.synchronize()
    v = f32[: n * 16].view(torch.int32).cpu().numpy().view(np.uint32).reshape(n, 4, 4)
    st = v[:, :, 0].astype(np.uint64) | (v[:, :, 1].astype(np.uint64) << 32)
    dur = v[:, :, 2].astype(np.float64) / 100.0
    used = st > 0
    t0 = st[used].min()
    start = np.where(used, (st.astype(np.float64) - float(t0)) / 100.0, np.nan)
    end = np.where(used, start + dur, np.nan)
    tile_end = np.nanmax(end, axis=1)
    print(f"rep {rep}: hot slots {ctx.stats().hot_tiles}, span {np.nanmax(end):.1f} us, split tiles {int((used[:, 1:]).any(axis=1).sum())}")
    if rep == 5:
        for i in np.argsort(-tile_end)[:10]:
            parts = [(round(float(start[i, p]), 1), round(float(dur[i, p]), 1)) for p in range(4) if used[i, p]]
            print(f"  tile ({i % gx * 8}, {i // gx * 8}) ends {tile_end[i]:.1f}: parts (start, us) {parts}")
ctx.close()
