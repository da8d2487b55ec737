"""Diagnostic: sdf-showcase at 3840x2160 with RRTE_TILE_ORDER=2 (fixed hot list, split tiles) vs image
order, three renders per variant (RGBA8 and linear floats), reporting how many pixels differ and in
which tiles (split or not).  Variants: split with the uncached exchange, split plus agent-scope fences
(RRTE_SPLIT_FENCE=1), hot order without splits.  usage: python tools/split_diag.py"""
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from rrte_amd import LoweredScene, abi, scenes  # noqa: E402
from rrte_amd.renderer import Context  # noqa: E402
import torch  # noqa: E402

W, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (3840, 2160)
objs, lights, cam, cfg = scenes.sdf_showcase(W, H)
sc, prm = LoweredScene(objs, lights, cam), cfg.lower()


def ctx_with(env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    c = Context(0, jit=abi.JIT_ON)
    for k, v in old.items():
        if v is None:
            os.environ.pop(k)
        else:
            os.environ[k] = v
    return c


def render(c, linear):
    p = abi.RenderParams.from_buffer_copy(prm)
    if linear:
        p.flags |= abi.FLAG_F32_LINEAR
        buf = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
        c.check(c.lib.rrte_hip_render_async(c.h, sc.ref(), C.byref(p), None, buf.data_ptr(), None))
    else:
        buf = torch.full((W * H,), -1, dtype=torch.int32, device="cuda")
        c.check(c.lib.rrte_hip_render_async(c.h, sc.ref(), C.byref(p), buf.data_ptr(), None, None))
    c.check(c.lib.rrte_hip_synchronize(c.h))
    return buf.cpu().numpy().view(np.uint32).reshape(H, W, -1)


ref = ctx_with({"RRTE_TILE_ORDER": "0"})
want = {lin: render(ref, lin) for lin in (False, True)}
ref.close()
for name, env in [("split", {"RRTE_TILE_ORDER": "2"}), ("split+fence", {"RRTE_TILE_ORDER": "2", "RRTE_SPLIT_FENCE": "1"}),
                  ("nosplit", {"RRTE_TILE_ORDER": "2", "RRTE_TILE_SPLIT": "0"})]:
    c = ctx_with(env)
    for rep in range(3):
        for lin in (False, True):
            got = render(c, lin)
            bad = np.any(got != want[lin], axis=2)
            ys, xs = np.nonzero(bad)
            tiles = sorted(set(zip((xs // 8).tolist(), (ys // 8).tolist())))
            print(f"{name} rep {rep} {'linear' if lin else 'rgba8'}: {int(bad.sum())} pixels differ in {len(tiles)} tiles "
                  f"{tiles[:6]}", flush=True)
            if bad.any():
                y, x = ys[0], xs[0]
                print("   first", (x, y), "got", got[y, x].view(np.float32) if lin else got[y, x],
                      "want", want[lin][y, x].view(np.float32) if lin else want[lin][y, x], flush=True)
    c.close()
