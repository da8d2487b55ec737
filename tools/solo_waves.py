"""Duration of the slowest waves of a frame under full load vs alone on the GPU (diagnostic).
First a stamped frame (RRTE_DEBUG=16) finds the slowest waves; then, for each of their workgroups,
a context with RRTE_DEBUG bit 5 runs only that workgroup (ray_kernels.hpp ray_kernel_body).
usage: python tools/solo_waves.py [scene] [W H] [n]"""
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from rrte_amd import LoweredScene, abi, scenes  # noqa: E402
from rrte_amd.renderer import Context  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "sdf-showcase"
W, H = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1920, 1080)
N = int(sys.argv[4]) if len(sys.argv) > 4 else 8
import torch  # noqa: E402

objs, lights, cam, cfg = scenes.SCENES[name](W, H)
sc = LoweredScene(objs, lights, cam)
prm = cfg.lower()
dev = torch.device("cuda", 0)
rgba = torch.empty(W * H, dtype=torch.int32, device=dev)
f32 = torch.zeros(W * H * 4 + 4096, dtype=torch.float32, device=dev)
gx, gy = (W + 15) // 16, (H + 15) // 16
n = gx * gy * 4


def stamped(debug):
    os.environ["RRTE_DEBUG"] = str(debug)
    ctx = Context(0, jit=abi.JIT_ON)
    f32.zero_()
    for _ in range(3):
        ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(prm), rgba.data_ptr(), f32.data_ptr(), None))
    torch.cuda.synchronize()
    ctx.close()
    v = f32[: n * 4].view(torch.int32).cpu().numpy().view(np.uint32).reshape(n, 4)
    return v[:, 2].astype(np.float64) / 100.0  # us


full = stamped(16)
slow = np.argsort(-full)[:N]
print(f"{name} {W}x{H}: loaded p50 {np.median(full):.1f} us, max {full.max():.1f} us")
for i in slow:
    blk, w = divmod(int(i), 4)
    alone = stamped(16 | 32 | (blk << 16))
    prim = stamped(16 | 32 | 2 | (blk << 16))  # primary visibility only
    noshadow = stamped(16 | 32 | 1 | (blk << 16))  # + attributes and shading, no shadow tests
    by, bx = divmod(blk, gx)
    px, py = bx * 16 + (w & 1) * 8, by * 16 + (w >> 1) * 8
    others = ", ".join(f"{alone[blk * 4 + k]:.1f}" for k in range(4))
    print(f"  wave {i} tile ({px},{py}): loaded {full[i]:.1f} us, alone {alone[i]:.1f} us (its workgroup alone: {others}); "
          f"alone primary-only {prim[i]:.1f}, no shadow tests {noshadow[i]:.1f}")
