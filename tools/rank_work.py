"""Where a frame's work lies under the multi-GPU band partition (diagnostic): renders one frame with
per-wave time stamps (RRTE_DEBUG=16: each 8x8 tile's wave writes its start and duration into the f32
buffer, ray_kernels.hpp ray_kernel_body), then sums the tiles' wave time per rank for N = 2 / 4 / 8
under the partition the library picks (rrte_hip_band_layout; device_scene.hpp band_owner).  A rank's
share of the summed wave time against its share of the rows says whether the ranks' frames follow
their work or something else.
usage: RRTE_DEBUG=16 python tools/rank_work.py [scene] [W H]"""
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from rrte_amd import LoweredScene, abi, scenes  # noqa: E402
from rrte_amd.renderer import Context  # noqa: E402

assert int(os.environ.get("RRTE_DEBUG", "0"), 0) & 16, "run with RRTE_DEBUG=16"
name = sys.argv[1] if len(sys.argv) > 1 else "sdf-showcase"
W, H = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1920, 1080)
import torch  # noqa: E402

objs, lights, cam, cfg = scenes.SCENES[name](W, H)
cfg.band_rows = 16
sc = LoweredScene(objs, lights, cam)
prm = cfg.lower()
ctx = Context(0, jit=abi.JIT_ON)
dev = torch.device("cuda", 0)
rgba = torch.empty(W * H, dtype=torch.int32, device=dev)
f32 = torch.zeros(W * H * 4 + 4096, dtype=torch.float32, device=dev)
tx, ty = (W + 7) // 8, (H + 7) // 8
durs = []
for it in range(6):
    ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(prm), rgba.data_ptr(), f32.data_ptr(), None))
    torch.cuda.synchronize()
    if it >= 2:  # (after the tile profile: the frames as the bench runs them)
        v = f32[: tx * ty * 16].view(torch.int32).cpu().numpy().view(np.uint32).reshape(tx * ty, 4, 4)[:, 0, :]
        durs.append(v[:, 2].astype(np.float64) / 100.0)  # us per 8x8 tile's wave
dur = np.mean(durs, axis=0).reshape(ty, tx)
row_work = dur.sum(axis=1)  # per 8-row tile row
print(f"{name} {W}x{H}: {tx * ty} tiles, summed wave time {dur.sum():.0f} us per frame")
for n in (2, 4, 8):
    sky, rb, pb = abi.band_layout(sc.ref(), C.byref(prm), n)
    L = rb + (n - 1) * pb
    nb = (H + 15) // 16
    owner = []
    for b in range(nb):
        if b < sky:
            owner.append(0)
            continue
        slot = (b - sky) % L
        owner.append(0 if slot < rb else 1 + (slot - rb) % (n - 1))
    work = np.zeros(n)
    rows = np.zeros(n)
    for b in range(nb):
        r0, r1 = b * 16, min(b * 16 + 16, H)
        work[owner[b]] += row_work[r0 // 8:(r1 + 7) // 8].sum()
        rows[owner[b]] += r1 - r0
    share = work / work.sum()
    print(f"N={n} partition sky {sky} root:peer {rb}:{pb}: work share per rank " +
          " ".join(f"{s:.3f}" for s in share) + f"  (max {share.max():.3f} vs 1/N {1 / n:.3f}); rows " +
          " ".join(str(int(r)) for r in rows))
ctx.close()
