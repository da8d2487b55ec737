"""Per-tile durations and start times of one lone frame and of a frame inside a 4-deep stream
(RRTE_DEBUG=16 stamps: each wave writes its start, duration and CU into the f32 buffer) -- diagnostic
input for the dispatch-order simulation in tools/tile_sim.py.  usage: python tools/tile_dump.py [scene] [W H]"""
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
import torch  # noqa: E402

objs, lights, cam, cfg = scenes.SCENES[name](W, H)
sc = LoweredScene(objs, lights, cam)
prm = cfg.lower()
dev = torch.device("cuda", 0)
gx, gy = (W + 7) // 8, (H + 7) // 8
n = gx * gy
os.environ["RRTE_DEBUG"] = "16"
ctx = Context(0, jit=abi.JIT_ON)
rgba = [torch.empty(W * H, dtype=torch.int32, device=dev) for _ in range(4)]
f32 = [torch.zeros(W * H * 4 + 4096, dtype=torch.float32, device=dev) for _ in range(4)]
streams = [torch.cuda.Stream() for _ in range(4)]
out = {}
for rep in range(3):  # lone frames
    f32[0].zero_()
    torch.cuda.synchronize()
    ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(prm), rgba[0].data_ptr(), f32[0].data_ptr(), None))
    torch.cuda.synchronize()
    v = f32[0][: n * 16].view(torch.int32).cpu().numpy().view(np.uint32).reshape(n, 4, 4)[:, 0, :].copy()
    out[f"lone{rep}"] = v
# a stream of 16 frames, 4 in flight on 4 streams: keep frame 12's stamps
for f in range(16):
    s = streams[f % 4]
    with torch.cuda.stream(s):
        ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(prm), rgba[f % 4].data_ptr(),
                                                f32[f % 4].data_ptr(), C.c_void_p(s.cuda_stream)))
torch.cuda.synchronize()
for k in range(4):
    out[f"stream{k}"] = f32[k][: n * 16].view(torch.int32).cpu().numpy().view(np.uint32).reshape(n, 4, 4)[:, 0, :].copy()
ctx.close()
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed(f"gpurun_out/tiles_{name}_{W}x{H}.npz", gx=gx, gy=gy, **out)
for k, v in out.items():
    d = v[:, 2].astype(np.float64) / 100.0
    st = (v[:, 0].astype(np.uint64) | (v[:, 1].astype(np.uint64) << 32))
    st = (st - st.min()).astype(np.float64) / 100.0
    print(k, "span %.1f us, dur p50 %.1f p99 %.1f max %.1f, tiles > 40 us: %d" %
          ((st + d).max(), np.median(d), np.percentile(d, 99), d.max(), int((d > 40).sum())))
