"""Per-wave durations of one frame (diagnostic): RRTE_DEBUG=16 makes the ray kernel write each wave's
start (100 MHz wall clock), duration and CU id into the f32 buffer instead of colours (ray_kernels.hpp
ray_kernel_body); see DESIGN.md §Performance (tail analysis).
usage: RRTE_DEBUG=16 python tools/wave_times.py [scene] [W H] [jit]"""
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
jit = int(sys.argv[4]) if len(sys.argv) > 4 else abi.JIT_ON
import torch  # noqa: E402

objs, lights, cam, cfg = scenes.SCENES[name](W, H)
sc = LoweredScene(objs, lights, cam)
prm = cfg.lower()
ctx = Context(0, jit=jit)
dev = torch.device("cuda", 0)
rgba = torch.empty(W * H, dtype=torch.int32, device=dev)
f32 = torch.zeros(W * H * 4 + 4096, dtype=torch.float32, device=dev)
for _ in range(3):
    ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(prm), rgba.data_ptr(), f32.data_ptr(), None))
torch.cuda.synchronize()
gx, gy = (W + 15) // 16, (H + 15) // 16
n = gx * gy * 4
v = f32[: n * 4].view(torch.int32).cpu().numpy().view(np.uint32).reshape(n, 4)
start = v[:, 0].astype(np.uint64) | (v[:, 1].astype(np.uint64) << 32)
dur = v[:, 2].astype(np.float64) / 100.0  # us
cu = v[:, 3]
start = (start - start.min()).astype(np.float64) / 100.0
end = start + dur
print(f"{name} {W}x{H} jit={jit}: {n} waves, kernel span {end.max():.1f} us, sum of wave time {dur.sum():.0f} us")
q = np.percentile(dur, [50, 90, 99, 99.9, 100])
print("wave duration us p50 %.1f p90 %.1f p99 %.1f p99.9 %.1f max %.1f" % tuple(q))
slow = np.argsort(-dur)[:10]
for i in slow:
    b, w = divmod(int(i), 4)
    by, bx = divmod(b, gx)
    px, py = bx * 16 + (w & 1) * 8, by * 16 + (w >> 1) * 8
    print(f"  wave {i}: tile ({px},{py}) start {start[i]:.1f} dur {dur[i]:.1f} end {end[i]:.1f} cu {cu[i]}")
# how much of the span is the tail: time when 99% of waves have finished
print("99%% of waves done at %.1f us; last start %.1f us" % (np.percentile(end, 99), start.max()))
# the slowest wave of each start-time decile: is the tail made of late starters or slow waves?
order = np.argsort(start)
for k, part in enumerate(np.array_split(order, 10)):
    print(f"  start decile {k}: starts {start[part].min():6.1f}-{start[part].max():6.1f} us, "
          f"mean dur {dur[part].mean():5.1f}, max dur {dur[part].max():6.1f}, last end {end[part].max():6.1f}")
# concurrency over time (waves resident), 10 us bins
edges = np.arange(0.0, end.max() + 10.0, 10.0)
res = [int(((start < b + 10.0) & (end > b)).sum()) for b in edges[:-1]]
print("resident waves per 10 us bin:", res)
tiles = dur.reshape(gy, gx, 2, 2).transpose(0, 2, 1, 3).reshape(gy * 2, gx * 2)
os.makedirs("gpurun_out", exist_ok=True)
np.save("gpurun_out/wave_dur_%s_%dx%d.npy" % (name, W, H), tiles)
