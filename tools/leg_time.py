"""Time one workload on the GPU (frames in flight, as bench.py's legs) and print one JSON line:
ms per frame, lone-launch ms, shadow rays, jit kind and a hash of the frame (A/B runs of exact
variants must print the same hash).  Variants are environment settings of separate processes, e.g.
    RRTE_JIT_EXTRA_OPTS=-O3 python tools/leg_time.py --scene deformation-stress --width 3840 --height 2160
usage: python tools/leg_time.py [--scene S] [--width W] [--height H] [--mode M] [--jit on|off] [--frames N]"""
import argparse
import ctypes as C
import hashlib
import json
import os
import sys
import time
from pathlib import Path

os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("RRTE_BENCH_HW_QUEUES", "32")  # (as bench.py)
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from rrte_amd import LoweredScene, abi, scenes  # noqa: E402
from rrte_amd.renderer import Context  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="deformation-stress")
ap.add_argument("--width", type=int, default=3840)
ap.add_argument("--height", type=int, default=2160)
ap.add_argument("--mode", default="lambert_shadow")
ap.add_argument("--jit", default="on", choices=["on", "off"])
ap.add_argument("--frames", type=int, default=0, help="0: about 1 s of frames")
ap.add_argument("--inflight", type=int, default=4)
a = ap.parse_args()
dev = torch.device("cuda", 0)
objs, lights, cam, cfg = scenes.SCENES[a.scene](a.width, a.height, mode=a.mode)
sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
W, H, F = a.width, a.height, a.inflight
ctx = Context(0, jit=abi.JIT_ON if a.jit == "on" else abi.JIT_OFF)
streams = [torch.cuda.Stream(dev) for _ in range(F)]
sp = [C.c_void_p(s.cuda_stream) for s in streams]
outs = [torch.empty(W * H, dtype=torch.int32, device=dev) for _ in range(F)]


def go(i):
    ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(prm), outs[i % F].data_ptr(), None, sp[i % F]))


for i in range(4):
    go(i)
torch.cuda.synchronize(dev)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(streams[0])
for _ in range(5):
    go(0)
e1.record(streams[0])
torch.cuda.synchronize(dev)
lone = e0.elapsed_time(e1) / 5
n = a.frames or max(8, int(1000.0 / max(lone, 1e-3)))
ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
ctx.stats()
t0 = time.perf_counter()
for i in range(n):
    go(i)
torch.cuda.synchronize(dev)
dt = (time.perf_counter() - t0) / n
ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
st = ctx.stats()
h = hashlib.sha256(outs[0].cpu().numpy().tobytes()).hexdigest()[:16]
print(json.dumps({"scene": a.scene, "size": f"{W}x{H}", "mode": a.mode, "jit": int(st.jit_active),
                  "ms_per_frame": round(dt * 1e3, 4), "lone_launch_ms": round(lone, 4), "frames": n,
                  "shadow_rays_per_frame": int(st.shadow_rays) // n, "sha": h,
                  "env": {k: v for k, v in os.environ.items() if k.startswith("RRTE_")}}), flush=True)
ctx.close()
