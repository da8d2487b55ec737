"""Host-side cost of the asynchronous frame call for a small frame (is a small-frame leg host-bound?).
Times N rrte_hip_render_async calls with 4 frames in flight two ways: the enqueue loop alone (no sync
inside, the device still working when it ends) and enqueue + drain; and the same through a Python loop
over the bare ctypes function (the bench legs' harness cost is the difference).  One JSON line.
usage: python tools/enqueue_rate.py [--scene basic-demo] [--width 640] [--height 480] [--frames 2000]"""
import argparse
import ctypes as C
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
ap.add_argument("--scene", default="basic-demo")
ap.add_argument("--width", type=int, default=640)
ap.add_argument("--height", type=int, default=480)
ap.add_argument("--mode", default=None)
ap.add_argument("--frames", type=int, default=2000)
ap.add_argument("--animated", action="store_true",
                help="a new scene every frame (8-frame value animation, cycled; the topology kernel), as "
                     "bench.py's topology_animated kind")
a = ap.parse_args()
if a.animated:
    os.environ["RRTE_JIT_TOPO"] = "1"  # (read at context creation)

dev = torch.device("cuda", 0)
objs, lights, cam, cfg = scenes.SCENES[a.scene](a.width, a.height)
if a.mode:
    cfg.mode = a.mode
sc = LoweredScene(objs, lights, cam)
prm = cfg.lower()
frames = [scenes.animate_values(LoweredScene(objs, lights, cam), f) for f in range(8)] if a.animated else [sc]
c = Context(0, jit=abi.JIT_ON)
lib = c.lib
F = 4
streams = [torch.cuda.Stream(dev) for _ in range(F)]
sp = [C.c_void_p(s.cuda_stream) for s in streams]
outs = [torch.empty(a.width * a.height, dtype=torch.int32, device=dev) for _ in range(F)]
optr = [o.data_ptr() for o in outs]
h, pref = c.h, C.byref(prm)
refs = [f.ref() for f in frames]
K = len(refs)
fn = lib.rrte_hip_render_async
for i in range(50):
    assert fn(h, refs[i % K], pref, optr[i % F], None, sp[i % F]) == 0
torch.cuda.synchronize(dev)
res = {"scene": a.scene, "width": a.width, "height": a.height, "frames": a.frames, "animated": a.animated}
for rep in range(2):
    t0 = time.perf_counter()
    for i in range(a.frames):
        fn(h, refs[i % K], pref, optr[i % F], None, sp[i % F])
    t1 = time.perf_counter()
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    res[f"enqueue_us_per_frame_{rep}"] = round((t1 - t0) / a.frames * 1e6, 3)
    res[f"total_us_per_frame_{rep}"] = round((t2 - t0) / a.frames * 1e6, 3)
# the Python loop alone (an arithmetic-only call of the same library, 4 arguments: the harness's share)
nop = lib.rrte_hip_band_rows_for_rank
t0 = time.perf_counter()
for i in range(a.frames):
    nop(1080, 16, 8, 3)
res["python_ctypes_call_us"] = round((time.perf_counter() - t0) / a.frames * 1e6, 3)
st = c.stats()
res["kernel_ms_last"] = round(st.kernel_ms, 5)
res["jit_active"] = int(st.jit_active)
print(json.dumps(res))
c.close()
