"""Where the fixed cost of a short timed region goes (diagnostic): the bench's frames-in-flight loop
for K frames with a HIP event before and after every frame on its own stream plus the host time of
every enqueue, all relative to the start of the timed region.
usage: python tools/ramp.py [K] [inflight] [gather] [H]
gather=1: the multi-GPU frame path through a 1-rank RCCL communicator (RRTE_FORCE_GATHER=1)"""
import ctypes as C
import os
import sys
import time
from pathlib import Path

os.environ.setdefault("GPU_MAX_HW_QUEUES", "32")
os.environ["RRTE_FORCE_GATHER"] = "1"
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from rrte_amd import LoweredScene, abi, scenes  # noqa: E402
from rrte_amd.renderer import Context  # noqa: E402

import torch  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
F = int(sys.argv[2]) if len(sys.argv) > 2 else 12
G = len(sys.argv) > 3 and sys.argv[3] == "1"
W, H = 1920, int(sys.argv[4]) if len(sys.argv) > 4 else 1080
objs, lights, cam, cfg = scenes.SCENES["sdf-showcase"](W, H)
sc = LoweredScene(objs, lights, cam)
prm = cfg.lower()
ctx = Context(0, jit=abi.JIT_ON)
if G:
    uid = (C.c_uint8 * abi.UNIQUE_ID_BYTES)()
    ctx.check(ctx.lib.rrte_hip_comm_unique_id(uid))
    ctx.check(ctx.lib.rrte_hip_comm_init(ctx.h, 1, 0, uid))
dev = torch.device("cuda", 0)
streams = [torch.cuda.Stream(dev) for _ in range(F)]
outs = [torch.empty(W * H, dtype=torch.int32, device=dev) for _ in range(F)]
sp = [C.c_void_p(s.cuda_stream) for s in streams]
ref, pp = sc.ref(), C.byref(prm)


def enqueue(i):
    if G:
        ctx.check(ctx.lib.rrte_hip_render_gather_async(ctx.h, ref, pp, 0, outs[i % F].data_ptr(), sp[i % F]))
    else:
        ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, ref, pp, outs[i % F].data_ptr(), None, sp[i % F]))


for i in range(10):
    enqueue(i)
torch.cuda.synchronize()
for rep in range(3):
    ev0 = torch.cuda.Event(enable_timing=True)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    host = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(streams[0])
    for i in range(K):
        s = streams[i % F]
        evs[i][0].record(s)
        enqueue(i)
        evs[i][1].record(s)
        host.append(time.perf_counter() - t0)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t1 = time.perf_counter() - t0
    print(f"rep {rep}: K={K} F={F} gather={G} H={H} wall {t1 * 1e3:.3f} ms = {t1 / K * 1e3:.4f} ms/frame; "
          f"host enqueue of all frames {t_enq * 1e3:.3f} ms ({t_enq / K * 1e6:.1f} us/frame)")
    for i in range(K):
        a, b = ev0.elapsed_time(evs[i][0]), ev0.elapsed_time(evs[i][1])
        print(f"  frame {i:3d}: host enq done {host[i] * 1e3:7.3f} ms  gpu start {a:7.3f} end {b:7.3f} dur {b - a:6.3f}")
ctx.close()
