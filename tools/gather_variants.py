"""Wall time per frame of the multi-GPU frame path on ONE GPU (diagnostic, 1-rank RCCL communicators,
RRTE_FORCE_GATHER=1) for a rank-sized frame against the plain render, plus the same with a timing
event recorded after every frame, gathering every frame on its own (its gather chained to the previous
frame's across the F streams) or in batches of B frames (rrte_hip_set_gather_batch: one ncclGather per
batch on the comm stream).  usage: python tools/gather_variants.py [W H] [F] [frames] [B]"""
import ctypes as C
import os
import sys
import time
from pathlib import Path

os.environ["GPU_MAX_HW_QUEUES"] = "32"
os.environ["RRTE_FORCE_GATHER"] = "1"
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from rrte_amd import LoweredScene, abi, scenes  # noqa: E402
from rrte_amd.renderer import Context  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 2 else 1920
H = int(sys.argv[2]) if len(sys.argv) > 2 else 136
F = int(sys.argv[3]) if len(sys.argv) > 3 else 8
N = int(sys.argv[4]) if len(sys.argv) > 4 else 200
B = int(sys.argv[5]) if len(sys.argv) > 5 else F
objs, lights, cam, cfg = scenes.sdf_showcase(W, H)
sc = LoweredScene(objs, lights, cam)
prm = cfg.lower()
ctx = Context(0, jit=abi.JIT_ON)
lib = ctx.lib
uid = (C.c_uint8 * abi.UNIQUE_ID_BYTES)()
ctx.check(lib.rrte_hip_comm_unique_id(uid))
ctx.check(lib.rrte_hip_comm_init(ctx.h, 1, 0, uid))
dev = torch.device("cuda", 0)
streams = [torch.cuda.Stream(dev) for _ in range(F)]
outs = [torch.empty(W * H, dtype=torch.int32, device=dev) for _ in range(F)]
sp = [C.c_void_p(s.cuda_stream) for s in streams]
ref = sc.ref()


def run(kind, flags=0, events=False, batch=1, one_stream=False):
    ctx.check(lib.rrte_hip_set_gather_batch(ctx.h, batch))
    prm.flags = flags
    p = C.byref(prm)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(F)]

    def one(i):
        if kind == "plain":
            st = lib.rrte_hip_render_async(ctx.h, ref, p, outs[i % F].data_ptr(), None, sp[i % F])
        else:
            st = lib.rrte_hip_render_gather_async(ctx.h, ref, p, 0, outs[i % F].data_ptr(),
                                                  sp[0] if one_stream else sp[i % F])
        if st:
            ctx.check(st)
        if events:
            evs[i % F].record(streams[i % F])

    for i in range(30):
        one(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(N):
        one(i)
    t1 = time.perf_counter()
    ctx.check(lib.rrte_hip_flush(ctx.h))
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return 1e6 * (t1 - t0) / N, 1e6 * (t2 - t0) / N


for rep in range(int(os.environ.get("GV_REPS", "2"))):
    for name, kind, ev, batch, one in [("plain", "plain", False, 1, False),
                                       ("gather per frame", "gather", False, 1, False),
                                       ("gather per frame+ev", "gather", True, 1, False),
                                       (f"gather batch {B}", "gather", False, B, False),
                                       (f"gather batch {B} 1 stream", "gather", False, B, True),
                                       (f"gather batch {B}+ev", "gather", True, B, False)]:
        enq, wall = run(kind, 0, ev, batch, one)
        print(f"{name:26s} {W}x{H} F={F}: "
              f"host {enq:6.1f} us/frame, wall {wall:6.1f} us/frame", flush=True)
ctx.close()
