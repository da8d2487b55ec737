"""Host cost of enqueueing one frame (diagnostic): the plain path (rrte_hip_render_async) and the
multi-GPU path (rrte_hip_render_gather_async through a 1-rank RCCL communicator with
RRTE_FORCE_GATHER=1: band render -> ncclGather -> de-interleave, as a rank of an N-GPU job issues
them), for a frame the size of one rank's share at N = 8 (1920 x 136) with F frames in flight.
Host enqueue time per frame vs wall time per frame: when the first reaches the second the job is
host-bound.  usage: python tools/host_enqueue.py [W H] [F] [frames]"""
import ctypes as C
import os
import sys
import time
from pathlib import Path

os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("GPU_MAX_HW_QUEUES_OVERRIDE", "32")
os.environ["RRTE_FORCE_GATHER"] = "1"
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from rrte_amd import LoweredScene, abi, scenes  # noqa: E402
from rrte_amd.renderer import Context  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 2 else 1920
H = int(sys.argv[2]) if len(sys.argv) > 2 else 136
F = int(sys.argv[3]) if len(sys.argv) > 3 else 8
N = int(sys.argv[4]) if len(sys.argv) > 4 else 400
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
ref, p = sc.ref(), C.byref(prm)


def run(kind):
    fn = lib.rrte_hip_render_async if kind == "plain" else lib.rrte_hip_render_gather_async

    def one(i):
        if kind == "plain":
            st = fn(ctx.h, ref, p, outs[i % F].data_ptr(), None, sp[i % F])
        else:
            st = fn(ctx.h, ref, p, 0, outs[i % F].data_ptr(), sp[i % F])
        if st:
            ctx.check(st)

    for i in range(30):
        one(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(N):
        one(i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return 1e6 * (t1 - t0) / N, 1e6 * (t2 - t0) / N


for kind in ("plain", "gather", "plain", "gather"):
    enq, wall = run(kind)
    print(f"{kind:6s} {W}x{H} F={F}: host enqueue {enq:6.1f} us/frame, wall {wall:6.1f} us/frame")
ctx.close()
