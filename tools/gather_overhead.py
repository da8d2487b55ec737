"""Per-frame cost of the multi-GPU frame path on ONE GPU (diagnostic): a 1-rank RCCL communicator with
RRTE_FORCE_GATHER=1 runs band render -> ncclGather -> de-interleave exactly as a rank of an N-GPU
job would (minus the xGMI transfer), frames pipelined over F streams, against plain
rrte_hip_render_async of the same frame.  The difference bounds the fixed per-frame cost the gather
path adds (RCCL kernel launch, events, de-interleave).
usage: python tools/gather_overhead.py [W H] [F] [frames]"""
import ctypes as C
import os
import sys
import time
from pathlib import Path

os.environ.setdefault("GPU_MAX_HW_QUEUES", "32")
os.environ["RRTE_FORCE_GATHER"] = "1"
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from rrte_amd import LoweredScene, abi, scenes  # noqa: E402
from rrte_amd.renderer import Context  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 2 else 1920
H = int(sys.argv[2]) if len(sys.argv) > 2 else 1080
F = int(sys.argv[3]) if len(sys.argv) > 3 else 12
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
ref = sc.ref()


def run(kind, flags):
    prm.flags = flags
    p = C.byref(prm)

    def one(i):
        if kind == "plain":
            ctx.check(lib.rrte_hip_render_async(ctx.h, ref, p, outs[i % F].data_ptr(), None, sp[i % F]))
        else:
            ctx.check(lib.rrte_hip_render_gather_async(ctx.h, ref, p, 0, outs[i % F].data_ptr(), sp[i % F]))

    for i in range(30):
        one(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(N):
        one(i)
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / N


base = prm.flags
for kind, flags, name in (("plain", base, "render_async"),
                          ("gather", base | abi.FLAG_GATHER_OVERLAP, "gather path, pipelined"),
                          ("gather", base, "gather path, one stream per frame"),
                          ("plain", base, "render_async")):
    print(f"{W}x{H} F={F} {name}: {run(kind, flags):.4f} ms/frame", flush=True)
