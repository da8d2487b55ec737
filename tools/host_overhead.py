"""Host cost per frame call (diagnostic): enqueue-only timing of rrte_hip_render_async on a
tiny frame, vs the GPU-side throughput, for F streams in flight.
usage: python tools/host_overhead.py [scene] [W H] [F...]"""
import ctypes as C
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from rrte_amd import LoweredScene, abi, scenes  # noqa: E402
from rrte_amd.renderer import Context  # noqa: E402
import torch  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "sdf-showcase"
W, H = int(sys.argv[2]), int(sys.argv[3])
Fs = [int(a) for a in sys.argv[4:]] or [1, 4, 8]
objs, lights, cam, cfg = scenes.SCENES[name](W, H)
sc = LoweredScene(objs, lights, cam)
prm = cfg.lower()
ctx = Context(0, jit=abi.JIT_ON)
lib = ctx.lib
dev = torch.device("cuda", 0)
for F in Fs:
    streams = [torch.cuda.Stream(dev) for _ in range(F)]
    outs = [torch.empty(W * H, dtype=torch.int32, device=dev) for _ in range(F)]
    sp = [C.c_void_p(s.cuda_stream) for s in streams]
    ref, p = sc.ref(), C.byref(prm)
    for i in range(20):
        lib.rrte_hip_render_async(ctx.h, ref, p, outs[i % F].data_ptr(), None, sp[i % F])
    torch.cuda.synchronize()
    n = 400
    t0 = time.perf_counter()
    for i in range(n):
        lib.rrte_hip_render_async(ctx.h, ref, p, outs[i % F].data_ptr(), None, sp[i % F])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name} {W}x{H} F={F}: host enqueue {1e6 * (t1 - t0) / n:.1f} us/frame, "
          f"end-to-end {1e6 * (t2 - t0) / n:.1f} us/frame")
