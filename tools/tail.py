"""Tail analysis of one frame, 64-thread workgroups (one 8x8 tile per wave) -- diagnostic only.
A stamped frame (RRTE_DEBUG=16: each wave writes its start, duration and CU into the f32 buffer)
gives the per-wave durations under full load; then each of the N slowest tiles runs ALONE
(RRTE_DEBUG bit 5 + the workgroup index in bits 16+) in several ablations: full, primary visibility
only (bit 1), no shadow tests (bit 0), and the shadow tests of one light only (bit 8, light in bits
9-11).  usage: python tools/tail.py [scene] [W H] [N]"""
import ctypes as C
import json
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from rrte_amd import LoweredScene, abi, scenes  # noqa: E402
from rrte_amd.renderer import Context  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "sdf-showcase"
W, H = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1920, 1080)
N = int(sys.argv[4]) if len(sys.argv) > 4 else 6
import torch  # noqa: E402

objs, lights, cam, cfg = scenes.SCENES[name](W, H)
sc = LoweredScene(objs, lights, cam)
prm = cfg.lower()
dev = torch.device("cuda", 0)
rgba = torch.empty(W * H, dtype=torch.int32, device=dev)
f32 = torch.zeros(W * H * 4 + 4096, dtype=torch.float32, device=dev)
gx, gy = (W + 7) // 8, (H + 7) // 8
n = gx * gy
nl = len(lights)


def stamped(debug, reps=3):
    os.environ["RRTE_DEBUG"] = str(debug)
    ctx = Context(0, jit=abi.JIT_ON)
    best = None
    for _ in range(reps):
        f32.zero_()
        ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(prm), rgba.data_ptr(), f32.data_ptr(), None))
        torch.cuda.synchronize()
        v = f32[: n * 16].view(torch.int32).cpu().numpy().view(np.uint32).reshape(n, 4, 4)[:, 0, :]
        d = v[:, 2].astype(np.float64) / 100.0
        best = d if best is None else np.minimum(best, d)
    st = v
    ctx.close()
    return best, st


full, st = stamped(16)
start = st[:, 0].astype(np.uint64) | (st[:, 1].astype(np.uint64) << 32)
start = (start - start.min()).astype(np.float64) / 100.0
end = start + full
q = np.percentile(full, [50, 90, 99, 99.9, 100])
out = {"scene": name, "W": W, "H": H, "waves": n, "span_us": float(end.max()),
       "dur_p50_p90_p99_p999_max": [round(float(x), 1) for x in q], "slow": []}
print(f"{name} {W}x{H}: {n} waves, span {end.max():.1f} us; wave us p50 %.1f p90 %.1f p99 %.1f p99.9 %.1f max %.1f" % tuple(q))
slow = np.argsort(-full)[:N]
for i in slow:
    blk = int(i)
    base = 16 | 32 | (blk << 16)
    row = {"tile": [blk % gx * 8, blk // gx * 8], "loaded": float(full[i]), "loaded_start": float(start[i])}
    row["alone"] = float(stamped(base)[0][i])
    row["primary"] = float(stamped(base | 2)[0][i])
    row["no_shadow"] = float(stamped(base | 1)[0][i])
    row["one_light"] = [float(stamped(base | 256 | (li << 9))[0][i]) for li in range(nl)]
    out["slow"].append(row)
    print(f"  tile {row['tile']}: loaded {row['loaded']:.1f} (start {row['loaded_start']:.1f}), alone {row['alone']:.1f}, "
          f"primary {row['primary']:.1f}, no shadow {row['no_shadow']:.1f}, one light "
          + " ".join(f"{x:.1f}" for x in row["one_light"]))
os.makedirs("gpurun_out", exist_ok=True)
Path(f"gpurun_out/tail_{name}_{W}x{H}.json").write_text(json.dumps(out, indent=1))
