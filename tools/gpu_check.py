"""Quick GPU-vs-oracle parity sweep over the BASELINE scenes (diagnostic tool).

Usage: python tools/gpu_check.py [W H]
"""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import oracle  # noqa: E402
from rrte_amd import LoweredScene, Raytracer, scenes  # noqa: E402

W, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (480, 270)
for name, fn in scenes.SCENES.items():
    for mode in ("refcompat", "lambert_shadow"):
        objs, lights, cam, cfg = fn(W, H, mode=mode)
        rt = Raytracer(cfg)
        t = time.time()
        g8, gf = rt.render_f32(objs, lights, [], cam)
        tg = time.time() - t
        st = rt.stats()
        t = time.time()
        r8, rf, rsh = oracle.render(LoweredScene(objs, lights, cam), cfg.lower(), nthreads=16)
        tc = time.time() - t
        d = gf.astype(np.float64) - rf
        rms = np.sqrt(np.mean(d ** 2))
        du8 = np.abs(g8.astype(np.int16) - r8.astype(np.int16))
        npix_diff = int((du8.reshape(-1, 4).max(1) > 0).sum())
        print(f"{name:22s} {mode:15s} rms={rms:.3e} maxabs={np.abs(d).max():.3e} u8max={du8.max()} "
              f"pixdiff={npix_diff} shadow gpu/ref={st.shadow_rays}/{rsh} kernel={st.kernel_ms:.3f}ms "
              f"gpu_call={tg*1e3:.1f}ms cpu={tc*1e3:.1f}ms", flush=True)
