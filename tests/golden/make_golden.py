"""Regenerate tests/golden/*.npz from the CPU oracle (run from the repo root):

    python tests/golden/make_golden.py [--force]

The reference ships no golden images; these fixtures freeze the
oracle's output for every BASELINE scene and both shading modes at small sizes,
including the build-defined SDF/CSG/deformer scenes.  Each fixture holds the
RGBA8 image, the SHA-256 of the linear (pre-gamma) f32 buffer and the
shadow-ray count.
"""
import hashlib
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import oracle  # noqa: E402
from rrte_amd import LoweredScene, scenes  # noqa: E402

CASES = [(name, mode, 64, 36) for name in scenes.SCENES for mode in ("refcompat", "lambert_shadow")]


def render_case(name, mode, w, h):
    objs, lights, cam, cfg = scenes.SCENES[name](w, h, mode=mode)
    sc = LoweredScene(objs, lights, cam)
    rgba8, _, shadow = oracle.render(sc, cfg.lower(), nthreads=4, want_f32=False)
    _, lin, _ = oracle.render(sc, cfg.lower(), nthreads=4, linear=True)
    return rgba8.reshape(h, w, 4), hashlib.sha256(lin.tobytes()).hexdigest(), shadow


def main():
    out = Path(__file__).resolve().parent
    force = "--force" in sys.argv  # default: only write fixtures that do not exist yet
    for name, mode, w, h in CASES:
        if not force and (out / f"{name}_{mode}_{w}x{h}.npz").exists():
            continue
        img, lin_hash, shadow = render_case(name, mode, w, h)
        np.savez_compressed(out / f"{name}_{mode}_{w}x{h}.npz", rgba8=img, linear_sha256=np.array(lin_hash),
                            shadow_rays=np.array(shadow, np.int64))
        print(name, mode, lin_hash[:12], shadow)


if __name__ == "__main__":
    main()
