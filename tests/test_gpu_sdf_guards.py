"""CSG early-outs on the GPU (sdf_guard.hip): renders with guards off (RRTE_CSG_GUARDS=0),
at the default policy and on every operand (=1) are bit-identical (linear image, shadow-ray count)
and match the oracle, for the generic and the scene-specialised kernels."""
import ctypes as C

import numpy as np
import pytest

import scenes_extra as se
from rrte_amd import Raytracer, abi, scenes
from test_gpu_parity import compare

pytestmark = pytest.mark.gpu


def _render(args, jit):
    objs, lights, cam, cfg = args
    rt = Raytracer(cfg, device=0, jit=jit)
    _, lin = rt.render_f32(objs, lights, [], cam, linear=True)
    return lin.view(np.uint32).copy(), int(rt.stats().shadow_rays)


@pytest.mark.parametrize("jit", [abi.JIT_OFF, abi.JIT_ON])
@pytest.mark.parametrize("case", ["deformation-stress", "random-csg-1", "random-csg-2", "sdf-showcase", "nan-left"])
def test_csg_guards_are_exact(case, jit, monkeypatch):
    if case == "deformation-stress":
        args = scenes.deformation_stress(384, 216)
    elif case == "sdf-showcase":
        args = scenes.sdf_showcase(320, 180)
    elif case == "nan-left":
        args = se.nan_left_operand_scene(320, 180)
    else:
        args = se.random_csg_scene(320, 180, "lambert_shadow", seed=int(case[-1]))
    out = {}
    for g in ("0", "2", "1"):
        monkeypatch.setenv("RRTE_CSG_GUARDS", g)
        out[g] = _render(args, jit)
    assert np.array_equal(out["0"][0], out["2"][0]) and out["0"][1] == out["2"][1]
    assert np.array_equal(out["0"][0], out["1"][0]) and out["0"][1] == out["1"][1]
    monkeypatch.setenv("RRTE_CSG_GUARDS", "1")
    compare(*args, jit=jit)


def test_random_csg_refcompat_matches_oracle():
    compare(*se.random_csg_scene(200, 120, "refcompat", seed=3), jit=abi.JIT_ON)
