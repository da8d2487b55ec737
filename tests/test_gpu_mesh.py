"""Triangle meshes on the GPU (BVH traversal) against the oracle's linear triangle scan and against
the same geometry as individual Triangle objects."""
import ctypes as C

import numpy as np
import pytest

import oracle
from rrte_amd import (Color, LambertianMaterial, LoweredScene, Mesh, PointLight, Raytracer, Sphere, abi,
                      scenes)
from rrte_amd.mesh import icosphere, torus
from test_gpu_parity import compare
from test_mesh import _cam, _cfg

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["refcompat", "lambert_shadow"])
@pytest.mark.parametrize("jit", [abi.JIT_OFF, abi.JIT_ON])
def test_mesh_demo_matches_oracle(mode, jit):
    objs, lights, cam, cfg = scenes.mesh_demo(320, 180, mode=mode, detail=0.3)
    info = compare(objs, lights, cam, cfg, jit=jit)
    print(info)


@pytest.mark.parametrize("jit", [abi.JIT_OFF, abi.JIT_ON])
def test_mesh_demo_full_detail(jit):
    """~56 K triangles (BVH depth ~16) at 240x135 against the oracle's linear scan."""
    compare(*scenes.mesh_demo(240, 135), jit=jit)


@pytest.mark.parametrize("jit", [abi.JIT_OFF, abi.JIT_ON])
def test_mesh_equals_its_triangles_on_the_gpu(jit):
    mat = LambertianMaterial(Color.rgb(0.7, 0.5, 0.3))
    meshes = [icosphere((-1.2, 1.0, 0.0), 0.9, 2, mat), torus((1.3, 1.0, 0.0), 0.8, 0.3, 16, 8, mat)]
    ground = Sphere((0, -1000, 0), 1000, LambertianMaterial(Color.rgb(0.3, 0.3, 0.3)))
    lights = [PointLight((3, 6, 4), Color.rgb(1, 1, 1), 4.0)]
    w, h = 200, 120
    cfg = _cfg(w, h, "lambert_shadow")
    out = []
    for objs in ([ground] + meshes, [ground] + [t for m in meshes for t in m.triangles()]):
        rt = Raytracer(cfg, device=0, jit=jit)
        _, lin = rt.render_f32(objs, lights, [], _cam(w, h), linear=True)
        out.append((lin.view(np.uint32).copy(), int(rt.stats().shadow_rays)))
    assert np.array_equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1]


def test_mesh_edge_cases():
    mat = LambertianMaterial(Color.rgb(0.5, 0.5, 0.5))
    w, h = 64, 48
    cfg = _cfg(w, h, "lambert_shadow")
    lights = [PointLight((2, 5, 3), Color.rgb(1, 1, 1), 3.0)]
    empty = Mesh(np.zeros((0, 3)), np.zeros((0, 3)), np.zeros((0, 3)), mat)
    flat = Mesh([(0, 1, 0), (1, 1, 0), (2, 1, 0)], [(0, 1, 2)], [(0, 1, 0)] * 3, mat)  # degenerate triangle
    one = Mesh([(-1, 0.5, -1), (1, 0.5, -1), (0, 2.0, 0.5)], [(0, 1, 2)], None, mat)
    for objs in ([empty], [flat], [one], [empty, one, flat]):
        compare(objs, lights, _cam(w, h), cfg)


def test_invalid_mesh_input_fails_loudly():
    m = icosphere((0, 0, 0), 1.0, 0)
    sc = LoweredScene([m], [], _cam(8, 8))
    sc._mesh_idx[4] = 999
    from rrte_amd.renderer import Context
    ctx = Context(0)
    buf = np.zeros(8 * 8 * 4, dtype=np.uint8)
    prm = _cfg(8, 8, "lambert_shadow").lower()
    st = ctx.lib.rrte_hip_render(ctx.h, sc.ref(), C.byref(prm), buf.ctypes.data_as(C.POINTER(C.c_uint8)))
    assert st == abi.RRTE_INVALID_ARG
    ctx.close()
