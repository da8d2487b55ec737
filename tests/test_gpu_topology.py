"""Topology-specialised kernels (jit.hip JitTopo, ray_kernels.hpp TopoPrim / TopoNode / TopoLight;
VERDICT r02 #8).  A topology kernel compiles in only the scene's structure and reads every value --
SDF leaf centres and sizes, smooth-op k, CSG-guard spheres, light positions and intensities, material
colours -- from the uploaded records, so an animated scene compiles ONE kernel instead of one per
frame.  It must reproduce the oracle exactly like the full and generic kernels: bit-identical linear
image and identical shadow-ray count on every frame."""
import ctypes as C

import numpy as np
import pytest

import oracle
from rrte_amd import LoweredScene, abi, scenes
from rrte_amd.renderer import Context
from test_gpu_parity import SCENE_CASES, compare

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,mode", SCENE_CASES)
def test_topology_kernels_match_oracle(name, mode, monkeypatch):
    monkeypatch.setenv("RRTE_JIT_TOPO", "1")
    compare(*scenes.SCENES[name](160, 90, mode=mode), jit=abi.JIT_ON, expect_jit=2)


def _animate(sc: LoweredScene, f: int):
    """Frame f of a value-only animation: every SDF leaf and smooth op moves/changes, every light moves
    and dims, every material changes colour -- the topology stays."""
    for i in range(sc.ir.num_sdf_nodes):
        n = sc.nodes[i]
        if n.op < 32:  # leaves: centre x, z
            n.f[0] = np.float32(n.f[0] + 0.15 * f)
            n.f[2] = np.float32(n.f[2] - 0.1 * f)
        elif 35 <= n.op <= 37:  # smooth ops: k
            n.f[0] = np.float32(n.f[0] * (1.0 + 0.2 * f))
    for i in range(sc.ir.num_lights):
        L = sc.lights[i]
        L.position[1] = np.float32(L.position[1] - 0.7 * f)
        L.intensity = np.float32(L.intensity * (1.0 - 0.05 * f))
    for i in range(sc.ir.num_materials):
        m = sc.mats[i]
        m.albedo[0] = np.float32(min(1.0, m.albedo[0] + 0.05 * f))


def _render(ctx, sc, prm, w, h):
    out8 = np.empty(w * h * 4, np.uint8)
    lin = np.empty(w * h * 4, np.float32)
    ctx.check(ctx.lib.rrte_hip_render_f32(ctx.h, sc.ref(), C.byref(prm), out8.ctypes.data, lin.ctypes.data))
    return lin, ctx.stats()


@pytest.mark.parametrize("name", ["sdf-showcase", "deformation-stress"])
def test_animation_compiles_one_topology_kernel(name, tmp_path, monkeypatch):
    """Adaptive policy (default): frame 0 gets the full kernel; every later frame changes values only,
    so frames 1.. run ONE topology kernel (one more code object, not one per frame); once the scene
    stops changing for 16 frames the full kernel of the final scene takes over.  Every frame exact."""
    monkeypatch.setenv("RRTE_JIT_CACHE_DIR", str(tmp_path))
    monkeypatch.delenv("RRTE_JIT_TOPO", raising=False)
    w, h = 128, 72
    objs, lights, cam, cfg = scenes.SCENES[name](w, h)
    prm = cfg.lower()
    prm.flags |= abi.FLAG_F32_LINEAR
    ctx = Context(0, jit=abi.JIT_ON)
    for f in range(5):
        sc = LoweredScene(objs, lights, cam)
        _animate(sc, f)
        lin, st = _render(ctx, sc, prm, w, h)
        _, want, wsh = oracle.render(sc, prm, nthreads=16, linear=True)
        assert np.array_equal(lin.view(np.uint32), want.view(np.uint32)), f"frame {f}"
        assert int(st.shadow_rays) == wsh, f
        assert st.jit_active == (1 if f == 0 else 2), (f, st.jit_active)
        assert len(list(tmp_path.glob("*.hsaco"))) == (1 if f == 0 else 2), f
    for k in range(17):  # the last frame's scene, unchanged
        lin, st = _render(ctx, sc, prm, w, h)
    assert st.jit_active == 1
    assert np.array_equal(lin.view(np.uint32), want.view(np.uint32))
    assert len(list(tmp_path.glob("*.hsaco"))) == 3
    ctx.close()


def test_topology_change_leaves_the_topology_kernel(monkeypatch):
    """A structural change (another object kind) is not a value edit: the next frame gets a full
    kernel again, and stays exact."""
    monkeypatch.delenv("RRTE_JIT_TOPO", raising=False)
    w, h = 96, 54
    objs, lights, cam, cfg = scenes.sdf_showcase(w, h)
    prm = cfg.lower()
    prm.flags |= abi.FLAG_F32_LINEAR
    ctx = Context(0, jit=abi.JIT_ON)
    for f, expect in [(0, 1), (1, 2)]:
        sc = LoweredScene(objs, lights, cam)
        _animate(sc, f)
        _, st = _render(ctx, sc, prm, w, h)
        assert st.jit_active == expect
    objs2, lights2, cam2, _ = scenes.sdf_showcase_literal(w, h)
    sc = LoweredScene(objs2, lights2, cam2)
    lin, st = _render(ctx, sc, prm, w, h)
    _, want, wsh = oracle.render(sc, prm, nthreads=16, linear=True)
    assert st.jit_active == 1
    assert np.array_equal(lin.view(np.uint32), want.view(np.uint32)) and int(st.shadow_rays) == wsh
    ctx.close()
