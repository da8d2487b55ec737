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
    """Frame f of a value-only animation (rrte_amd.scenes.animate_values): every SDF leaf and smooth op
    moves/changes, every light moves and dims, every material changes colour -- the topology stays."""
    scenes.animate_values(sc, f)


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


@pytest.mark.parametrize("jit_topo", ["1", "2"])
def test_animation_in_flight_is_exact(jit_topo, monkeypatch):
    """a scene change per frame with frames in flight -- 5 animation frames issued on 4
    streams without a synchronisation between them (each scene uploaded into the next version of the
    scene ring while the earlier frames still read theirs) -- every frame's linear image bit-exact
    against the oracle and the shadow-ray total exact; topology kernel forced (1) or adaptive (2)."""
    import torch
    monkeypatch.setenv("RRTE_JIT_TOPO", jit_topo)
    w, h = 160, 96
    objs, lights, cam, cfg = scenes.sdf_showcase(w, h)
    prm = cfg.lower()
    prm.flags |= abi.FLAG_F32_LINEAR
    frames = [_animate_copy(objs, lights, cam, f) for f in range(5)]
    want = [oracle.render(sc, prm, nthreads=16, linear=True) for sc in frames]
    ctx = Context(0, jit=abi.JIT_ON)
    streams = [torch.cuda.Stream() for _ in range(4)]
    outs = [torch.zeros(w * h * 4, dtype=torch.float32, device="cuda") for _ in frames]
    torch.cuda.synchronize()
    for rnd in range(2):  # round 0 compiles; round 1 runs the animation on warm kernels
        for i, sc in enumerate(frames):
            ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(prm), None, outs[i].data_ptr(),
                                                    C.c_void_p(streams[i % 4].cuda_stream)))
        ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
        assert int(ctx.stats().shadow_rays) == sum(wsh for _, _, wsh in want)
        for i, o in enumerate(outs):
            got = o.cpu().numpy().view(np.uint32)
            assert np.array_equal(got, want[i][1].view(np.uint32)), f"round {rnd} frame {i}"
    assert ctx.stats().jit_active == 2
    ctx.close()


def _animate_copy(objs, lights, cam, f):
    sc = LoweredScene(objs, lights, cam)
    _animate(sc, f)
    return sc
