"""The blocking drop-in entry point (rrte_hip_render: Raytracer::render's signature, raytracer.rs:45-89,
host RGBA8 out) with its pipelined host copy: the render counts finished workgroups per row band, a copy
kernel running beside it moves each finished band into pinned host memory and flags it, host threads
copy flagged bands into the caller's buffer (rrte_hip.hip band_copy_kernel / pipe_copy).  Its bytes
must equal the plain path's (RRTE_BOUNDARY_PIPE=0: render, then one hipMemcpy) and the oracle's, for
sizes whose rows are and are not a multiple of the 8-row tiles and 32-row bands, at 4K (the band cap),
into reused and fresh buffers, frame after frame."""
import ctypes as C

import numpy as np
import pytest

import oracle
from rrte_amd import LoweredScene, abi, scenes
from rrte_amd.renderer import Context

pytestmark = pytest.mark.gpu


def _blocking(ctx, sc, prm, out):
    ctx.check(ctx.lib.rrte_hip_render(ctx.h, sc.ref(), C.byref(prm), out.ctypes.data_as(C.POINTER(C.c_uint8))))
    return out


@pytest.mark.parametrize("name,w,h", [("sdf-showcase", 1920, 1080), ("sdf-showcase", 333, 97),
                                      ("sdf-showcase", 64, 7), ("basic-demo", 640, 480),
                                      ("sdf-showcase", 3840, 2160), ("mesh-demo", 200, 120)])
def test_pipelined_blocking_render_matches_plain_path(name, w, h, monkeypatch):
    objs, lights, cam, cfg = scenes.SCENES[name](w, h)
    sc = LoweredScene(objs, lights, cam)
    prm = cfg.lower()
    monkeypatch.setenv("RRTE_BOUNDARY_PIPE", "0")
    plain = Context(0, jit=abi.JIT_ON)
    want = _blocking(plain, sc, prm, np.zeros(w * h * 4, np.uint8))
    plain.close()
    monkeypatch.setenv("RRTE_BOUNDARY_PIPE", "1")
    ctx = Context(0, jit=abi.JIT_ON)
    reused = np.full(w * h * 4, 7, np.uint8)
    for f in range(3):  # reused buffer, frame after frame (flag generations)
        got = _blocking(ctx, sc, prm, reused)
        assert np.array_equal(got, want), f"frame {f}: {int((got != want).sum())} bytes differ"
    fresh = _blocking(ctx, sc, prm, np.zeros(w * h * 4, np.uint8))
    assert np.array_equal(fresh, want)
    assert ctx.stats().primary_rays == w * h
    if w * h <= 400 * 120:
        r8, _, rsh = oracle.render(sc, prm, nthreads=16)
        assert np.abs(want.astype(int) - r8.astype(int)).max() <= 1
        assert int(ctx.stats().shadow_rays) == rsh
    ctx.close()


def test_pipelined_blocking_render_generic_kernel_and_size_changes(monkeypatch):
    """The generic kernel counts bands too; a smaller and a larger frame on one context reuse / regrow
    the stage and the band flags."""
    monkeypatch.setenv("RRTE_BOUNDARY_PIPE", "1")
    ctx = Context(0, jit=abi.JIT_OFF)
    for w, h in [(320, 180), (96, 40), (1280, 720), (320, 180)]:
        objs, lights, cam, cfg = scenes.sdf_showcase(w, h)
        sc = LoweredScene(objs, lights, cam)
        prm = cfg.lower()
        got = _blocking(ctx, sc, prm, np.zeros(w * h * 4, np.uint8))
        r8, _, rsh = oracle.render(sc, prm, nthreads=16)
        assert np.abs(got.astype(int) - r8.astype(int)).max() <= 1, (w, h)
        assert int(ctx.stats().shadow_rays) == rsh
    ctx.close()
