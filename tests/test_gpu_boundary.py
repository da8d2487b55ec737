"""The blocking drop-in entry point (rrte_hip_render: Raytracer::render's signature, raytracer.rs:45-89,
host RGBA8 out, D2H included): its bytes must equal the device-buffer path's (rrte_hip_render_async +
a copy) and the oracle's, for sizes whose rows are and are not a multiple of the 8-row tiles, at 4K,
into reused and fresh buffers, frame after frame, on the specialised and the generic kernels."""
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
def test_blocking_render_matches_device_path(name, w, h):
    import torch
    objs, lights, cam, cfg = scenes.SCENES[name](w, h)
    sc = LoweredScene(objs, lights, cam)
    prm = cfg.lower()
    ctx = Context(0, jit=abi.JIT_ON)
    dev = torch.zeros(w * h, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()  # the fill ran on torch's stream; the renders run on others
    ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(prm), dev.data_ptr(), None, None))
    ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
    want = dev.cpu().numpy().view(np.uint8)
    reused = np.full(w * h * 4, 7, np.uint8)
    for f in range(3):  # reused buffer, frame after frame
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


def test_blocking_render_generic_kernel_and_size_changes():
    """The generic kernel's blocking frames; smaller and larger frames on one context."""
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


@pytest.mark.parametrize("chunks", ["1", "3", "8"])
@pytest.mark.parametrize("w,h", [(1920, 1080), (333, 97), (200, 40)])
def test_chunked_blocking_render_is_exact(chunks, w, h, monkeypatch):
    """rrte_hip_render renders row chunks on their own streams, each chunk's D2H starting when the
    chunk is done (RRTE_BND_CHUNKS; rrte_hip.hip render_chunked): every chunk count, sizes whose
    chunks end mid-tile or leave a short last chunk, and enough frames for each chunk's measured tile
    order to land (its own profile slot) -- always the device path's bytes and shadow-ray count."""
    import torch
    objs, lights, cam, cfg = scenes.sdf_showcase(w, h)
    sc = LoweredScene(objs, lights, cam)
    prm = cfg.lower()
    ref = Context(0, jit=abi.JIT_ON)
    dev = torch.zeros(w * h, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ref.check(ref.lib.rrte_hip_render_async(ref.h, sc.ref(), C.byref(prm), dev.data_ptr(), None, None))
    ref.check(ref.lib.rrte_hip_synchronize(ref.h))
    want, want_shadow = dev.cpu().numpy().view(np.uint8), int(ref.stats().shadow_rays)
    ref.close()
    monkeypatch.setenv("RRTE_BND_CHUNKS", chunks)
    ctx = Context(0, jit=abi.JIT_ON)
    buf = np.full(w * h * 4, 7, np.uint8)
    for f in range(6):
        got = _blocking(ctx, sc, prm, buf)
        assert np.array_equal(got, want), f"frame {f}: {int((got != want).sum())} bytes differ"
        assert int(ctx.stats().shadow_rays) == want_shadow
    ctx.close()


@pytest.mark.parametrize("name,w,h", [("sdf-showcase", 1920, 1080), ("sdf-showcase", 333, 97),
                                      ("mesh-demo", 200, 120)])
def test_pinned_buffers_are_written_directly(name, w, h):
    """A registered buffer (rrte_hip_host_register, pinned once) and a caller-pinned buffer (torch
    pin_memory: hipHostMalloc) take the zero-copy route -- the kernel stores the frame into host memory
    -- and must hold exactly the copy path's bytes, frame after frame; unregistering is checked."""
    import torch
    objs, lights, cam, cfg = scenes.SCENES[name](w, h)
    sc = LoweredScene(objs, lights, cam)
    prm = cfg.lower()
    ctx = Context(0, jit=abi.JIT_ON)
    want = _blocking(ctx, sc, prm, np.zeros(w * h * 4, np.uint8)).copy()
    reg = np.full(w * h * 4 + 64, 7, np.uint8)[16:16 + w * h * 4]  # (not page aligned)
    ctx.check(ctx.lib.rrte_hip_host_register(ctx.h, reg.ctypes.data, reg.nbytes))
    for f in range(3):
        reg[:] = 7
        got = _blocking(ctx, sc, prm, reg)
        assert np.array_equal(got, want), f"registered, frame {f}: {int((got != want).sum())} bytes differ"
    ctx.check(ctx.lib.rrte_hip_host_unregister(ctx.h, reg.ctypes.data))
    assert ctx.lib.rrte_hip_host_unregister(ctx.h, reg.ctypes.data) == abi.RRTE_INVALID_ARG
    reg[:] = 7
    assert np.array_equal(_blocking(ctx, sc, prm, reg), want)  # pageable again: the copy path
    pinned = torch.full((w * h * 4,), 7, dtype=torch.uint8).pin_memory()
    for f in range(2):
        ctx.check(ctx.lib.rrte_hip_render(ctx.h, sc.ref(), C.byref(prm),
                                          C.cast(pinned.data_ptr(), C.POINTER(C.c_uint8))))
        got = pinned.numpy()
        assert np.array_equal(got, want), f"pinned, frame {f}: {int((got != want).sum())} bytes differ"
    ctx.close()


@pytest.mark.parametrize("jit", [abi.JIT_ON, abi.JIT_OFF])
def test_engine_loop_render_into_is_the_blocking_frame(jit):
    """Engine::render_frame's loop (rust/patches/0002, Raytracer::render_into in the Python mirror):
    one buffer reused every frame, pinned once through the C ABI (rrte_hip_host_register) so the
    kernel stores into it; every frame must be rrte_hip_render's bytes into a pageable buffer; a
    second buffer (a resized engine) unpins the first and pins itself."""
    from rrte_amd import Raytracer
    objs, lights, cam, cfg = scenes.sdf_showcase(640, 360)
    rt = Raytracer(cfg, device=0, jit=jit)
    want = rt.render(objs, lights, [], cam)  # pageable copy path
    buf = np.full(640 * 360 * 4, 7, np.uint8)
    for f in range(4):
        buf[:] = 7
        rt.render_into(objs, lights, [], cam, buf)
        assert np.array_equal(buf, want), f"frame {f}"
    assert rt._pinned == (buf.ctypes.data, buf.nbytes)
    buf2 = np.zeros_like(buf)
    rt.render_into(objs, lights, [], cam, buf2)
    assert np.array_equal(buf2, want) and rt._pinned == (buf2.ctypes.data, buf2.nbytes)
    ctx = rt.ctx
    assert ctx.lib.rrte_hip_host_unregister(ctx.h, buf.ctypes.data) == abi.RRTE_INVALID_ARG  # (unpinned)
    ctx.close()
