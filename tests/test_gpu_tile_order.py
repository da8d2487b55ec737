"""Measured-cost tile order (KParams::hot, rrte_hip.hip plan_tile_order): a launch may dispatch its
tiles in any order -- the default measures every tile on a profiled launch and, once the durations
arrive, dispatches every tile slowest first.  Pixels are independent (raytracer.rs:57-60), so every
order must give the same bytes, linear floats and shadow-ray counts as image order.
RRTE_TILE_ORDER=2 forces a fixed scrambled permutation of the tiles on every launch (no profile), so
these tests run the list path on every kernel kind, mode and launch shape; RRTE_TILE_ORDER=0 is image
order.  The timed configuration itself -- the default policy with 4 frames in flight at 1080p and 4K,
after the measured list has landed -- is checked against the ORACLE."""
import ctypes as C
import os

import numpy as np
import pytest

import oracle
from rrte_amd import LoweredScene, abi, scenes
from rrte_amd.math import vec3
from rrte_amd.renderer import Context

import scenes_extra as se  # noqa: E402  (tests/ is on sys.path, as for test_gpu_parity)

pytestmark = pytest.mark.gpu


def _ctx(monkeypatch, order, jit, **env):
    if order is None:
        monkeypatch.delenv("RRTE_TILE_ORDER", raising=False)
    else:
        monkeypatch.setenv("RRTE_TILE_ORDER", order)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    ctx = Context(0, jit=jit)
    monkeypatch.delenv("RRTE_TILE_ORDER", raising=False)
    for k in env:
        monkeypatch.delenv(k)
    return ctx


def _render(ctx, sc, prm, rows=None):
    """(RGBA8 bytes, linear floats, shadow rays, hot tiles) of one frame through render_async."""
    import torch
    rows = prm.height if rows is None else rows
    p = abi.RenderParams.from_buffer_copy(prm)
    rgba = torch.full((rows * p.width,), -1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()  # the fill ran on torch's stream; the renders run on others
    ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(p), rgba.data_ptr(), None, None))
    ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
    s1 = ctx.stats()
    p.flags |= abi.FLAG_F32_LINEAR
    f32 = torch.zeros(rows * p.width * 4, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()  # the fill ran on torch's stream; the renders run on others
    ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(p), None, f32.data_ptr(), None))
    ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
    return (rgba.cpu().numpy().view(np.uint8), f32.cpu().numpy().view(np.uint32), s1.shadow_rays, s1.hot_tiles)


SCENES = dict(scenes.SCENES, **{"all-lights": se.all_lights_scene, "mixed": se.mixed_scene})
# (scene, W, H, mode, spp): odd sizes (a partial last slot row), every light kind, REFCOMPAT with
# samples and bounces, the deformer and mesh kernels
CASES = [("sdf-showcase", 320, 200, "lambert_shadow", 1), ("sdf-showcase", 162, 90, "lambert_shadow", 1),
         ("advanced-demo", 200, 120, "lambert_shadow", 1), ("all-lights", 120, 72, "lambert_shadow", 1),
         ("mixed", 96, 64, "lambert_shadow", 1), ("sdf-showcase", 96, 64, "refcompat", 3),
         ("deformation-stress", 64, 40, "lambert_shadow", 1), ("mesh-demo", 160, 96, "lambert_shadow", 1)]


@pytest.mark.parametrize("jit", [abi.JIT_OFF, abi.JIT_ON])
@pytest.mark.parametrize("name,w,h,mode,spp", CASES)
def test_fixed_tile_list_is_exact(name, w, h, mode, spp, jit, monkeypatch):
    objs, lights, cam, cfg = SCENES[name](w, h, mode=mode)
    if spp > 1:
        cfg.samples_per_pixel, cfg.max_depth, cfg.jitter = spp, 5, "random"
    sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
    ref = _ctx(monkeypatch, "0", jit)
    a = _render(ref, sc, prm)
    assert a[3] == 0
    tiles = ((w + 7) // 8) * ((h + 7) // 8)
    hot = _ctx(monkeypatch, "2", jit)
    b = _render(hot, sc, prm)
    assert b[3] == tiles
    assert np.array_equal(a[0], b[0]), (a[0] != b[0]).sum()
    assert np.array_equal(a[1], b[1])
    assert a[2] == b[2]
    hot.close()
    ref.close()


@pytest.mark.parametrize("nranks,rank", [(3, 1), (8, 0), (8, 7)])
def test_fixed_tile_list_on_band_mapped_ranks(nranks, rank, monkeypatch):
    """One rank's packed interleaved bands (RRTE_EMULATE_RANK): slots address the rank's local tile
    rows, the camera-tile mask maps them to image rows."""
    w, h, band = 256, 200, 16
    objs, lights, cam, cfg = scenes.sdf_showcase(w, h)
    cfg.band_rows = band
    sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
    lib = abi.load()
    rows = lib.rrte_hip_band_rows_for_rank_ex(h, band, nranks, rank, *abi.band_layout(sc.ref(), C.byref(prm), nranks))
    env = {"RRTE_EMULATE_RANK": f"{nranks}:{rank}"}
    ref = _ctx(monkeypatch, "0", abi.JIT_ON, **env)
    hot = _ctx(monkeypatch, "2", abi.JIT_ON, **env)
    a, b = _render(ref, sc, prm, rows), _render(hot, sc, prm, rows)
    assert b[3] == 32 * ((rows + 7) // 8)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2]
    ref.close()
    hot.close()


def test_measured_order(monkeypatch):
    """The default policy: the first launch of a shape is profiled, the durations come back
    asynchronously and a later launch dispatches every tile in measured-cost order; every frame on
    the way is identical to image order."""
    objs, lights, cam, cfg = scenes.sdf_showcase(640, 360)
    sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
    ref = _ctx(monkeypatch, "0", abi.JIT_ON)
    want = _render(ref, sc, prm)
    ref.close()
    ctx = _ctx(monkeypatch, None, abi.JIT_ON)
    seen = 0
    for _ in range(6):
        got = _render(ctx, sc, prm)
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1]) and got[2] == want[2]
        seen = max(seen, got[3])
    assert seen == 80 * 45  # one slot per tile
    ctx.close()


def test_fixed_tile_list_in_batched_gathers(monkeypatch):
    """Multi-frame launches of the batched gather path (blockIdx.y = frame): every frame's slots, 8
    frames per launch, a partial last batch."""
    import torch
    frames = []
    for i in range(11):
        objs, lights, cam, cfg = scenes.sdf_showcase(320, 200)
        cam.transform.position = vec3(0.7 * i, 8.0 - 0.3 * i, 20.0)
        cam.look_at((0, 2, 0))
        frames.append((LoweredScene(objs, lights, cam), cfg.lower()))
    ref = _ctx(monkeypatch, "0", abi.JIT_ON)
    want = []
    for sc, prm in frames:
        buf = np.zeros(prm.width * prm.height * 4, dtype=np.uint8)
        ref.check(ref.lib.rrte_hip_render(ref.h, sc.ref(), C.byref(prm), buf.ctypes.data_as(C.POINTER(C.c_uint8))))
        want.append(buf)
    ref.close()
    ctx = _ctx(monkeypatch, "2", abi.JIT_ON, RRTE_FORCE_GATHER="1")
    lib = ctx.lib
    uid = (C.c_uint8 * abi.UNIQUE_ID_BYTES)()
    ctx.check(lib.rrte_hip_comm_unique_id(uid))
    ctx.check(lib.rrte_hip_comm_init(ctx.h, 1, 0, uid))
    ctx.check(lib.rrte_hip_set_gather_batch(ctx.h, 8))
    streams = [torch.cuda.Stream() for _ in range(2)]
    outs = [torch.full((p.width * p.height,), -1, dtype=torch.int32, device="cuda") for _, p in frames]
    torch.cuda.synchronize()  # the fill ran on torch's stream; the renders run on others
    for i, ((sc, prm), o) in enumerate(zip(frames, outs)):
        ctx.check(lib.rrte_hip_render_gather_async(ctx.h, sc.ref(), C.byref(prm), 0, o.data_ptr(),
                                                    C.c_void_p(streams[i % 2].cuda_stream)))
    ctx.check(lib.rrte_hip_flush(ctx.h))
    ctx.check(lib.rrte_hip_synchronize(ctx.h))
    assert ctx.stats().hot_tiles == 40 * 25
    for i, o in enumerate(outs):
        got = o.cpu().numpy().view(np.uint8)
        assert np.array_equal(got, want[i]), f"frame {i}: {(got != want[i]).sum()} bytes differ"
    ctx.close()


def test_list_versions_recycle_in_flight(monkeypatch):
    """RRTE_TEST_RECYCLE=1: a new tile-list version per launch, so the pool of 16 versions wraps
    while frames are in flight on 4 streams; a version is only reused after the launches that read
    it have completed (no device synchronisation), and every frame stays exact."""
    import torch
    objs, lights, cam, cfg = scenes.sdf_showcase(320, 200)
    sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
    ref = _ctx(monkeypatch, "0", abi.JIT_ON)
    want = _render(ref, sc, prm)
    ref.close()
    ctx = _ctx(monkeypatch, "2", abi.JIT_ON, RRTE_TEST_RECYCLE="1")
    streams = [torch.cuda.Stream() for _ in range(4)]
    outs = [torch.full((320 * 200,), -1, dtype=torch.int32, device="cuda") for _ in range(4)]
    torch.cuda.synchronize()
    n = 40
    for i in range(n):
        ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(prm), outs[i % 4].data_ptr(), None,
                                                C.c_void_p(streams[i % 4].cuda_stream)))
    ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
    assert ctx.stats().hot_tiles == 40 * 25
    assert int(ctx.stats().shadow_rays) == n * int(want[2])
    for o in outs:
        assert np.array_equal(o.cpu().numpy().view(np.uint8), want[0])
    ctx.close()


def _threads():
    return int(os.environ.get("RRTE_ORACLE_THREADS", min(16, os.cpu_count() or 1)))


@pytest.mark.parametrize("w,h", [(1920, 1080), (3840, 2160)])
def test_timed_configuration_matches_oracle(w, h, monkeypatch):
    """the bench's own configuration -- default tile policy, 4 frames in flight on 4
    streams, scene-specialised kernel, RGBA8 frames -- run until the measured whole-frame order has
    landed (hot_tiles == tiles); then the last frames in flight are compared byte for byte with the
    ORACLE's frame and the shadow-ray count of every frame with the oracle's, and the same policy's
    linear floats bit for bit with the oracle's linear image."""
    import torch
    objs, lights, cam, cfg = scenes.sdf_showcase(w, h)
    sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
    want8, _, want_shadow = oracle.render(sc, prm, nthreads=_threads(), want_f32=False)
    _, want_lin, _ = oracle.render(sc, prm, nthreads=_threads(), linear=True)
    ctx = _ctx(monkeypatch, None, abi.JIT_ON)
    F = 4
    streams = [torch.cuda.Stream() for _ in range(F)]
    outs = [torch.full((w * h,), -1, dtype=torch.int32, device="cuda") for _ in range(F)]
    torch.cuda.synchronize()
    tiles = ((w + 7) // 8) * ((h + 7) // 8)
    go = lambda i: ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(prm), outs[i % F].data_ptr(),  # noqa: E731
                                                           None, C.c_void_p(streams[i % F].cuda_stream)))
    landed, i = False, 0
    for _ in range(40):  # rounds of F frames until the profile's list is in use
        for _ in range(F):
            go(i)
            i += 1
        landed = ctx.stats().hot_tiles == tiles
        if landed:
            break
        ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
    assert landed, "the measured tile order never landed"
    for _ in range(2 * F):  # frames in flight on the measured order
        go(i)
        i += 1
    assert ctx.stats().hot_tiles == tiles
    ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
    assert int(ctx.stats().shadow_rays) == 3 * F * want_shadow  # the landing round + 2 rounds, since the last sync
    for o in outs:
        got = o.cpu().numpy().view(np.uint8)
        d = np.abs(got.astype(np.int16) - want8.astype(np.int16))
        assert d.max() <= 1, f"u8 max diff {d.max()}"
        # glibc's powf and the device's differ by an ulp on a few inputs near byte boundaries (the
        # linear image is compared bit for bit below): 35 of 33 M bytes at 4K on the first GPU run
        assert (d != 0).sum() <= max(16, d.size // 100000), f"{int((d != 0).sum())} bytes differ (gamma powf ulps only)"
    # linear floats of the same policy (f32 output: the powf gamma path), frames in flight
    p = abi.RenderParams.from_buffer_copy(prm)
    p.flags |= abi.FLAG_F32_LINEAR
    f32s = [torch.zeros(w * h * 4, dtype=torch.float32, device="cuda") for _ in range(F)]
    torch.cuda.synchronize()
    for j in range(2 * F):
        ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(p), None, f32s[j % F].data_ptr(),
                                                C.c_void_p(streams[j % F].cuda_stream)))
    assert ctx.stats().hot_tiles == tiles
    ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
    assert int(ctx.stats().shadow_rays) == 2 * F * want_shadow
    for f in f32s:
        got = f.cpu().numpy().view(np.uint32)
        bad = (got != want_lin.view(np.uint32)).reshape(-1, 4).any(-1)
        assert not bad.any(), f"{int(bad.sum())} pixels differ from the oracle's linear image"
    ctx.close()
