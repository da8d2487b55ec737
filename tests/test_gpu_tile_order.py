"""Hot-first tile order and split hot tiles (KParams::hot, rrte_hip.hip plan_tile_order): a launch
may dispatch a list of tiles first and skip them in image order, and a hot tile may be rendered as
one workgroup per shadow-casting light, the last of which sums the lights' terms in light order.
Pixels are independent (raytracer.rs:57-60) and adding a light that contributes nothing as +0 is
exact, so every order and split must give the same bytes, linear floats and shadow-ray counts as
image order.  RRTE_TILE_ORDER=2 forces a fixed list of tiles spread over the frame (first and last
tile included, every other one split when RRTE_TILE_SPLIT=1 and splitting applies) on every launch,
so these tests run the hot slots, split parts, the partial hot row and the image-order skip on every
kernel kind, mode and launch shape; RRTE_TILE_ORDER=0 is image order.  The default measures the tiles
on a profiled launch and, once the durations arrive, dispatches every tile slowest first
(RRTE_TILE_ORDER=3; =1 only the 1024 slowest first; no splits by default: measured slower)."""
import ctypes as C

import numpy as np
import pytest

from rrte_amd import LoweredScene, abi, scenes
from rrte_amd.math import vec3
from rrte_amd.renderer import Context

import scenes_extra as se  # noqa: E402  (tests/ is on sys.path, as for test_gpu_parity)

pytestmark = pytest.mark.gpu


def _ctx(monkeypatch, order, jit, **env):
    monkeypatch.setenv("RRTE_TILE_ORDER", order)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    ctx = Context(0, jit=jit)
    monkeypatch.delenv("RRTE_TILE_ORDER")
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


MAX_SLOTS = 1024  # device_scene.hpp kMaxHotTiles


def _fixed_slots(tiles, parts):
    """Slots of RRTE_TILE_ORDER=2's list (rrte_hip.hip compose_slots): m tiles, every other one split."""
    m = min(tiles, MAX_SLOTS)
    while m > 1 and (m + 1) // 2 * parts + m // 2 > MAX_SLOTS:
        m -= 1
    return (m + 1) // 2 * parts + m // 2


SCENES = dict(scenes.SCENES, **{"all-lights": se.all_lights_scene, "mixed": se.mixed_scene})
# (scene, W, H, mode, spp): 3 lights (3 parts), 5 point lights (4 parts, round robin), point +
# directional + spot + ambient (3 parts, ambient in part 0), odd sizes, REFCOMPAT (never split)
CASES = [("sdf-showcase", 320, 200, "lambert_shadow", 1), ("sdf-showcase", 162, 90, "lambert_shadow", 1),
         ("advanced-demo", 200, 120, "lambert_shadow", 1), ("all-lights", 120, 72, "lambert_shadow", 1),
         ("mixed", 96, 64, "lambert_shadow", 1), ("sdf-showcase", 96, 64, "refcompat", 3),
         ("deformation-stress", 64, 40, "lambert_shadow", 1), ("mesh-demo", 160, 96, "lambert_shadow", 1)]


@pytest.mark.parametrize("jit", [abi.JIT_OFF, abi.JIT_ON])
@pytest.mark.parametrize("name,w,h,mode,spp", CASES)
def test_fixed_hot_list_is_exact(name, w, h, mode, spp, jit, monkeypatch):
    objs, lights, cam, cfg = SCENES[name](w, h, mode=mode)
    if spp > 1:
        cfg.samples_per_pixel, cfg.max_depth, cfg.jitter = spp, 5, "random"
    sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
    ref = _ctx(monkeypatch, "0", jit)
    a = _render(ref, sc, prm)
    assert a[3] == 0
    tiles = ((w + 7) // 8) * ((h + 7) // 8)
    casters = sum(1 for lt in sc.lights[:sc.ir.num_lights] if lt.kind != abi.LIGHT_AMBIENT)
    for split in ("0", "1"):
        hot = _ctx(monkeypatch, "2", jit, RRTE_TILE_SPLIT=split)
        b = _render(hot, sc, prm)
        parts = min(casters, 4) if split == "1" and mode == "lambert_shadow" and spp == 1 else 1
        assert b[3] == _fixed_slots(tiles, parts if parts > 1 else 1)
        assert np.array_equal(a[0], b[0]), (split, (a[0] != b[0]).sum())
        assert np.array_equal(a[1], b[1]), split
        assert a[2] == b[2], split
        hot.close()
    ref.close()


@pytest.mark.parametrize("nranks,rank", [(3, 1), (8, 0), (8, 7)])
def test_fixed_hot_list_on_band_mapped_ranks(nranks, rank, monkeypatch):
    """One rank's packed interleaved bands (RRTE_EMULATE_RANK): hot tiles address the rank's local
    tile rows, the camera-tile mask maps them to image rows."""
    w, h, band = 256, 200, 16
    objs, lights, cam, cfg = scenes.sdf_showcase(w, h)
    cfg.band_rows = band
    sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
    rows = abi.load().rrte_hip_band_rows_for_rank(h, band, nranks, rank)
    env = {"RRTE_EMULATE_RANK": f"{nranks}:{rank}"}
    ref = _ctx(monkeypatch, "0", abi.JIT_ON, **env)
    hot = _ctx(monkeypatch, "2", abi.JIT_ON, **env)
    a, b = _render(ref, sc, prm, rows), _render(hot, sc, prm, rows)
    assert b[3] > 0
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2]
    ref.close()
    hot.close()


def test_fixed_hot_list_at_4k(monkeypatch):
    """BASELINE configs[3]'s size: 480 x 270 tiles (270 tile rows: the row bitmap's upper words) and
    16x16 camera-culling blocks."""
    objs, lights, cam, cfg = scenes.sdf_showcase(3840, 2160)
    sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
    ref = _ctx(monkeypatch, "0", abi.JIT_ON)
    hot = _ctx(monkeypatch, "2", abi.JIT_ON, RRTE_TILE_SPLIT="1")
    a, b = _render(ref, sc, prm), _render(hot, sc, prm)
    assert b[3] == _fixed_slots(480 * 270, 3)  # 3 lights: 256 split tiles of 3 parts + 256 whole ones
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2]
    ref.close()
    hot.close()


def test_measured_hot_list(monkeypatch):
    """The default policy: the first launch of a shape is profiled, the durations come back
    asynchronously and a later launch dispatches every tile in measured-cost order; every frame on
    the way is identical to image order."""
    objs, lights, cam, cfg = scenes.sdf_showcase(640, 360)
    sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
    ref = _ctx(monkeypatch, "0", abi.JIT_ON)
    want = _render(ref, sc, prm)
    ref.close()
    monkeypatch.delenv("RRTE_TILE_ORDER", raising=False)
    ctx = Context(0, jit=abi.JIT_ON)
    seen = 0
    for _ in range(6):
        got = _render(ctx, sc, prm)
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1]) and got[2] == want[2]
        seen = max(seen, got[3])
    assert seen == 80 * 45  # the default whole-frame order: one slot per tile
    ctx.close()


def test_fixed_hot_list_in_batched_gathers(monkeypatch):
    """Multi-frame launches of the batched gather path (blockIdx.y = frame): every frame's hot tiles
    first, 8 frames per launch, a partial last batch."""
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
    ctx = _ctx(monkeypatch, "2", abi.JIT_ON, RRTE_FORCE_GATHER="1", RRTE_TILE_SPLIT="1")
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
    assert ctx.stats().hot_tiles == _fixed_slots(40 * 25, 3)  # per launch: split tiles x 3 parts + whole tiles
    for i, o in enumerate(outs):
        got = o.cpu().numpy().view(np.uint8)
        assert np.array_equal(got, want[i]), f"frame {i}: {(got != want[i]).sum()} bytes differ"
    ctx.close()


@pytest.mark.parametrize("split", ["0", "1"])
def test_measured_lpt_order(split, monkeypatch):
    """RRTE_TILE_ORDER=3: after the profile every tile of the frame is dispatched in measured-cost
    order (no image-order rows), the slowest ones optionally split; identical to image order."""
    objs, lights, cam, cfg = scenes.sdf_showcase(480, 272)
    sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
    ref = _ctx(monkeypatch, "0", abi.JIT_ON)
    want = _render(ref, sc, prm)
    ref.close()
    ctx = _ctx(monkeypatch, "3", abi.JIT_ON, RRTE_TILE_SPLIT=split)
    tiles = 60 * 34
    seen = 0
    for _ in range(5):
        got = _render(ctx, sc, prm)
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1]) and got[2] == want[2]
        seen = max(seen, got[3])
    assert seen >= tiles  # every tile has a slot (split parts add more)
    ctx.close()
