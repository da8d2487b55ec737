"""GPU parity: librrte_hip.so (HIP kernels on the MI355X, called through the C ABI) against
the CPU oracle on identical scenes.  Tolerance (north_star): per-channel RMS <= 1e-4 on the
post-gamma/post-clamp float image; additionally u8 max |diff| <= 1, identical shadow-ray
counts, and the pre-gamma linear image bit-exact (the device reproduces the reference's f32
arithmetic op for op; only powf in the gamma step may differ by an ulp)."""
import ctypes as C
import hashlib
import sys
from pathlib import Path

import numpy as np
import pytest

import oracle
import scenes_extra as se
from rrte_amd import LoweredScene, Raytracer, RaytracerConfig, abi, scenes
from rrte_amd.renderer import Context

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-4


def compare(objs, lights, cam, cfg, linear_exact=True, threads=16, jit=abi.JIT_OFF, expect_jit=None):
    rt = Raytracer(cfg, device=0, jit=jit)
    g8, gf = rt.render_f32(objs, lights, [], cam)
    st = rt.stats()
    _, glin = rt.render_f32(objs, lights, [], cam, linear=True)
    sc = LoweredScene(objs, lights, cam)
    r8, rf, rsh = oracle.render(sc, cfg.lower(), nthreads=threads)
    _, rlin, _ = oracle.render(sc, cfg.lower(), nthreads=threads, linear=True)
    d = gf.astype(np.float64) - rf.astype(np.float64)
    both_nan = np.isnan(gf) & np.isnan(rf)
    d[both_nan] = 0.0
    rms = float(np.sqrt(np.mean(d ** 2)))
    u8 = int(np.abs(g8.astype(np.int16) - r8.astype(np.int16)).max())
    info = dict(rms=rms, u8=u8, shadow=(int(st.shadow_rays), rsh), kernel_ms=st.kernel_ms,
                diff_pixels=int((np.abs(g8.astype(np.int16) - r8.astype(np.int16)).reshape(-1, 4).max(1) > 0).sum()))
    assert rms <= RMS_TOL, info
    assert u8 <= 1, info
    assert int(st.shadow_rays) == rsh, info
    assert st.primary_rays == cfg.width * cfg.height * cfg.samples_per_pixel
    if expect_jit is None:
        expect_jit = 1 if jit == abi.JIT_ON else 0
    assert st.jit_active == expect_jit, "unexpected kernel path"
    if linear_exact:
        assert np.array_equal(glin.view(np.uint32), rlin.view(np.uint32)), info
    return info


SCENE_CASES = [(n, m) for n in scenes.SCENES for m in ("refcompat", "lambert_shadow")]


@pytest.mark.parametrize("name,mode", SCENE_CASES)
def test_baseline_scenes_160x90(name, mode):
    compare(*scenes.SCENES[name](160, 90, mode=mode))


@pytest.mark.parametrize("name,mode,w,h", [c for c in __import__("test_golden").make_golden.CASES])
def test_golden_fixtures_on_gpu(name, mode, w, h):
    fx = np.load(Path(__file__).parent / "golden" / f"{name}_{mode}_{w}x{h}.npz")
    objs, lights, cam, cfg = scenes.SCENES[name](w, h, mode=mode)
    rt = Raytracer(cfg, device=0)
    g8 = rt.render(objs, lights, [], cam)
    assert int(rt.stats().shadow_rays) == int(fx["shadow_rays"])
    assert np.abs(g8.reshape(h, w, 4).astype(int) - fx["rgba8"].astype(int)).max() <= 1
    _, lin = rt.render_f32(objs, lights, [], cam, linear=True)
    assert hashlib.sha256(lin.tobytes()).hexdigest() == str(fx["linear_sha256"])


@pytest.mark.parametrize("jit", [abi.JIT_OFF, abi.JIT_ON])
def test_sdf_showcase_full_1080p(jit):
    """BASELINE configs[1] at full size (the bench workload), generic and scene-specialised kernels."""
    info = compare(*scenes.sdf_showcase(1920, 1080), jit=jit)
    print(info)


@pytest.mark.parametrize("name,mode", SCENE_CASES)
def test_scene_specialised_kernels_match_oracle(name, mode):
    """The hiprtc-specialised kernel (jit.hip) must reproduce the oracle exactly like the generic one."""
    compare(*scenes.SCENES[name](160, 90, mode=mode), jit=abi.JIT_ON)


def test_advanced_demo_full_1080p():
    """BASELINE configs[2]: 6 spheres, 5 point lights with shadow rays."""
    compare(*scenes.advanced_demo(1920, 1080))


def test_basic_demo_reference_cpu_config_640x480():
    """BASELINE configs[0]: the reference CPU raytracer's formula (REFCOMPAT)."""
    compare(*scenes.basic_demo(640, 480, mode="refcompat"))


@pytest.mark.parametrize("jit", [abi.JIT_OFF, abi.JIT_ON])
def test_deformation_stress_4k(jit):
    """BASELINE configs[4] workload on one GPU (64-node CSG + bend/twist/noise, 3840x2160)."""
    compare(*scenes.deformation_stress(3840, 2160), threads=16, jit=jit)


@pytest.mark.parametrize("fn", [se.mixed_scene, se.all_lights_scene, se.deformers_scene, se.ortho_scene,
                                se.convex_sdf_scene])
@pytest.mark.parametrize("mode", ["refcompat", "lambert_shadow"])
@pytest.mark.parametrize("jit", [abi.JIT_OFF, abi.JIT_ON])
def test_extra_scenes(fn, mode, jit):
    # spot lights use acosf (libm vs device ocml): allow an ulp in the linear image there
    compare(*fn(200, 120, mode), linear_exact=fn is not se.all_lights_scene, jit=jit)


@pytest.mark.parametrize("jit", [abi.JIT_OFF, abi.JIT_ON])
@pytest.mark.parametrize("case", ["cull_stress", "cull_stress_66", "mixed", "all_lights", "advanced-demo",
                                  "sdf-showcase", "deformers"])
def test_shadow_culling_is_exact(case, jit, monkeypatch):
    """Shadow-ray culling (RRTE_CULL forces it on/off regardless of the scene policy) never changes
    a bit: culled and unculled renders are identical (linear image and shadow-ray count), and both
    match the oracle.  cull_stress_66 has > 64 objects, where culling must switch itself off."""
    if case.startswith("cull_stress"):
        args = se.cull_stress_scene(240, 160, "lambert_shadow", n_spheres=60 if case.endswith("66") else 40)
    elif case in ("mixed", "all_lights", "deformers"):
        args = getattr(se, case + "_scene")(200, 120, "lambert_shadow")
    else:
        args = scenes.SCENES[case](320, 180)
    objs, lights, cam, cfg = args
    out = {}
    for cull in ("0", "1"):
        monkeypatch.setenv("RRTE_CULL", cull)
        # spot lights use acosf (libm vs device ocml): an ulp in the linear image vs the oracle
        compare(*args, linear_exact=case not in ("all_lights", "cull_stress", "cull_stress_66"), jit=jit)
        rt = Raytracer(cfg, device=0, jit=jit)
        _, lin = rt.render_f32(objs, lights, [], cam, linear=True)
        out[cull] = (lin.view(np.uint32).copy(), int(rt.stats().shadow_rays))
    assert np.array_equal(out["0"][0], out["1"][0])
    assert out["0"][1] == out["1"][1]


@pytest.mark.parametrize("scene", ["convex", "csg_parts"])
@pytest.mark.parametrize("size", [(240, 160), (641, 359)])
def test_convex_secant_early_miss_is_exact(size, scene, monkeypatch):
    """Scene-specialised any-hit marches of convex SDF objects stop once the secant bound proves
    that no later step can hit (ray_kernels.hpp sdf_march CONVEX), and those of two-leaf CSG objects
    once every part their value is bounded by is proven (sdf_parts_plan, round 6).  Exact: the image
    and the shadow-ray count match the oracle bit for bit, and match the same kernel compiled without
    the early misses (RRTE_JIT_EXTRA_OPTS=-DRRTE_SECANT_EXIT=0), with grazing and near-horizon lights,
    degenerate sizes and controls the exits must leave alone."""
    fn = se.convex_sdf_scene if scene == "convex" else se.csg_parts_scene
    objs, lights, cam, cfg = fn(*size)
    compare(objs, lights, cam, cfg, jit=abi.JIT_ON)
    out = {}
    # (the part-wise exit is an off-by-default switch: -DRRTE_PARTS_EXIT=1 checks it)
    opts = ("", "-DRRTE_PARTS_EXIT=1", "-DRRTE_SECANT_EXIT=0")
    for opt in opts:
        monkeypatch.setenv("RRTE_JIT_EXTRA_OPTS", opt)
        rt = Raytracer(cfg, device=0, jit=abi.JIT_ON)
        _, lin = rt.render_f32(objs, lights, [], cam, linear=True)
        st = rt.stats()
        assert st.jit_active == 1
        out[opt] = (lin.view(np.uint32).copy(), int(st.shadow_rays))
    for opt in opts[:2]:
        assert np.array_equal(out[opt][0], out["-DRRTE_SECANT_EXIT=0"][0]), opt
        assert out[opt][1] == out["-DRRTE_SECANT_EXIT=0"][1], opt


@pytest.mark.parametrize("jit", [abi.JIT_OFF, abi.JIT_ON])
def test_stochastic_multibounce_materials(jit):
    """Reference default workload shape: spp > 1, random jitter, depth > 1, Lambertian/Metal/
    Dielectric/Emissive scatter (§8f rank 1).  Same counter-based RNG stream on both sides;
    the device accumulates the recursion forward (rounding-level differences beyond depth 2).
    JIT_ON: the scene-specialised kernel with runtime sample/bounce loops."""
    objs, lights, cam, cfg = se.materials_scene(160, 100, spp=4, depth=8)
    compare(objs, lights, cam, cfg, linear_exact=False, jit=jit)


@pytest.mark.parametrize("jit", [abi.JIT_OFF, abi.JIT_ON])
def test_stock_config_depth2_is_bit_exact(jit):
    """spp 4, random jitter and scatter, depth 2 (forward accumulation is exact up to depth 2)."""
    objs, lights, cam, cfg = scenes.sdf_showcase(160, 90, mode="refcompat")
    cfg.samples_per_pixel, cfg.max_depth, cfg.jitter = 4, 2, "random"
    compare(objs, lights, cam, cfg, jit=jit)


@pytest.mark.parametrize("w,h", [(1, 1), (17, 13), (64, 1), (1, 64), (33, 47)])
def test_odd_sizes(w, h):
    compare(*scenes.sdf_showcase(w, h))


def test_empty_scene_no_lights_depth0_and_no_material():
    objs, lights, cam, cfg = scenes.basic_demo(40, 30)
    compare([], [], cam, cfg)
    compare(objs, [], cam, cfg)
    cfg0 = RaytracerConfig(**{**cfg.__dict__, "max_depth": 0})
    compare(objs, lights, cam, cfg0)
    for o in objs:
        o.material = None
    compare(objs, lights, cam, cfg)


def test_jit_auto_policy_specialises_in_the_background():
    """AUTO (the default): the second render of an unchanged scene starts a background compile;
    frames keep running on the generic kernel until the specialised one is loaded, and every frame is
    identical whichever kernel rendered it."""
    import time
    objs, lights, cam, cfg = scenes.sdf_showcase(96, 54)
    rt = Raytracer(cfg, device=0, jit=abi.JIT_AUTO)
    a = rt.render(objs, lights, [], cam)
    assert rt.stats().jit_active == 0
    t0, frames = time.time(), 1
    while True:
        b = rt.render(objs, lights, [], cam)
        frames += 1
        assert np.array_equal(a, b)
        if rt.stats().jit_active:
            break
        assert time.time() - t0 < 120, "the background compile never landed"
    # frame 1 ran on the generic kernel; frame 2 started the compile -- with the persistent code-object
    # cache warm it can land within frame 2 itself (a later row chunk of the blocking frame)
    assert frames >= 2 and rt.stats().jit_compile_ms > 0
    cam.transform.position = (cam.transform.position[0], cam.transform.position[1] + np.float32(0.5),
                              cam.transform.position[2])
    c = rt.render(objs, lights, [], cam)  # camera motion: no recompile, still specialised
    assert rt.stats().jit_active == 1 and not np.array_equal(a, c)
    compare(objs, lights, cam, cfg)


@pytest.mark.parametrize("name", ["sdf-showcase", "sdf-showcase-literal", "basic-demo"])
def test_camera_motion_on_one_specialised_kernel(name):
    """One scene-specialised context, the camera moved between frames (camera state is a kernel
    argument, never compiled in): poses inside an object's bounding sphere and next to a
    transformed analytic object, then an orthographic camera (per-lane ray origins) -- every
    frame's linear image bit-exact against the oracle."""
    objs, lights, cam, cfg = scenes.SCENES[name](96, 54, mode="lambert_shadow")
    rt = Raytracer(cfg, device=0, jit=abi.JIT_ON)
    poses = [((0.0, 8.0, 20.0), (0.0, 2.0, 0.0)), ((-11.5, 2.2, -7.6), (4.0, 2.0, -8.0)),
             ((-8.0, 2.0, 1.0), (-8.0, 2.0, -8.0)), ((3.0, 0.5, 4.0), (0.0, 1.0, 0.0))]
    for pos, tgt in poses:
        c = scenes._camera(96, 54, pos, tgt, 50.0)
        g8, _ = rt.render_f32(objs, lights, [], c)
        assert rt.stats().jit_active == 1
        _, glin = rt.render_f32(objs, lights, [], c, linear=True)
        sc = LoweredScene(objs, lights, c)
        r8, _, rsh = oracle.render(sc, cfg.lower(), nthreads=16)
        _, rlin, _ = oracle.render(sc, cfg.lower(), nthreads=16, linear=True)
        assert np.array_equal(glin.view(np.uint32), rlin.view(np.uint32)), (name, pos)
        assert int(np.abs(g8.astype(np.int16) - r8.astype(np.int16)).max()) <= 1
    from rrte_amd.renderer import Camera
    oc = Camera.new_orthographic(-8, 8, -4.5, 4.5, 0.1, 100.0)
    oc.transform.position = scenes.vec3((0.0, 8.0, 20.0))
    oc.look_at(scenes.vec3((0.0, 2.0, 0.0)), scenes.vec3((0, 1, 0)))
    compare(objs, lights, oc, cfg, jit=abi.JIT_ON)


@pytest.mark.parametrize("jit", [abi.JIT_OFF, abi.JIT_ON])
@pytest.mark.parametrize("name", ["sdf-showcase", "sdf-showcase-literal", "advanced-demo", "basic-demo"])
def test_camera_tile_culling_is_exact(name, jit, monkeypatch):
    """Camera-ray tile culling (KParams::tile_rect: an 8x8 tile, or a 16x16 block in frames wider
    than 2048, skips objects whose bounding sphere projects outside it) never changes a bit: off and on give identical linear images and shadow-ray
    counts for poses with objects off screen, at the frame edge, close to the eye and behind it,
    a wide and a narrow field of view, odd frame sizes and random jitter."""
    poses = [((0.0, 8.0, 20.0), (0.0, 2.0, 0.0), 45.0), ((-11.0, 2.5, -3.0), (4.0, 2.0, -8.0), 80.0),
             ((-8.0, 2.0, 1.5), (-8.0, 2.0, -8.0), 30.0), ((3.0, 1.0, 3.0), (12.0, 2.0, 0.0), 100.0),
             ((0.0, 3.0, 0.0), (0.0, 2.0, 10.0), 60.0), ((14.0, 6.0, 9.0), (-2.0, 1.0, -4.0), 20.0)]
    rts = {}
    for tc in ("0", "1"):  # the switch is read when a context is created
        monkeypatch.setenv("RRTE_TILE_CULL", tc)
        rts[tc] = Raytracer(scenes.SCENES[name](64, 36, mode="lambert_shadow")[3], device=0, jit=jit)
    for w, h in ((131, 77), (200, 112), (2101, 40)):  # 8x8 tiles; 16x16 blocks past 2048 pixels
        for k, (pos, tgt, fov) in enumerate(poses):
            objs, lights, _, cfg = scenes.SCENES[name](w, h, mode="lambert_shadow")
            if k == 5:
                cfg.samples_per_pixel, cfg.jitter = 2, "random"
            cam = scenes._camera(w, h, pos, tgt, fov)
            out = {}
            for tc, rt in rts.items():
                rt.update_config(cfg)
                _, lin = rt.render_f32(objs, lights, [], cam, linear=True)
                out[tc] = (lin.view(np.uint32).copy(), int(rt.stats().shadow_rays))
            assert np.array_equal(out["0"][0], out["1"][0]), (name, w, h, pos)
            assert out["0"][1] == out["1"][1]


@pytest.mark.parametrize("jit", [abi.JIT_OFF, abi.JIT_ON])
@pytest.mark.parametrize("name", ["sdf-showcase", "advanced-demo"])
def test_camera_tile_culling_in_the_path_loop_is_exact(name, jit, monkeypatch):
    """REFCOMPAT with spp > 1 and depth > 1 (the path-regeneration loop): the tile mask applies while
    every active lane of a wave is on its camera ray; culling on and off give identical images."""
    rts = {}
    for tc in ("0", "1"):
        monkeypatch.setenv("RRTE_TILE_CULL", tc)
        rts[tc] = Raytracer(scenes.SCENES[name](64, 36, mode="refcompat")[3], device=0, jit=jit)
    for w, h in ((131, 77), (2101, 40)):
        for pos, tgt, fov in [((0.0, 8.0, 20.0), (0.0, 2.0, 0.0), 45.0), ((3.0, 1.0, 3.0), (12.0, 2.0, 0.0), 100.0)]:
            objs, lights, _, cfg = scenes.SCENES[name](w, h, mode="refcompat")
            cfg.samples_per_pixel, cfg.max_depth, cfg.jitter = 3, 6, "random"
            cam = scenes._camera(w, h, pos, tgt, fov)
            out = {}
            for tc, rt in rts.items():
                rt.update_config(cfg)
                _, lin = rt.render_f32(objs, lights, [], cam, linear=True)
                out[tc] = lin.view(np.uint32).copy()
            assert np.array_equal(out["0"], out["1"]), (name, w, h, pos)


@pytest.mark.parametrize("jit", [abi.JIT_OFF, abi.JIT_ON])
@pytest.mark.parametrize("band", [8, 16])
def test_camera_tile_culling_with_band_mapping(band, jit, monkeypatch):
    """Tile culling on one rank's share of a multi-GPU frame (KParams::band_rows > 0: local rows map
    to interleaved image rows through image_row): rank 1 of 3 emulated on one GPU
    (RRTE_EMULATE_RANK, rrte_hip_render_async renders exactly that rank's packed bands).  Culling
    on and off give identical linear rows, and they are the matching rows of the full frame."""
    import torch
    name, nranks, rank = "sdf-showcase", 3, 1
    poses = [((0.0, 8.0, 20.0), (0.0, 2.0, 0.0), 45.0), ((-11.0, 2.5, -3.0), (4.0, 2.0, -8.0), 80.0),
             ((3.0, 1.0, 3.0), (12.0, 2.0, 0.0), 100.0)]
    full_rt = Raytracer(scenes.SCENES[name](64, 36, mode="lambert_shadow")[3], device=0, jit=jit)
    ctxs = {}
    monkeypatch.setenv("RRTE_EMULATE_RANK", f"{nranks}:{rank}")
    for tc in ("0", "1"):  # both switches are read when a context is created
        monkeypatch.setenv("RRTE_TILE_CULL", tc)
        ctxs[tc] = Context(0, jit=jit)
    monkeypatch.delenv("RRTE_EMULATE_RANK")
    lib = abi.load()
    from test_gpu_4k import band_owner
    for w, h in ((131, 77), (200, 112), (2101, 40)):  # 8x8 tiles; 16x16 blocks past 2048 pixels
        for pos, tgt, fov in poses:
            objs, lights, _, cfg = scenes.SCENES[name](w, h, mode="lambert_shadow")
            cfg.band_rows = band
            cam = scenes._camera(w, h, pos, tgt, fov)
            full_rt.update_config(cfg)
            _, full_lin = full_rt.render_f32(objs, lights, [], cam, linear=True)
            full_lin = full_lin.view(np.uint32).reshape(h, w, 4)
            sc = LoweredScene(objs, lights, cam)
            prm = cfg.lower()
            prm.flags |= abi.FLAG_F32_LINEAR
            # this pose's band partition (sky bands on rank 0, the rest round robin)
            part = abi.band_layout(sc.ref(), C.byref(prm), nranks)
            rows = lib.rrte_hip_band_rows_for_rank_ex(h, band, nranks, rank, *part)
            img_rows = [y for y in range(h) if band_owner(y // band, nranks, *part) == rank]
            assert len(img_rows) == rows
            out = {}
            for tc, ctx in ctxs.items():
                f32 = torch.zeros(rows * w * 4, dtype=torch.float32, device="cuda")
                torch.cuda.synchronize()  # the fill ran on torch's stream; the renders run on others
                ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(prm), None, f32.data_ptr(), None))
                ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
                out[tc] = f32.cpu().numpy().view(np.uint32).reshape(rows, w, 4)
            assert np.array_equal(out["0"], out["1"]), (w, h, pos)
            assert np.array_equal(out["1"], full_lin[img_rows]), (w, h, pos)
    for ctx in ctxs.values():
        ctx.close()


def test_jit_cache_eviction_with_frames_in_flight(monkeypatch):
    """The scene-specialised kernel cache holds 32 modules; the 33rd (scene, mode, variant) evicts
    them all.  A mode or sample-count change does not re-upload the scene (upload_scene's device sync
    does not run), so the eviction itself must wait for frames still running from the old modules on
    other streams.  Nine small scenes x up to four variants, every frame on one of four
    streams without synchronising in between, the 33rd module requested on a same-scene variant
    switch; every frame must equal the generic kernel's.  Full kernels only (RRTE_JIT_TOPO=0): the
    nine scenes differ in values only, so the adaptive policy would share one topology kernel."""
    import torch
    monkeypatch.setenv("RRTE_JIT_TOPO", "0")
    W, H = 48, 32
    variants = [("refcompat", 1), ("refcompat", 2), ("lambert_shadow", 1), ("lambert_shadow", 2)]
    plan = []
    for k in range(9):
        n = 3 if k == 7 else 4  # 7*4 + 3 + 1 = 32 modules, then scene 9's second variant evicts
        plan += [(k, v) for v in variants[:n]]
    ctx = Context(0, jit=abi.JIT_ON)
    streams = [torch.cuda.Stream() for _ in range(4)]
    frames = []
    for i, (k, (mode, spp)) in enumerate(plan):
        objs, lights, cam, cfg = scenes.basic_demo(W, H, mode=mode)
        objs[1].radius = np.float32(0.6 + 0.05 * k)  # a distinct scene per k
        cfg.samples_per_pixel, cfg.jitter = spp, ("random" if spp > 1 else "center")
        sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
        for j in range(3):  # several frames of each variant in flight on different streams
            buf = torch.zeros(W * H, dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()  # the fill ran on torch's stream; the renders run on others
            st = streams[(i + j) % 4]
            ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(prm), buf.data_ptr(), None,
                                                    C.c_void_p(st.cuda_stream)))
            frames.append((objs, lights, cam, cfg, buf))
    ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
    assert ctx.stats().jit_active == 1
    ctx.close()
    rt = Raytracer(frames[0][3], device=0, jit=abi.JIT_OFF)
    for objs, lights, cam, cfg, buf in frames[::3]:
        rt.update_config(cfg)
        ref = rt.render(objs, lights, [], cam)
        assert np.array_equal(buf.cpu().numpy().view(np.uint8), ref)
    for i in range(0, len(frames), 3):  # the other frames of each variant are identical to the first
        a = frames[i][4].cpu()
        assert all(torch.equal(a, frames[i + j][4].cpu()) for j in (1, 2))


def test_scene_cache_invalidates_on_change():
    objs, lights, cam, cfg = scenes.sdf_showcase(96, 54)
    rt = Raytracer(cfg, device=0, jit=abi.JIT_OFF)
    a = rt.render(objs, lights, [], cam)
    b = rt.render(objs, lights, [], cam)
    assert np.array_equal(a, b)
    assert rt.stats().upload_ms == 0.0  # second frame served from the HBM scene cache
    lights[0].intensity = np.float32(lights[0].intensity * 0.5)
    c = rt.render(objs, lights, [], cam)
    assert not np.array_equal(a, c)
    compare(objs, lights, cam, cfg)


def test_async_device_output_matches_blocking():
    import torch
    objs, lights, cam, cfg = scenes.sdf_showcase(320, 180)
    ctx = Context(0)
    sc = LoweredScene(objs, lights, cam)
    prm = cfg.lower()
    buf = torch.zeros(320 * 180, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()  # the fill ran on torch's stream; the renders run on others
    s = torch.cuda.Stream()
    ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(prm), buf.data_ptr(), None,
                                            C.c_void_p(s.cuda_stream)))
    ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
    rt = Raytracer(cfg, device=0)
    ref = rt.render(objs, lights, [], cam)
    assert np.array_equal(buf.cpu().numpy().view(np.uint8), ref)


def test_invalid_inputs_fail_loudly():
    objs, lights, cam, cfg = scenes.sdf_showcase(32, 18)
    ctx = Context(0)
    sc = LoweredScene(objs, lights, cam)
    out = np.zeros(32 * 18 * 4, np.uint8)
    prm = cfg.lower()
    prm.width = 0
    assert ctx.lib.rrte_hip_render(ctx.h, sc.ref(), C.byref(prm), out.ctypes.data) == abi.RRTE_INVALID_ARG
    assert b"zero-sized" in ctx.lib.rrte_hip_last_error(ctx.h)
    prm = cfg.lower()
    prm.mode = 7
    assert ctx.lib.rrte_hip_render(ctx.h, sc.ref(), C.byref(prm), out.ctypes.data) == abi.RRTE_INVALID_ARG
    bad = LoweredScene(objs, lights, cam)
    bad.nodes[0].op = 255  # unknown SDF op in the first SDF object's program
    assert ctx.lib.rrte_hip_render(ctx.h, bad.ref(), C.byref(cfg.lower()), out.ctypes.data) == abi.RRTE_INVALID_ARG
    bad2 = LoweredScene(objs, lights, cam)
    bad2.prims[0].kind = 42
    assert ctx.lib.rrte_hip_render(ctx.h, bad2.ref(), C.byref(cfg.lower()), out.ctypes.data) == abi.RRTE_UNSUPPORTED_PRIM
    h = C.c_void_p()
    assert ctx.lib.rrte_hip_create(99, C.byref(h)) == abi.RRTE_NO_DEVICE


def test_jit_code_objects_persist_across_contexts(tmp_path, monkeypatch):
    """The persistent code-object cache (jit.hip): a second context specialising the same scene loads
    the compiled kernel from RRTE_JIT_CACHE_DIR instead of running hiprtc again, and renders the same
    bytes; a different scene misses the cache."""
    monkeypatch.setenv("RRTE_JIT_CACHE_DIR", str(tmp_path))
    objs, lights, cam, cfg = scenes.sdf_showcase(96, 54)
    a = Raytracer(cfg, device=0, jit=abi.JIT_ON)
    img_a = a.render(objs, lights, [], cam)
    cold = a.stats().jit_compile_ms
    assert a.stats().jit_active == 1 and len(list(tmp_path.glob("*.hsaco"))) == 1
    b = Raytracer(cfg, device=0, jit=abi.JIT_ON)
    img_b = b.render(objs, lights, [], cam)
    warm = b.stats().jit_compile_ms
    assert b.stats().jit_active == 1 and np.array_equal(img_a, img_b)
    assert warm < 0.2 * cold, (cold, warm)
    lights[0].intensity = np.float32(lights[0].intensity * 0.5)  # another scene: another kernel
    b.render(objs, lights, [], cam)
    assert len(list(tmp_path.glob("*.hsaco"))) == 2
