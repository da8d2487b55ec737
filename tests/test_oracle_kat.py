"""Known-answer tests for the CPU oracle, derived by hand from the reference source
(Melthizar/RRTE; file:line per test).  The reference ships no tests or fixtures
(SURVEY.md §4), so these closed-form answers are what pins the oracle."""
import ctypes as C
import math

import numpy as np
import pytest

import oracle
from rrte_amd import (Camera, Capsule, Color, Cone, Cube, Cylinder, LambertianMaterial, LoweredScene, Plane,
                      PointLight, RaytracerConfig, Sphere, Transform, Triangle, abi, to_radians)
from rrte_amd.math import quat_from_rotation_arc, vec3

f32 = np.float32


def one(obj):
    cam = Camera.new_perspective(to_radians(45.0), 1.0, 0.1, 100.0)
    return LoweredScene([obj], [], cam)


def hit(obj, o, d, tmin=0.001, tmax=float("inf")):
    sc = one(obj)
    h = oracle.OracleHit()
    ok = oracle.load().rrte_oracle_intersect(C.byref(sc.ir), 0, oracle.farr(o), oracle.farr(d), tmin, tmax, C.byref(h))
    return (h.t, list(h.point), list(h.normal), bool(h.front_face)) if ok else None


def test_sphere_front_hit():  # primitives.rs:57-81, ray.rs:45-56
    t, p, n, front = hit(Sphere((0, 0, 0), 1.0), (0, 0, 5), (0, 0, -1))
    assert t == 4.0 and p == [0, 0, 1] and n == [0, 0, 1] and front


def test_sphere_from_inside_takes_far_root_and_flips_normal():  # primitives.rs:71-76
    t, p, n, front = hit(Sphere((0, 0, 0), 2.0), (0, 0, 0), (1, 0, 0))
    assert t == 2.0 and n == [-1, 0, 0] and not front


def test_sphere_miss_and_tmax():
    assert hit(Sphere((0, 0, 0), 1.0), (0, 5, 5), (0, 0, -1)) is None
    assert hit(Sphere((0, 0, 0), 1.0), (0, 0, 5), (0, 0, -1), tmax=3.9) is None


def test_plane():  # primitives.rs:133-149: normal = denom<0 ? n : -n, then HitInfo flips again
    t, p, n, front = hit(Plane((0, 0, 0), (0, 1, 0)), (0, 5, 0), (0, -1, 0))
    assert t == 5.0 and n == [0, 1, 0] and front
    assert hit(Plane((0, 0, 0), (0, 1, 0)), (0, 5, 0), (1, 0, 0)) is None  # parallel: |denom| < 1e-6


def test_triangle():  # primitives.rs:208-244
    tri = Triangle((-1, -1, 0), (1, -1, 0), (0, 1, 0))
    t, p, n, front = hit(tri, (0, 0, 5), (0, 0, -1))
    assert t == 5.0 and n == [0, 0, 1] and front
    assert hit(tri, (2, 2, 5), (0, 0, -1)) is None


def test_cube_slab():  # primitives.rs:301-364
    t, p, n, front = hit(Cube((0, 0, 0), (2, 2, 2)), (0, 0, 5), (0, 0, -1))
    assert t == 4.0 and p == [0, 0, 1] and n == [0, 0, 1] and front
    t, p, n, front = hit(Cube((0, 0, 0), (2, 2, 2)), (5, 0.25, 0.5), (-1, 0, 0))
    assert t == 4.0 and n == [1, 0, 0]


def test_cube_origin_inside_quirk_nan_normal():  # primitives.rs:312-354: t = t_min, normal ZERO -> NaN
    t, p, n, front = hit(Cube((0, 0, 0), (2, 2, 2)), (0, 0, 0), (0, 0, -1))
    assert t == pytest.approx(0.001) and all(math.isnan(v) for v in n)


def test_cube_rotated_transform():  # transform.rs:50-57: local ray through inverse_matrix
    c = Cube((0, 0, 0), (2, 2, 2))
    s = math.sqrt(0.5)
    c.transform = Transform(position=(0, 0, 0), rotation=(0, s, 0, s), scale=(1, 1, 1))  # 90 deg about Y
    t, p, n, front = hit(c, (0, 0, 5), (0, 0, -1))
    assert abs(t - 4.0) < 1e-6 and abs(n[2] - 1.0) < 1e-6 and front


def test_cylinder_side_and_axis_parallel():  # primitives.rs:419-465 (no caps)
    t, p, n, front = hit(Cylinder((0, 0, 0), 1.0, 2.0), (5, 0, 0), (-1, 0, 0))
    assert t == 4.0 and n == [1, 0, 0]
    assert hit(Cylinder((0, 0, 0), 1.0, 2.0), (0, 5, 0), (0, -1, 0)) is None  # a = 0: no caps, no hit


def test_cone_side_normal_quirk():  # primitives.rs:520-571
    t, p, n, front = hit(Cone((0, 0, 0), 1.0, 2.0), (5, -0.5, 0), (-1, 0, 0))
    # radius at y=-0.5: k*(h/2 - y) = 0.5*1.5 = 0.75 -> t = 4.25; normal = normalize(x/r, k, z/r) = (1, .5, 0)/|.|
    assert t == pytest.approx(4.25, abs=1e-6)
    assert n == pytest.approx([2 / math.sqrt(5), 1 / math.sqrt(5), 0], abs=1e-6)


def test_capsule_top_cap():  # primitives.rs:626-725
    t, p, n, front = hit(Capsule((0, 0, 0), 0.5, 2.0), (0, 5, 0), (0, -1, 0))
    assert t == 3.5 and n == [0, 1, 0]
    t, p, n, front = hit(Capsule((0, 0, 0), 0.5, 2.0), (5, 0.2, 0), (-1, 0, 0))
    assert t == 4.5 and n == [1, 0, 0]


def test_look_at_quaternions():  # camera.rs:85-95 (Quat::from_rotation_arc(-Z, forward); up ignored)
    q = (C.c_float * 4)()
    oracle.load().rrte_oracle_look_at(oracle.farr([0, 0, 5]), oracle.farr([0, 0, 0]), q)
    assert list(q) == [0, 0, 0, 1]
    oracle.load().rrte_oracle_look_at(oracle.farr([5, 0, 0]), oracle.farr([0, 0, 0]), q)
    s = np.float32(1) / np.sqrt(np.float32(2))
    assert list(q) == pytest.approx([0, s, 0, s], abs=1e-7)
    # the Python mirror restates the same algorithm with numpy f32: bit-identical
    for pos, tgt in [((6, 4, 6), (0, 1, 0)), ((0, 8, 20), (0, 2, 0)), ((12, 6, 0), (0, 1, 0))]:
        oracle.load().rrte_oracle_look_at(oracle.farr(pos), oracle.farr(tgt), q)
        from rrte_amd.math import normalize, sub
        mine = quat_from_rotation_arc(vec3(0, 0, -1), normalize(sub(vec3(tgt), vec3(pos))))
        assert np.array(list(q), np.float32).tobytes() == np.array(mine, np.float32).tobytes()


def test_generate_ray_centre_is_forward():  # camera.rs:98-117
    cam = Camera.new_perspective(to_radians(45.0), 1.0, 0.1, 100.0)
    cam.transform.position = vec3(0, 0, 5)
    cam.look_at((0, 0, 0))
    o, d = (C.c_float * 3)(), (C.c_float * 3)()
    oracle.load().rrte_oracle_generate_ray(C.byref(cam.lower()), 0.5, 0.5, o, d)
    assert list(o) == [0, 0, 5] and list(d) == [0, 0, -1]
    # v = 0 is the TOP row: ndc_y = +1 (camera.rs:101)
    oracle.load().rrte_oracle_generate_ray(C.byref(cam.lower()), 0.5, 0.0, o, d)
    assert d[1] > 0


def _render(objs, lights, cfg, cam=None):
    cam = cam or Camera.new_perspective(to_radians(45.0), f32(cfg.width) / f32(cfg.height), 0.1, 100.0)
    if cam.transform.position == vec3(0, 0, 0):
        cam.transform.position = vec3(0, 0, 5)
        cam.look_at((0, 0, 0))
    o8, of, sh = oracle.render(LoweredScene(objs, lights, cam), cfg.lower(), nthreads=2)
    return o8.reshape(cfg.height, cfg.width, 4), of.reshape(cfg.height, cfg.width, 4), sh


def test_background_gamma_and_truncation():  # raytracer.rs:76-85, color.rs:58-65
    cfg = RaytracerConfig(max_depth=1, samples_per_pixel=1, width=4, height=3, jitter="center")
    img, f, _ = _render([], [], cfg)
    g = np.float32(1) / np.float32(2.2)
    exp = [int(np.float32(np.power(np.float32(c), g)) * np.float32(255)) for c in (0.5, 0.7, 1.0)]
    assert exp == [186, 216, 255]
    assert (img[..., :3] == exp).all() and (img[..., 3] == 255).all()


def test_depth_zero_is_black():  # raytracer.rs:100-101
    cfg = RaytracerConfig(max_depth=0, samples_per_pixel=1, width=4, height=3, jitter="center")
    img, _, _ = _render([Sphere((0, 0, 0), 1.0, LambertianMaterial(Color.rgb(1, 0, 0)))], [], cfg)
    assert (img[..., :3] == 0).all() and (img[..., 3] == 255).all()


def test_no_material_is_black():  # raytracer.rs:139-143
    cfg = RaytracerConfig(max_depth=1, samples_per_pixel=1, width=5, height=5, jitter="center")
    img, _, _ = _render([Sphere((0, 0, 0), 1.0)], [], cfg)
    assert (img[2, 2, :3] == 0).all()


def test_refcompat_formula_centre_pixel():  # raytracer.rs:121-136 + light.rs:170-194
    alb = Color.rgb(0.2, 0.4, 0.6)
    light = PointLight((0, 0, 10), Color.rgb(1.0, 0.5, 0.25), 2.0)
    cfg = RaytracerConfig(max_depth=1, samples_per_pixel=1, width=5, height=5, jitter="center",
                          background_color=Color(0, 0, 0, 1))
    _, f, _ = _render([Sphere((0, 0, 0), 1.0, LambertianMaterial(alb))], [light], cfg)
    # centre pixel hits (0,0,1); distance to light 9
    d = np.float32(9)
    att = np.float32(1) / ((np.float32(1) + np.float32(0.09) * d) + (np.float32(0.032) * d) * d)
    for k, (a, lc) in enumerate([(0.2, 1.0), (0.4, 0.5), (0.6, 0.25)]):
        lin = (np.float32(0) + (np.float32(a) * np.float32(0.1)) * np.float32(0.1)) + (np.float32(lc) * np.float32(2)) * att
        exp = min(1.0, float(np.power(lin, np.float32(1) / np.float32(2.2))))
        assert f[2, 2, k] == pytest.approx(exp, abs=1e-7)


def test_lambert_shadow_occlusion_and_count():  # build-defined LAMBERT_SHADOW
    mat = LambertianMaterial(Color.rgb(0.5, 0.5, 0.5))
    light = PointLight((0, 10, 0), Color.rgb(1, 1, 1), 3.0)
    plane_y0 = Plane((0, 0, 0), (0, 1, 0), mat)
    blocker = Sphere((2, 2, 0), 0.5, mat)
    cam = Camera.new_perspective(to_radians(60.0), 1.0, 0.1, 100.0)
    cam.transform.position = vec3(0, 8, 8)
    cam.look_at((0, 0, 0))
    cfg = RaytracerConfig(max_depth=1, samples_per_pixel=1, width=33, height=33, jitter="center",
                          mode="lambert_shadow", background_color=Color(0, 0, 0, 1))
    lit, _, n_lit = _render([plane_y0], [light], cfg, cam)
    shad, _, n_sh = _render([plane_y0, blocker], [light], cfg, cam)
    assert n_lit == (lit[..., 0] > 0).sum()  # every plane pixel faces the light -> one shadow ray each
    assert n_sh > 0
    # pixels whose view ray hits the plane behind the blocker are darker than the unblocked image
    assert (shad[..., 0] < lit[..., 0]).any()
