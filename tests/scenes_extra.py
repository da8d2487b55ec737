"""Extra test scenes: transformed analytic prims, every light kind, every material kind,
orthographic camera."""
import math

from rrte_amd import (AmbientLight, Camera, Capsule, Color, Cone, Cube, Cylinder, DielectricMaterial,
                      DirectionalLight, EmissiveMaterial, LambertianMaterial, MetalMaterial, Plane, PointLight,
                      RaytracerConfig, SDFObject, SDFSphere, SDFTorus, Sphere, SpotLight, Transform, Triangle,
                      TwistDeformer, TaperDeformer, WaveDeformer, DeformedSDF, SDFBox, to_radians)
from rrte_amd.math import f32, vec3


def mixed_scene(w, h, mode):
    mats = [LambertianMaterial(Color.rgb(*c)) for c in [(0.6, 0.3, 0.2), (0.2, 0.5, 0.7), (0.4, 0.6, 0.3)]]
    s = math.sqrt(0.5)
    rot = Cube((1.5, 1.0, 0.0), (1.0, 1.5, 0.8), mats[0])
    rot.transform = Transform(position=(0.1, 0.0, 0.2), rotation=(0.0, 0.38268343, 0.0, 0.92387953), scale=(1, 1.2, 1))
    cyl = Cylinder((-1.5, 1.0, 0.5), 0.6, 1.5, mats[1])
    cyl.transform = Transform(position=(0, 0, 0), rotation=(s * 0.5, 0.0, 0.0, math.sqrt(1 - 0.125)), scale=(1, 1, 1))
    objs = [Plane((0, 0, 0), (0, 1, 0), mats[2]), rot, cyl, Cone((0.0, 1.2, -1.5), 0.8, 1.6, mats[0]),
            Capsule((0.0, 1.0, 1.8), 0.4, 1.0, mats[1]),
            Triangle((-3, 0.1, -3), (3, 0.1, -3), (0, 3, -3), mats[2])]
    lights = [PointLight((3, 6, 4), Color.rgb(1, 1, 1), 4.0), PointLight((-4, 3, -1), Color.rgb(0.5, 0.6, 1.0), 2.5)]
    cam = Camera.new_perspective(to_radians(50.0), f32(w) / f32(h), 0.1, 100.0)
    cam.transform.position = vec3(4, 3.5, 6)
    cam.look_at((0, 1, 0))
    cfg = RaytracerConfig(max_depth=1, samples_per_pixel=1, width=w, height=h, jitter="center", mode=mode,
                          background_color=Color(0.1, 0.1, 0.15, 1))
    return objs, lights, cam, cfg


def all_lights_scene(w, h, mode):
    objs, _, cam, cfg = mixed_scene(w, h, mode)
    lights = [PointLight((3, 6, 4), Color.rgb(1, 1, 1), 2.0),
              DirectionalLight((-0.3, -1.0, -0.3), Color(1.0, 0.95, 0.8, 1.0), 0.6),
              SpotLight((0, 5, 0), (0, -1, 0), Color.rgb(1, 0.8, 0.6), 6.0, 0.3, 0.6),
              AmbientLight.default_ambient()]
    return objs, lights, cam, cfg


def materials_scene(w, h, spp=4, depth=6):
    objs = [Sphere((0, -1000, 0), 1000, LambertianMaterial(Color.rgb(0.5, 0.5, 0.5))),
            Sphere((-2.2, 1, 0), 1.0, MetalMaterial(Color.rgb(0.8, 0.6, 0.2), 0.1)),
            Sphere((0, 1, 0), 1.0, DielectricMaterial(1.5)),
            Sphere((2.2, 1, 0), 1.0, EmissiveMaterial(Color.rgb(1.0, 0.3, 0.2), 4.0)),
            SDFObject(DeformedSDF(SDFTorus((0, 0.5, 2.2), 0.7, 0.25), TwistDeformer((0, 1, 0), 1.5, (0, 0.5, 2.2))),
                      LambertianMaterial(Color.rgb(0.3, 0.7, 0.4)))]
    lights = [PointLight((0, 6, 4), Color.rgb(1, 1, 1), 0.3)]
    cam = Camera.new_perspective(to_radians(45.0), f32(w) / f32(h), 0.1, 100.0)
    cam.transform.position = vec3(0, 3, 9)
    cam.look_at((0, 1, 0))
    cfg = RaytracerConfig(max_depth=depth, samples_per_pixel=spp, width=w, height=h, jitter="random", seed=1234,
                          mode="refcompat", background_color=Color(0.5, 0.7, 1.0, 1.0))
    return objs, lights, cam, cfg


def deformers_scene(w, h, mode):
    m = LambertianMaterial(Color.rgb(0.7, 0.6, 0.4))
    objs = [Plane((0, 0, 0), (0, 1, 0), LambertianMaterial(Color.rgb(0.3, 0.3, 0.3))),
            SDFObject(DeformedSDF(SDFBox((-2, 1, 0), (1, 1.6, 1)), TaperDeformer((0, 1, 0), 1.0, 0.4, 1.6, (-2, 1, 0))), m),
            SDFObject(DeformedSDF(SDFBox((0, 1, 0), (1.2, 1, 1)), WaveDeformer((1, 0, 0), 0.15, 6.0, (0, 1, 0), (0, 1, 0))), m),
            SDFObject(DeformedSDF(SDFSphere((2, 1, 0), 0.8), TwistDeformer((0, 1, 0), 2.0, (2, 1, 0))), m)]
    lights = [PointLight((2, 6, 5), Color.rgb(1, 1, 1), 5.0)]
    cam = Camera.new_perspective(to_radians(45.0), f32(w) / f32(h), 0.1, 100.0)
    cam.transform.position = vec3(0, 3, 8)
    cam.look_at((0, 1, 0))
    cfg = RaytracerConfig(max_depth=1, samples_per_pixel=1, width=w, height=h, jitter="center", mode=mode,
                          background_color=Color(0.1, 0.1, 0.15, 1))
    return objs, lights, cam, cfg


def ortho_scene(w, h, mode):
    objs, lights, _, cfg = mixed_scene(w, h, mode)
    cam = Camera.new_orthographic(-4, 4, -3, 3, 0.1, 100.0)
    cam.transform.position = vec3(0, 2, 10)
    return objs, lights, cam, cfg


def cull_stress_scene(w, h, mode, n_spheres=40, seed=7):
    """Shadow-culling edge cases: many small close objects casting grazing shadows, transformed
    analytic prims, a plane with a NON-unit normal (shadow origins offset by |n|*bias), a
    directional light with a non-unit direction, a point light inside the object cloud."""
    import random
    rnd = random.Random(seed)
    mats = [LambertianMaterial(Color.rgb(0.3 + 0.6 * rnd.random(), 0.3 + 0.6 * rnd.random(), 0.3 + 0.6 * rnd.random()))
            for _ in range(4)]
    objs = [Plane((0, 0, 0), (0, 2.5, 0), mats[0])]
    for i in range(n_spheres):
        objs.append(Sphere((rnd.uniform(-4, 4), rnd.uniform(0.2, 2.5), rnd.uniform(-4, 4)), rnd.uniform(0.08, 0.35),
                           mats[i % 4]))
    cube = Cube((0.0, 0.6, 0.0), (0.8, 0.5, 1.2), mats[1])
    cube.transform = Transform(position=(0.5, 0.1, -0.5), rotation=(0.0, 0.38268343, 0.0, 0.92387953), scale=(1.5, 1, 0.7))
    objs += [cube, Cylinder((2.5, 0.8, 2.0), 0.3, 1.2, mats[2]), Cone((-2.5, 0.8, 2.0), 0.5, 1.0, mats[3]),
             Capsule((0.0, 0.5, 3.0), 0.25, 0.6, mats[1]), Triangle((-3, 0.05, -4), (3, 0.05, -4), (0, 2.5, -4), mats[2]),
             SDFObject(SDFTorus((2.0, 1.5, -2.0), 0.6, 0.2), mats[3])]
    lights = [PointLight((0.3, 1.5, 0.2), Color.rgb(1, 0.9, 0.8), 1.5),
              DirectionalLight((-0.6, -2.0, -0.4), Color(1.0, 0.95, 0.8, 1.0), 0.5),
              SpotLight((0, 6, 0), (0, -1, 0), Color.rgb(0.6, 0.8, 1.0), 5.0, 0.4, 0.8)]
    cam = Camera.new_perspective(to_radians(55.0), f32(w) / f32(h), 0.1, 100.0)
    cam.transform.position = vec3(5, 4, 7)
    cam.look_at((0, 1, 0))
    cfg = RaytracerConfig(max_depth=1, samples_per_pixel=1, width=w, height=h, jitter="center", mode=mode,
                          background_color=Color(0.1, 0.1, 0.15, 1))
    return objs, lights, cam, cfg


def random_csg_scene(w, h, mode, seed=11, n_objects=4, depth=4):
    """SDF objects built from random CSG trees over every leaf kind and every op (smooth k random),
    some subtrees under deformers: exercises the CSG early-outs (sdf_guard.hip) at every nesting."""
    import numpy as np
    from rrte_amd import renderer as R

    rng = np.random.default_rng(seed)
    ops = ["union", "smooth_union", "difference", "smooth_difference", "intersection", "smooth_intersection"]

    def leaf(c):
        k = int(rng.integers(10))
        s = float(rng.uniform(0.3, 0.9))
        c = tuple(float(v) for v in c)
        return [R.SDFSphere(c, s), R.SDFBox(c, (s * 1.5, s, s * 1.2)), R.SDFCylinder(c, s * 0.6, s * 1.6),
                R.SDFPrism(c, (s, s * 1.5, s)), R.SDFTorus(c, s, s * 0.3), R.SDFTube(c, s, s * 0.6, s * 1.4),
                R.SDFRing(c, s, s * 0.25), R.SDFCone(c, s * 0.7, s * 1.5), R.SDFCapsule(c, s * 0.4, s),
                R.SDFEllipsoid(c, (s, s * 0.3, s * 0.8))][k]

    def tree(c, d):
        if d == 0 or rng.uniform() < 0.15:
            return leaf(c)
        spread = 0.35 * d
        a = tree(np.asarray(c) + rng.uniform(-spread, spread, 3), d - 1)
        b = tree(np.asarray(c) + rng.uniform(-spread, spread, 3), d - 1)
        t = R.CSGComposite(a, b, ops[int(rng.integers(6))] if d < depth else "union", float(rng.uniform(0.05, 0.5)))
        if d == 2 and rng.uniform() < 0.3:
            t = R.DeformedSDF(t, R.TwistDeformer((0, 1, 0), float(rng.uniform(0.2, 0.8)), tuple(c)))
        return t

    m = [LambertianMaterial(Color.rgb(0.7, 0.5, 0.3)), LambertianMaterial(Color.rgb(0.3, 0.6, 0.8))]
    objs = [Sphere((0.0, -1000.0, 0.0), 1000.0, LambertianMaterial(Color.rgb(0.2, 0.2, 0.2)))]
    for i in range(n_objects):
        c = (-4.5 + 3.0 * i, 1.8, float(rng.uniform(-1, 1)))
        objs.append(SDFObject(tree(c, depth), m[i % 2], max_steps=160))
    lights = [PointLight((0, 8, 6), Color.rgb(1, 1, 1), 25.0), PointLight((-6, 5, -3), Color.rgb(1, 0.8, 0.6), 15.0)]
    cam = Camera.new_perspective(to_radians(45.0), f32(w) / f32(h), 0.1, 100.0)
    cam.transform.position = vec3(0, 4, 12)
    cam.look_at((0, 1.5, 0))
    cfg = RaytracerConfig(max_depth=1, samples_per_pixel=1, width=w, height=h, jitter="center", mode=mode,
                          background_color=Color(0.05, 0.05, 0.08, 1))
    return objs, lights, cam, cfg


def nan_left_operand_scene(w, h, mode="lambert_shadow"):
    """Differences and smooth differences whose LEFT operand is NaN almost everywhere (an ellipsoid
    with a zero radius: k0 (k0 - 1) / k1 = inf * inf / inf) and whose right operand is a guarded
    union of two spheres: a NaN left value must fail the CSG early-out (sdf_guard.hip), since the
    plain op gives smx(NaN, -b) = -b (IEEE maxNum), not NaN."""
    from rrte_amd import renderer as R

    m = LambertianMaterial(Color.rgb(0.7, 0.5, 0.3))
    objs = [Sphere((0.0, -1000.0, 0.0), 1000.0, LambertianMaterial(Color.rgb(0.2, 0.2, 0.2)))]
    for i, op in enumerate(["difference", "smooth_difference", "union"]):
        c = (-3.0 + 3.0 * i, 1.5, 0.0)
        right = R.CSGComposite(R.SDFSphere((c[0] - 0.4, c[1], c[2]), 0.6), R.SDFSphere((c[0] + 0.4, c[1], c[2]), 0.6),
                               "union")
        left = R.SDFEllipsoid(c, (1.2, 0.0, 1.2))
        objs.append(SDFObject(R.CSGComposite(left, right, op, 0.3), m, max_steps=64))
    lights = [PointLight((0, 8, 6), Color.rgb(1, 1, 1), 25.0)]
    cam = Camera.new_perspective(to_radians(45.0), f32(w) / f32(h), 0.1, 100.0)
    cam.transform.position = vec3(0, 3, 9)
    cam.look_at((0, 1.5, 0))
    cfg = RaytracerConfig(max_depth=1, samples_per_pixel=1, width=w, height=h, jitter="center", mode=mode,
                          background_color=Color(0.05, 0.05, 0.08, 1))
    return objs, lights, cam, cfg


def convex_sdf_scene(w, h, mode="lambert_shadow"):
    """Every convex SDF kind the secant early miss applies to (sphere, box, cylinder, prism, cone,
    capsule, intersections and smooth intersections; degenerate sizes: a negative box extent, an inverted capsule) packed
    close together with non-convex controls (torus, union, cone with a negative radius), lit by a
    light near the horizon and one overhead: many grazing shadow rays, and shadow rays that start on
    one convex object and skim its neighbours (ray_kernels.hpp sdf_march CONVEX)."""
    from rrte_amd import renderer as R

    ms = [LambertianMaterial(Color.rgb(*c)) for c in [(0.7, 0.5, 0.3), (0.3, 0.6, 0.8), (0.5, 0.8, 0.4)]]
    y = 1.0
    sdfs = [R.SDFSphere((-3.0, y, -1.0), 0.9), R.SDFBox((-1.6, y, -1.2), (1.2, 1.6, 1.0)),
            R.SDFCylinder((-0.2, y, -1.0), 0.6, 1.8), R.SDFPrism((1.2, y, -1.1), (1.2, 1.6, 0.8)),
            R.SDFCone((2.6, y, -1.0), 0.8, 1.9), R.SDFCapsule((-2.4, y, 0.9), 0.5, 1.2),
            R.CSGComposite(R.SDFSphere((-0.6, y, 1.0), 0.9), R.SDFBox((-0.3, y, 1.0), (1.2, 1.2, 1.2)),
                           "intersection"),
            R.SDFBox((0.9, y, 1.1), (1.0, -0.5, 1.0)), R.SDFCapsule((2.2, y, 1.0), 0.45, -0.6),
            R.CSGComposite(R.SDFSphere((3.4, y, 0.2), 0.8), R.SDFCylinder((3.7, y, 0.2), 0.6, 1.6),
                           "smooth_intersection", 0.3),
            R.CSGComposite(R.SDFCone((-3.6, 0.8, 2.2), 0.7, 1.6), R.SDFSphere((-3.5, 0.8, 2.2), 0.7),
                           "smooth_intersection", 0.05),
            R.SDFTorus((0.4, 0.4, 2.6), 0.7, 0.25),
            R.CSGComposite(R.SDFSphere((-2.0, 0.6, 2.6), 0.6), R.SDFSphere((-1.4, 0.6, 2.6), 0.6), "union"),
            R.SDFCone((2.0, 0.7, 2.6), -0.6, 1.2)]
    objs = [Sphere((0.0, -1000.0, 0.0), 1000.0, LambertianMaterial(Color.rgb(0.2, 0.2, 0.2)))]
    objs += [SDFObject(s, ms[i % 3]) for i, s in enumerate(sdfs)]
    lights = [PointLight((-12.0, 1.3, 0.3), Color.rgb(1.0, 0.9, 0.8), 30.0),
              PointLight((0.5, 7.0, 0.5), Color.rgb(0.6, 0.7, 1.0), 12.0),
              DirectionalLight((1.0, -0.05, -0.2), Color.rgb(0.9, 0.9, 1.0), 0.5)]
    cam = Camera.new_perspective(to_radians(50.0), f32(w) / f32(h), 0.1, 100.0)
    cam.transform.position = vec3(1.0, 4.5, 8.0)
    cam.look_at((0.0, 0.8, 0.5))
    cfg = RaytracerConfig(max_depth=1, samples_per_pixel=1, width=w, height=h, jitter="center", mode=mode,
                          background_color=Color(0.05, 0.05, 0.08, 1))
    return objs, lights, cam, cfg


def csg_parts_scene(w, h, mode="lambert_shadow"):
    """Two-leaf CSG objects the part-wise secant early miss applies to (ray_kernels.hpp sdf_parts_plan):
    unions and smooth unions of two convex leaves (both parts proven), differences and smooth
    differences with a convex left leaf (the left part proven; the right one may be anything, here a
    torus too), a large smooth k, degenerate sizes, and controls the plan must leave alone (a union with
    a torus, a smooth union with k = 0), packed together under a near-horizon light and an overhead
    one: grazing shadow rays leaving one object and skimming the next."""
    from rrte_amd import renderer as R

    ms = [LambertianMaterial(Color.rgb(*c)) for c in [(0.8, 0.4, 0.3), (0.3, 0.7, 0.6), (0.6, 0.6, 0.9)]]
    y = 0.9
    sdfs = [R.CSGComposite(R.SDFSphere((-3.0, y, -1.0), 0.8), R.SDFBox((-2.4, y, -1.1), (0.9, 1.4, 0.9)), "union"),
            R.CSGComposite(R.SDFCapsule((-1.2, y, -1.0), 0.4, 1.0), R.SDFCylinder((-0.8, y, -0.9), 0.5, 1.4),
                           "smooth_union", 0.3),
            R.CSGComposite(R.SDFBox((0.6, y, -1.0), (1.4, 1.4, 1.4)), R.SDFSphere((0.9, y + 0.3, -0.7), 0.8),
                           "difference"),
            R.CSGComposite(R.SDFSphere((2.4, y, -1.0), 0.9), R.SDFBox((2.8, y, -1.0), (0.8, 0.8, 2.0)),
                           "smooth_difference", 0.2),
            R.CSGComposite(R.SDFSphere((-2.6, 0.7, 1.2), 0.6), R.SDFSphere((-1.7, 0.7, 1.3), 0.5),
                           "smooth_union", 0.8),
            R.CSGComposite(R.SDFCone((-0.4, 0.8, 1.2), 0.7, 1.6), R.SDFTorus((-0.4, 0.8, 1.2), 0.6, 0.2),
                           "difference"),
            R.CSGComposite(R.SDFPrism((1.1, 0.8, 1.2), (1.2, 1.6, 0.8)), R.SDFCapsule((1.3, 0.8, 1.4), 0.3, 0.8),
                           "smooth_difference", 0.15),
            R.CSGComposite(R.SDFSphere((2.8, 0.6, 1.3), 0.6), R.SDFTorus((2.8, 0.6, 1.3), 0.7, 0.15), "union"),
            R.CSGComposite(R.SDFBox((-1.0, 0.5, 2.9), (1.0, -0.4, 1.0)), R.SDFCapsule((-0.6, 0.5, 2.9), 0.4, -0.5),
                           "union"),
            R.CSGComposite(R.SDFSphere((1.0, 0.5, 2.9), 0.5), R.SDFSphere((1.5, 0.5, 2.9), 0.5), "smooth_union", 0.0)]
    objs = [Sphere((0.0, -1000.0, 0.0), 1000.0, LambertianMaterial(Color.rgb(0.2, 0.2, 0.2)))]
    objs += [SDFObject(s, ms[i % 3]) for i, s in enumerate(sdfs)]
    lights = [PointLight((-12.0, 1.2, 0.4), Color.rgb(1.0, 0.9, 0.8), 30.0),
              PointLight((0.3, 7.0, 0.6), Color.rgb(0.6, 0.7, 1.0), 12.0),
              DirectionalLight((1.0, -0.04, -0.25), Color.rgb(0.9, 0.9, 1.0), 0.5)]
    cam = Camera.new_perspective(to_radians(50.0), f32(w) / f32(h), 0.1, 100.0)
    cam.transform.position = vec3(0.8, 4.2, 8.0)
    cam.look_at((0.0, 0.8, 0.8))
    cfg = RaytracerConfig(max_depth=1, samples_per_pixel=1, width=w, height=h, jitter="center", mode=mode,
                          background_color=Color(0.05, 0.05, 0.08, 1))
    return objs, lights, cam, cfg
