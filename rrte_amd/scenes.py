"""The BASELINE.json scenes, built through the reference-shaped API.

basic_demo      examples/basic-demo/src/main.rs:174-257   (ground + 3 spheres, 2 point lights)
simple_demo     examples/simple-demo/src/main.rs:169-221  (ground + cube, 1 light)
advanced_demo   examples/advanced-demo/src/main.rs:238-322 (5 spheres + ground, 5 lights, dark bg)
sdf_showcase_literal  examples/sdf-showcase/src/main.rs:168-381 (the 17 analytic stand-ins, as written)
sdf_showcase    the same layout with real SDFs: 10 SL/advanced primitives + 6 CSG ops (build-defined
                parameters after README.md:212-244, 303-328)
deformation_stress  64-node CSG tree (32 leaves, 31 ops) under Bend -> Twist -> Noise

Each builder returns (objects, lights, camera, config) for `Raytracer.render`.
"""
from __future__ import annotations

import numpy as np

from .math import Color, f32, to_radians, vec3
from .renderer import (BendDeformer, Camera, Capsule, Cone, CSGComposite, Cube, Cylinder, DeformedSDF,
                       LambertianMaterial, NoiseDeformer, PointLight, RaytracerConfig, SDFBox, SDFCapsule,
                       SDFCone, SDFCylinder, SDFEllipsoid, SDFObject, SDFPrism, SDFRing, SDFSphere, SDFTorus,
                       SDFTube, Sphere, TwistDeformer)

SEED = 0x5EED2025


def _camera(width, height, position, target, fov_deg=45.0) -> Camera:
    # Engine::new: perspective fov 45deg, aspect = w/h (engine.rs:97-98); demos then set fov + look_at.
    cam = Camera.new_perspective(to_radians(45.0), f32(width) / f32(height), 0.1, 100.0)
    cam.fov = to_radians(fov_deg)
    cam.transform.position = vec3(position)
    cam.look_at(vec3(target), vec3(0, 1, 0))
    return cam


def _config(width, height, bg, mode, spp=1, max_depth=1, jitter="center"):
    return RaytracerConfig(max_depth=max_depth, samples_per_pixel=spp, width=width, height=height,
                           background_color=bg, mode=mode, jitter=jitter)


def basic_demo(width=640, height=480, mode="refcompat"):
    ground = LambertianMaterial(Color.rgb(0.5, 0.5, 0.5))
    red = LambertianMaterial(Color.rgb(0.7, 0.3, 0.3))
    blue = LambertianMaterial(Color.rgb(0.3, 0.3, 0.7))
    green = LambertianMaterial(Color.rgb(0.3, 0.7, 0.3))
    objects = [
        Sphere((0.0, -1000.0, 0.0), 1000.0, ground),
        Sphere((0.0, 1.0, 0.0), 1.0, red),
        Sphere((-2.5, 1.0, 0.0), 1.0, blue),
        Sphere((2.5, 1.0, 0.0), 1.0, green),
    ]
    lights = [PointLight((0.0, 5.0, 5.0), Color.rgb(1.0, 1.0, 1.0), 50.0),
              PointLight((-5.0, 3.0, -2.0), Color.rgb(0.8, 0.9, 1.0), 30.0)]
    cam = _camera(width, height, (6.0, 4.0, 6.0), (0.0, 1.0, 0.0), 45.0)
    return objects, lights, cam, _config(width, height, Color(0.5, 0.7, 1.0, 1.0), mode)


def simple_demo(width=640, height=480, mode="refcompat"):
    objects = [Sphere((0.0, -1000.0, 0.0), 1000.0, LambertianMaterial(Color.rgb(0.5, 0.5, 0.5))),
               Cube((0.0, 1.0, 0.0), (2.0, 2.0, 2.0), LambertianMaterial(Color.rgb(0.8, 0.3, 0.3)))]
    lights = [PointLight((5.0, 10.0, 5.0), Color.rgb(1.0, 1.0, 1.0), 50.0)]
    cam = _camera(width, height, (5.0, 3.0, 5.0), (0.0, 1.0, 0.0), 45.0)
    return objects, lights, cam, _config(width, height, Color(0.5, 0.7, 1.0, 1.0), mode)


def advanced_demo(width=1920, height=1080, mode="lambert_shadow"):
    mats = [LambertianMaterial(Color.rgb(*c)) for c in
            [(0.3, 0.05, 0.05), (0.05, 0.1, 0.3), (0.05, 0.2, 0.05), (0.2, 0.05, 0.2), (0.3, 0.15, 0.02)]]
    very_dark = LambertianMaterial(Color.rgb(0.1, 0.1, 0.1))
    spheres = [((-6.0, 1.0, 0.0), 1.2), ((-3.0, 1.0, 0.0), 0.8), ((0.0, 1.0, 0.0), 0.8), ((3.0, 1.0, 0.0), 0.9),
               ((6.0, 1.0, 0.0), 0.7)]
    objects = [Sphere(p, r, m) for (p, r), m in zip(spheres, mats)]
    objects.append(Sphere((0.0, -1000.0, 0.0), 1000.0, very_dark))
    lights = [PointLight(p, Color.rgb(*c), i) for p, c, i in [
        ((0.0, 8.0, 0.0), (0.2, 0.1, 0.4), 15.0),
        ((-8.0, 3.0, 4.0), (0.4, 0.1, 0.05), 12.0),
        ((8.0, 4.0, -4.0), (0.05, 0.2, 0.3), 10.0),
        ((-2.0, 1.5, -8.0), (0.1, 0.3, 0.05), 8.0),
        ((4.0, 6.0, 6.0), (0.3, 0.05, 0.3), 6.0)]]
    cam = _camera(width, height, (12.0, 6.0, 0.0), (0.0, 1.0, 0.0), 60.0)
    return objects, lights, cam, _config(width, height, Color(0.05, 0.05, 0.1, 1.0), mode)


def _showcase_lights():
    return [PointLight((-10.0, 15.0, 10.0), Color.rgb(1.0, 1.0, 1.0), 25.0),
            PointLight((10.0, 10.0, 15.0), Color.rgb(0.6, 0.7, 1.0), 15.0),
            PointLight((0.0, 5.0, -15.0), Color.rgb(1.0, 0.8, 0.6), 10.0)]


def sdf_showcase_literal(width=1920, height=1080, mode="refcompat"):
    """examples/sdf-showcase/src/main.rs:168-381 exactly as written (analytic stand-ins), in
    Scene::get_objects() order (add_sphere and add_object both append to `objects`)."""
    sl = LambertianMaterial(Color.rgb(0.2, 0.6, 0.9))
    adv = LambertianMaterial(Color.rgb(0.9, 0.4, 0.2))
    csg = LambertianMaterial(Color.rgb(0.6, 0.9, 0.3))
    ground = LambertianMaterial(Color.rgb(0.2, 0.2, 0.2))
    y = 2.0
    objects = [
        Sphere((0.0, -1000.0, 0.0), 1000.0, ground),
        Cube((-12.0, y, -8.0), (2.0, 2.0, 2.0), sl),
        Sphere((-8.0, y, -8.0), 1.2, sl),
        Cylinder((-4.0, y, -8.0), 1.0, 2.0, sl),
        Cube((0.0, y, -8.0), (1.5, 2.0, 1.0), sl),
        Sphere((4.0, y, -8.0), 1.0, sl),
        Sphere((8.0, y, -8.0), 1.0, sl),
        Sphere((12.0, y, -8.0), 1.0, sl),
        Cone((-8.0, y, 0.0), 1.2, 2.5, adv),
        Capsule((-4.0, y, 0.0), 0.8, 2.0, adv),
        Sphere((0.0, y, 0.0), 1.0, adv),
        Sphere((4.0, y, 0.0), 0.8, csg), Sphere((5.0, y, 0.0), 0.8, csg),
        Sphere((8.0, y, 0.0), 1.2, csg), Sphere((8.5, y, 0.0), 0.6, csg),
        Sphere((12.0, y, 0.0), 1.0, csg), Sphere((12.5, y, 0.0), 1.0, csg),
    ]
    cam = _camera(width, height, (0.0, 8.0, 20.0), (0.0, 2.0, 0.0), 45.0)
    return objects, _showcase_lights(), cam, _config(width, height, Color(0.05, 0.05, 0.08, 1.0), mode)


def sdf_showcase(width=1920, height=1080, mode="lambert_shadow"):
    """The sdf-showcase layout with real SDFs: 10 SL/advanced primitives (Box, Sphere, Cylinder,
    Prism, Torus, Tube, Ring, Cone, Capsule, Ellipsoid) + 6 CSG ops (Union, Difference,
    Intersection and their smooth forms, k = 0.3), each an SDFObject, over the analytic ground."""
    sl = LambertianMaterial(Color.rgb(0.2, 0.6, 0.9))
    adv = LambertianMaterial(Color.rgb(0.9, 0.4, 0.2))
    csg = LambertianMaterial(Color.rgb(0.6, 0.9, 0.3))
    ground = LambertianMaterial(Color.rgb(0.2, 0.2, 0.2))
    y = 2.0
    S = SDFSphere
    sdfs = [
        (SDFBox((-12.0, y, -8.0), (2.0, 2.0, 2.0)), sl),
        (SDFSphere((-8.0, y, -8.0), 1.2), sl),
        (SDFCylinder((-4.0, y, -8.0), 1.0, 2.0), sl),
        (SDFPrism((0.0, y, -8.0), (1.5, 2.0, 1.0)), sl),
        (SDFTorus((4.0, y, -8.0), 0.8, 0.3), sl),
        (SDFTube((8.0, y, -8.0), 1.0, 0.6, 1.5), sl),
        (SDFRing((12.0, y, -8.0), 0.8, 0.15), sl),
        (SDFCone((-8.0, y, 0.0), 1.2, 2.5), adv),
        (SDFCapsule((-4.0, y, 0.0), 0.8, 2.0), adv),
        (SDFEllipsoid((0.0, y, 0.0), (1.2, 0.8, 1.0)), adv),
        (CSGComposite.union(S((4.0, y, 0.0), 0.8), S((5.0, y, 0.0), 0.8)), csg),
        (CSGComposite.difference(S((8.0, y, 0.0), 1.2), S((8.5, y, 0.0), 0.6)), csg),
        (CSGComposite.intersection(S((12.0, y, 0.0), 1.0), S((12.5, y, 0.0), 1.0)), csg),
        (CSGComposite.smooth_union(S((4.0, y, 4.0), 0.8), S((5.0, y, 4.0), 0.8), 0.3), csg),
        (CSGComposite.smooth_difference(S((8.0, y, 4.0), 1.2), S((8.5, y, 4.0), 0.6), 0.3), csg),
        (CSGComposite.smooth_intersection(S((12.0, y, 4.0), 1.0), S((12.5, y, 4.0), 1.0), 0.3), csg),
    ]
    objects = [Sphere((0.0, -1000.0, 0.0), 1000.0, ground)] + [SDFObject(s, m) for s, m in sdfs]
    cam = _camera(width, height, (0.0, 8.0, 20.0), (0.0, 2.0, 0.0), 45.0)
    return objects, _showcase_lights(), cam, _config(width, height, Color(0.05, 0.05, 0.08, 1.0), mode)


def _balanced(leaves, ops):
    """Combine leaves pairwise into a balanced binary tree (value-stack depth <= log2(n)+1)."""
    level, k = list(leaves), 0
    while len(level) > 1:
        nxt = []
        for i in range(0, len(level) - 1, 2):
            op, kk = ops[k % len(ops)]
            k += 1
            nxt.append(CSGComposite(level[i], level[i + 1], op, kk))
        if len(level) % 2:
            nxt.append(level[-1])
        level = nxt
    return level[0], k


def deformation_stress(width=3840, height=2160, mode="lambert_shadow", seed=SEED):
    """32 SL leaves (16 overlapping pairs, uniform in [-10,10]x[0,6]x[-10,10],
    size 0.5-1.5) + 31 binary CSG ops: the 16 pair ops cycle all six CSG ops (k in [0.1, 0.5]),
    the 15 ops above them join the pairs with (smooth) unions; the tree sits under the root chain
    Bend(0.1) -> Twist(0.5 rad/unit) -> Noise(freq 2, amp 0.1, 4 octaves, persistence 0.5).
    63 CSG nodes + 3 deformers; march cap 256 steps, step scale 0.6, hit eps 1e-4*t."""
    rng = np.random.default_rng(seed)
    kinds = [SDFSphere, SDFBox, SDFCylinder, SDFTorus, SDFCapsule, SDFEllipsoid, SDFCone, SDFTube]

    def leaf(K, c, s):
        if K is SDFSphere:
            return K(c, s)
        if K is SDFBox:
            return K(c, (s * 1.6, s * 1.2, s * 1.4))
        if K is SDFEllipsoid:
            return K(c, (s, s * 0.7, s * 0.9))
        if K is SDFTorus:
            return K(c, s, s * 0.35)
        if K is SDFTube:
            return K(c, s, s * 0.6, s * 1.5)
        return K(c, s * 0.7, s * 1.8)  # cylinder, capsule, cone

    names = ["union", "smooth_union", "difference", "smooth_difference", "intersection", "smooth_intersection"]
    pairs = []
    for i in range(16):
        c = np.array([rng.uniform(-10, 10), rng.uniform(0.5, 5.5), rng.uniform(-10, 10)])
        s = rng.uniform(0.5, 1.5)
        off = rng.normal(size=3)
        off = off / np.linalg.norm(off) * s * rng.uniform(0.3, 0.8)
        a = leaf(kinds[(2 * i) % 8], tuple(c), s)
        b = leaf(kinds[(2 * i + 1) % 8], tuple(c + off), s * rng.uniform(0.5, 0.9))
        pairs.append(CSGComposite(a, b, names[i % 6], float(rng.uniform(0.1, 0.5))))
    joins = [("union", 0.0) if i % 2 == 0 else ("smooth_union", float(rng.uniform(0.1, 0.5))) for i in range(15)]
    tree, used = _balanced(pairs, joins)
    assert used == 15
    pivot = (0.0, 3.0, 0.0)
    deform = BendDeformer((0, 0, 1), (1, 0, 0), 0.1, pivot).chain(TwistDeformer((0, 1, 0), 0.5, pivot)) \
        .chain(NoiseDeformer(2.0, 0.1, pivot, seed=seed & 0xFFFF).with_octaves(4).with_persistence(0.5))
    obj = SDFObject(DeformedSDF(tree, deform), LambertianMaterial(Color.rgb(0.7, 0.5, 0.3)),
                    max_steps=256, step_scale=0.6, hit_eps=1e-4)
    objects = [Sphere((0.0, -1000.0, 0.0), 1000.0, LambertianMaterial(Color.rgb(0.2, 0.2, 0.2))), obj]
    cam = _camera(width, height, (0.0, 12.0, 26.0), (0.0, 2.0, 0.0), 45.0)
    return objects, _showcase_lights(), cam, _config(width, height, Color(0.05, 0.05, 0.08, 1.0), mode)


def mesh_demo(width=1920, height=1080, mode="lambert_shadow", detail=1.0):
    """Triangle meshes (§8f rank 4: MeshAsset-shaped data, RRTE_PRIM_MESH): a rolling heightfield
    terrain, an icosphere, a torus and a second icosphere over the analytic ground sphere, lit by
    the sdf-showcase lights.  `detail` scales the triangle counts (1.0: ~60 K triangles)."""
    from .mesh import heightfield, icosphere, torus
    n = max(8, int(129 * detail ** 0.5))
    terrain = heightfield((-12.0, 0.0, -12.0), 24.0, n,
                          lambda x, z: 0.6 * np.sin(0.45 * x) * np.cos(0.35 * z) + 0.25 * np.sin(1.3 * x + 0.7 * z),
                          LambertianMaterial(Color.rgb(0.45, 0.55, 0.35)))
    sub = 4 if detail >= 0.5 else 2
    ball = icosphere((-3.0, 2.2, 0.5), 1.6, sub, LambertianMaterial(Color.rgb(0.8, 0.35, 0.3)))
    ring = torus((3.0, 2.0, -1.0), 1.6, 0.5, max(12, int(128 * detail ** 0.5)), max(8, int(64 * detail ** 0.5)),
                 LambertianMaterial(Color.rgb(0.3, 0.5, 0.85)))
    small = icosphere((0.5, 1.4, 3.0), 0.9, sub - 1, LambertianMaterial(Color.rgb(0.85, 0.8, 0.4)))
    objects = [Sphere((0.0, -1000.0, 0.0), 1000.0, LambertianMaterial(Color.rgb(0.2, 0.2, 0.2))),
               terrain, ball, ring, small]
    cam = _camera(width, height, (0.0, 8.0, 16.0), (0.0, 1.5, 0.0), 45.0)
    return objects, _showcase_lights(), cam, _config(width, height, Color(0.05, 0.05, 0.08, 1.0), mode)


SCENES = {
    "basic-demo": basic_demo,
    "simple-demo": simple_demo,
    "advanced-demo": advanced_demo,
    "sdf-showcase-literal": sdf_showcase_literal,
    "sdf-showcase": sdf_showcase,
    "deformation-stress": deformation_stress,
    "mesh-demo": mesh_demo,
}


def animate_values(sc, f):
    """Frame f of a value-only animation of a lowered scene (rrte_amd.LoweredScene), in place: every
    SDF leaf moves in x and z, every smooth op's k grows, every light moves down and dims, every
    material's red channel rises -- the topology (object kinds, SDF structure, light kinds) stays, so
    one topology-specialised kernel serves every frame (the reference re-renders after
    scene_mut().update(dt) every frame, examples/sdf-showcase/src/main.rs:133-139)."""
    import numpy as np
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
    return sc
