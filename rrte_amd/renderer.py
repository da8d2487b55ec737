"""Host-side mirror of rrte-renderer's public surface (Melthizar/RRTE
crates/rrte-renderer/src/*.rs and the README-only SDF/CSG/Deformer API),
lowering a scene to the POD IR of include/rrte_hip.h and rendering it through
librrte_hip.so.  Names, argument meanings and defaults follow the reference;
file:line citations are relative to the reference root.

`Raytracer.render` is the drop-in for `Raytracer::render`
(raytracer.rs:45-89): same inputs, RGBA8 row-major output.  There is no CPU
path behind it.
"""
from __future__ import annotations

import ctypes as C
import itertools
import math
import os
from dataclasses import dataclass, field

import numpy as np

from . import abi
from .math import (NEG_Z, ONE, ZERO, Color, Transform, f32, normalize, quat_from_rotation_arc, sub, to_radians,
                   vec3)

# ===================================================================== materials
class Material:
    """Material trait (material.rs:5-19)."""
    kind = abi.MAT_LAMBERTIAN

    def albedo(self) -> Color:
        raise NotImplementedError

    def ambient_color(self) -> Color:  # material.rs:10-12
        a = self.albedo()
        return Color(a.r * f32(0.1), a.g * f32(0.1), a.b * f32(0.1), a.a * f32(0.1))

    def lower(self) -> abi.Material:
        m = abi.Material()
        m.kind = self.kind
        m.albedo[:] = list(self.albedo().as_tuple())
        m.fuzz = float(getattr(self, "roughness", 0.0))
        m.ior = float(getattr(self, "ior", 1.0))
        return m


class LambertianMaterial(Material):  # material.rs:45-81
    kind = abi.MAT_LAMBERTIAN

    def __init__(self, albedo: Color):
        self._albedo = albedo

    @staticmethod
    def new(albedo: Color) -> "LambertianMaterial":
        return LambertianMaterial(albedo)

    def albedo(self) -> Color:
        return self._albedo


class MetalMaterial(Material):  # material.rs:85-120
    kind = abi.MAT_METAL

    def __init__(self, albedo: Color, roughness: float):
        self._albedo = albedo
        self.roughness = f32(min(max(roughness, 0.0), 1.0))

    def albedo(self) -> Color:
        return self._albedo


class DielectricMaterial(Material):  # material.rs:124-183
    kind = abi.MAT_DIELECTRIC

    def __init__(self, ior: float, color: Color | None = None):
        self.ior = f32(ior)
        self.color = color if color is not None else Color.WHITE

    @staticmethod
    def with_color(ior: float, color: Color) -> "DielectricMaterial":
        return DielectricMaterial(ior, color)

    def albedo(self) -> Color:
        return self.color


class EmissiveMaterial(Material):  # material.rs:187-213
    kind = abi.MAT_EMISSIVE

    def __init__(self, color: Color, intensity: float):
        self.color = color
        self.intensity = f32(intensity)

    def albedo(self) -> Color:
        return self.color


# ======================================================================== lights
class Light:
    """Light trait (light.rs:5-26)."""
    transform: Transform

    def lower(self) -> abi.Light:
        raise NotImplementedError


def _light_struct(kind, color, intensity, position=ZERO, direction=ZERO, rng=100.0, lin=0.09, quad=0.032,
                  inner=0.0, outer=0.0) -> abi.Light:
    l = abi.Light()
    l.kind = kind
    l.intensity = float(intensity)
    l.range = float(rng)
    l.linear = float(lin)
    l.quadratic = float(quad)
    l.inner_angle = float(inner)
    l.outer_angle = float(outer)
    l.position[:] = [*vec3(position), 0.0]
    l.direction[:] = [*vec3(direction), 0.0]
    l.color[:] = list(color.as_tuple())
    return l


class PointLight(Light):  # light.rs:123-220
    def __init__(self, position, color: Color, intensity: float):
        self.position = vec3(position)
        self.color = color
        self.intensity = f32(intensity)
        self.range = f32(100.0)
        self.linear_attenuation = f32(0.09)
        self.quadratic_attenuation = f32(0.032)
        self.transform = Transform.identity()

    @staticmethod
    def new(position, color, intensity) -> "PointLight":
        return PointLight(position, color, intensity)

    @staticmethod
    def with_attenuation(position, color, intensity, rng, linear, quadratic) -> "PointLight":
        l = PointLight(position, color, intensity)
        l.range, l.linear_attenuation, l.quadratic_attenuation = f32(rng), f32(linear), f32(quadratic)
        return l

    def lower(self):
        return _light_struct(abi.LIGHT_POINT, self.color, self.intensity, position=self.position, rng=self.range,
                             lin=self.linear_attenuation, quad=self.quadratic_attenuation)


class DirectionalLight(Light):  # light.rs:57-121
    def __init__(self, direction, color: Color, intensity: float):
        self.direction = normalize(vec3(direction))
        self.color = color
        self.intensity = f32(intensity)
        self.transform = Transform.identity()

    @staticmethod
    def sun() -> "DirectionalLight":
        return DirectionalLight(normalize(vec3(-0.3, -1.0, -0.3)), Color(1.0, 0.95, 0.8, 1.0), 5.0)

    def lower(self):
        return _light_struct(abi.LIGHT_DIRECTIONAL, self.color, self.intensity, direction=self.direction)


class SpotLight(Light):  # light.rs:222-338
    def __init__(self, position, direction, color: Color, intensity: float, inner_angle: float, outer_angle: float):
        self.position = vec3(position)
        self.direction = normalize(vec3(direction))
        self.color = color
        self.intensity = f32(intensity)
        self.range = f32(100.0)
        self.inner_angle = f32(inner_angle)
        self.outer_angle = f32(outer_angle)
        self.linear_attenuation = f32(0.09)
        self.quadratic_attenuation = f32(0.032)
        self.transform = Transform.identity()

    def lower(self):
        return _light_struct(abi.LIGHT_SPOT, self.color, self.intensity, position=self.position,
                             direction=self.direction, rng=self.range, lin=self.linear_attenuation,
                             quad=self.quadratic_attenuation, inner=self.inner_angle, outer=self.outer_angle)


class AmbientLight(Light):  # light.rs:340-397
    def __init__(self, color: Color, intensity: float):
        self.color = color
        self.intensity = f32(intensity)
        self.transform = Transform.identity()

    @staticmethod
    def default_ambient() -> "AmbientLight":
        return AmbientLight(Color(0.2, 0.2, 0.3, 1.0), 0.3)

    def lower(self):
        return _light_struct(abi.LIGHT_AMBIENT, self.color, self.intensity)


# ======================================================================== camera
@dataclass
class Camera:
    """rrte_renderer::Camera (camera.rs:24-31) with ProjectionType (camera.rs:5-20)."""
    transform: Transform = field(default_factory=Transform.identity)
    projection: str = "perspective"
    fov: float = 0.0
    aspect_ratio: float = 1.0
    near: float = 0.1
    far: float = 100.0
    left: float = -1.0
    right: float = 1.0
    bottom: float = -1.0
    top: float = 1.0
    is_active: bool = True

    @staticmethod
    def new_perspective(fov, aspect_ratio, near, far) -> "Camera":
        return Camera(projection="perspective", fov=f32(fov), aspect_ratio=f32(aspect_ratio), near=f32(near),
                      far=f32(far))

    @staticmethod
    def new_orthographic(left, right, bottom, top, near, far) -> "Camera":
        return Camera(projection="orthographic", left=f32(left), right=f32(right), bottom=f32(bottom),
                      top=f32(top), near=f32(near), far=f32(far))

    def look_at(self, target, up=(0.0, 1.0, 0.0)):
        """camera.rs:85-95: rotation = Quat::from_rotation_arc(-Z, normalize(target - position)); `up` unused."""
        fwd = normalize(sub(vec3(target), self.transform.position))
        self.transform.rotation = quat_from_rotation_arc(NEG_Z, fwd)

    def lower(self) -> abi.Camera:
        c = abi.Camera()
        c.position[:] = list(self.transform.position)
        c.rotation[:] = list(self.transform.rotation)
        c.scale[:] = list(self.transform.scale)
        c.projection = abi.PERSPECTIVE if self.projection == "perspective" else abi.ORTHOGRAPHIC
        c.fov, c.aspect_ratio, c.near_plane, c.far_plane = self.fov, self.aspect_ratio, self.near, self.far
        c.left, c.right, c.bottom, c.top = self.left, self.right, self.bottom, self.top
        return c


# ================================================================ scene objects
class SceneObject:
    """SceneObject trait (primitives.rs:6-18)."""
    material: Material | None = None
    transform: Transform

    def set_material(self, material: Material):
        self.material = material

    def set_transform(self, transform: Transform):
        self.transform = transform

    def _prim(self, kind: int, params) -> abi.Prim:
        p = abi.Prim()
        p.kind = kind
        vals = [float(v) for v in params]
        p.p[: len(vals)] = vals
        p.trs[:] = [float(v) for v in self.transform.trs()]
        return p

    def lower(self, lowering: "_Lowering") -> abi.Prim:
        raise NotImplementedError


class Sphere(SceneObject):  # primitives.rs:20-94
    def __init__(self, center, radius, material: Material | None = None):
        self.center, self.radius, self.material = vec3(center), f32(radius), material
        self.transform = Transform.identity()

    @staticmethod
    def with_material(center, radius, material) -> "Sphere":
        return Sphere(center, radius, material)

    def lower(self, lw):
        return self._prim(abi.PRIM_SPHERE, [*self.center, self.radius])


class Plane(SceneObject):  # primitives.rs:96-161
    def __init__(self, point, normal, material: Material | None = None):
        self.point, self.normal, self.material = vec3(point), normalize(vec3(normal)), material
        self.transform = Transform.identity()

    @staticmethod
    def with_material(point, normal, material) -> "Plane":
        return Plane(point, normal, material)

    def lower(self, lw):
        return self._prim(abi.PRIM_PLANE, [*self.point, 0.0, *self.normal])


class Triangle(SceneObject):  # primitives.rs:163-257
    def __init__(self, v0, v1, v2, material: Material | None = None):
        v0, v1, v2 = vec3(v0), vec3(v1), vec3(v2)
        from .math import cross
        n = normalize(cross(sub(v1, v0), sub(v2, v0)))
        self.vertices, self.normals, self.material = [v0, v1, v2], [n, n, n], material
        self.transform = Transform.identity()

    @staticmethod
    def with_material(v0, v1, v2, material) -> "Triangle":
        return Triangle(v0, v1, v2, material)

    def set_normals(self, n0, n1, n2):
        self.normals = [normalize(vec3(n0)), normalize(vec3(n1)), normalize(vec3(n2))]

    def lower(self, lw):
        return self._prim(abi.PRIM_TRIANGLE, [c for v in self.vertices + self.normals for c in v])


class Cube(SceneObject):  # primitives.rs:259-377
    def __init__(self, center, size, material: Material | None = None):
        self.center, self.size, self.material = vec3(center), vec3(size), material
        self.transform = Transform.identity()

    @staticmethod
    def with_material(center, size, material) -> "Cube":
        return Cube(center, size, material)

    @staticmethod
    def unit() -> "Cube":
        return Cube(ZERO, ONE)

    def lower(self, lw):
        return self._prim(abi.PRIM_CUBE, [*self.center, 0.0, *self.size])


class _RadialPrim(SceneObject):
    KIND = -1

    def __init__(self, center, radius, height, material: Material | None = None):
        self.center, self.radius, self.height, self.material = vec3(center), f32(radius), f32(height), material
        self.transform = Transform.identity()

    @classmethod
    def with_material(cls, center, radius, height, material):
        return cls(center, radius, height, material)

    def lower(self, lw):
        return self._prim(self.KIND, [*self.center, self.radius, self.height])


class Cylinder(_RadialPrim):  # primitives.rs:379-478
    KIND = abi.PRIM_CYLINDER


class Cone(_RadialPrim):  # primitives.rs:480-584
    KIND = abi.PRIM_CONE


class Capsule(_RadialPrim):  # primitives.rs:586-738
    KIND = abi.PRIM_CAPSULE


# ===================================================== SDF / CSG / deformers
# README.md:458-510 gives only signatures; formulas are build-defined
#  and frozen by tests/golden fixtures.

def _axis_index(axis) -> int:
    a = vec3(axis)
    for i in range(3):
        if abs(float(a[i])) == 1.0 and all(float(a[j]) == 0.0 for j in range(3) if j != i):
            return i
    raise abi.RrteError(abi.RRTE_UNSUPPORTED_PRIM, f"deformer axis {axis} must be a coordinate axis")


def _node(op, f=(), i=()) -> abi.SdfNode:
    n = abi.SdfNode()
    n.op = op
    fv = [float(v) for v in f]
    n.f[: len(fv)] = fv
    iv = [int(v) for v in i]
    n.i[: len(iv)] = iv
    return n


def _merge(b1, b2):
    (c1, r1), (c2, r2) = b1, b2
    d = math.dist(c1, c2)
    if d + r2 <= r1:
        return b1
    if d + r1 <= r2:
        return b2
    r = (d + r1 + r2) * 0.5
    t = (r - r1) / d if d > 0 else 0.0
    c = tuple(c1[k] + (c2[k] - c1[k]) * t for k in range(3))
    return (c, r)


class SDF:
    """SDF trait (README.md:458-467): distance / material_at / intersect.  Here
    an SDF lowers to a postfix node program plus a conservative bounding sphere."""

    def emit(self, out: list):
        raise NotImplementedError

    def bound(self):
        """(center, radius) of a sphere containing the zero set."""
        raise NotImplementedError

    def has_deformer(self) -> bool:
        return False


class _Leaf(SDF):
    OP = 0

    def __init__(self, center, *params, material: Material | None = None):
        self.center = vec3(center)
        self.params = params
        self.material = material

    @classmethod
    def with_material(cls, center, *params):
        *params, material = params
        return cls(center, *params, material=material)

    def floats(self):
        raise NotImplementedError

    def emit(self, out):
        out.append(_node(self.OP, self.floats()))


class SDFSphere(_Leaf):
    OP = abi.SDF_SPHERE

    def floats(self):
        return [*self.center, self.params[0]]

    def bound(self):
        return (tuple(map(float, self.center)), float(self.params[0]))


class SDFBox(_Leaf):  # size = full extents, like Cube
    OP = abi.SDF_BOX

    def floats(self):
        return [*self.center, 0.0, *vec3(self.params[0])]

    def bound(self):
        s = vec3(self.params[0])
        return (tuple(map(float, self.center)), 0.5 * math.sqrt(sum(float(v) ** 2 for v in s)))


class SDFCylinder(_Leaf):  # (radius, height), Y axis
    OP = abi.SDF_CYLINDER

    def floats(self):
        return [*self.center, self.params[0], self.params[1]]

    def bound(self):
        r, h = map(float, self.params[:2])
        return (tuple(map(float, self.center)), math.hypot(r, h * 0.5))


class SDFPrism(_Leaf):  # size: triangle in XY (size.y = triangle size), depth size.z
    OP = abi.SDF_PRISM

    def floats(self):
        return [*self.center, 0.0, *vec3(self.params[0])]

    def bound(self):
        s = [float(v) for v in vec3(self.params[0])]
        # |x|*0.866 + y*0.5 <= sy/4 and -y <= sy/4: the triangle spans y in [-sy/4, sy/2], |x| <= sy*0.433
        return (tuple(map(float, self.center)), math.sqrt((s[1] * 0.5) ** 2 + (s[1] * 0.433) ** 2 + (s[2] * 0.5) ** 2))


class SDFTorus(_Leaf):  # (major, minor), ring in XZ
    OP = abi.SDF_TORUS

    def floats(self):
        return [*self.center, self.params[0], self.params[1]]

    def bound(self):
        return (tuple(map(float, self.center)), float(self.params[0]) + float(self.params[1]))


class SDFTube(_Leaf):  # (outer, inner, height)
    OP = abi.SDF_TUBE

    def floats(self):
        return [*self.center, self.params[0], self.params[1], self.params[2]]

    def bound(self):
        ro, ri, h = map(float, self.params[:3])
        return (tuple(map(float, self.center)), math.hypot(ro, h * 0.5))


class SDFRing(_Leaf):  # (major, minor), standing ring in XY
    OP = abi.SDF_RING

    def floats(self):
        return [*self.center, self.params[0], self.params[1]]

    def bound(self):
        return (tuple(map(float, self.center)), float(self.params[0]) + float(self.params[1]))


class SDFCone(_Leaf):  # (radius, height), apex +Y
    OP = abi.SDF_CONE

    def floats(self):
        return [*self.center, self.params[0], self.params[1]]

    def bound(self):
        r, h = map(float, self.params[:2])
        return (tuple(map(float, self.center)), math.hypot(r, h * 0.5))


class SDFCapsule(_Leaf):  # (radius, height)
    OP = abi.SDF_CAPSULE

    def floats(self):
        return [*self.center, self.params[0], self.params[1]]

    def bound(self):
        r, h = map(float, self.params[:2])
        return (tuple(map(float, self.center)), h * 0.5 + r)


class SDFEllipsoid(_Leaf):  # radii (x, y, z)
    OP = abi.SDF_ELLIPSOID

    def floats(self):
        return [*self.center, 0.0, *vec3(self.params[0])]

    def bound(self):
        return (tuple(map(float, self.center)), max(float(v) for v in vec3(self.params[0])))


_CSG_OPS = {
    "union": abi.SDF_UNION, "difference": abi.SDF_DIFFERENCE, "intersection": abi.SDF_INTERSECTION,
    "smooth_union": abi.SDF_SMOOTH_UNION, "smooth_difference": abi.SDF_SMOOTH_DIFFERENCE,
    "smooth_intersection": abi.SDF_SMOOTH_INTERSECTION,
}


class CSGComposite(SDF):
    """CSGOperation (README.md:475-482) applied to two SDFs."""

    def __init__(self, a: SDF, b: SDF, op: str, k: float = 0.0):
        if op not in _CSG_OPS:
            raise ValueError(op)
        self.a, self.b, self.op, self.k = a, b, op, f32(k)

    union = staticmethod(lambda a, b: CSGComposite(a, b, "union"))
    difference = staticmethod(lambda a, b: CSGComposite(a, b, "difference"))
    intersection = staticmethod(lambda a, b: CSGComposite(a, b, "intersection"))
    smooth_union = staticmethod(lambda a, b, k: CSGComposite(a, b, "smooth_union", k))
    smooth_difference = staticmethod(lambda a, b, k: CSGComposite(a, b, "smooth_difference", k))
    smooth_intersection = staticmethod(lambda a, b, k: CSGComposite(a, b, "smooth_intersection", k))

    def emit(self, out):
        self.a.emit(out)
        self.b.emit(out)
        out.append(_node(_CSG_OPS[self.op], [self.k]))

    def bound(self):
        ba, bb = self.a.bound(), self.b.bound()
        k = abs(float(self.k))
        if self.op in ("union", "smooth_union"):
            c, r = _merge(ba, bb)
        elif self.op in ("difference", "smooth_difference"):
            c, r = ba
        else:
            c, r = ba if ba[1] <= bb[1] else bb
        return (c, r + k)

    def has_deformer(self):
        return self.a.has_deformer() or self.b.has_deformer()


class Deformer:
    """Deformer trait (README.md:496-502): deform(point) -> point, chainable."""
    pivot = (0.0, 0.0, 0.0)

    def nodes(self) -> list:
        raise NotImplementedError

    def grow(self, c, r):
        """Bound of the deformed shape given the undeformed bound (c, r)."""
        raise NotImplementedError

    def chain(self, other: "Deformer") -> "ChainDeformer":
        return ChainDeformer([self, other])


class ChainDeformer(Deformer):
    def __init__(self, parts):
        self.parts = []
        for p in parts:
            self.parts.extend(p.parts if isinstance(p, ChainDeformer) else [p])

    def chain(self, other):
        return ChainDeformer(self.parts + [other])

    def nodes(self):
        return [n for p in self.parts for n in p.nodes()]

    def grow(self, c, r):
        # the deformed zero set is the preimage through d1 then d2 ...: grow innermost-first
        for p in reversed(self.parts):
            c, r = p.grow(c, r)
        return c, r


def _about_pivot(pivot, c, r):
    d = math.dist(tuple(map(float, pivot)), tuple(map(float, c)))
    return tuple(map(float, pivot)), d + r


class TwistDeformer(Deformer):  # rotate the plane normal to `axis` by rate * q[axis]
    def __init__(self, axis, rate, pivot=ZERO):
        self.axis, self.rate, self.pivot = _axis_index(axis), f32(rate), vec3(pivot)

    def nodes(self):
        return [_node(abi.SDF_TWIST, [*self.pivot, self.rate], [self.axis])]

    def grow(self, c, r):
        return _about_pivot(self.pivot, c, r)


class BendDeformer(Deformer):  # rotate the plane normal to `axis` by amount * q[direction]
    def __init__(self, axis, direction, amount, pivot=ZERO):
        self.axis, self.direction, self.amount = _axis_index(axis), _axis_index(direction), f32(amount)
        self.pivot = vec3(pivot)

    def nodes(self):
        return [_node(abi.SDF_BEND, [*self.pivot, self.amount], [self.axis, self.direction])]

    def grow(self, c, r):
        return _about_pivot(self.pivot, c, r)


class TaperDeformer(Deformer):  # scale across `axis` from `start` to `end` over `length`
    def __init__(self, axis, start, end, length, pivot=ZERO):
        self.axis, self.start, self.end, self.length = _axis_index(axis), f32(start), f32(end), f32(length)
        self.pivot = vec3(pivot)

    def nodes(self):
        return [_node(abi.SDF_TAPER, [*self.pivot, self.start, self.end, self.length], [self.axis])]

    def grow(self, c, r):
        pc, pr = _about_pivot(self.pivot, c, r)
        return pc, pr * max(1.0, abs(float(self.start)), abs(float(self.end)))


class NoiseDeformer(Deformer):  # p + amplitude * fbm3(frequency * (p - pivot))
    def __init__(self, frequency, amplitude, pivot=ZERO, seed=0):
        self.frequency, self.amplitude, self.pivot = f32(frequency), f32(amplitude), vec3(pivot)
        self.octaves, self.persistence, self.seed = 1, f32(0.5), int(seed)

    def with_octaves(self, n):
        if n > abi.SDF_MAX_OCTAVES:
            raise ValueError(f"octaves <= {abi.SDF_MAX_OCTAVES}")
        self.octaves = int(n)
        return self

    def with_persistence(self, p):
        self.persistence = f32(p)
        return self

    def nodes(self):
        return [_node(abi.SDF_NOISE, [*self.pivot, self.frequency, self.amplitude, self.persistence],
                      [self.octaves, self.seed])]

    def grow(self, c, r):
        total = sum(abs(float(self.persistence)) ** o for o in range(self.octaves))
        return c, r + math.sqrt(3.0) * abs(float(self.amplitude)) * total


class WaveDeformer(Deformer):  # q[displaced] += amplitude * sin(frequency * q[axis])
    def __init__(self, axis, amplitude, frequency, displaced_axis=None, pivot=ZERO):
        self.axis = _axis_index(axis)
        self.displaced = (self.axis + 1) % 3 if displaced_axis is None else _axis_index(displaced_axis)
        self.amplitude, self.frequency, self.pivot = f32(amplitude), f32(frequency), vec3(pivot)

    def nodes(self):
        return [_node(abi.SDF_WAVE, [*self.pivot, self.amplitude, self.frequency], [self.axis, self.displaced])]

    def grow(self, c, r):
        return c, r + abs(float(self.amplitude))


class DeformedSDF(SDF):
    def __init__(self, sdf: SDF, deformer: Deformer):
        self.sdf, self.deformer = sdf, deformer

    def emit(self, out):
        nodes = self.deformer.nodes()
        out.extend(nodes)
        self.sdf.emit(out)
        out.extend(_node(abi.SDF_POP_POINT) for _ in nodes)

    def bound(self):
        c, r = self.sdf.bound()
        return self.deformer.grow(c, r)

    def has_deformer(self):
        return True


class SDFObject(SceneObject):
    """A SceneObject whose intersect sphere-traces an SDF (README.md:458-467,
    'ray marching with adaptive stepping')."""

    def __init__(self, sdf: SDF, material: Material | None = None, max_steps: int = 128,
                 step_scale: float | None = None, hit_eps: float = 1e-4):
        self.sdf, self.material = sdf, material
        self.max_steps = int(max_steps)
        self.step_scale = f32(step_scale if step_scale is not None else (0.6 if sdf.has_deformer() else 1.0))
        self.hit_eps = f32(hit_eps)
        self.transform = Transform.identity()

    @staticmethod
    def with_material(sdf, material) -> "SDFObject":
        return SDFObject(sdf, material)

    def lower(self, lw):
        nodes = []
        self.sdf.emit(nodes)
        c, r = self.sdf.bound()
        r = r * 1.001 + 1e-3
        p = self._prim(abi.PRIM_SDF, [c[0], c[1], c[2], r])
        p.sdf_first = len(lw.nodes)
        p.sdf_count = len(nodes)
        p.sdf_max_steps = self.max_steps
        p.sdf_step_scale = float(self.step_scale)
        p.sdf_hit_eps = float(self.hit_eps)
        lw.nodes.extend(nodes)
        return p


# ===================================================================== renderer
@dataclass
class RaytracerConfig:
    """RaytracerConfig (raytracer.rs:8-26) + the build-defined knobs of this path."""
    max_depth: int = 50
    samples_per_pixel: int = 100
    width: int = 800
    height: int = 600
    background_color: Color = field(default_factory=lambda: Color(0.5, 0.7, 1.0, 1.0))
    mode: str = "refcompat"          # "refcompat" (raytracer.rs:92-148) | "lambert_shadow"
    jitter: str = "random"           # "random" (raytracer.rs:67-68) | "center" (deterministic)
    seed: int = 0
    t_min: float = 0.001             # raytracer.rs:107
    shadow_bias: float = 1e-3
    gamma: float = 2.2               # raytracer.rs:79
    band_rows: int = 16              # multi-GPU row-band height

    def lower(self) -> abi.RenderParams:
        p = abi.RenderParams()
        p.width, p.height = self.width, self.height
        p.samples_per_pixel, p.max_depth = self.samples_per_pixel, self.max_depth
        p.mode = {"refcompat": abi.MODE_REFCOMPAT, "lambert_shadow": abi.MODE_LAMBERT_SHADOW}[self.mode]
        p.jitter = {"random": abi.JITTER_RANDOM, "center": abi.JITTER_CENTER}[self.jitter]
        p.seed = self.seed & 0xFFFFFFFF
        p.background[:] = list(self.background_color.as_tuple())
        p.t_min, p.shadow_bias, p.gamma = self.t_min, self.shadow_bias, self.gamma
        p.band_rows = self.band_rows
        return p


_MESH_VERSION = itertools.count(1)


class _Lowering:
    def __init__(self):
        self.nodes: list = []
        self.materials: list = []
        self._mat_index: dict = {}
        self.mesh_pos: list = []      # per mesh: (N, 3) float32
        self.mesh_nrm: list = []
        self.mesh_idx: list = []      # per mesh: (M, 3) uint32, offset into the shared vertex pool
        self._nverts = 0
        self._ntris = 0

    def add_mesh(self, pos, nrm, idx):
        """Append a mesh to the shared pools; returns (first triangle, triangle count)."""
        first = self._ntris
        self.mesh_pos.append(pos)
        self.mesh_nrm.append(nrm)
        self.mesh_idx.append(idx.astype(np.uint32) + np.uint32(self._nverts))
        self._nverts += len(pos)
        self._ntris += len(idx)
        return first, len(idx)

    def material_index(self, m: Material | None) -> int:
        if m is None:
            return -1
        k = id(m)  # dedupe by identity, like the Arc-pointer dedupe of gpu_renderer.rs:483-523
        if k not in self._mat_index:
            self._mat_index[k] = len(self.materials)
            self.materials.append(m)
        return self._mat_index[k]


class LoweredScene:
    """A scene lowered to include/rrte_hip.h's rrte_scene_ir (keeps the arrays alive)."""

    def __init__(self, objects, lights, camera: Camera):
        lw = _Lowering()
        prims = []
        for o in objects:
            p = o.lower(lw)
            p.material = lw.material_index(o.material)
            prims.append(p)
        self.prims = (abi.Prim * max(1, len(prims)))(*prims)
        mats = [m.lower() for m in lw.materials]
        self.mats = (abi.Material * max(1, len(mats)))(*mats)
        lts = [l.lower() for l in lights]
        self.lights = (abi.Light * max(1, len(lts)))(*lts)
        self.nodes = (abi.SdfNode * max(1, len(lw.nodes)))(*lw.nodes)
        ir = abi.SceneIR()
        ir.prims, ir.num_prims = self.prims, len(prims)
        ir.materials, ir.num_materials = self.mats, len(mats)
        ir.lights, ir.num_lights = self.lights, len(lts)
        ir.sdf_nodes, ir.num_sdf_nodes = self.nodes, len(lw.nodes)
        ir.camera = camera.lower()
        if lw.mesh_pos:
            vtx = np.concatenate([np.concatenate([p, n], axis=1) for p, n in zip(lw.mesh_pos, lw.mesh_nrm)])
            self._mesh_vtx = np.ascontiguousarray(vtx, dtype=np.float32)
            self._mesh_idx = np.ascontiguousarray(np.concatenate(lw.mesh_idx).reshape(-1), dtype=np.uint32)
            ir.mesh_vertices = self._mesh_vtx.ctypes.data_as(C.POINTER(abi.MeshVertex))
            ir.num_mesh_vertices = len(self._mesh_vtx)
            ir.mesh_indices = self._mesh_idx.ctypes.data_as(C.POINTER(C.c_uint32))
            ir.num_mesh_indices = len(self._mesh_idx)
            ir.mesh_version = next(_MESH_VERSION)  # arrays are immutable for this object's lifetime
        self.ir = ir

    def ref(self):
        return C.byref(self.ir)


class Context:
    """Owns one rrte_ctx (one HIP device, its stream and HBM scene cache)."""

    def __init__(self, device: int | None = None, jit: int | None = None):
        self.lib = abi.load()
        if device is None:
            device = int(os.environ.get("RRTE_HIP_DEVICE", "0"))
        h = C.c_void_p()
        st = self.lib.rrte_hip_create(device, C.byref(h))
        if st != abi.RRTE_OK:
            raise abi.RrteError(st, f"rrte_hip_create(device={device}) failed")
        self.h = h
        if jit is not None:
            self.check(self.lib.rrte_hip_set_jit(self.h, int(jit)))

    def check(self, st):
        if st != abi.RRTE_OK:
            raise abi.RrteError(st, self.lib.rrte_hip_last_error(self.h).decode())

    def stats(self) -> abi.Stats:
        s = abi.Stats()
        self.check(self.lib.rrte_hip_stats(self.h, C.byref(s)))
        return s

    def close(self):
        if self.h:
            self.lib.rrte_hip_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Raytracer:
    """Raytracer (raytracer.rs:28-149), rendering on an MI355X."""

    def __init__(self, config: RaytracerConfig | None = None, device: int | None = None, jit: int | None = None):
        """jit: abi.JIT_OFF / JIT_ON / JIT_AUTO (None = library default, AUTO)."""
        self.config = config or RaytracerConfig()
        self._device = device
        self._jit = jit
        self._ctx: Context | None = None

    @staticmethod
    def new(config: RaytracerConfig) -> "Raytracer":
        return Raytracer(config)

    def update_config(self, new_config: RaytracerConfig):
        self.config = new_config

    @property
    def ctx(self) -> Context:
        if self._ctx is None:
            self._ctx = Context(self._device, self._jit)
        return self._ctx

    def render(self, objects, lights, materials, camera: Camera) -> np.ndarray:
        """raytracer.rs:45-89: returns W*H*4 RGBA8 bytes, row-major, row 0 = top."""
        out, _ = self.render_f32(objects, lights, materials, camera, want_f32=False)
        return out

    def render_into(self, objects, lights, materials, camera: Camera, out: np.ndarray) -> np.ndarray:
        """Engine::render_frame's loop (engine.rs:82,293; rust/patches/0002): the frame into the
        caller's buffer, reused every frame and pinned once (rrte_hip_host_register) so the kernel
        stores the frame straight into it -- the boundary's fast path.  `out` is a C-contiguous
        uint8 array of W*H*4 bytes (the caller keeps it alive until it passes another buffer or the
        context closes; a different buffer unpins this one first).  A buffer that cannot be pinned
        (one of its pages already pinned elsewhere) takes the copy path.  Returns `out`."""
        cfg = self.config
        need = cfg.width * cfg.height * 4
        if out.dtype != np.uint8 or out.size != need or not out.flags.c_contiguous:
            raise ValueError(f"render_into needs a C-contiguous uint8 buffer of {need} bytes")
        ctx = self.ctx
        addr = out.ctypes.data
        pinned = getattr(self, "_pinned", None)
        if pinned is not None and pinned != (addr, need):
            ctx.check(ctx.lib.rrte_hip_host_unregister(ctx.h, pinned[0]))
            self._pinned = pinned = None
        if pinned is None and getattr(self, "_unpinnable", None) != addr:
            if ctx.lib.rrte_hip_host_register(ctx.h, addr, need) == abi.RRTE_OK:
                self._pinned = (addr, need)
            else:
                self._unpinnable = addr
        scene = LoweredScene(objects, lights, camera)
        prm = cfg.lower()
        ctx.check(ctx.lib.rrte_hip_render(ctx.h, scene.ref(), C.byref(prm), addr))
        return out

    def render_f32(self, objects, lights, materials, camera: Camera, want_f32=True, linear=False):
        """Parity variant: also returns the post-gamma/clamp (or linear) f32 RGBA buffer."""
        cfg = self.config
        scene = LoweredScene(objects, lights, camera)
        prm = cfg.lower()
        if linear:
            prm.flags |= abi.FLAG_F32_LINEAR
        out8 = np.empty(cfg.width * cfg.height * 4, dtype=np.uint8)
        outf = np.empty(cfg.width * cfg.height * 4, dtype=np.float32) if want_f32 else None
        ctx = self.ctx
        ctx.check(ctx.lib.rrte_hip_render_f32(ctx.h, scene.ref(), C.byref(prm), out8.ctypes.data,
                                              outf.ctypes.data if outf is not None else None))
        return out8, outf

    def stats(self) -> abi.Stats:
        return self.ctx.stats()
