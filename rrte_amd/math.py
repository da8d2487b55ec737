"""f32 value types of rrte-math (Melthizar/RRTE crates/rrte-math/src/*.rs), restated
with numpy float32 scalars so host-side computations (camera look_at, light
colours) round exactly like the reference's f32 code (no FMA, one rounding per
op).  glam 0.24.2 algorithms are restated from glam's published source
(parity unpinned: glam is not vendored in the reference).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

f32 = np.float32
PI_F32 = f32(np.pi)


def vec3(x, y=None, z=None) -> tuple:
    """Vec3::new as a tuple of float32 (accepts a 3-sequence or 3 scalars)."""
    if y is None:
        x, y, z = x
    return (f32(x), f32(y), f32(z))


X = vec3(1, 0, 0)
Y = vec3(0, 1, 0)
Z = vec3(0, 0, 1)
NEG_Z = vec3(0, 0, -1)
ZERO = vec3(0, 0, 0)
ONE = vec3(1, 1, 1)


def to_radians(deg) -> np.float32:
    """f32::to_radians: self * (PI / 180.0) in f32."""
    return f32(deg) * (PI_F32 / f32(180.0))


def dot(a, b) -> np.float32:  # glam Vec3::dot, left to right
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def cross(a, b) -> tuple:
    return (a[1] * b[2] - b[1] * a[2], a[2] * b[0] - b[2] * a[0], a[0] * b[1] - b[0] * a[1])


def sub(a, b) -> tuple:
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def normalize(a) -> tuple:  # glam Vec3::normalize: self * (1 / length)
    r = f32(1.0) / np.sqrt(dot(a, a))
    return (a[0] * r, a[1] * r, a[2] * r)


def length(a) -> np.float32:
    return np.sqrt(dot(a, a))


@dataclass
class Color:
    """rrte_math::Color (color.rs:6-11): RGBA f32."""
    r: float
    g: float
    b: float
    a: float = 1.0

    def __post_init__(self):
        self.r, self.g, self.b, self.a = f32(self.r), f32(self.g), f32(self.b), f32(self.a)

    @staticmethod
    def rgb(r, g, b) -> "Color":
        return Color(r, g, b, 1.0)

    @staticmethod
    def gray(v) -> "Color":
        return Color(v, v, v, 1.0)

    def as_tuple(self):
        return (self.r, self.g, self.b, self.a)


Color.BLACK = Color(0, 0, 0, 1)
Color.WHITE = Color(1, 1, 1, 1)


def quat_from_rotation_arc(frm, to) -> tuple:
    """glam Quat::from_rotation_arc (used by Camera::look_at, camera.rs:85-95)."""
    one_minus_eps = f32(1.0) - f32(2.0) * f32(1.1920929e-7)
    d = dot(frm, to)
    if d > one_minus_eps:
        return (f32(0), f32(0), f32(0), f32(1))
    if d < -one_minus_eps:
        # from_axis_angle(from.any_orthonormal_vector(), PI)
        half = PI_F32 * f32(0.5)
        ax = (f32(1), f32(0), f32(0))
        s = f32(np.sin(np.float64(half)))
        return (ax[0] * s, ax[1] * s, ax[2] * s, f32(np.cos(np.float64(half))))
    c = cross(frm, to)
    x, y, z, w = c[0], c[1], c[2], f32(1.0) + d
    # glam Vec4 (SSE2) dot: (x*x + z*z) + (y*y + w*w); normalize divides by the length
    ln = np.sqrt((x * x + z * z) + (y * y + w * w))
    return (x / ln, y / ln, z / ln, w / ln)


@dataclass
class Transform:
    """rrte_math::Transform (transform.rs:6-10)."""
    position: tuple = ZERO
    rotation: tuple = (f32(0), f32(0), f32(0), f32(1))
    scale: tuple = ONE

    def __post_init__(self):
        self.position = vec3(self.position)
        self.rotation = tuple(f32(v) for v in self.rotation)
        self.scale = vec3(self.scale)

    @staticmethod
    def identity() -> "Transform":
        return Transform()

    @staticmethod
    def from_position(p) -> "Transform":
        return Transform(position=p)

    def trs(self) -> list:
        return [*self.position, *self.rotation, *self.scale]
