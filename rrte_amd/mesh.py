"""Triangle meshes: the rrte-assets MeshAsset / SceneAsset surface (crates/rrte-assets/src/asset.rs:53-146)
lowered to RRTE_PRIM_MESH.

In the reference a mesh has no ray-tracing path yet (MeshAsset and SceneAsset are defined and
serialisable but nothing renders them).  The build defines a mesh the way the
renderer already defines its one triangle type: every mesh triangle is `Triangle::intersect`
(primitives.rs:208-244) with `set_normals(n0, n1, n2)` (normals normalised, primitives.rs:196-198),
and the mesh is the closest hit over its triangles in index order -- exactly a `Vec<Triangle>` in the
object list.  Vertex arrays are float32 throughout; every host computation below is written op by op
in f32 so the lowered vertices are reproducible.

JSON layouts follow serde's derive output for the reference structs, with glam's `serde` feature
(Vec2/Vec3 as [x, y(, z)], Quat as [x, y, z, w]) and Color as {"r","g","b","a"}.
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

from . import abi
from .math import Color, Transform, f32

F = np.float32


def normalize_rows(v: np.ndarray) -> np.ndarray:
    """glam Vec3::normalize per row: v * (1 / sqrt((x*x + y*y) + z*z)), f32, one rounding per op."""
    v = np.asarray(v, dtype=F)
    d = (v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2]
    with np.errstate(divide="ignore", invalid="ignore"):
        r = F(1.0) / np.sqrt(d)
    return v * r[:, None]


def face_normals(pos: np.ndarray, idx: np.ndarray) -> np.ndarray:
    """Triangle::new's normal (primitives.rs:175-177): normalize(cross(v1 - v0, v2 - v0))."""
    v0, v1, v2 = pos[idx[:, 0]], pos[idx[:, 1]], pos[idx[:, 2]]
    a, b = v1 - v0, v2 - v0
    c = np.stack([a[:, 1] * b[:, 2] - b[:, 1] * a[:, 2], a[:, 2] * b[:, 0] - b[:, 2] * a[:, 0],
                  a[:, 0] * b[:, 1] - b[:, 0] * a[:, 1]], axis=1).astype(F)
    return normalize_rows(c)


def _quat_rotate(q, v: np.ndarray) -> np.ndarray:
    """glam Quat * Vec3, per row: v*(w*w - b.b) + b*(2*(v.b)) + (b x v)*(2*w), f32."""
    x, y, z, w = (F(c) for c in q)
    bb = (x * x + y * y) + z * z
    s = w * w - bb
    vb = (v[:, 0] * x + v[:, 1] * y) + v[:, 2] * z
    t = F(2.0) * vb
    cx = y * v[:, 2] - v[:, 1] * z
    cy = z * v[:, 0] - v[:, 2] * x
    cz = x * v[:, 1] - v[:, 0] * y
    w2 = F(2.0) * w
    out = np.empty_like(v)
    out[:, 0] = (v[:, 0] * s + x * t) + cx * w2
    out[:, 1] = (v[:, 1] * s + y * t) + cy * w2
    out[:, 2] = (v[:, 2] * s + z * t) + cz * w2
    return out


class Mesh:
    """A triangle mesh object (RRTE_PRIM_MESH): float32 positions (N, 3), unit normals (N, 3) and
    uint32 triangles (M, 3).  Normals are normalised at construction (Triangle::set_normals)."""

    def __init__(self, positions, indices, normals=None, material=None, name: str = ""):
        self.positions = np.ascontiguousarray(positions, dtype=F).reshape(-1, 3)
        self.indices = np.ascontiguousarray(indices, dtype=np.uint32).reshape(-1, 3)
        if self.indices.size and int(self.indices.max()) >= len(self.positions):
            raise ValueError("mesh index out of range")
        if normals is None:  # area-weighted vertex normals from the faces, then normalised
            acc = np.zeros_like(self.positions)
            fn = face_normals(self.positions, self.indices)
            for k in range(3):
                np.add.at(acc, self.indices[:, k], fn)
            normals = acc
        self.normals = normalize_rows(np.asarray(normals, dtype=F).reshape(-1, 3))
        self.material = material
        self.transform = Transform.identity()  # ignored, like Triangle's (bake transforms into vertices)
        self.name = name

    # ---- SceneObject surface
    def set_material(self, material):
        self.material = material

    def set_transform(self, transform: Transform):
        self.transform = transform

    @property
    def num_triangles(self) -> int:
        return len(self.indices)

    def lower(self, lw) -> abi.Prim:
        p = abi.Prim()
        p.kind = abi.PRIM_MESH
        p.sdf_first, p.sdf_count = lw.add_mesh(self.positions, self.normals, self.indices)
        p.trs[:] = [float(v) for v in self.transform.trs()]
        return p

    def triangles(self, material=None):
        """The same geometry as individual Triangle objects (the reference's object model)."""
        from .renderer import Triangle
        out = []
        for a, b, c in self.indices:
            t = Triangle(self.positions[a], self.positions[b], self.positions[c], material or self.material)
            t.normals = [tuple(F(x) for x in self.normals[i]) for i in (a, b, c)]
            out.append(t)
        return out

    def transformed(self, tr: Transform) -> "Mesh":
        """Bake an entity transform (SceneEntity.transform) into the vertices: positions through
        glam's Mat4::from_scale_rotation_translation(...).transform_point3, normals through the
        inverse-transpose (rotate(n / scale)) and normalised."""
        s = np.array(tr.scale, dtype=F)
        p = _quat_rotate(tr.rotation, self.positions * s[None, :]) + np.array(tr.position, dtype=F)[None, :]
        with np.errstate(divide="ignore", invalid="ignore"):
            n = _quat_rotate(tr.rotation, self.normals / s[None, :])
        m = Mesh(p.astype(F), self.indices, n, self.material, self.name)
        return m

    # ---- MeshAsset JSON (serde layout of asset.rs:53-65)
    @staticmethod
    def from_asset(src, material=None) -> "Mesh":
        d = _load_json(src)
        verts = d["vertices"]
        pos = np.array([v["position"] for v in verts], dtype=F).reshape(-1, 3)
        nrm = np.array([v["normal"] for v in verts], dtype=F).reshape(-1, 3)
        idx = np.array(d["indices"], dtype=np.uint32).reshape(-1, 3)
        name = d.get("metadata", {}).get("path", "")
        return Mesh(pos, idx, nrm, material, name)

    def to_asset(self, path: str = "") -> dict:
        meta = {"path": path, "asset_type": "Mesh", "size": 0,
                "created": {"secs_since_epoch": 0, "nanos_since_epoch": 0},
                "modified": {"secs_since_epoch": 0, "nanos_since_epoch": 0}, "dependencies": []}
        return {"vertices": [{"position": [float(c) for c in self.positions[i]],
                              "normal": [float(c) for c in self.normals[i]], "uv": [0.0, 0.0],
                              "color": {"r": 1.0, "g": 1.0, "b": 1.0, "a": 1.0}}
                             for i in range(len(self.positions))],
                "indices": [int(i) for i in self.indices.reshape(-1)], "metadata": meta}


def _load_json(src):
    if isinstance(src, dict):
        return src
    p = Path(src)
    return json.loads(p.read_text())


# ------------------------------------------------------------- procedural meshes (test scenes)
def icosphere(center, radius, subdivisions=3, material=None) -> Mesh:
    t = (1.0 + 5.0 ** 0.5) / 2.0
    v = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
         (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    f = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2),
         (10, 7, 6), (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11),
         (6, 2, 10), (8, 6, 7), (9, 8, 1)]
    verts = [np.array(p, dtype=np.float64) / np.linalg.norm(p) for p in v]
    for _ in range(subdivisions):
        cache, nf = {}, []

        def mid(a, b):
            k = (min(a, b), max(a, b))
            if k not in cache:
                m = verts[a] + verts[b]
                verts.append(m / np.linalg.norm(m))
                cache[k] = len(verts) - 1
            return cache[k]
        for a, b, c in f:
            ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
            nf += [(a, ab, ca), (b, bc, ab), (c, ca, bc), (ab, bc, ca)]
        f = nf
    unit = np.array(verts)
    pos = (unit * float(radius) + np.array(center, dtype=np.float64)).astype(F)
    return Mesh(pos, np.array(f, dtype=np.uint32), unit.astype(F), material, "icosphere")


def torus(center, major, minor, nu=96, nv=48, material=None) -> Mesh:
    u = np.linspace(0, 2 * np.pi, nu, endpoint=False)
    v = np.linspace(0, 2 * np.pi, nv, endpoint=False)
    uu, vv = np.meshgrid(u, v, indexing="ij")
    cx = np.cos(uu) * (major + minor * np.cos(vv))
    cz = np.sin(uu) * (major + minor * np.cos(vv))
    cy = minor * np.sin(vv)
    pos = np.stack([cx, cy, cz], -1).reshape(-1, 3) + np.array(center, dtype=np.float64)
    nrm = np.stack([np.cos(uu) * np.cos(vv), np.sin(vv), np.sin(uu) * np.cos(vv)], -1).reshape(-1, 3)
    idx = []
    for i in range(nu):
        for j in range(nv):
            a, b = i * nv + j, ((i + 1) % nu) * nv + j
            c, d = ((i + 1) % nu) * nv + (j + 1) % nv, i * nv + (j + 1) % nv
            idx += [(a, d, b), (b, d, c)]
    return Mesh(pos.astype(F), np.array(idx, dtype=np.uint32), nrm.astype(F), material, "torus")


def heightfield(origin, size, n, height, material=None) -> Mesh:
    """n x n grid over [x0, x0+size] x [z0, z0+size]; height(x, z) -> y (numpy-vectorised)."""
    xs = np.linspace(0.0, size, n) + origin[0]
    zs = np.linspace(0.0, size, n) + origin[2]
    xx, zz = np.meshgrid(xs, zs, indexing="ij")
    yy = height(xx, zz) + origin[1]
    pos = np.stack([xx, yy, zz], -1).reshape(-1, 3)
    idx = []
    for i in range(n - 1):
        for j in range(n - 1):
            a, b, c, d = i * n + j, (i + 1) * n + j, (i + 1) * n + j + 1, i * n + j + 1
            idx += [(a, d, b), (b, d, c)]
    return Mesh(pos.astype(F), np.array(idx, dtype=np.uint32), None, material, "heightfield")


# ------------------------------------------------------------------------ SceneAsset loader
def _material_from_asset(d):
    """MaterialAsset (asset.rs:84-100) -> a renderer material.  Build-defined mapping (the reference
    has none): emission > 0 -> Emissive; metallic >= 0.5 -> Metal(albedo, fuzz = roughness);
    ior > 1 with albedo alpha < 1 -> Dielectric(ior); else Lambertian(albedo)."""
    from .renderer import DielectricMaterial, EmissiveMaterial, LambertianMaterial, MetalMaterial
    a = d.get("albedo", {"r": 0.8, "g": 0.8, "b": 0.8, "a": 1.0})
    alb = Color(a["r"], a["g"], a["b"], a.get("a", 1.0))
    e = d.get("emission", {"r": 0, "g": 0, "b": 0, "a": 1})
    if max(e["r"], e["g"], e["b"]) > 0:
        return EmissiveMaterial(Color(e["r"], e["g"], e["b"], 1.0), 1.0)
    if d.get("metallic", 0.0) >= 0.5:
        return MetalMaterial(alb, d.get("roughness", 0.0))
    if d.get("ior", 1.0) > 1.0 and alb.a < 1.0:
        return DielectricMaterial(d["ior"])
    return LambertianMaterial(alb)


def load_scene_asset(src, aspect_ratio: float, base_dir=None):
    """SceneAsset JSON (asset.rs:103-146) -> (objects, lights, camera).  Entity meshes/materials
    are asset paths (resolved against the scene file's directory) or inline asset dicts; the
    entity transform is baked into the mesh vertices.  Light types: point, directional, spot,
    ambient (light.rs).  SceneCamera.fov is in radians (Camera::new_perspective)."""
    from .renderer import (AmbientLight, Camera, DirectionalLight, LambertianMaterial, PointLight,
                           SpotLight)
    d = _load_json(src)
    if base_dir is None:
        base_dir = Path(src).parent if not isinstance(src, dict) else Path(".")

    def res(x):
        return x if isinstance(x, dict) else Path(base_dir) / x

    def tr(t):
        return Transform(position=tuple(t["position"]), rotation=tuple(t["rotation"]), scale=tuple(t["scale"]))

    objects, mat_cache = [], {}
    for ent in d.get("entities", []):
        if not ent.get("mesh"):
            continue
        mkey = json.dumps(ent["material"], sort_keys=True) if isinstance(ent.get("material"), dict) else ent.get("material")
        if mkey not in mat_cache:
            mat_cache[mkey] = (_material_from_asset(_load_json(res(ent["material"]))) if ent.get("material")
                               else LambertianMaterial(Color(0.8, 0.8, 0.8, 1.0)))
        mesh = Mesh.from_asset(res(ent["mesh"]), mat_cache[mkey]).transformed(tr(ent["transform"]))
        mesh.name = ent.get("name", mesh.name)
        objects.append(mesh)
    lights = []
    for L in d.get("lights", []):
        c = L["color"]
        col = Color(c["r"], c["g"], c["b"], c.get("a", 1.0))
        kind = L["light_type"].lower()
        if kind == "point":
            lights.append(PointLight(tuple(L["position"]), col, L["intensity"]))
        elif kind == "directional":
            lights.append(DirectionalLight(tuple(L["direction"]), col, L["intensity"]))
        elif kind == "spot":
            lights.append(SpotLight(tuple(L["position"]), tuple(L["direction"]), col, L["intensity"],
                                    L.get("inner_angle", 0.3), L.get("outer_angle", 0.6)))
        elif kind == "ambient":
            lights.append(AmbientLight(col, L["intensity"]))
        else:
            raise ValueError(f"unknown light_type {L['light_type']!r}")
    sc = d["camera"]
    cam = Camera.new_perspective(sc["fov"], aspect_ratio, sc["near"], sc["far"])
    cam.transform = tr(sc["transform"])
    return objects, lights, cam
