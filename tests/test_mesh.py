"""Triangle meshes (RRTE_PRIM_MESH, §8f rank 4) on the CPU side: a mesh is exactly the Vec<Triangle>
it stands for (oracle, bit for bit), MeshAsset/SceneAsset JSON in serde's layout, lowering and
validation, and the scene-specialised kernel compiles for a mesh scene (hiprtc, no device)."""
import json

import numpy as np
import pytest

import oracle
from rrte_amd import (Camera, Color, LambertianMaterial, LoweredScene, Mesh, PointLight, RaytracerConfig,
                      Sphere, Transform, abi, load_scene_asset, scenes, to_radians, vec3)
from rrte_amd.math import f32
from rrte_amd.mesh import heightfield, icosphere, torus


def _cam(w, h, pos=(0, 3, 8), target=(0, 1, 0)):
    cam = Camera.new_perspective(to_radians(45.0), f32(w) / f32(h), 0.1, 100.0)
    cam.transform.position = vec3(pos)
    cam.look_at(target)
    return cam


def _cfg(w, h, mode):
    return RaytracerConfig(max_depth=1, samples_per_pixel=1, width=w, height=h, jitter="center", mode=mode,
                           background_color=Color(0.1, 0.1, 0.15, 1))


def _small_meshes(mat):
    return [icosphere((-1.2, 1.0, 0.0), 0.9, 1, mat), torus((1.3, 1.0, 0.0), 0.8, 0.3, 10, 6, mat)]


@pytest.mark.parametrize("mode", ["refcompat", "lambert_shadow"])
def test_mesh_is_exactly_its_triangles_in_the_oracle(mode):
    mat = LambertianMaterial(Color.rgb(0.7, 0.5, 0.3))
    ground = Sphere((0, -1000, 0), 1000, LambertianMaterial(Color.rgb(0.3, 0.3, 0.3)))
    meshes = _small_meshes(mat)
    lights = [PointLight((3, 6, 4), Color.rgb(1, 1, 1), 4.0), PointLight((-4, 3, 2), Color.rgb(0.6, 0.7, 1), 3.0)]
    w, h = 96, 64
    a = LoweredScene([ground] + meshes, lights, _cam(w, h))
    tris = [t for m in meshes for t in m.triangles()]
    b = LoweredScene([ground] + tris, lights, _cam(w, h))
    cfg = _cfg(w, h, mode)
    _, la, sa = oracle.render(a, cfg.lower(), nthreads=4, linear=True)
    _, lb, sb = oracle.render(b, cfg.lower(), nthreads=4, linear=True)
    assert np.array_equal(la.view(np.uint32), lb.view(np.uint32))
    assert sa == sb
    assert (la.reshape(-1, 4)[:, 0] != np.float32(0.1)).sum() > 500  # the meshes are in view


def test_mesh_normals_are_normalised_and_faces_default():
    m = Mesh([(0, 0, 0), (1, 0, 0), (0, 1, 0)], [(0, 1, 2)], normals=[(0, 0, 3), (0, 0, 2), (0, 0, 1)])
    assert np.allclose(np.linalg.norm(m.normals, axis=1), 1.0, atol=1e-6)
    m2 = Mesh([(0, 0, 0), (1, 0, 0), (0, 1, 0)], [(0, 1, 2)])
    assert np.allclose(m2.normals, [[0, 0, 1]] * 3)
    with pytest.raises(ValueError):
        Mesh([(0, 0, 0)], [(0, 1, 2)])


def test_mesh_asset_json_round_trip(tmp_path):
    m = icosphere((0, 1, 0), 1.0, 1)
    d = m.to_asset("ball.json")
    p = tmp_path / "ball.json"
    p.write_text(json.dumps(d))
    m2 = Mesh.from_asset(p)
    assert np.array_equal(m2.positions, m.positions)
    assert np.array_equal(m2.indices, m.indices)
    assert np.allclose(m2.normals, m.normals, atol=1e-7)
    # serde layout of MeshAsset / Vertex (asset.rs:53-65)
    v = d["vertices"][0]
    assert set(v) == {"position", "normal", "uv", "color"} and len(v["position"]) == 3
    assert set(v["color"]) == {"r", "g", "b", "a"}
    assert len(d["indices"]) == 3 * m.num_triangles


def test_scene_asset_loader(tmp_path):
    (tmp_path / "ball.json").write_text(json.dumps(icosphere((0, 0, 0), 1.0, 1).to_asset("ball.json")))
    (tmp_path / "red.json").write_text(json.dumps({
        "name": "red", "albedo": {"r": 0.8, "g": 0.2, "b": 0.2, "a": 1.0}, "metallic": 0.0, "roughness": 0.5,
        "specular": 0.5, "emission": {"r": 0, "g": 0, "b": 0, "a": 1}, "ior": 1.5, "albedo_texture": None,
        "normal_texture": None, "metallic_texture": None, "roughness_texture": None, "metadata": {}}))
    ident = {"position": [0, 0, 0], "rotation": [0, 0, 0, 1], "scale": [1, 1, 1]}
    scene = {"name": "s", "metadata": {},
             "entities": [{"name": "a", "transform": {"position": [2, 1, 0], "rotation": [0, 0, 0, 1],
                                                       "scale": [0.5, 0.5, 0.5]}, "mesh": "ball.json",
                           "material": "red.json"},
                          {"name": "empty", "transform": ident, "mesh": None, "material": None}],
             "lights": [{"name": "sun", "light_type": "directional", "position": [0, 0, 0],
                         "direction": [-0.3, -1, -0.2], "color": {"r": 1, "g": 1, "b": 1, "a": 1}, "intensity": 1.0},
                        {"name": "p", "light_type": "point", "position": [0, 5, 5], "direction": [0, 0, 0],
                         "color": {"r": 1, "g": 0.9, "b": 0.8, "a": 1}, "intensity": 20.0}],
             "camera": {"transform": {"position": [0, 2, 8], "rotation": [0, 0, 0, 1], "scale": [1, 1, 1]},
                        "fov": 0.8, "near": 0.1, "far": 100.0}}
    (tmp_path / "scene.json").write_text(json.dumps(scene))
    objs, lights, cam = load_scene_asset(tmp_path / "scene.json", aspect_ratio=1.5)
    assert len(objs) == 1 and len(lights) == 2
    m = objs[0]
    assert np.allclose(m.positions.min(0), [1.5, 0.5, -0.5], atol=1e-6)
    assert np.allclose(m.positions.max(0), [2.5, 1.5, 0.5], atol=1e-6)
    assert np.allclose(m.material.albedo().as_tuple()[:3], (0.8, 0.2, 0.2))
    cfg = _cfg(48, 32, "lambert_shadow")
    r8, _, _ = oracle.render(LoweredScene(objs, lights, cam), cfg.lower(), nthreads=2)
    assert r8.reshape(-1, 4)[:, 0].max() > 100  # the red ball is lit


def test_entity_transform_rotates_normals():
    m = Mesh([(0, 0, 0), (1, 0, 0), (0, 1, 0)], [(0, 1, 2)])
    q = (0.0, np.sin(np.pi / 4), 0.0, np.cos(np.pi / 4))  # 90 degrees about Y
    t = m.transformed(Transform(position=(0, 0, 0), rotation=q, scale=(2, 2, 2)))
    assert np.allclose(t.normals, [[1, 0, 0]] * 3, atol=1e-6)
    assert np.allclose(t.positions[1], [0, 0, -2], atol=1e-6)


def test_lowering_shares_one_vertex_pool():
    mat = LambertianMaterial(Color.rgb(0.5, 0.5, 0.5))
    ms = _small_meshes(mat)
    sc = LoweredScene(ms, [], _cam(8, 8))
    ir = sc.ir
    assert ir.num_mesh_vertices == sum(len(m.positions) for m in ms)
    assert ir.num_mesh_indices == 3 * sum(m.num_triangles for m in ms)
    assert ir.mesh_version > 0
    assert ir.prims[0].kind == abi.PRIM_MESH and ir.prims[1].kind == abi.PRIM_MESH
    assert ir.prims[1].sdf_first == ms[0].num_triangles and ir.prims[1].sdf_count == ms[1].num_triangles
    idx = np.ctypeslib.as_array(ir.mesh_indices, shape=(ir.num_mesh_indices,))
    assert idx[3 * ms[0].num_triangles:].min() >= len(ms[0].positions)  # second mesh offset into the pool


def test_oracle_rejects_out_of_range_mesh_indices():
    m = icosphere((0, 0, 0), 1.0, 0)
    sc = LoweredScene([m], [], _cam(8, 8))
    sc._mesh_idx[5] = 10_000
    with pytest.raises(ValueError):
        oracle.render(sc, _cfg(8, 8, "lambert_shadow").lower(), nthreads=1)


def test_scene_specialised_kernel_compiles_for_meshes():
    lib = abi.load()
    objs, lights, cam, cfg = scenes.mesh_demo(32, 18, detail=0.05)
    sc = LoweredScene(objs, lights, cam)
    import ctypes as C
    log = C.create_string_buffer(4096)
    assert lib.rrte_hip_jit_check(sc.ref(), abi.MODE_LAMBERT_SHADOW, log, 4096) == abi.RRTE_OK, log.value.decode()


def test_heightfield_grid_counts():
    m = heightfield((0, 0, 0), 1.0, 5, lambda x, z: 0 * x)
    assert m.num_triangles == 2 * 4 * 4 and len(m.positions) == 25
