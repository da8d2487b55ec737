"""The C++ mirror of the renderer API (include/rrte/rrte_renderer.hpp, rrte_amd/cpp/): it lowers
every scene to exactly the bytes the Python mirror produces, reports errors like the Python mirror,
and its Raytracer::render reproduces the oracle on the GPU."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle
from rrte_amd import (AmbientLight, BendDeformer, Capsule, Color, Cone, Cube, Cylinder, DeformedSDF,
                      DielectricMaterial, DirectionalLight, EmissiveMaterial, LambertianMaterial, LoweredScene,
                      Mesh, MetalMaterial, NoiseDeformer, Plane, PointLight, SDFBox, SDFCapsule, SDFObject,
                      SDFTorus, Sphere, SpotLight, TaperDeformer, Transform, Triangle, TwistDeformer,
                      WaveDeformer, abi, scenes)
from rrte_amd.scenes import _camera, _config

ROOT = Path(__file__).resolve().parents[1]
TOOL = ROOT / "rrte_amd" / "lib" / "cpp_mirror_tool"
F = np.float32


@pytest.fixture(scope="module", autouse=True)
def built():
    subprocess.run(["make", "-s", "-C", str(ROOT / "rrte_amd" / "cpp")], check=True)


def kitchen_sink(w, h, mode):
    """Python twin of rrte_amd/cpp/examples.cpp kitchen_sink (every object/light/material kind)."""
    m0, m1, m2 = (LambertianMaterial(Color.rgb(*c)) for c in [(0.6, 0.3, 0.2), (0.2, 0.5, 0.7), (0.4, 0.6, 0.3)])
    metal = MetalMaterial(Color.rgb(0.8, 0.7, 0.5), 0.2)
    glass = DielectricMaterial(1.5)
    glow = EmissiveMaterial(Color.rgb(1.0, 0.5, 0.2), 2.0)
    cube = Cube((1.5, 1.0, 0.0), (1.0, 1.5, 0.8), m0)
    cube.transform = Transform(position=(0.1, 0.0, 0.2), rotation=(0.0, 0.38268343, 0.0, 0.92387953), scale=(1.0, 1.2, 1.0))
    tri = Triangle((-3.0, 0.1, -3.0), (3.0, 0.1, -3.0), (0.0, 3.0, -3.0), m2)
    tri.set_normals((0.0, 0.0, 2.0), (0.1, 0.0, 1.0), (-0.1, 0.2, 1.0))
    pos = np.array([1, 0, 0, -1, 0, 0, 0, 1, 0, 0, -1, 0, 0, 0, 1, 0, 0, -1], dtype=F).reshape(-1, 3)
    pos = pos * F(0.6) + np.array([-1.5, 1.0, 1.8], dtype=F)
    idx = np.array([0, 2, 4, 2, 1, 4, 1, 3, 4, 3, 0, 4, 2, 0, 5, 1, 2, 5, 3, 1, 5, 0, 3, 5], dtype=np.uint32)
    oct_ = Mesh(pos, idx, None, metal)
    piv = (0.0, 0.6, 2.2)
    twisted = DeformedSDF(SDFTorus(piv, 0.7, 0.25), TwistDeformer((0, 1, 0), 1.5, piv).chain(
        NoiseDeformer(2.0, 0.05, piv, seed=7).with_octaves(3).with_persistence(0.5)))
    pv2 = (-2.0, 1.0, -1.0)
    tapered = DeformedSDF(SDFBox(pv2, (1.0, 1.6, 1.0)), TaperDeformer((0, 1, 0), 1.0, 0.4, 1.6, pv2).chain(
        WaveDeformer((1, 0, 0), 0.1, 5.0, (0, 1, 0), pv2)))
    pv3 = (2.5, 1.2, 2.0)
    bent = DeformedSDF(SDFCapsule(pv3, 0.3, 1.2), BendDeformer((0, 0, 1), (1, 0, 0), 0.3, pv3))
    objects = [Plane((0, 0, 0), (0, 1, 0), m2), cube, Cylinder((-1.5, 1.0, 0.5), 0.6, 1.5, m1),
               Cone((0.0, 1.2, -1.5), 0.8, 1.6, m0), Capsule((0.0, 1.0, 1.8), 0.4, 1.0, m1), tri,
               Sphere((2.2, 0.6, -1.8), 0.6, glass), Sphere((-2.6, 0.4, 2.6), 0.4, glow), oct_,
               SDFObject(twisted, m1), SDFObject(tapered, m0, max_steps=160, step_scale=0.5, hit_eps=2e-4),
               SDFObject(bent, metal)]
    lights = [PointLight((3, 6, 4), Color.rgb(1, 1, 1), 2.0),
              DirectionalLight((-0.3, -1.0, -0.3), Color(1.0, 0.95, 0.8, 1.0), 0.6),
              SpotLight((0, 5, 0), (0, -1, 0), Color.rgb(1, 0.8, 0.6), 6.0, 0.3, 0.6),
              AmbientLight.default_ambient(),
              PointLight.with_attenuation((-4, 3, -1), Color.rgb(0.5, 0.6, 1.0), 2.5, 50.0, 0.05, 0.01)]
    cam = _camera(w, h, (4.0, 3.5, 6.0), (0.0, 1.0, 0.0), 50.0)
    return objects, lights, cam, _config(w, h, Color(0.1, 0.1, 0.15, 1.0), mode)


PY_SCENES = {"basic-demo": scenes.basic_demo, "advanced-demo": scenes.advanced_demo,
             "sdf-showcase": scenes.sdf_showcase, "kitchen-sink": kitchen_sink}


def ir_bytes(sc: LoweredScene, params) -> bytes:
    ir = sc.ir
    b = bytearray()
    for ptr, n, T in [(ir.prims, ir.num_prims, abi.Prim), (ir.materials, ir.num_materials, abi.Material),
                      (ir.lights, ir.num_lights, abi.Light), (ir.sdf_nodes, ir.num_sdf_nodes, abi.SdfNode)]:
        b += bytes(memoryview((T * n).from_address(__import__("ctypes").addressof(ptr.contents)))) if n else b""
    b += bytes(ir.camera)
    if ir.num_mesh_vertices:
        b += sc._mesh_vtx.tobytes() + sc._mesh_idx.tobytes()
    return bytes(b) + bytes(params)


@pytest.mark.parametrize("name", sorted(PY_SCENES))
@pytest.mark.parametrize("mode", ["refcompat", "lambert_shadow"])
def test_cpp_and_python_mirrors_lower_identically(name, mode, tmp_path):
    out = tmp_path / "ir.bin"
    subprocess.run([str(TOOL), "ir", name, "160", "90", mode, str(out)], check=True)
    objs, lights, cam, cfg = PY_SCENES[name](160, 90, mode=mode) if name != "kitchen-sink" else kitchen_sink(160, 90, mode)
    want = ir_bytes(LoweredScene(objs, lights, cam), cfg.lower())
    got = out.read_bytes()
    assert len(got) == len(want)
    if got != want:
        d = np.nonzero(np.frombuffer(got, np.uint8) != np.frombuffer(want, np.uint8))[0]
        pytest.fail(f"{len(d)} bytes differ, first at {d[0]}")


def test_cpp_mirror_error_behaviour():
    r = subprocess.run([str(TOOL), "errors"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(PY_SCENES))
def test_cpp_raytracer_render_matches_oracle(name, tmp_path):
    w, h = 200, 120
    mode = "lambert_shadow"
    out = tmp_path / "img.bin"
    r = subprocess.run([str(TOOL), "render", name, str(w), str(h), mode, str(out)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    raw = out.read_bytes()
    g8 = np.frombuffer(raw[: w * h * 4], np.uint8)
    glin = np.frombuffer(raw[w * h * 4:], np.float32)
    objs, lights, cam, cfg = PY_SCENES[name](w, h, mode=mode) if name != "kitchen-sink" else kitchen_sink(w, h, mode)
    sc = LoweredScene(objs, lights, cam)
    r8, _, rsh = oracle.render(sc, cfg.lower(), nthreads=16)
    _, rlin, _ = oracle.render(sc, cfg.lower(), nthreads=16, linear=True)
    assert int(r.stdout.split()[-1]) == rsh
    assert np.abs(g8.astype(int) - r8.astype(int)).max() <= 1
    if name == "kitchen-sink":  # spot light: device acosf vs libm, an ulp in the linear image
        d = glin.astype(np.float64) - rlin.astype(np.float64)
        assert np.sqrt(np.mean(np.nan_to_num(d) ** 2)) <= 1e-4
    else:
        assert np.array_equal(glin.view(np.uint32), rlin.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("name,w,h", [("sdf-showcase", 1920, 1080), ("basic-demo", 333, 97)])
def test_cpp_engine_loop_render_into(name, w, h, tmp_path):
    """Engine::render_frame's loop through the C++ mirror (Raytracer::render_into: one reused buffer,
    pinned once, the kernel storing the frame straight into it; rust/patches/0002): every frame
    byte-identical to Raytracer::render's, and the last one to the oracle's."""
    out = tmp_path / "img.bin"
    r = subprocess.run([str(TOOL), "engine", name, str(w), str(h), "lambert_shadow", str(out), "8"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatched 0" in r.stdout, r.stdout
    g8 = np.frombuffer(out.read_bytes(), np.uint8)
    objs, lights, cam, cfg = PY_SCENES[name](w, h, mode="lambert_shadow")
    r8, _, _ = oracle.render(LoweredScene(objs, lights, cam), cfg.lower(), nthreads=16, want_f32=False)
    assert np.abs(g8.astype(int) - r8.astype(int)).max() <= 1
