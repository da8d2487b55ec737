"""The C oracle vs an independent numpy float32 restatement (tests/numpy_ref.py) of the
reference loop, written from the reference source: linear colours must agree bit-for-bit,
gamma'd bytes within 1 (numpy's float32 power may use a vector libm)."""
import math

import numpy as np
import pytest

import numpy_ref
import oracle
from rrte_amd import (Camera, Capsule, Color, Cone, Cube, Cylinder, LambertianMaterial, LoweredScene, Plane,
                      PointLight, RaytracerConfig, Sphere, Transform, Triangle, scenes, to_radians)
from rrte_amd.math import f32, vec3


from scenes_extra import mixed_scene as _mixed_scene  # noqa: E402


CASES = [(name, mode) for name in ["basic-demo", "simple-demo", "advanced-demo", "sdf-showcase-literal", "mixed"]
         for mode in ["refcompat", "lambert_shadow"]]


@pytest.mark.parametrize("name,mode", CASES)
def test_oracle_matches_numpy_restatement(name, mode):
    w, h = 48, 32
    objs, lights, cam, cfg = (_mixed_scene(w, h, mode) if name == "mixed" else scenes.SCENES[name](w, h, mode=mode))
    sc = LoweredScene(objs, lights, cam)
    n8, nf, nsh = numpy_ref.render(sc.ir, cfg.lower())
    o8, of, osh = oracle.render(sc, cfg.lower(), nthreads=2)
    _, of_lin, _ = oracle.render(sc, cfg.lower(), nthreads=2, linear=True)
    o8 = o8.reshape(h, w, 4)
    of = of.reshape(h, w, 4)
    assert osh == nsh
    # post-gamma floats within an ulp-level tolerance, bytes within 1
    assert np.nanmax(np.abs(of - nf)) <= 2e-7
    assert np.abs(o8.astype(int) - n8.astype(int)).max() <= 1
    # the linear (pre-gamma) buffer involves no transcendental: exact
    lin_np = numpy_ref_linear(sc, cfg)
    assert np.array_equal(of_lin.reshape(h, w, 4).view(np.uint32), lin_np.view(np.uint32))


def numpy_ref_linear(sc, cfg):
    """numpy_ref.render's pre-gamma colour: re-run with gamma 1 (x^1 is exact) and no clamp."""
    prm = cfg.lower()
    prm.gamma = 1.0
    import numpy_ref as nr
    saved = np.clip
    try:
        np.clip = lambda x, a, b: x  # noqa: E731  (linear buffer is unclamped)
        _, lin, _ = nr.render(sc.ir, prm)
    finally:
        np.clip = saved
    return lin


def test_sdf_leaf_formulas_match_numpy():
    """Build-defined SDF leaves + smooth_min (README.md:485-488): oracle == numpy, bit-exact."""
    import ctypes as C

    from rrte_amd import (SDFCapsule, SDFCylinder, SDFObject, SDFRing, SDFSphere, SDFTorus, SDFTube, abi,
                          CSGComposite)
    rng = np.random.default_rng(7)
    pts = rng.uniform(-2.5, 2.5, size=(200, 3)).astype(np.float32)
    leaves = [SDFSphere((0.1, 0.2, -0.3), 1.1), SDFCylinder((0, 0.1, 0), 0.7, 1.5), SDFTorus((0.2, 0, 0), 1.0, 0.3),
              SDFRing((0, 0, 0.1), 0.9, 0.2), SDFCapsule((0, 0, 0), 0.5, 1.2), SDFTube((0, 0, 0), 1.0, 0.6, 1.4)]
    cam = Camera.new_perspective(1.0, 1.0, 0.1, 100.0)
    lib = oracle.load()
    for leaf in leaves:
        sc = LoweredScene([SDFObject(leaf)], [], cam)
        node = sc.nodes[0]
        exp = numpy_ref.sdf_leaf(node.op, list(node.f), [pts[:, 0], pts[:, 1], pts[:, 2]])
        got = np.array([lib.rrte_oracle_sdf_eval(C.byref(sc.ir), 0, oracle.farr(p)) for p in pts], np.float32)
        assert np.array_equal(got.view(np.uint32), exp.astype(np.float32).view(np.uint32)), type(leaf).__name__
    a, b = SDFSphere((0, 0, 0), 1.0), SDFSphere((0.8, 0, 0), 0.7)
    sc = LoweredScene([SDFObject(CSGComposite.smooth_union(a, b, 0.3))], [], cam)
    da = numpy_ref.sdf_leaf(abi.SDF_SPHERE, list(sc.nodes[0].f), [pts[:, 0], pts[:, 1], pts[:, 2]])
    db = numpy_ref.sdf_leaf(abi.SDF_SPHERE, list(sc.nodes[1].f), [pts[:, 0], pts[:, 1], pts[:, 2]])
    exp = numpy_ref.smin(da, db, 0.3)
    got = np.array([lib.rrte_oracle_sdf_eval(C.byref(sc.ir), 0, oracle.farr(p)) for p in pts], np.float32)
    assert np.array_equal(got.view(np.uint32), exp.astype(np.float32).view(np.uint32))


def test_trig_and_noise_are_well_behaved():
    """Build-defined sin/cos: within 2e-7 of libm over the deformer range;
    value noise in [-1, 1) and continuous."""
    lib = oracle.load()
    xs = np.linspace(-40, 40, 4001, dtype=np.float32)
    s = np.array([lib.rrte_oracle_sinf(float(x)) for x in xs])
    c = np.array([lib.rrte_oracle_cosf(float(x)) for x in xs])
    assert np.abs(s - np.sin(xs.astype(np.float64))).max() < 5e-7
    assert np.abs(c - np.cos(xs.astype(np.float64))).max() < 5e-7
    v = np.array([lib.rrte_oracle_value_noise(float(x), 0.37, -1.3, 11) for x in np.linspace(-3, 3, 601)])
    assert v.min() >= -1 and v.max() < 1 and np.abs(np.diff(v)).max() < 0.2
