"""CSG early-out bounds (rrte_amd/csrc/sdf_guard.hip, DESIGN.md §5 CSG guards), checked on the CPU.

The renderer may skip the right operand B of a union / difference when a lower bound of B decides
the op.  That is exact only if B >= lambda (|p - c| - R) holds for the f32 formulas wherever the
guard is used (R <= |p - c| <= smax).  These tests take the decoration the library computes
(rrte_hip_sdf_guards) and check the claim against the oracle's f32 evaluation of B (test
infrastructure: oracle/rrte_oracle.c sdf_eval) at many points, for every leaf kind with random and
extreme parameters and for random CSG subtrees.  The GPU tests (test_gpu_sdf_guards.py) then check
that renders with guards on and off are bit-identical.
"""
import ctypes as C
import math

import numpy as np
import pytest

import oracle
from rrte_amd import abi, renderer as R
from rrte_amd import LoweredScene, Camera

LEAVES = ["sphere", "box", "cylinder", "prism", "torus", "tube", "ring", "cone", "capsule", "ellipsoid"]


def leaf(kind, rng, c=None, scale=1.0):
    c = tuple(rng.uniform(-3, 3, 3)) if c is None else c
    u = lambda lo=0.05, hi=2.0: float(rng.uniform(lo, hi)) * scale  # noqa: E731
    if kind == "sphere":
        return R.SDFSphere(c, u())
    if kind == "box":
        return R.SDFBox(c, (u(), u(), u()))
    if kind == "cylinder":
        return R.SDFCylinder(c, u(), u())
    if kind == "prism":
        return R.SDFPrism(c, (u(), u(), u()))
    if kind == "torus":
        return R.SDFTorus(c, u(), u())
    if kind == "tube":
        o = u()
        return R.SDFTube(c, o, o * float(rng.uniform(0.0, 1.0)), u())
    if kind == "ring":
        return R.SDFRing(c, u(), u())
    if kind == "cone":
        return R.SDFCone(c, u(), u())
    if kind == "capsule":
        return R.SDFCapsule(c, u(), u())
    # extreme aspect ratios too: lambda = (rmin/rmax)^2 gets small
    return R.SDFEllipsoid(c, (u(0.01, 3.0), u(0.01, 3.0), u(0.01, 3.0)))


OPS = ["union", "smooth_union", "difference", "smooth_difference", "intersection", "smooth_intersection"]


def tree(rng, depth):
    if depth == 0 or rng.uniform() < 0.2:
        return leaf(LEAVES[rng.integers(len(LEAVES))], rng)
    return R.CSGComposite(tree(rng, depth - 1), tree(rng, depth - 1), OPS[rng.integers(len(OPS))],
                          float(rng.uniform(0.05, 0.8)))


def program(sdf):
    out = []
    sdf.emit(out)
    return out


def guards_of(nodes, min_leaves=1):
    arr = (abi.SdfNode * len(nodes))(*nodes)
    out = (abi.SdfNode * len(nodes))()
    n = C.c_uint32()
    assert abi.load().rrte_hip_sdf_guards(arr, len(nodes), min_leaves, out, C.byref(n)) == abi.RRTE_OK
    return list(out), n.value


class SdfEval:
    """The oracle's f32 evaluation of one SDF program (a scene holding just that SDFObject)."""

    def __init__(self, sdf_or_nodes):
        cam = Camera.new_perspective(1.0, 1.0, 0.1, 100.0)
        if isinstance(sdf_or_nodes, list):
            self.scene = LoweredScene([R.SDFObject(R.SDFSphere((0, 0, 0), 1.0))], [], cam)
            self.nodes = (abi.SdfNode * len(sdf_or_nodes))(*sdf_or_nodes)
            self.scene.ir.sdf_nodes, self.scene.ir.num_sdf_nodes = self.nodes, len(sdf_or_nodes)
            self.scene.prims[0].sdf_first, self.scene.prims[0].sdf_count = 0, len(sdf_or_nodes)
        else:
            self.scene = LoweredScene([R.SDFObject(sdf_or_nodes)], [], cam)
        self.lib = oracle.load()

    def __call__(self, p):
        v = (C.c_float * 3)(*[float(x) for x in p])
        return self.lib.rrte_oracle_sdf_eval(C.byref(self.scene.ir), 0, v)


def shell_points(rng, c, r0, r1, n):
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    # half the samples hug the inner radius (where the bound is tightest)
    t = np.concatenate([r0 * (1.0 + rng.uniform(0, 1e-3, n // 2)), rng.uniform(r0, r1, n - n // 2)])
    return np.asarray(c, np.float64)[None, :] + d * t[:, None]


def check_guard(g, operand, rng, n):
    """The bound stored in op node g must hold for the operand program at points of its range."""
    c, Rg, lam, smax = np.array(g.f[4:7], np.float64), float(g.f[7]), float(g.f[8]), float(g.f[9])
    assert 0 < lam <= 1 and Rg > 0 and smax > Rg
    ev = SdfEval(operand)
    worst = math.inf
    for p in shell_points(rng, c, Rg, smax, n):
        # the device's f32 point: the bound must hold for it
        p32 = p.astype(np.float32).astype(np.float64)
        s = float(np.linalg.norm(p32 - c))
        if s < Rg or s > smax:
            continue
        v = ev(p32)
        L = lam * (s - Rg)
        assert v >= L, (p32, v, L)
        worst = min(worst, v - L)
    return worst


def check_bound(sdf, rng, n=400):
    """Guard the SDF as the right operand of a union with a far-away sphere and check every
    guard of the decorated program (the outer one and any inside the SDF)."""
    nodes = [*program(R.SDFSphere((50.0, 0.0, 0.0), 0.5)), *program(sdf)]
    nodes.append(R._node(abi.SDF_UNION))
    out, ng = guards_of(nodes)
    assert ng >= 1 and out[1].i[2] == len(nodes)
    for start, nd in enumerate(out):
        link = nd.i[2]
        if link:
            check_guard(out[link - 1], nodes[start:link - 1], rng, n if start == 1 else n // 3)


@pytest.mark.parametrize("kind", LEAVES)
def test_leaf_bounds_hold(kind):
    rng = np.random.default_rng(abs(hash(kind)) % (1 << 32))
    for _ in range(12):
        check_bound(leaf(kind, rng), rng)


@pytest.mark.parametrize("kind", LEAVES)
def test_leaf_bounds_hold_far_from_origin_and_large(kind):
    """Large coordinates and sizes: the f32 error grows with |p|, the margin with R + |c|."""
    rng = np.random.default_rng(7 + LEAVES.index(kind))
    for _ in range(6):
        check_bound(leaf(kind, rng, c=tuple(rng.uniform(-200, 200, 3)), scale=20.0), rng, n=200)


def test_subtree_bounds_hold():
    rng = np.random.default_rng(0x5EED)
    checked = 0
    for _ in range(40):
        t = tree(rng, 3)
        nodes = [*program(R.SDFSphere((50.0, 0.0, 0.0), 0.5)), *program(t), R._node(abi.SDF_UNION)]
        if guards_of(nodes)[0][1].i[2] == len(nodes):
            check_bound(t, rng, n=150)
            checked += 1
    assert checked >= 20


def test_default_policy_and_off():
    """min_leaves 2 (the renderer's default) guards multi-leaf operands and the long single
    formulas; 0 guards nothing; caller bytes in i[2] are never taken for links."""
    rng = np.random.default_rng(3)
    a, b = leaf("sphere", rng), leaf("box", rng)
    pair = R.CSGComposite(leaf("box", rng), leaf("capsule", rng), "union")
    for B, expect in [(b, 0), (pair, 1), (leaf("ellipsoid", rng), 1), (leaf("cone", rng), 1)]:
        nodes = [*program(a), *program(B), R._node(abi.SDF_UNION)]
        assert guards_of(nodes, 2)[1] == expect
        assert guards_of(nodes, 0)[1] == 0
    nodes = [*program(a), *program(b), R._node(abi.SDF_INTERSECTION)]
    for n in nodes:
        n.i[2] = 12345
    out, ng = guards_of(nodes, 1)
    assert ng == 0 and all(n.i[2] == 0 for n in out)


def test_no_guard_across_deformers_or_for_intersections():
    rng = np.random.default_rng(5)
    a = leaf("sphere", rng)
    pair = R.CSGComposite(leaf("box", rng), leaf("torus", rng), "smooth_union", 0.3)
    deformed = R.DeformedSDF(pair, R.TwistDeformer((0, 1, 0), 0.5))
    for op, B in [(abi.SDF_UNION, deformed), (abi.SDF_INTERSECTION, pair), (abi.SDF_SMOOTH_INTERSECTION, pair)]:
        nodes = [*program(a), *program(B), R._node(op, [0.3])]
        out, _ = guards_of(nodes, 1)
        assert all(n.i[2] != len(nodes) for n in out)  # the outer op is never guarded
    # a deformed left operand does not stop a guard on a clean right operand
    nodes = [*program(deformed), *program(pair), R._node(abi.SDF_DIFFERENCE)]
    out, ng = guards_of(nodes, 1)
    assert ng >= 1 and out[len(program(deformed))].i[2] == len(nodes)
    # inside a deformed subtree, guards use the deformed point: allowed
    inner = R.DeformedSDF(R.CSGComposite(a, pair, "union"), R.TwistDeformer((0, 1, 0), 0.5))
    assert guards_of(program(inner), 1)[1] >= 1


def test_smooth_union_with_zero_k_is_not_guarded():
    rng = np.random.default_rng(9)
    pair = R.CSGComposite(leaf("box", rng), leaf("torus", rng), "union")
    nodes = [*program(leaf("sphere", rng)), *program(pair), R._node(abi.SDF_SMOOTH_UNION, [0.0])]
    out, ng = guards_of(nodes, 1)
    assert out[len(nodes) - 1].i[2] == 0 and all(n.i[2] != len(nodes) for n in out)
