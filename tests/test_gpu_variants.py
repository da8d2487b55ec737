"""Kernel variants behind build switches, each held to the parity bar against the oracle (linear image
bit-exact, shadow-ray counts exact): the branch-free correctly rounded square root
(RRTE_SQRT_BRANCHFREE; its exhaustive proof is tests/test_gpu_fpexact.py), and the generic kernel's
all-features build next to the per-scene feature variants the host picks (RRTE_GENERIC_ALL), with and
without the one-leaf march dispatch and the short-program fast paths (RRTE_SDF_LEAF_DISPATCH,
RRTE_SDF_FASTPATH are build switches of the library: their A/B builds are tools/generic_ab.sh's)."""
import pytest

import scenes_extra as se
from rrte_amd import AmbientLight, scenes
from rrte_amd import abi
from test_gpu_parity import compare

pytestmark = pytest.mark.gpu


def _ambient_showcase(w, h, mode="lambert_shadow"):
    """sdf-showcase with an ambient light between its point lights."""
    objs, lights, cam, cfg = scenes.sdf_showcase(w, h, mode=mode)
    lights.insert(1, AmbientLight.default_ambient())
    return objs, lights, cam, cfg


CASES = {
    "sdf-showcase": lambda: scenes.sdf_showcase(320, 180),
    "sdf-showcase-1080p": lambda: scenes.sdf_showcase(1920, 1080),
    "advanced-demo": lambda: scenes.advanced_demo(320, 180),      # 5 point lights
    "basic-demo": lambda: scenes.basic_demo(320, 240, mode="lambert_shadow"),
    "ambient": lambda: _ambient_showcase(320, 180),  # an ambient light between point lights
    "deformers": lambda: se.deformers_scene(200, 120, "lambert_shadow"),
    "cull-stress": lambda: se.cull_stress_scene(240, 160, "lambert_shadow", n_spheres=40),
    "all-lights": lambda: se.all_lights_scene(200, 120, "lambert_shadow"),  # point, directional, spot, ambient
}


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("opt", ["-DRRTE_SQRT_BRANCHFREE"])
def test_specialised_kernel_variant_matches_oracle(case, opt, monkeypatch):
    monkeypatch.setenv("RRTE_JIT_EXTRA_OPTS", opt)
    # (spot lights use acosf -- libm against the device's ocml: an ulp in the linear image, as in
    # test_gpu_parity.py's culling tests)
    compare(*CASES[case](), linear_exact=case not in ("all-lights", "cull-stress"), jit=abi.JIT_ON)


@pytest.mark.parametrize("name,mode", [("sdf-showcase", "lambert_shadow"), ("basic-demo", "refcompat"),
                                       ("sdf-showcase-literal", "lambert_shadow"), ("mesh-demo", "lambert_shadow")])
def test_generic_all_features_build(name, mode, monkeypatch):
    """The generic kernel with every feature compiled in (RRTE_GENERIC_ALL=1) and the feature
    variant the host picks for the scene both match the oracle."""
    for flag in ("1", "0"):
        monkeypatch.setenv("RRTE_GENERIC_ALL", flag)
        compare(*scenes.SCENES[name](200, 120, mode=mode), jit=abi.JIT_OFF)


@pytest.mark.parametrize("case", ["sdf-showcase", "deformers", "advanced-demo", "cull-stress"])
@pytest.mark.parametrize("policy", ["0", "1"])
def test_guard_flavours_match_oracle(case, policy, monkeypatch):
    """Both guard flavours of the specialised kernel (RRTE_GUARD_POLICY=1: wave-uniform fallback
    branches, the streaming entry points' default; 0: divergent, the blocking frame's) are exact."""
    monkeypatch.setenv("RRTE_GUARD_POLICY", policy)
    compare(*CASES[case](), linear_exact=case != "cull-stress", jit=abi.JIT_ON)
