"""The oracle's instrumented counting build (flop tally for the roofline):
same results as the timed build, exact event counts on scenes where they are known in
closed form, thread-count independence."""
import numpy as np

import oracle
from rrte_amd import LoweredScene, scenes


def test_counting_build_counts_basic_demo_exactly():
    objs, lights, cam, cfg = scenes.basic_demo(64, 48, mode="lambert_shadow")
    sc = LoweredScene(objs, lights, cam)
    cnt, flops = oracle.count(sc, cfg.lower(), nthreads=3)
    _, _, shadow = oracle.render(sc, cfg.lower(), nthreads=3)
    px = 64 * 48
    assert cnt.pixels == px and cnt.samples == px * cfg.samples_per_pixel
    assert cnt.shadow_rays == shadow
    # every camera ray tests every object once (linear scan, raytracer.rs:106-113)
    assert cnt.isect_calls[0] >= cnt.samples * len(objs)
    assert cnt.light_evals[0] == cnt.shaded_hits * len(lights)
    assert cnt.lambert_lights == cnt.shaded_hits * len(lights)
    assert 0 < cnt.lambert_terms <= cnt.shadow_rays
    assert flops > 0


def test_counts_independent_of_thread_count_and_sdf_events():
    objs, lights, cam, cfg = scenes.sdf_showcase(96, 54)
    sc = LoweredScene(objs, lights, cam)
    a, fa = oracle.count(sc, cfg.lower(), nthreads=1)
    b, fb = oracle.count(sc, cfg.lower(), nthreads=5)
    assert bytes(a) == bytes(b) and fa == fb
    assert a.sdf_steps > 0 and sum(a.sdf_nodes) > a.sdf_steps
    # each SDF hit runs one tetrahedral normal estimate
    assert a.sdf_normals == a.isect_hits[7]


def test_timed_build_matches_counting_build_output():
    objs, lights, cam, cfg = scenes.sdf_showcase(48, 27)
    sc = LoweredScene(objs, lights, cam)
    r8, rf, sh = oracle.render(sc, cfg.lower(), nthreads=2)
    cnt, _ = oracle.count(sc, cfg.lower(), nthreads=2)
    assert cnt.shadow_rays == sh
    assert np.isfinite(rf).all()
