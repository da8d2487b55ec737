"""The sky bands of rrte_hip_band_layout (include/rrte_hip.h) -- the leading bands the multi-GPU band
partition hands to the root because no object reaches them -- hold only background pixels: checked
against the CPU oracle's frame over camera poses.  (The partition only decides which rank renders a
band, never a pixel; this checks the silhouette geometry its work model relies on.)"""
import ctypes as C

import numpy as np
import pytest

import oracle
from rrte_amd import LoweredScene, abi, scenes

W, H, BAND = 320, 180, 4
# (eye, target, fov): the showcase pose, higher / lower / wider / sideways views
POSES = [(None, None, None),
         ((0.0, 2.0, 14.0), (0.0, 1.0, 0.0), 45.0),
         ((7.0, 3.0, 9.0), (0.0, 1.0, 0.0), 50.0),
         ((-9.0, 6.0, 7.0), (0.0, 0.0, 0.0), 40.0),
         ((0.0, 1.0, 16.0), (0.0, 2.0, 0.0), 30.0),
         ((2.0, 9.0, 6.0), (0.0, 0.0, 0.0), 70.0)]


def _render(objs, lights, cam, cfg):
    sc = LoweredScene(objs, lights, cam)
    img, _, _ = oracle.render(sc, cfg.lower(), nthreads=8, want_f32=False)
    return sc, img.reshape(H, W, 4)


@pytest.mark.parametrize("n", [2, 8])
def test_sky_bands_hold_only_background(n):
    skies = []
    for eye, tgt, fov in POSES:
        objs, lights, cam, cfg = scenes.sdf_showcase(W, H)
        cfg.band_rows = BAND
        if eye is not None:
            cam = scenes._camera(W, H, eye, tgt, fov)
        sc, img = _render(objs, lights, cam, cfg)
        prm = cfg.lower()
        sky, rb, pb = abi.band_layout(sc.ref(), C.byref(prm), n)
        assert 0 <= rb <= 8 and 1 <= pb <= 8 and (rb or sky)
        skies.append(sky)
        if sky == 0:
            continue
        _, empty = _render([], lights, cam, cfg)  # every camera ray misses: the background
        rows = min(sky * BAND, H)
        assert np.array_equal(img[:rows], empty[:rows]), (eye, sky)
        # how loose the bound is (culling spheres enclose the objects, plus one band of margin): the
        # first row an object reaches lies within H/6 below the sky (measured: 10-23 of 180 rows)
        first = int(np.where((img != empty).any(axis=(1, 2)))[0][0])
        assert rows <= first < rows + H // 6, (eye, sky, first)
    assert sum(1 for s in skies if s > 0) >= 3  # most poses see sky above the objects
