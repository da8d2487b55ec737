"""Host-side planning of the hot-first tile order (rrte_hip_tile_order_plan, the code a context runs
after a profile; no device needed): the hot list holds the slowest tiles, at most 1024 slots, sorted
by row then column with a split tile's parts consecutive; the whole-frame LPT order is a permutation
of every tile, slowest first, split tiles first; slots decode to in-range tiles."""
import ctypes as C

import numpy as np
import pytest

from rrte_amd import abi

MAX_SLOTS = 1024


def _plan(costs, tiles_x, lpt, parts=1, frac=0.7, cap=None):
    lib = abi.load()  # (signatures from abi.EXPORTS)
    c = np.ascontiguousarray(costs, dtype=np.uint32)
    cap = cap if cap is not None else len(c) * 4 + 16
    out = np.zeros(cap, dtype=np.uint32)
    n = C.c_uint32()
    st = lib.rrte_hip_tile_order_plan(c.ctypes.data_as(C.POINTER(C.c_uint32)), len(c), tiles_x, lpt, parts, frac,
                                      out.ctypes.data_as(C.POINTER(C.c_uint32)), cap, C.byref(n))
    return st, out[: n.value]


def _decode(s):
    return (s >> 4) & 0xFFF, s >> 16, s & 3, ((s >> 2) & 3) + 1


def _costs(tx=240, ty=135, seed=3):
    rng = np.random.default_rng(seed)
    c = rng.gamma(2.0, 600.0, size=tx * ty).astype(np.uint32) + 200
    c[rng.choice(tx * ty, 40, replace=False)] = rng.integers(8000, 10000, 40)  # a silhouette tail
    return c, tx, ty


@pytest.mark.parametrize("parts", [1, 3])
def test_hot_list(parts):
    c, tx, ty = _costs()
    st, s = _plan(c, tx, 0, parts)
    assert st == abi.RRTE_OK and 0 < len(s) <= MAX_SLOTS
    assert np.all(np.diff(s.astype(np.int64)) > 0)  # ascending: row, column, parts, part
    x, y, part, np_ = _decode(s)
    assert np.all(x < tx) and np.all(y < ty)
    tiles = y * tx + x
    thr = max(2.0 * c.mean(), 0.25 * c.max())
    assert np.all(c[tiles] >= np.floor(thr))  # only slow tiles
    assert c.argmax() in set(tiles.tolist())  # the slowest is there
    uniq = np.unique(tiles)
    for t in uniq:  # a split tile's parts are consecutive, 0..P-1, and only the slowest split
        idx = np.nonzero(tiles == t)[0]
        assert np.array_equal(idx, np.arange(idx[0], idx[0] + len(idx)))
        assert list(part[idx]) == list(range(len(idx))) and np.all(np_[idx] == len(idx))
        assert len(idx) in ((1,) if parts == 1 else (1, parts))
        if len(idx) > 1:
            assert c[t] >= 0.7 * c.max()


@pytest.mark.parametrize("parts", [1, 3])
def test_lpt_order_is_a_permutation(parts):
    c, tx, ty = _costs(64, 40, seed=5)
    st, s = _plan(c, tx, 1, parts)
    assert st == abi.RRTE_OK
    x, y, part, np_ = _decode(s)
    tiles = (y * tx + x).astype(np.int64)
    first = part == 0
    assert sorted(tiles[first].tolist()) == list(range(tx * ty))  # every tile once
    cost_order = c[tiles[first]].astype(np.int64)
    # slowest first, up to the 65536 cost buckets of the counting sort
    assert np.all(np.diff(cost_order) <= c.max() // 65535 + 1)
    if parts > 1:
        split = np.nonzero(np_ > 1)[0]
        assert len(split) > 0 and split.max() < MAX_SLOTS and split[-1] == len(split) - 1  # split ones first


def test_rejects_bad_arguments_and_small_buffers():
    c, tx, _ = _costs(16, 8)
    assert _plan(c, 0, 0)[0] == abi.RRTE_INVALID_ARG
    assert _plan(c, tx, 0, parts=5)[0] == abi.RRTE_INVALID_ARG
    assert _plan(c, tx, 1, cap=10)[0] == abi.RRTE_INVALID_ARG
