"""Host-side planning of the measured-cost tile order (rrte_hip_tile_order_plan, the code a context
runs after a profile; no device needed): every tile once, slowest first; slots decode to in-range
tiles."""
import ctypes as C

import numpy as np

from rrte_amd import abi


def _plan(costs, tiles_x, cap=None):
    lib = abi.load()  # (signatures from abi.EXPORTS)
    c = np.ascontiguousarray(costs, dtype=np.uint32)
    cap = cap if cap is not None else len(c) + 16
    out = np.zeros(cap, dtype=np.uint32)
    n = C.c_uint32()
    st = lib.rrte_hip_tile_order_plan(c.ctypes.data_as(C.POINTER(C.c_uint32)), len(c), tiles_x,
                                      out.ctypes.data_as(C.POINTER(C.c_uint32)), cap, C.byref(n))
    return st, out[: n.value]


def _costs(tx=240, ty=135, seed=3):
    rng = np.random.default_rng(seed)
    c = rng.gamma(2.0, 600.0, size=tx * ty).astype(np.uint32) + 200
    k = min(40, tx * ty)
    c[rng.choice(tx * ty, k, replace=False)] = rng.integers(8000, 10000, k)  # a silhouette tail
    return c, tx, ty


def test_lpt_order_is_a_permutation_slowest_first():
    for tx, ty, seed in ((64, 40, 5), (240, 135, 3), (480, 270, 7), (1, 9, 1), (13, 1, 2)):
        c, tx, ty = _costs(tx, ty, seed)
        st, s = _plan(c, tx)
        assert st == abi.RRTE_OK
        x, y = s & 0xFFFF, s >> 16
        assert np.all(x < tx) and np.all(y < ty)
        tiles = (y.astype(np.int64) * tx + x)
        assert sorted(tiles.tolist()) == list(range(tx * ty))  # every tile once
        order = c[tiles].astype(np.int64)
        # slowest first, up to the 65536 cost buckets of the counting sort
        assert np.all(np.diff(order) <= c.max() // 65535 + 1)
        assert tiles[0] == int(np.argmax(c)) or c[tiles[0]] >= c.max() - c.max() // 65535 - 1


def test_equal_costs_keep_tile_order():
    c = np.full(37, 5, dtype=np.uint32)
    st, s = _plan(c, 5)
    assert st == abi.RRTE_OK
    assert ((s >> 16) * 5 + (s & 0xFFFF)).tolist() == list(range(37))


def test_rejects_bad_arguments_and_small_buffers():
    c, tx, _ = _costs(16, 8)
    assert _plan(c, 0)[0] == abi.RRTE_INVALID_ARG
    assert _plan(c, tx, cap=10)[0] == abi.RRTE_INVALID_ARG
