"""CPU proof of device_scene.hpp vnorm_unit's bit formula: for x = 1 + k ulp (|k| <= 1024),
RN(1 / RN(sqrt(x))) == bits(1.0f) - (k >= 0 ? k & ~1 : k >> 2), exhaustively (numpy float32 sqrt and
division are correctly rounded); the formula's first failure is at |k| = 2898, so the device guard
(|k| <= 1024) has margin.  Not GPU code: the integer ops are exact on any target."""
import numpy as np


def _formula(k):
    return (0x3F800000 - np.where(k >= 0, k & ~1, k >> 2)).astype(np.uint32).view(np.float32)


def _reference(k):
    x = (0x3F800000 + k).astype(np.uint32).view(np.float32)
    return (np.float32(1.0) / np.sqrt(x)).astype(np.float32)


def test_vnorm_unit_formula_exact_on_the_guarded_range():
    k = np.arange(-1024, 1025, dtype=np.int64)
    assert np.array_equal(_formula(k).view(np.uint32), _reference(k).view(np.uint32))


def test_vnorm_unit_formula_first_failure_is_outside_the_guard():
    k = np.arange(-(1 << 14), (1 << 14) + 1, dtype=np.int64)
    bad = np.abs(k[_formula(k).view(np.uint32) != _reference(k).view(np.uint32)])
    assert bad.min() == 2898
