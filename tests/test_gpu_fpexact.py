"""The kernels' short correctly rounded f32 sequences (device_scene.hpp sqrt_rn, rcp_rn and the
constant-divisor step of div_rn) are bit-identical to the compiler's full sequences.

sqrt and 1/x are checked over every one of the 2^32 f32 bit patterns (a few seconds each on an
MI355X).  The constant-divisor division step is exponent-invariant inside its range guard, so
its proof is the sweep over all 2^46 significand pairs (`python tools/fpexact.py div`, about a
minute); the test runs a strided eighth of the b significands plus the edge significands.
"""
import ctypes as C

import pytest

from rrte_amd import abi

pytestmark = pytest.mark.gpu


def _check(kind, lo, hi):
    out = C.c_uint64(0)
    st = abi.load().rrte_hip_fpcheck(0, kind, lo, hi, C.byref(out))
    assert st == 0, abi.STATUS_NAMES.get(st, st)
    return out.value


def test_sqrt_rn_all_inputs():
    assert _check(abi.FPCHECK_SQRT, 0, 1 << 32) == 0


def test_sqrt_rn_branchfree_all_inputs():
    """The branch-free form (tiny inputs scaled by 2^64, +-0 / +inf through v_cmp_class)."""
    assert _check(abi.FPCHECK_SQRT_BF, 0, 1 << 32) == 0


def test_sweep_detects_one_ulp_errors():
    """Control: the bare hardware v_sqrt_f32 is only faithful; the same sweep must see it
    (about 3.4e8 of the 2^32 patterns differ from the correctly rounded result)."""
    assert _check(abi.FPCHECK_SQRT_HW, 0, 1 << 32) > 100_000_000


def test_rcp_rn_all_inputs():
    assert _check(abi.FPCHECK_RCP, 0, 1 << 32) == 0


def test_gamma_byte_all_inputs():
    """The frame's gamma-2.2 byte from v_log_f32 / v_exp_f32 with a powf fallback near byte
    boundaries equals to_u8(clamp(powf(c, 1/2.2))) for every f32 c."""
    assert _check(abi.FPCHECK_GAMMA_U8, 0, 1 << 32) == 0


@pytest.mark.parametrize("lo,hi", [(0, 1 << 12), ((1 << 23) - (1 << 12), 1 << 23)]
                         + [(k << 20, (k << 20) + (1 << 17)) for k in range(8)])
def test_constant_divisor_step(lo, hi):
    assert _check(abi.FPCHECK_DIV, lo, hi) == 0

