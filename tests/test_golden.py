"""Frozen oracle outputs (tests/golden/, made by tests/golden/make_golden.py): the oracle must
reproduce them exactly; on the GPU the product must match them (see test_gpu_parity.py)."""
import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))
import make_golden  # noqa: E402

GOLDEN = Path(__file__).resolve().parent / "golden"


@pytest.mark.parametrize("name,mode,w,h", make_golden.CASES)
def test_oracle_reproduces_golden(name, mode, w, h):
    fx = np.load(GOLDEN / f"{name}_{mode}_{w}x{h}.npz")
    img, lin_hash, shadow = make_golden.render_case(name, mode, w, h)
    assert int(fx["shadow_rays"]) == shadow
    assert str(fx["linear_sha256"]) == lin_hash
    assert np.array_equal(fx["rgba8"], img)
