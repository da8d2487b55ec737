"""Register / scratch budget of the headline's scene-specialised kernel (CPU: hipcc cross-compiles the
generated source for gfx950, tools/jit_isa.sh).  A kernel-wide regression -- e.g. a debug helper left
out of line, whose call made the compiler spill the 3.5 KB kernel-argument block to scratch (2160
bytes per lane, every light scene ~10x slower) -- shows up here before a GPU run."""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="needs hipcc")
@pytest.mark.parametrize("scene,max_vgprs", [("sdf-showcase", 64), ("basic-demo", 64), ("advanced-demo", 64)])
def test_specialised_kernel_has_no_scratch(scene, max_vgprs, tmp_path):
    r = subprocess.run(["bash", str(ROOT / "tools" / "jit_isa.sh"), scene, str(tmp_path / "k.s")],
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    out = r.stdout + r.stderr
    scratch = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", out)
    vgprs = re.search(r"VGPRs: (\d+)", out)
    assert scratch and vgprs, out[-2000:]
    assert int(scratch.group(1)) == 0, out[-2000:]
    assert int(vgprs.group(1)) <= max_vgprs, out[-2000:]
