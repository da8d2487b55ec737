import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librrte_hip.so on a HIP device)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the product library and the oracle once per session (no-ops when up to date)."""
    jobs = str(min(8, os.cpu_count() or 1))
    subprocess.run(["make", "-s", "-j", jobs, "-C", str(ROOT / "rrte_amd" / "csrc")], check=True)
    subprocess.run(["make", "-s", "-j", jobs, "-C", str(ROOT / "oracle")], check=True)
