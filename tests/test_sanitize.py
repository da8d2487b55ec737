"""Host-only code under AddressSanitizer + UndefinedBehaviorSanitizer: the CPU oracle,
the C++ mirror, and the host parts of librrte_hip -- validation and lowering, the BVH builder, the
CSG-guard analysis, the scene-specialised kernel's source generation and hiprtc compile -- built by
tools/sanitize.sh with clang's sanitizer runtime and driven by tests/cpp/sanitize_driver.cpp (oracle
renders at 1 and 4 threads must agree byte for byte; every SDF program through the guard analysis;
the ABI's error paths).  Device code is not instrumented (no GPU sanitizers on this pool)."""
import os
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def test_host_code_is_clean_under_asan_and_ubsan():
    env = dict(os.environ)
    r = subprocess.run(["bash", str(ROOT / "tools" / "sanitize.sh")], capture_output=True, text=True, env=env,
                       timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "sanitize_driver: all checks passed" in out, out[-2000:]
    assert "runtime error" not in out and "ERROR: AddressSanitizer" not in out, out[-4000:]


def test_host_threads_are_clean_under_tsan():
    """tools/tsan.sh: the host code a context runs on its worker threads (JIT source generation and
    hiprtc compile, tile-order planning, SceneIR dump / load, cache keys) and the mirror's lowering, on
    several threads at once, plus the oracle's thread pool, under ThreadSanitizer (tests/cpp/tsan_driver.cpp).
    It found the C++ mirror's mesh stamp counter racing (two meshes lowered on two threads could share
    a stamp, which keys the library's BVH cache); now atomic."""
    r = subprocess.run(["bash", str(ROOT / "tools" / "tsan.sh")], capture_output=True, text=True,
                       env=dict(os.environ), timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "tsan_driver: all checks passed" in out, out[-2000:]
    assert "ThreadSanitizer" not in out, out[-4000:]
