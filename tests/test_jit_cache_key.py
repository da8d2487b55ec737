"""The persistent JIT code-object cache key (rrte_amd/csrc/jit.hip cache_key): a
specialised kernel is a function of its generated source AND of the device headers compiled into the
library (the generated source only says #include "ray_kernels.hpp") AND of the hiprtc options, so
the key must change with each of them -- a rebuilt library whose ray_kernels.hpp changed must miss
the cache instead of loading a code object with a stale argument layout.  Host only."""
import ctypes as C

from rrte_amd import abi


def _key(src, hdr=None):
    out = C.create_string_buffer(64)
    st = abi.load().rrte_hip_jit_cache_key(src.encode(), hdr.encode() if hdr is not None else None, out, 64)
    assert st == abi.RRTE_OK
    return out.value.decode()


def test_key_is_stable_and_hex():
    k = _key("extern \"C\" __global__ void rrte_jit_kernel() {}")
    assert k == _key("extern \"C\" __global__ void rrte_jit_kernel() {}")
    assert len(k) == 32 and all(ch in "0123456789abcdef" for ch in k)


def test_key_changes_with_the_source():
    assert _key("a") != _key("b")


def test_an_edited_header_misses_the_cache():
    """headers_override stands in for the embedded kHdrApi/kHdrDeviceScene/kHdrRayKernels of a
    rebuilt library: any change of their text changes the key."""
    src = "#include \"ray_kernels.hpp\"\n"
    base = _key(src)
    hdr = "struct KParams { unsigned width, height; };"
    edited = "struct KParams { unsigned width, height, rows; };"
    assert _key(src, hdr) != base
    assert _key(src, hdr) != _key(src, edited)
    assert _key(src, hdr) == _key(src, hdr)


def test_key_changes_with_the_compile_options(monkeypatch):
    src = "x"
    monkeypatch.delenv("RRTE_JIT_EXTRA_OPTS", raising=False)
    plain = _key(src)
    monkeypatch.setenv("RRTE_JIT_EXTRA_OPTS", "-DRRTE_SECANT_EXIT=0")
    assert _key(src) != plain
    monkeypatch.setenv("RRTE_JIT_EXTRA_OPTS", "-DRRTE_SECANT_EXIT=0 -DX")
    assert _key(src) != plain


def test_rejects_bad_arguments():
    out = C.create_string_buffer(8)
    assert abi.load().rrte_hip_jit_cache_key(b"x", None, out, 8) == abi.RRTE_INVALID_ARG
    assert abi.load().rrte_hip_jit_cache_key(None, None, C.create_string_buffer(64), 64) == abi.RRTE_INVALID_ARG
