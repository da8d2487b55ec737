"""TEST INFRASTRUCTURE ONLY — ctypes loader for the CPU oracle (oracle/rrte_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / the CPU baseline.  See rrte_oracle.h for
the parity status ("parity unpinned" against the Rust binary, which cannot be
built here).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

from rrte_amd import abi

_HERE = Path(__file__).resolve().parent
LIB = _HERE / "build" / "librrte_oracle.so"


class OracleHit(C.Structure):
    _fields_ = [("t", C.c_float), ("point", C.c_float * 3), ("normal", C.c_float * 3), ("front_face", C.c_int32)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not LIB.exists():
        build()
    lib = C.CDLL(str(LIB))
    lib.rrte_oracle_render.restype = C.c_int
    lib.rrte_oracle_render.argtypes = [C.POINTER(abi.SceneIR), C.POINTER(abi.RenderParams), C.c_void_p, C.c_void_p,
                                       C.POINTER(C.c_uint64), C.c_int, C.c_uint32, C.c_uint32]
    lib.rrte_oracle_intersect.restype = C.c_int
    lib.rrte_oracle_intersect.argtypes = [C.POINTER(abi.SceneIR), C.c_uint32, C.POINTER(C.c_float),
                                          C.POINTER(C.c_float), C.c_float, C.c_float, C.POINTER(OracleHit)]
    lib.rrte_oracle_generate_ray.restype = None
    lib.rrte_oracle_generate_ray.argtypes = [C.POINTER(abi.Camera), C.c_float, C.c_float,
                                             C.POINTER(C.c_float), C.POINTER(C.c_float)]
    lib.rrte_oracle_look_at.restype = None
    lib.rrte_oracle_look_at.argtypes = [C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float)]
    lib.rrte_oracle_sdf_eval.restype = C.c_float
    lib.rrte_oracle_sdf_eval.argtypes = [C.POINTER(abi.SceneIR), C.c_uint32, C.POINTER(C.c_float)]
    lib.rrte_oracle_mat4_srt.restype = None
    lib.rrte_oracle_mat4_srt.argtypes = [C.POINTER(C.c_float), C.POINTER(C.c_float)]
    lib.rrte_oracle_mat4_inverse.restype = None
    lib.rrte_oracle_mat4_inverse.argtypes = [C.POINTER(C.c_float), C.POINTER(C.c_float)]
    for fn in ("rrte_oracle_sinf", "rrte_oracle_cosf"):
        getattr(lib, fn).restype = C.c_float
        getattr(lib, fn).argtypes = [C.c_float]
    lib.rrte_oracle_value_noise3.restype = None
    lib.rrte_oracle_value_noise3.argtypes = [C.c_float, C.c_float, C.c_float, C.c_uint32, C.POINTER(C.c_float)]
    _lib = lib
    return lib


def farr(vals):
    return (C.c_float * len(vals))(*[float(v) for v in vals])


def render(scene, params, nthreads=None, rows=None, want_f32=True, linear=False):
    """Render with the oracle.  Returns (rgba8 flat uint8, f32 flat or None, shadow_rays)."""
    lib = load()
    prm = abi.RenderParams.from_buffer_copy(params)
    if linear:
        prm.flags |= abi.FLAG_F32_LINEAR
    n = prm.width * prm.height * 4
    out8 = np.zeros(n, dtype=np.uint8)
    outf = np.zeros(n, dtype=np.float32) if want_f32 else None
    sh = C.c_uint64(0)
    r0, r1 = rows if rows else (0, 0)
    if nthreads is None:
        nthreads = int(os.environ.get("RRTE_ORACLE_THREADS", os.cpu_count() or 1))
    st = lib.rrte_oracle_render(C.byref(scene.ir), C.byref(prm), out8.ctypes.data,
                                outf.ctypes.data if outf is not None else None, C.byref(sh), nthreads, r0, r1)
    if st != 0:
        raise ValueError(f"oracle rejected the scene/params (status {st})")
    return out8, outf, sh.value


class Counts(C.Structure):
    """Mirror of rrte_oracle_counts (rrte_oracle.h)."""
    _fields_ = [("samples", C.c_uint64), ("pixels", C.c_uint64), ("isect_calls", C.c_uint64 * 16),
                ("isect_hits", C.c_uint64 * 16), ("mesh_tri_tests", C.c_uint64), ("root_checks", C.c_uint64),
                ("sdf_steps", C.c_uint64),
                ("sdf_normals", C.c_uint64), ("sdf_nodes", C.c_uint64 * 128), ("noise_octaves", C.c_uint64),
                ("light_evals", C.c_uint64 * 4), ("shaded_hits", C.c_uint64), ("lambert_lights", C.c_uint64),
                ("shadow_rays", C.c_uint64), ("lambert_terms", C.c_uint64), ("ref_light_terms", C.c_uint64),
                ("scatters", C.c_uint64 * 4), ("sphere_samples", C.c_uint64)]


_clib = None


def load_counting():
    """The counting build (librrte_oracle_count.so): same source, event counters compiled in."""
    global _clib
    if _clib is not None:
        return _clib
    path = _HERE / "build" / "librrte_oracle_count.so"
    if not path.exists():
        build()
    lib = C.CDLL(str(path))
    lib.rrte_oracle_render_counted.restype = C.c_int
    lib.rrte_oracle_render_counted.argtypes = [C.POINTER(abi.SceneIR), C.POINTER(abi.RenderParams),
                                               C.POINTER(Counts), C.c_int, C.c_uint32, C.c_uint32]
    lib.rrte_oracle_flops.restype = C.c_double
    lib.rrte_oracle_flops.argtypes = [C.POINTER(Counts)]
    _clib = lib
    return lib


def count(scene, params, nthreads=None, rows=None):
    """Instrumented event counts of one render and their algorithmic FP32 op total
    (SURVEY.md §8d).  Returns (Counts, flops)."""
    lib = load_counting()
    prm = abi.RenderParams.from_buffer_copy(params)
    cnt = Counts()
    r0, r1 = rows if rows else (0, 0)
    if nthreads is None:
        nthreads = int(os.environ.get("RRTE_ORACLE_THREADS", os.cpu_count() or 1))
    if lib.rrte_oracle_render_counted(C.byref(scene.ir), C.byref(prm), C.byref(cnt), nthreads, r0, r1) != 0:
        raise ValueError("oracle rejected the scene/params")
    return cnt, float(lib.rrte_oracle_flops(C.byref(cnt)))
