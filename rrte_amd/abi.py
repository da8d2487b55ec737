"""ctypes mirror of include/rrte_hip.h and the loader for librrte_hip.so.

The shared library is the product: if it is missing (not built, or built for
another arch) importing this module raises — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("RRTE_HIP_LIB", _HERE / "lib" / "librrte_hip.so"))

# ----------------------------------------------------------------- enums
RRTE_OK, RRTE_INVALID_ARG, RRTE_HIP_ERROR, RRTE_RCCL_ERROR, RRTE_UNSUPPORTED_PRIM, RRTE_NO_DEVICE = range(6)
STATUS_NAMES = {0: "OK", 1: "INVALID_ARG", 2: "HIP_ERROR", 3: "RCCL_ERROR", 4: "UNSUPPORTED_PRIM", 5: "NO_DEVICE"}

PRIM_SPHERE, PRIM_PLANE, PRIM_TRIANGLE, PRIM_CUBE, PRIM_CYLINDER, PRIM_CONE, PRIM_CAPSULE, PRIM_SDF, PRIM_MESH = range(9)
MAT_LAMBERTIAN, MAT_METAL, MAT_DIELECTRIC, MAT_EMISSIVE = range(4)
LIGHT_POINT, LIGHT_DIRECTIONAL, LIGHT_SPOT, LIGHT_AMBIENT = range(4)
PERSPECTIVE, ORTHOGRAPHIC = 0, 1
MODE_REFCOMPAT, MODE_LAMBERT_SHADOW = 0, 1
JITTER_CENTER, JITTER_RANDOM = 0, 1
ABI_VERSION = 2  # include/rrte_hip.h RRTE_ABI_VERSION
FLAG_F32_LINEAR = 1
FLAG_GATHER_OVERLAP = 2

SDF_SPHERE, SDF_BOX, SDF_CYLINDER, SDF_PRISM, SDF_TORUS = 1, 2, 3, 4, 5
SDF_TUBE, SDF_RING, SDF_CONE, SDF_CAPSULE, SDF_ELLIPSOID = 6, 7, 8, 9, 10
SDF_UNION, SDF_DIFFERENCE, SDF_INTERSECTION = 32, 33, 34
SDF_SMOOTH_UNION, SDF_SMOOTH_DIFFERENCE, SDF_SMOOTH_INTERSECTION = 35, 36, 37
SDF_BEND, SDF_TWIST, SDF_TAPER, SDF_NOISE, SDF_WAVE = 64, 65, 66, 67, 68
SDF_POP_POINT = 96
SDF_MAX_STACK, SDF_MAX_POINT_STACK, SDF_MAX_OCTAVES = 8, 4, 8
UNIQUE_ID_BYTES = 128
JIT_OFF, JIT_ON, JIT_AUTO = 0, 1, 2
FPCHECK_SQRT, FPCHECK_RCP, FPCHECK_DIV, FPCHECK_SQRT_HW, FPCHECK_GAMMA_U8, FPCHECK_SQRT_BF = 0, 1, 2, 3, 4, 5


# --------------------------------------------------------------- structs
class Prim(C.Structure):
    _fields_ = [
        ("kind", C.c_uint32), ("material", C.c_int32), ("sdf_first", C.c_uint32), ("sdf_count", C.c_uint32),
        ("sdf_max_steps", C.c_uint32), ("sdf_step_scale", C.c_float), ("sdf_hit_eps", C.c_float),
        ("flags", C.c_uint32), ("p", C.c_float * 20), ("trs", C.c_float * 10), ("_pad", C.c_float * 10),
    ]


class Material(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("fuzz", C.c_float), ("ior", C.c_float), ("_pad0", C.c_float),
                ("albedo", C.c_float * 4)]


class Light(C.Structure):
    _fields_ = [
        ("kind", C.c_uint32), ("intensity", C.c_float), ("range", C.c_float), ("linear", C.c_float),
        ("quadratic", C.c_float), ("inner_angle", C.c_float), ("outer_angle", C.c_float), ("_pad0", C.c_float),
        ("position", C.c_float * 4), ("direction", C.c_float * 4), ("color", C.c_float * 4),
    ]


class SdfNode(C.Structure):
    _fields_ = [("op", C.c_uint32), ("i", C.c_uint32 * 3), ("f", C.c_float * 12)]


class Camera(C.Structure):
    _fields_ = [
        ("position", C.c_float * 3), ("projection", C.c_uint32), ("rotation", C.c_float * 4),
        ("scale", C.c_float * 3), ("fov", C.c_float), ("aspect_ratio", C.c_float), ("near_plane", C.c_float),
        ("far_plane", C.c_float), ("left", C.c_float), ("right", C.c_float), ("bottom", C.c_float),
        ("top", C.c_float), ("_pad", C.c_float * 1),
    ]


class RenderParams(C.Structure):
    _fields_ = [
        ("width", C.c_uint32), ("height", C.c_uint32), ("samples_per_pixel", C.c_uint32),
        ("max_depth", C.c_uint32), ("mode", C.c_uint32), ("jitter", C.c_uint32), ("seed", C.c_uint32),
        ("flags", C.c_uint32), ("background", C.c_float * 4), ("t_min", C.c_float), ("shadow_bias", C.c_float),
        ("gamma", C.c_float), ("band_rows", C.c_uint32),
    ]


class MeshVertex(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("normal", C.c_float * 3)]


class SceneIR(C.Structure):
    _fields_ = [
        ("prims", C.POINTER(Prim)), ("num_prims", C.c_uint32),
        ("materials", C.POINTER(Material)), ("num_materials", C.c_uint32),
        ("lights", C.POINTER(Light)), ("num_lights", C.c_uint32),
        ("sdf_nodes", C.POINTER(SdfNode)), ("num_sdf_nodes", C.c_uint32),
        ("camera", Camera),
        ("mesh_vertices", C.POINTER(MeshVertex)), ("num_mesh_vertices", C.c_uint32),
        ("mesh_indices", C.POINTER(C.c_uint32)), ("num_mesh_indices", C.c_uint32),
        ("mesh_version", C.c_uint64),
    ]


class Stats(C.Structure):
    _fields_ = [("primary_rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("kernel_ms", C.c_double),
                ("gather_ms", C.c_double), ("upload_ms", C.c_double), ("frames", C.c_uint64),
                ("jit_active", C.c_uint32), ("hot_tiles", C.c_uint32), ("jit_compile_ms", C.c_double)]


assert C.sizeof(Prim) == 192 and C.sizeof(Material) == 32 and C.sizeof(Light) == 80
assert C.sizeof(SdfNode) == 64 and C.sizeof(Camera) == 80 and C.sizeof(RenderParams) == 64

# Every entry point include/rrte_hip.h declares: name -> (restype, argtypes)
_P = C.c_void_p
EXPORTS = {
    "rrte_hip_abi_version": (C.c_uint32, []),
    "rrte_hip_create": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "rrte_hip_destroy": (None, [_P]),
    "rrte_hip_last_error": (C.c_char_p, [_P]),
    "rrte_hip_render": (C.c_int, [_P, C.POINTER(SceneIR), C.POINTER(RenderParams), _P]),
    "rrte_hip_render_f32": (C.c_int, [_P, C.POINTER(SceneIR), C.POINTER(RenderParams), _P, _P]),
    "rrte_hip_render_async": (C.c_int, [_P, C.POINTER(SceneIR), C.POINTER(RenderParams), _P, _P, _P]),
    "rrte_hip_synchronize": (C.c_int, [_P]),
    "rrte_hip_query": (C.c_int, [_P, C.POINTER(C.c_uint32)]),
    "rrte_hip_stats": (C.c_int, [_P, C.POINTER(Stats)]),
    "rrte_hip_set_jit": (C.c_int, [_P, C.c_int]),
    "rrte_hip_jit_check": (C.c_int, [C.POINTER(SceneIR), C.c_int, C.c_char_p, C.c_size_t]),
    "rrte_hip_fpcheck": (C.c_int, [C.c_int, C.c_int, C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64)]),
    "rrte_hip_sdf_guards": (C.c_int, [C.POINTER(SdfNode), C.c_uint32, C.c_uint32, C.POINTER(SdfNode),
                                      C.POINTER(C.c_uint32)]),
    "rrte_hip_tile_order_plan": (C.c_int, [C.POINTER(C.c_uint32), C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32),
                                           C.c_uint32, C.POINTER(C.c_uint32)]),
    "rrte_hip_jit_cache_key": (C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p, C.c_size_t]),
    "rrte_hip_check_word": (C.c_int, [_P, C.POINTER(C.c_uint64)]),
    "rrte_hip_scene_dump": (C.c_int, [C.POINTER(SceneIR), C.POINTER(RenderParams), C.c_char_p]),
    "rrte_hip_scene_load": (C.c_int, [C.c_char_p, C.POINTER(SceneIR), C.POINTER(RenderParams), C.POINTER(_P)]),
    "rrte_hip_scene_free": (None, [_P]),
    "rrte_hip_comm_unique_id": (C.c_int, [_P]),
    "rrte_hip_comm_init": (C.c_int, [_P, C.c_int, C.c_int, _P]),
    "rrte_hip_render_gather": (C.c_int, [_P, C.POINTER(SceneIR), C.POINTER(RenderParams), C.c_int, _P]),
    "rrte_hip_render_gather_async": (C.c_int, [_P, C.POINTER(SceneIR), C.POINTER(RenderParams), C.c_int, _P, _P]),
    "rrte_hip_band_rows_for_rank": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_int, C.c_int]),
    "rrte_hip_band_layout": (C.c_int, [C.POINTER(SceneIR), C.POINTER(RenderParams), C.c_int, C.c_int,
                                       C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "rrte_hip_band_rows_for_rank_ex": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_int, C.c_int, C.c_uint32, C.c_uint32,
                                                    C.c_uint32]),
    "rrte_hip_set_gather_batch": (C.c_int, [_P, C.c_uint32]),
    "rrte_hip_flush": (C.c_int, [_P]),
    "rrte_hip_gather_info": (C.c_int, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]),
    "rrte_hip_build_id": (C.c_int, [C.c_char_p, C.c_size_t]),
    "rrte_hip_host_register": (C.c_int, [_P, C.c_void_p, C.c_size_t]),
    "rrte_hip_host_unregister": (C.c_int, [_P, C.c_void_p]),
    "rrte_hip_set_comm_timeout": (C.c_int, [_P, C.c_uint32]),
}

_lib = None


def load() -> C.CDLL:
    """Load librrte_hip.so (raises if it is absent: no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise RuntimeError(
            f"librrte_hip.so not found at {LIB_PATH}; build it with `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    # torch-rocm bundles its own libamdhip64.so.7 / librccl.so.1 (same SONAMEs as /opt/rocm).
    # Two HIP runtimes in one process corrupt each other at exit, so if torch is installed it is
    # loaded first and librrte_hip.so binds to the runtime torch already mapped (one per process).
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    lib = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.rrte_hip_abi_version() != ABI_VERSION:
        raise RuntimeError("librrte_hip.so ABI version mismatch")
    _lib = lib
    return lib


class RrteError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"rrte_hip {STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


def band_layout(scene_ref, params_ref, nranks: int, root: int = 0) -> tuple:
    """(sky_bands, root_bands, peer_bands) of rrte_hip_band_layout (include/rrte_hip.h) for a scene and
    params passed by reference; raises on an error status."""
    sky, rb, pb = C.c_uint32(), C.c_uint32(), C.c_uint32()
    st = load().rrte_hip_band_layout(scene_ref, params_ref, nranks, root, C.byref(sky), C.byref(rb), C.byref(pb))
    if st != RRTE_OK:
        raise RuntimeError(f"rrte_hip_band_layout: status {st}")
    return sky.value, rb.value, pb.value


def build_id() -> str:
    """rrte_hip_build_id: the device code's identity (headers, hiprtc options, hiprtc version)."""
    buf = C.create_string_buffer(64)
    st = load().rrte_hip_build_id(buf, 64)
    if st != RRTE_OK:
        raise RuntimeError(f"rrte_hip_build_id: status {st}")
    return buf.value.decode()
