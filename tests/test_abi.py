"""The C-ABI boundary (include/rrte_hip.h): the library loads, exports every declared
entry point, struct layouts match, and host-side argument checks work without a GPU."""
import ctypes as C
import os
import re
from pathlib import Path

import numpy as np
import pytest

from rrte_amd import abi

HEADER = Path(__file__).resolve().parents[1] / "include" / "rrte_hip.h"


def declared_functions():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(rrte_hip_\w+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = abi.load()
    names = declared_functions()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
        assert n in abi.EXPORTS, f"{n} missing from the ctypes mirror"
    assert lib.rrte_hip_abi_version() == 2


def test_struct_layouts_match_header_comments():
    assert C.sizeof(abi.Prim) == 192
    assert C.sizeof(abi.Material) == 32
    assert C.sizeof(abi.Light) == 80
    assert C.sizeof(abi.SdfNode) == 64
    assert C.sizeof(abi.Camera) == 80
    assert C.sizeof(abi.RenderParams) == 64
    assert C.sizeof(abi.MeshVertex) == 24
    assert C.sizeof(abi.SceneIR) == 4 * 16 + 80 + 2 * 16 + 8  # (pointer, count) pairs, camera, mesh pairs, version
    text = HEADER.read_text()
    for name, size in [("rrte_material", 32), ("rrte_light", 80), ("rrte_sdf_node", 64), ("rrte_camera", 80),
                       ("rrte_render_params", 64)]:
        assert re.search(r"\}\s*" + name + r";\s*/\*\s*" + str(size) + " bytes", text), name


def test_null_arguments_are_rejected_without_a_device():
    lib = abi.load()
    assert lib.rrte_hip_create(0, None) == abi.RRTE_INVALID_ARG
    assert lib.rrte_hip_render(None, None, None, None) == abi.RRTE_INVALID_ARG
    assert lib.rrte_hip_stats(None, None) == abi.RRTE_INVALID_ARG
    assert lib.rrte_hip_comm_unique_id(None) == abi.RRTE_INVALID_ARG
    assert lib.rrte_hip_last_error(None) == b"null context"
    lib.rrte_hip_destroy(None)  # no-op


@pytest.mark.parametrize("name", ["sdf-showcase", "deformation-stress", "sdf-showcase-literal"])
def test_scene_specialised_kernel_source_compiles(name):
    """jit.hip: the generated per-scene HIP source compiles with hiprtc for gfx950 (no device needed)."""
    from rrte_amd import LoweredScene, scenes
    objs, lights, cam, cfg = scenes.SCENES[name](32, 18)
    sc = LoweredScene(objs, lights, cam)
    log = C.create_string_buffer(1 << 16)
    st = abi.load().rrte_hip_jit_check(sc.ref(), 1, log, len(log))
    assert st == abi.RRTE_OK, log.value.decode()[:4000]


def test_create_reports_no_device_off_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    h = C.c_void_p()
    assert abi.load().rrte_hip_create(0, C.byref(h)) == abi.RRTE_NO_DEVICE


@pytest.mark.parametrize("H,band,n", [(1080, 16, 2), (1080, 16, 8), (2160, 16, 8), (1000, 16, 3), (7, 16, 4),
                                      (1080, 1, 8), (1, 16, 1)])
def test_band_partition_covers_every_row_once(H, band, n):
    lib = abi.load()
    rows = [lib.rrte_hip_band_rows_for_rank(H, band, n, r) for r in range(n)]
    assert sum(rows) == H
    assert rows[0] == max(rows)  # rank 0 owns the most rows: the gather slot size
    # mirror of the device mapping image_row(): local row -> image row, a bijection onto [0, H)
    seen = []
    for r in range(n):
        for lr in range(rows[r]):
            b, w = divmod(lr, band)
            seen.append((b * n + r) * band + w if n > 1 else lr)
    assert sorted(seen) == list(range(H))


def test_fpcheck_rejects_bad_ranges():
    """Argument validation happens before any device call (runs without a GPU)."""
    import ctypes as C

    out = C.c_uint64(0)
    lib = abi.load()
    assert lib.rrte_hip_fpcheck(0, abi.FPCHECK_DIV, 0, (1 << 23) + 1, C.byref(out)) == 1
    assert lib.rrte_hip_fpcheck(0, 7, 0, 1, C.byref(out)) == 1
    assert lib.rrte_hip_fpcheck(0, -1, 0, 1, C.byref(out)) == 1
    assert lib.rrte_hip_fpcheck(0, abi.FPCHECK_SQRT, 5, 4, C.byref(out)) == 1
    assert lib.rrte_hip_fpcheck(0, abi.FPCHECK_SQRT, 0, 1, None) == 1


def _band_of_local(rank, lb, n, sky, rb, pb):
    """Mirror of device_scene.hpp band_of_local (rb root bands, then pb rounds over the peers, per cycle)."""
    L = rb + (n - 1) * pb
    if rank == 0:
        if lb < sky:
            return lb
        t = lb - sky
        return sky + (t // rb) * L + t % rb
    return sky + (lb // pb) * L + rb + (rank - 1) + (lb % pb) * (n - 1)


@pytest.mark.parametrize("H,band,n", [(1080, 16, 2), (1080, 16, 8), (2160, 16, 8), (1000, 16, 3), (7, 16, 4),
                                      (480, 16, 8), (1080, 8, 5)])
@pytest.mark.parametrize("sky,rb,pb", [(0, 1, 1), (3, 1, 1), (16, 0, 1), (16, 1, 1), (40, 0, 1), (0, 1, 2), (12, 1, 3),
                                       (5, 1, 8), (0, 2, 3), (7, 3, 4), (9, 8, 1)])
def test_sky_band_partition_covers_every_row_once(H, band, n, sky, rb, pb):
    """rrte_hip_band_rows_for_rank_ex and the device mapping (band_of_local) for a partition with sky
    bands on rank 0: every image row exactly once, packed in image order per rank."""
    lib = abi.load()
    nb = (H + band - 1) // band
    sky = min(sky, nb - 1)
    if rb == 0 and sky == 0:
        return  # (not a layout band_layout produces: the root would own nothing)
    rows = [lib.rrte_hip_band_rows_for_rank_ex(H, band, n, r, sky, rb, pb) for r in range(n)]
    assert sum(rows) == H
    seen = []
    for r in range(n):
        prev = -1
        for lr in range(rows[r]):
            b, w = divmod(lr, band)
            y = _band_of_local(r, b, n, sky, rb, pb) * band + w
            assert y > prev  # packed in image order
            prev = y
            seen.append(y)
    assert sorted(seen) == list(range(H))


def test_band_layout_of_the_showcase():
    """The showcase camera sees sky above every object: the leading bands go to rank 0; none with one
    rank, none with RRTE_BAND_SKY=0 (the plain interleave), none for the all-covering ground views."""
    from rrte_amd import LoweredScene, scenes
    lib = abi.load()
    objs, lights, cam, cfg = scenes.sdf_showcase(1920, 1080)
    cfg.band_rows = 16
    sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
    sky, rb, pb = C.c_uint32(), C.c_uint32(), C.c_uint32()

    def layout(n, root=0):
        assert lib.rrte_hip_band_layout(sc.ref(), C.byref(prm), n, root, C.byref(sky), C.byref(rb),
                                        C.byref(pb)) == abi.RRTE_OK
        return sky.value, rb.value, pb.value
    s8, rb8, pb8 = layout(8)
    assert 8 <= s8 < 34 and rb8 < pb8  # ~a quarter of the rows is sky; at 8 ranks a smaller root share
    s2, rb2, pb2 = layout(2)
    assert s2 == s8 and rb2 >= 1  # at 2 ranks the root also takes a round-robin share
    assert layout(1) == (0, 1, 1)
    assert layout(8, root=3) == (0, 1, 1)  # a root other than rank 0: the plain interleave
    assert lib.rrte_hip_band_layout(sc.ref(), C.byref(prm), 0, 0, C.byref(sky), C.byref(rb),
                                    C.byref(pb)) == abi.RRTE_INVALID_ARG
    for bad in [(0, 9, 1), (0, 1, 0), (0, 1, 9), (0, 0, 1)]:  # outside the documented ranges
        assert lib.rrte_hip_band_rows_for_rank_ex(1080, 16, 8, 1, *bad) == 0


def test_jit_compile_writes_nothing_outside_its_temporary_directory(tmp_path):
    """jit.hip rtc_compile: hiprtc writes the named headers under its own temporary directory
    ($TMPDIR/comgr-*/include), resolving each name as a path; a name with "../" once put the API header
    at $TMPDIR/include/rrte_hip.h, shared by every process on the machine, so concurrent compiles
    (test workers, the ranks of a node) read each other's half-written copy and failed at random."""
    import subprocess
    import sys
    code = ("import ctypes as C\nfrom rrte_amd import abi, LoweredScene, scenes\n"
            "objs, lights, cam, cfg = scenes.SCENES['sdf-showcase'](32, 18)\n"
            "sc = LoweredScene(objs, lights, cam)\nlog = C.create_string_buffer(1 << 16)\n"
            "assert abi.load().rrte_hip_jit_check(sc.ref(), 1, log, len(log)) == abi.RRTE_OK, log.value[:2000]\n")
    env = dict(os.environ, TMPDIR=str(tmp_path))
    r = subprocess.run([sys.executable, "-c", code], cwd=str(Path(__file__).resolve().parents[1]), env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert not (tmp_path / "include").exists()
