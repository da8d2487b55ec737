"""SceneIR dump / load (SURVEY §5 repro; rrte_amd/csrc/scene_io.hip): a dumped frame reloads to the
same IR bytes and parameters and replays bit for bit on the CPU oracle; damaged files are refused.
The device side -- RRTE_DUMP_SCENE writing the frame a render call was given -- is in
test_scene_io_gpu below."""
import ctypes as C

import numpy as np
import pytest

import oracle
from rrte_amd import LoweredScene, abi, scenes, sceneio


def _arrays(ir):
    """The IR's arrays as bytes (pointer-free), for comparison."""
    def arr(ptr, n, T):
        return bytes(C.string_at(ptr, n * C.sizeof(T))) if n else b""
    return (arr(ir.prims, ir.num_prims, abi.Prim), arr(ir.materials, ir.num_materials, abi.Material),
            arr(ir.lights, ir.num_lights, abi.Light), arr(ir.sdf_nodes, ir.num_sdf_nodes, abi.SdfNode),
            bytes(ir.camera), arr(ir.mesh_vertices, ir.num_mesh_vertices, abi.MeshVertex),
            arr(ir.mesh_indices, ir.num_mesh_indices, C.c_uint32), ir.mesh_version)


@pytest.mark.parametrize("name", ["deformation-stress", "mesh-demo", "sdf-showcase-literal"])
def test_dump_load_roundtrip_replays_on_the_oracle(name, tmp_path):
    objs, lights, cam, cfg = scenes.SCENES[name](48, 27)
    sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
    path = tmp_path / "frame.rrtesir"
    sceneio.dump(sc.ref(), prm, str(path))
    ld = sceneio.load(str(path))
    assert _arrays(ld.ir) == _arrays(sc.ir)
    assert bytes(ld.params) == bytes(prm)
    a8, _, ash = oracle.render(sc, prm, nthreads=4, want_f32=False)
    b8, _, bsh = oracle.render(ld, ld.params, nthreads=4, want_f32=False)
    assert np.array_equal(a8, b8) and ash == bsh
    ld.close()


def test_damaged_dumps_are_refused(tmp_path):
    objs, lights, cam, cfg = scenes.sdf_showcase(16, 9)
    sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
    path = tmp_path / "f.rrtesir"
    sceneio.dump(sc.ref(), prm, str(path))
    raw = path.read_bytes()
    for bad in (raw[:-1], raw[:100], raw[:40] + bytes([raw[40] ^ 1]) + raw[41:], b"RRTESIR\x00" + raw[8:20]):
        path.write_bytes(bad)
        with pytest.raises(abi.RrteError):
            sceneio.load(str(path))
    with pytest.raises(abi.RrteError):
        sceneio.load(str(tmp_path / "missing"))


@pytest.mark.gpu
def test_scene_io_gpu(tmp_path, monkeypatch):
    """RRTE_DUMP_SCENE: the library writes the frame a render call was given; replayed on the device
    it renders the same bytes, and on the oracle the same image (u8 <= 1, the gamma powf ulp)."""
    from rrte_amd.renderer import Context
    path = tmp_path / "last.rrtesir"
    monkeypatch.setenv("RRTE_DUMP_SCENE", str(path))
    objs, lights, cam, cfg = scenes.deformation_stress(200, 120)
    sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
    ctx = Context(0, jit=abi.JIT_OFF)
    out = np.empty(200 * 120 * 4, np.uint8)
    ctx.check(ctx.lib.rrte_hip_render(ctx.h, sc.ref(), C.byref(prm), out.ctypes.data))
    ctx.close()
    monkeypatch.delenv("RRTE_DUMP_SCENE")
    ld = sceneio.load(str(path))
    ctx = Context(0, jit=abi.JIT_OFF)
    again = np.empty_like(out)
    ctx.check(ctx.lib.rrte_hip_render(ctx.h, ld.ref(), C.byref(ld.params), again.ctypes.data))
    ctx.close()
    assert np.array_equal(out, again)
    r8, _, _ = oracle.render(ld, ld.params, nthreads=16, want_f32=False)
    assert np.abs(r8.astype(int) - out.astype(int)).max() <= 1
