"""Multi-GPU frame path on one GPU: a 1-rank RCCL communicator with RRTE_FORCE_GATHER=1 drives
rrte_hip_render_gather(_async) through the real band render -> ncclGather -> de-interleave
sequence, in both the single-stream and the pipelined (RRTE_FLAG_GATHER_OVERLAP) form.  Every
frame must equal the plain single-context render bit for bit.  (N > 1 needs more GPUs than the
test box has; the band partition itself is covered by tests/test_dist.py with gloo.)"""
import ctypes as C

import numpy as np
import pytest

from rrte_amd import LambertianMaterial, LoweredScene, abi, scenes
from rrte_amd.math import Color, vec3
from rrte_amd.renderer import Context

pytestmark = pytest.mark.gpu


def _frames(n, w=320, h=200, alpha=None):
    """`alpha`: None = the stock scene (every alpha byte 255: RGB24 slabs); "material" = one material
    with albedo alpha -150 (its pixels' alpha byte 127); "spp2" = 2 samples under a background alpha
    of 0.2 (sky pixels 178).  The last two must fall back to RGBA8 slabs."""
    out = []
    for i in range(n):
        objs, lights, cam, cfg = scenes.sdf_showcase(w, h)
        cam.transform.position = vec3(0.0 + 0.7 * i, 8.0 - 0.3 * i, 20.0)
        cam.look_at((0, 2, 0))
        if alpha == "material":
            objs[3].material = LambertianMaterial(Color(0.2, 0.6, 0.9, -150.0))
        elif alpha == "spp2":
            cfg.samples_per_pixel = 2
            cfg.background_color = Color(0.05, 0.05, 0.08, 0.2)
        out.append((LoweredScene(objs, lights, cam), cfg.lower()))
    return out


@pytest.mark.parametrize("comms", ["1", "2"])
@pytest.mark.parametrize("overlap", [False, True])
@pytest.mark.parametrize("jit", [abi.JIT_OFF, abi.JIT_ON])
def test_gather_path_matches_plain_render(overlap, jit, comms, monkeypatch):
    _check_gather(overlap, jit, comms, monkeypatch, None)


@pytest.mark.parametrize("alpha,rgb24", [(None, "0"), ("material", "1"), ("spp2", "1")])
def test_gather_slab_formats(alpha, rgb24, monkeypatch):
    """RGBA8 slabs when forced (RRTE_GATHER_RGB24=0) or when some alpha byte is not 255; every
    frame still equal to the plain render, alpha bytes included."""
    monkeypatch.setenv("RRTE_GATHER_RGB24", rgb24)
    _check_gather(True, abi.JIT_ON, "1", monkeypatch, alpha)


def _check_gather(overlap, jit, comms, monkeypatch, alpha):
    import torch

    monkeypatch.setenv("RRTE_FORCE_GATHER", "1")
    monkeypatch.setenv("RRTE_GATHER_COMMS", comms)
    frames = _frames(7, alpha=alpha)
    w, h = frames[0][1].width, frames[0][1].height
    ref = Context(0, jit=jit)
    want = []
    for sc, prm in frames:
        buf = np.zeros(w * h * 4, dtype=np.uint8)
        ref.check(ref.lib.rrte_hip_render(ref.h, sc.ref(), C.byref(prm), buf.ctypes.data_as(C.POINTER(C.c_uint8))))
        want.append(buf)
    ref.close()

    ctx = Context(0, jit=jit)
    lib = ctx.lib
    uid = (C.c_uint8 * abi.UNIQUE_ID_BYTES)()
    ctx.check(lib.rrte_hip_comm_unique_id(uid))
    ctx.check(lib.rrte_hip_comm_init(ctx.h, 1, 0, uid))
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(dev) for _ in range(3)]  # frames in flight, as bench.py runs them
    outs = [torch.empty(w * h, dtype=torch.int32, device=dev) for _ in frames]
    for i, ((sc, prm), o) in enumerate(zip(frames, outs)):
        p = abi.RenderParams.from_buffer_copy(prm)
        if overlap:
            p.flags |= abi.FLAG_GATHER_OVERLAP
        ctx.check(lib.rrte_hip_render_gather_async(ctx.h, sc.ref(), C.byref(p), 0, o.data_ptr(),
                                                    C.c_void_p(streams[i % 3].cuda_stream)))
    ctx.check(lib.rrte_hip_synchronize(ctx.h))
    for i, o in enumerate(outs):
        got = o.cpu().numpy().view(np.uint8)
        assert np.array_equal(got, want[i]), f"frame {i}: {(got != want[i]).sum()} bytes differ"
    if alpha is not None:  # the scene really has alpha bytes below 255
        assert (want[0].reshape(-1, 4)[:, 3] < 255).any()
    # blocking variant to host memory
    buf = np.zeros(w * h * 4, dtype=np.uint8)
    sc, prm = frames[2]
    ctx.check(lib.rrte_hip_render_gather(ctx.h, sc.ref(), C.byref(prm), 0, buf.ctypes.data_as(C.POINTER(C.c_uint8))))
    assert np.array_equal(buf, want[2])
    ctx.close()


def test_gather_requires_comm_and_root_buffer(monkeypatch):
    monkeypatch.setenv("RRTE_FORCE_GATHER", "1")
    (sc, prm), = _frames(1, 64, 48)
    ctx = Context(0)
    uid = (C.c_uint8 * abi.UNIQUE_ID_BYTES)()
    ctx.check(ctx.lib.rrte_hip_comm_unique_id(uid))
    ctx.check(ctx.lib.rrte_hip_comm_init(ctx.h, 1, 0, uid))
    assert ctx.lib.rrte_hip_render_gather_async(ctx.h, sc.ref(), C.byref(prm), 0, None, None) == abi.RRTE_INVALID_ARG
    assert ctx.lib.rrte_hip_render_gather_async(ctx.h, sc.ref(), C.byref(prm), 1, None, None) == abi.RRTE_INVALID_ARG
    ctx.close()
