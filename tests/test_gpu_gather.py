"""Multi-GPU frame path on one GPU: a 1-rank RCCL communicator with RRTE_FORCE_GATHER=1 drives
rrte_hip_render_gather(_async) through the real band render -> RCCL (ncclGather per frame; grouped
send / receive per batch, the root's own bands rendered in place or, RRTE_GATHER_SELF, sent to
itself) -> expansion sequence, with frames in flight on three streams, gathered per frame or in batches of 3 or 8
(rrte_hip_set_gather_batch: one ncclGather for a batch of frames on the comm stream; 7 frames leave
a partial batch for the flush), and with the (now ignored) RRTE_FLAG_GATHER_OVERLAP.  Every frame
must equal the plain single-context render bit for bit.  (N > 1 needs more GPUs than the
test box has; the band partition itself is covered by tests/test_dist.py with gloo.)"""
import ctypes as C

import numpy as np
import pytest

from rrte_amd import LambertianMaterial, LoweredScene, abi, scenes
from rrte_amd.math import Color, vec3
from rrte_amd.renderer import Context

pytestmark = pytest.mark.gpu


def _frames(n, w=320, h=200, alpha=None, first=0):
    """`alpha`: None = the stock scene (every alpha byte 255: RGB24 slabs); "material" = one material
    with albedo alpha -150 (its pixels' alpha byte 127); "spp2" = 2 samples under a background alpha
    of 0.2 (sky pixels 178).  The last two must fall back to RGBA8 slabs.  Frame i's camera is the
    (first + i)-th of a fly-by."""
    out = []
    for i in range(first, first + n):
        objs, lights, cam, cfg = scenes.sdf_showcase(w, h)
        cam.transform.position = vec3(0.0 + 0.7 * i, 8.0 - 0.3 * i, 20.0)
        cam.look_at((0, 2, 0))
        if alpha == "material":
            objs[3].material = LambertianMaterial(Color(0.2, 0.6, 0.9, -150.0))
        elif alpha == "recolour":  # another scene, same slab format
            objs[3].material = LambertianMaterial(Color(0.9, 0.3, 0.1, 1.0))
        elif alpha == "spp2":
            cfg.samples_per_pixel = 2
            cfg.background_color = Color(0.05, 0.05, 0.08, 0.2)
        out.append((LoweredScene(objs, lights, cam), cfg.lower()))
    return out


@pytest.mark.parametrize("route", ["in_place", "self"])
@pytest.mark.parametrize("batch", [1, 3, 8])
@pytest.mark.parametrize("overlap", [False, True])
@pytest.mark.parametrize("jit", [abi.JIT_OFF, abi.JIT_ON])
def test_gather_path_matches_plain_render(overlap, jit, batch, route, monkeypatch):
    """route in_place: the batched root renders its bands straight into the frames; self
    (RRTE_GATHER_SELF=1): the root's bands go through the peers' path -- packed slab, RCCL send and
    receive (to itself), expansion into the frames -- the path every peer's bands take at N > 1."""
    if route == "self":
        monkeypatch.setenv("RRTE_GATHER_SELF", "1")
    _check_gather(overlap, jit, batch, monkeypatch, None)


@pytest.mark.parametrize("route", ["in_place", "self"])
@pytest.mark.parametrize("batch", [3, 8])
def test_per_frame_batch_launches(batch, route, monkeypatch):
    """RRTE_BATCH_LAUNCH=0: each frame of a batch launched at its call on its caller's stream (the
    root in place, a peer into its send-slab slot) with only the exchange batched -- an A/B policy
    (measured slower than the default multi-frame launches)."""
    monkeypatch.setenv("RRTE_BATCH_LAUNCH", "0")
    if route == "self":
        monkeypatch.setenv("RRTE_GATHER_SELF", "1")
    _check_gather(False, abi.JIT_ON, batch, monkeypatch, None)


@pytest.mark.parametrize("alpha,rgb24", [(None, "0"), ("material", "1"), ("spp2", "1")])
def test_gather_slab_formats(alpha, rgb24, monkeypatch):
    """RGBA8 slabs when forced (RRTE_GATHER_RGB24=0) or when some alpha byte is not 255; every
    frame still equal to the plain render, alpha bytes included (the slab path: RRTE_GATHER_SELF)."""
    monkeypatch.setenv("RRTE_GATHER_RGB24", rgb24)
    monkeypatch.setenv("RRTE_GATHER_SELF", "1")
    _check_gather(True, abi.JIT_ON, 1, monkeypatch, alpha)
    _check_gather(False, abi.JIT_ON, 4, monkeypatch, alpha)


def _check_gather(overlap, jit, batch, monkeypatch, alpha):
    import torch

    monkeypatch.setenv("RRTE_FORCE_GATHER", "1")
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
    ctx.check(lib.rrte_hip_set_gather_batch(ctx.h, batch))
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(dev) for _ in range(3)]  # frames in flight, as bench.py runs them
    outs = [torch.empty(w * h, dtype=torch.int32, device=dev) for _ in frames]
    torch.cuda.synchronize()  # the fill ran on torch's stream; the renders run on others
    for i, ((sc, prm), o) in enumerate(zip(frames, outs)):
        p = abi.RenderParams.from_buffer_copy(prm)
        if overlap:
            p.flags |= abi.FLAG_GATHER_OVERLAP
        ctx.check(lib.rrte_hip_render_gather_async(ctx.h, sc.ref(), C.byref(p), 0, o.data_ptr(),
                                                    C.c_void_p(streams[i % 3].cuda_stream)))
    ctx.check(lib.rrte_hip_flush(ctx.h))  # the partial batch's gather (collective)
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


def test_gather_batch_arguments_and_size_change(monkeypatch):
    """Batch sizes outside [1, 16] are rejected; flushing with no open batch is a no-op; a frame of
    another size closes the open batch (its frames are gathered first), and every frame of a stream
    of alternating sizes (one of them not a multiple of 4 wide) still equals the plain render."""
    import torch

    monkeypatch.setenv("RRTE_FORCE_GATHER", "1")
    ctx = Context(0, jit=abi.JIT_ON)
    lib = ctx.lib
    uid = (C.c_uint8 * abi.UNIQUE_ID_BYTES)()
    ctx.check(lib.rrte_hip_comm_unique_id(uid))
    ctx.check(lib.rrte_hip_comm_init(ctx.h, 1, 0, uid))
    assert lib.rrte_hip_set_gather_batch(ctx.h, 0) == abi.RRTE_INVALID_ARG
    assert lib.rrte_hip_set_gather_batch(ctx.h, 17) == abi.RRTE_INVALID_ARG
    ctx.check(lib.rrte_hip_flush(ctx.h))
    ctx.check(lib.rrte_hip_set_gather_batch(ctx.h, 4))
    # widths 320 / 160: 4-pixel de-interleave; 162: the per-pixel form
    sizes = [(320, 200), (160, 96), (162, 90)]
    frames = [_frames(1, *sizes[i % 3])[0] for i in range(9)]
    ref = Context(0, jit=abi.JIT_OFF)
    want = []
    for sc, prm in frames:
        buf = np.zeros(prm.width * prm.height * 4, dtype=np.uint8)
        ref.check(ref.lib.rrte_hip_render(ref.h, sc.ref(), C.byref(prm), buf.ctypes.data_as(C.POINTER(C.c_uint8))))
        want.append(buf)
    ref.close()
    streams = [torch.cuda.Stream() for _ in range(2)]
    outs = [torch.empty(p.width * p.height, dtype=torch.int32, device="cuda") for _, p in frames]
    torch.cuda.synchronize()  # the fill ran on torch's stream; the renders run on others
    for i, ((sc, prm), o) in enumerate(zip(frames, outs)):
        ctx.check(lib.rrte_hip_render_gather_async(ctx.h, sc.ref(), C.byref(prm), 0, o.data_ptr(),
                                                    C.c_void_p(streams[i % 2].cuda_stream)))
    ctx.check(lib.rrte_hip_flush(ctx.h))
    ctx.check(lib.rrte_hip_synchronize(ctx.h))
    for i, o in enumerate(outs):
        assert np.array_equal(o.cpu().numpy().view(np.uint8), want[i]), f"frame {i}"
    ctx.close()


def test_gather_batch_multi_frame_launches_and_changes(monkeypatch):
    """A batch of 16 renders as two 8-frame launches (one camera per blockIdx.z); a scene change
    (another material), a sampling change (2 spp) or a new camera set mid-batch closes or joins the
    open batch as the header says, and every frame -- 26 of them, on two caller streams, the last
    batch partial -- equals the plain render of its own scene and camera."""
    import torch

    monkeypatch.setenv("RRTE_FORCE_GATHER", "1")
    frames = _frames(18)
    for sc_prm in _frames(3, first=18, alpha="recolour"):
        frames.insert(11, sc_prm)  # scene change in the middle of the first batch
    frames += _frames(3, first=21, alpha="spp2") + _frames(2, first=24)
    ref = Context(0, jit=abi.JIT_OFF)
    want = []
    for sc, prm in frames:
        buf = np.zeros(prm.width * prm.height * 4, dtype=np.uint8)
        ref.check(ref.lib.rrte_hip_render(ref.h, sc.ref(), C.byref(prm), buf.ctypes.data_as(C.POINTER(C.c_uint8))))
        want.append(buf)
    ref.close()
    assert not np.array_equal(want[0], want[1])  # every frame its own camera
    for jit in (abi.JIT_ON, abi.JIT_OFF):
        ctx = Context(0, jit=jit)
        lib = ctx.lib
        uid = (C.c_uint8 * abi.UNIQUE_ID_BYTES)()
        ctx.check(lib.rrte_hip_comm_unique_id(uid))
        ctx.check(lib.rrte_hip_comm_init(ctx.h, 1, 0, uid))
        ctx.check(lib.rrte_hip_set_gather_batch(ctx.h, 16))
        streams = [torch.cuda.Stream() for _ in range(2)]
        outs = [torch.full((p.width * p.height,), -1, dtype=torch.int32, device="cuda") for _, p in frames]
        torch.cuda.synchronize()  # the fill ran on torch's stream; the renders run on others
        for i, ((sc, prm), o) in enumerate(zip(frames, outs)):
            ctx.check(lib.rrte_hip_render_gather_async(ctx.h, sc.ref(), C.byref(prm), 0, o.data_ptr(),
                                                        C.c_void_p(streams[i % 2].cuda_stream)))
        ctx.check(lib.rrte_hip_flush(ctx.h))
        ctx.check(lib.rrte_hip_synchronize(ctx.h))
        for i, o in enumerate(outs):
            got = o.cpu().numpy().view(np.uint8)
            assert np.array_equal(got, want[i]), f"jit {jit} frame {i}: {(got != want[i]).sum()} bytes differ"
        ctx.close()


def test_query_reports_batched_work_done(monkeypatch):
    """rrte_hip_query: after a flush, polling until the context's own streams are idle is enough for
    every batched frame to be complete (the frames render and gather on the context's streams) --
    no device synchronisation before the outputs are read."""
    import torch

    monkeypatch.setenv("RRTE_FORCE_GATHER", "1")
    frames = _frames(6)
    ref = Context(0, jit=abi.JIT_ON)
    want = []
    for sc, prm in frames:
        buf = np.zeros(prm.width * prm.height * 4, dtype=np.uint8)
        ref.check(ref.lib.rrte_hip_render(ref.h, sc.ref(), C.byref(prm), buf.ctypes.data_as(C.POINTER(C.c_uint8))))
        want.append(buf)
    ref.close()
    ctx = Context(0, jit=abi.JIT_ON)
    lib = ctx.lib
    busy = C.c_uint32(7)
    ctx.check(lib.rrte_hip_query(ctx.h, C.byref(busy)))
    assert busy.value == 0  # nothing issued yet
    assert lib.rrte_hip_query(ctx.h, None) == abi.RRTE_INVALID_ARG
    uid = (C.c_uint8 * abi.UNIQUE_ID_BYTES)()
    ctx.check(lib.rrte_hip_comm_unique_id(uid))
    ctx.check(lib.rrte_hip_comm_init(ctx.h, 1, 0, uid))
    ctx.check(lib.rrte_hip_set_gather_batch(ctx.h, 4))
    stream = torch.cuda.Stream()
    outs = [torch.full((p.width * p.height,), -1, dtype=torch.int32, device="cuda") for _, p in frames]
    torch.cuda.synchronize()  # the fill ran on torch's stream; the renders run on others
    torch.cuda.synchronize()
    for (sc, prm), o in zip(frames, outs):
        ctx.check(lib.rrte_hip_render_gather_async(ctx.h, sc.ref(), C.byref(prm), 0, o.data_ptr(),
                                                    C.c_void_p(stream.cuda_stream)))
    ctx.check(lib.rrte_hip_flush(ctx.h))
    busy.value = 1
    while busy.value:
        ctx.check(lib.rrte_hip_query(ctx.h, C.byref(busy)))
    host = [torch.empty_like(o, device="cpu") for o in outs]
    side = torch.cuda.Stream()  # a stream that never waited on the library's work
    with torch.cuda.stream(side):
        for h, o in zip(host, outs):
            h.copy_(o)
    side.synchronize()
    for i, h in enumerate(host):
        assert np.array_equal(h.numpy().view(np.uint8), want[i]), f"frame {i}"
    ctx.check(lib.rrte_hip_synchronize(ctx.h))
    ctx.close()
