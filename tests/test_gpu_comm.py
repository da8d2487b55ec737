"""Gather-path control semantics on one GPU (a 1-rank RCCL communicator, RRTE_FORCE_GATHER=1):
which calls close a gather batch (collective) and which only render it (local), rrte_hip_comm_init
with a batch open, and collective failure detection -- a stalled gather surfaces as
RRTE_RCCL_ERROR after the communicator timeout instead of hanging the host (the reference
has no failure path beyond stopping its loop, examples/basic-demo/src/main.rs:145-150).  The stall
is injected on the device (RRTE_FAULT_STALL_GATHER: a kernel ahead of the N-th collective spins
until the host gives up on it), the stand-in for a dead peer on a one-GPU box."""
import ctypes as C
import time

import numpy as np
import pytest

from rrte_amd import LoweredScene, abi, scenes
from rrte_amd.math import vec3
from rrte_amd.renderer import Context

pytestmark = pytest.mark.gpu

W, H = 160, 96


def _frames(n, first=0):
    out = []
    for i in range(first, first + n):
        objs, lights, cam, cfg = scenes.sdf_showcase(W, H)
        cam.transform.position = vec3(0.0 + 0.7 * i, 8.0 - 0.3 * i, 20.0)
        cam.look_at((0, 2, 0))
        out.append((LoweredScene(objs, lights, cam), cfg.lower()))
    return out


def _want(frames):
    ref = Context(0, jit=abi.JIT_OFF)
    want = []
    for sc, prm in frames:
        buf = np.zeros(W * H * 4, dtype=np.uint8)
        ref.check(ref.lib.rrte_hip_render(ref.h, sc.ref(), C.byref(prm), buf.ctypes.data_as(C.POINTER(C.c_uint8))))
        want.append(buf)
    ref.close()
    return want


def _comm(ctx):
    uid = (C.c_uint8 * abi.UNIQUE_ID_BYTES)()
    ctx.check(ctx.lib.rrte_hip_comm_unique_id(uid))
    ctx.check(ctx.lib.rrte_hip_comm_init(ctx.h, 1, 0, uid))


def _gather(ctx, sc, prm, out, stream=None):
    return ctx.lib.rrte_hip_render_gather_async(ctx.h, sc.ref(), C.byref(prm), 0, out.data_ptr(),
                                                C.c_void_p(stream.cuda_stream) if stream else None)


def test_local_calls_render_but_do_not_close_a_batch(monkeypatch):
    """rrte_hip_synchronize and a preview render of ANOTHER scene through rrte_hip_render_async are
    local: the open batch's frames are rendered (with the scene they were issued with) but not
    gathered -- their outputs stay untouched -- until the batch fills; then every frame is exact."""
    import torch
    monkeypatch.setenv("RRTE_FORCE_GATHER", "1")
    # the root's bands through the slab + RCCL path (a single-rank root otherwise renders its bands
    # straight into the frames at render time, so the outputs would not show whether a collective ran)
    monkeypatch.setenv("RRTE_GATHER_SELF", "1")
    frames = _frames(4)
    objs, lights, cam, cfg = scenes.basic_demo(W, H, mode="lambert_shadow")
    preview = (LoweredScene(objs, lights, cam), cfg.lower())
    want = _want(frames + [preview])
    ctx = Context(0, jit=abi.JIT_ON)
    _comm(ctx)
    ctx.check(ctx.lib.rrte_hip_set_gather_batch(ctx.h, 4))
    outs = [torch.full((W * H,), -1, dtype=torch.int32, device="cuda") for _ in frames]
    torch.cuda.synchronize()  # the fill ran on torch's stream; the renders run on others
    for (sc, prm), o in zip(frames[:3], outs):
        ctx.check(_gather(ctx, sc, prm, o))
    pv = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()  # the fill ran on torch's stream; the renders run on others
    ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, preview[0].ref(), C.byref(preview[1]), pv.data_ptr(), None, None))
    ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
    assert np.array_equal(pv.cpu().numpy().view(np.uint8), want[4])
    for o in outs[:3]:  # rendered, not gathered: the collective waits for the batch to close
        assert (o.cpu() == -1).all()
    ctx.check(_gather(ctx, *frames[3], outs[3]))  # 4th frame: the batch is full and closes
    ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
    for i, o in enumerate(outs):
        assert np.array_equal(o.cpu().numpy().view(np.uint8), want[i]), f"frame {i}"
    ctx.close()


def test_comm_init_gathers_the_open_batch_first(monkeypatch):
    """Re-initialising the communicator with a partial batch open gathers that batch on the old
    communicator first (it used to be dropped), then the new communicator works."""
    import torch
    monkeypatch.setenv("RRTE_FORCE_GATHER", "1")
    frames = _frames(5)
    want = _want(frames)
    ctx = Context(0, jit=abi.JIT_ON)
    _comm(ctx)
    ctx.check(ctx.lib.rrte_hip_set_gather_batch(ctx.h, 4))
    outs = [torch.full((W * H,), -1, dtype=torch.int32, device="cuda") for _ in frames]
    torch.cuda.synchronize()  # the fill ran on torch's stream; the renders run on others
    for (sc, prm), o in zip(frames[:2], outs):
        ctx.check(_gather(ctx, sc, prm, o))
    _comm(ctx)
    for (sc, prm), o in zip(frames[2:], outs[2:]):
        ctx.check(_gather(ctx, sc, prm, o))
    ctx.check(ctx.lib.rrte_hip_flush(ctx.h))
    ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
    for i, o in enumerate(outs):
        assert np.array_equal(o.cpu().numpy().view(np.uint8), want[i]), f"frame {i}"
    ctx.close()


@pytest.mark.parametrize("batch", [1, 3])
def test_stalled_gather_surfaces_as_error(batch, monkeypatch):
    """The 2nd collective stalls on the device; the host's bounded wait gives up after the comm
    timeout (300 ms), aborts the communicator and returns RRTE_RCCL_ERROR with the reason.  Later
    gather calls fail fast until rrte_hip_comm_init; after it, frames are exact again."""
    import torch
    monkeypatch.setenv("RRTE_FORCE_GATHER", "1")
    monkeypatch.setenv("RRTE_FAULT_STALL_GATHER", "2")
    frames = _frames(3 * batch)
    want = _want(frames)
    ctx = Context(0, jit=abi.JIT_ON)
    _comm(ctx)
    ctx.check(ctx.lib.rrte_hip_set_comm_timeout(ctx.h, 300))
    assert ctx.lib.rrte_hip_set_comm_timeout(ctx.h, 0) == abi.RRTE_INVALID_ARG
    ctx.check(ctx.lib.rrte_hip_set_gather_batch(ctx.h, batch))
    stream = torch.cuda.Stream()
    outs = [torch.full((W * H,), -1, dtype=torch.int32, device="cuda") for _ in frames]
    torch.cuda.synchronize()  # the fill ran on torch's stream; the renders run on others
    for (sc, prm), o in zip(frames[:2 * batch], outs):  # collectives 1 and 2 (the stalled one)
        ctx.check(_gather(ctx, sc, prm, o, stream))
    t0 = time.perf_counter()
    rc = ctx.lib.rrte_hip_synchronize(ctx.h)
    dt = time.perf_counter() - t0
    msg = ctx.lib.rrte_hip_last_error(ctx.h)
    assert rc == abi.RRTE_RCCL_ERROR, (rc, msg)
    assert b"did not complete within 300 ms" in msg and b"aborted" in msg, msg
    assert 0.25 < dt < 4.0, dt  # the timeout, not the injected stall's own 5 s deadline
    assert _gather(ctx, *frames[0], outs[0], stream) == abi.RRTE_RCCL_ERROR
    assert b"rrte_hip_comm_init" in ctx.lib.rrte_hip_last_error(ctx.h)
    assert np.array_equal(outs[0].cpu().numpy().view(np.uint8), want[0])  # gathered before the stall
    _comm(ctx)  # recovery (the injected fault is one-shot)
    for (sc, prm), o in zip(frames[2 * batch:], outs[2 * batch:]):
        ctx.check(_gather(ctx, sc, prm, o, stream))
    ctx.check(ctx.lib.rrte_hip_flush(ctx.h))
    ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
    for i in range(2 * batch, 3 * batch):
        assert np.array_equal(outs[i].cpu().numpy().view(np.uint8), want[i]), f"frame {i}"
    ctx.close()


def _animated_frames(n):
    """Frames whose SCENE changes every frame (a light dimmed step by step): every frame call uploads
    a new scene version."""
    from rrte_amd.math import f32
    out = []
    for i in range(n):
        objs, lights, cam, cfg = scenes.sdf_showcase(W, H)
        lights[0].intensity = f32(25.0 - 0.5 * i)
        out.append((LoweredScene(objs, lights, cam), cfg.lower()))
    return out


@pytest.mark.parametrize("what", ["tile_list_recycle", "scene_change"])
def test_stall_during_recycle_or_scene_change_is_bounded(what, monkeypatch):
    """while the 2nd collective is stalled, frames keep arriving that (a) recycle the
    tile-list version pool every launch (RRTE_TEST_RECYCLE=1 with the fixed list) or (b) change the
    scene every frame, so the scene-version ring wraps onto versions read by renders queued behind the
    stalled gather.  Nothing may wait on the device unboundedly: (a) never waits at all (a version is
    reused only once its readers completed; otherwise the launch keeps its list), (b) waits for the
    version with the comm timeout.  The error surfaces as RRTE_RCCL_ERROR within the timeout, and
    after rrte_hip_comm_init frames are exact again."""
    import torch
    monkeypatch.setenv("RRTE_FORCE_GATHER", "1")
    monkeypatch.setenv("RRTE_FAULT_STALL_GATHER", "2")
    if what == "tile_list_recycle":
        monkeypatch.setenv("RRTE_TILE_ORDER", "2")
        monkeypatch.setenv("RRTE_TEST_RECYCLE", "1")
        frames = _frames(30)
    else:
        frames = _animated_frames(30)
    want = _want(frames[-3:])
    # compile the kernels the timed frames use (full, then topology once the values change) outside the
    # timed region: the JIT's disk cache then serves them, so `dt` measures the stall bound, not hiprtc
    warm = Context(0, jit=abi.JIT_ON)
    for sc, prm in frames[:2]:
        buf = np.zeros(W * H * 4, dtype=np.uint8)
        warm.check(warm.lib.rrte_hip_render(warm.h, sc.ref(), C.byref(prm), buf.ctypes.data_as(C.POINTER(C.c_uint8))))
    warm.close()
    ctx = Context(0, jit=abi.JIT_ON)
    _comm(ctx)
    ctx.check(ctx.lib.rrte_hip_set_comm_timeout(ctx.h, 300))
    ctx.check(ctx.lib.rrte_hip_set_gather_batch(ctx.h, 3))
    stream = torch.cuda.Stream()
    outs = [torch.full((W * H,), -1, dtype=torch.int32, device="cuda") for _ in frames]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rc = abi.RRTE_OK
    for (sc, prm), o in zip(frames[:27], outs):  # 9 batches: the 2nd one's gather stalls
        rc = _gather(ctx, sc, prm, o, stream)
        if rc != abi.RRTE_OK:
            break
    if rc == abi.RRTE_OK:
        rc = ctx.lib.rrte_hip_synchronize(ctx.h)
    dt = time.perf_counter() - t0
    msg = ctx.lib.rrte_hip_last_error(ctx.h)
    assert rc == abi.RRTE_RCCL_ERROR, (rc, msg)
    assert b"did not complete within 300 ms" in msg and b"aborted" in msg, msg
    assert dt < 4.0, dt  # the timeout, not the injected stall's own 5 s deadline
    _comm(ctx)  # recovery (the injected fault is one-shot)
    for (sc, prm), o in zip(frames[27:], outs[27:]):
        ctx.check(_gather(ctx, sc, prm, o, stream))
    ctx.check(ctx.lib.rrte_hip_flush(ctx.h))
    ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
    for j, i in enumerate(range(27, 30)):
        assert np.array_equal(outs[i].cpu().numpy().view(np.uint8), want[j]), f"frame {i}"
    ctx.close()


def _info(ctx):
    colls, open_frames = C.c_uint64(0), C.c_uint32(0)
    ctx.check(ctx.lib.rrte_hip_gather_info(ctx.h, C.byref(colls), C.byref(open_frames)))
    return colls.value, open_frames.value


def _recoloured_frames(n):
    """The same topology and array counts as _frames (sdf-showcase), another value: a material
    recoloured in place (a new material object would add a material record -- another count, which
    closes a batch on every rank alike)."""
    from rrte_amd.math import Color
    out = []
    for i in range(n):
        objs, lights, cam, cfg = scenes.sdf_showcase(W, H)
        objs[3].material._albedo = Color(0.9, 0.3, 0.1, 1.0)
        out.append((LoweredScene(objs, lights, cam), cfg.lower()))
    return out


def test_local_render_keeps_the_in_place_batch_open(monkeypatch):
    """the in-place root's batch stays open across local calls.  A scene change with
    unchanged array counts (same topology: the open batch is rendered locally first) and
    rrte_hip_synchronize (also renders it locally) must not change the batch-compatibility key, or
    the root alone would close the batch and issue a collective its peers do not (RGB24 slabs: the
    LAMBERT_SHADOW default).  No collective may be issued until the batch fills."""
    import torch
    monkeypatch.setenv("RRTE_FORCE_GATHER", "1")
    frames = _frames(3) + _recoloured_frames(2) + _frames(3, first=3)
    want = _want(frames)
    ctx = Context(0, jit=abi.JIT_ON)
    _comm(ctx)
    ctx.check(ctx.lib.rrte_hip_set_gather_batch(ctx.h, 8))
    outs = [torch.full((W * H,), -1, dtype=torch.int32, device="cuda") for _ in frames]
    torch.cuda.synchronize()  # the fill ran on torch's stream; the renders run on others
    for i, ((sc, prm), o) in enumerate(zip(frames[:7], outs)):
        ctx.check(_gather(ctx, sc, prm, o))
        assert _info(ctx) == (0, i + 1), f"after frame {i}"
        if i == 5:
            ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))  # local: renders the open batch, keeps it open
            assert _info(ctx) == (0, 6)
    ctx.check(_gather(ctx, *frames[7], outs[7]))  # the 8th frame fills the batch: one exchange
    assert _info(ctx) == (1, 0)
    ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
    for i, o in enumerate(outs):
        assert np.array_equal(o.cpu().numpy().view(np.uint8), want[i]), f"frame {i}"
    ctx.close()


def test_wait_without_communicator_is_unbounded(monkeypatch):
    """without a communicator nothing can stall a frame, so rrte_hip_synchronize
    waits as long as the device needs -- far past the communicator timeout -- and returns RRTE_OK.
    ADVICE r05 (low): the wait keeps a limit far above any frame (RRTE_NOCOMM_WAIT_MS, default 10
    minutes, 0 = none) so a hung kernel still returns; a short limit returns RRTE_HIP_ERROR."""
    import torch
    objs, lights, cam, cfg = scenes.deformation_stress(1920, 1080)
    sc, prm = LoweredScene(objs, lights, cam), cfg.lower()
    out = torch.empty(1920 * 1080, dtype=torch.int32, device="cuda")
    for limit in (None, "1"):
        if limit:
            monkeypatch.setenv("RRTE_NOCOMM_WAIT_MS", limit)
        ctx = Context(0, jit=abi.JIT_ON)
        ctx.check(ctx.lib.rrte_hip_set_comm_timeout(ctx.h, 1))
        if limit is None:
            ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(prm), out.data_ptr(), None, None))
            ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))  # (compile + first frame)
        t0 = time.perf_counter()
        for _ in range(24):  # ~5 ms each: >> the 1 ms comm timeout
            ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(prm), out.data_ptr(), None, None))
        rc = ctx.lib.rrte_hip_synchronize(ctx.h)
        dt = time.perf_counter() - t0
        if limit is None:
            assert rc == abi.RRTE_OK, ctx.lib.rrte_hip_last_error(ctx.h)
            assert dt > 0.02, dt  # the wait really outlasted the comm timeout
        else:
            assert rc == abi.RRTE_HIP_ERROR, rc
            assert b"did not complete within 1 ms" in ctx.lib.rrte_hip_last_error(ctx.h)
        torch.cuda.synchronize()
        ctx.close()
