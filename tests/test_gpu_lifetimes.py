"""Buffer lifetimes around the blocking entry points.

Round 5 recorded one "illegal memory access" at the f32 read-back of the second blocking render of a
fresh JIT_ON context (test_gpu_parity.py::test_convex_secant_early_miss_is_exact[641x359]).  This file
sets up that precondition deterministically and repeats it: a new context per iteration, a gamma
f32 render, stats, a linear f32 render, into caller buffers that are freed and re-allocated between
calls -- numpy heap buffers and anonymous mappings that are unmapped and mapped again (so the next
buffer lands at the address of one the runtime copied into a moment before) -- at odd frame sizes,
with the measured-cost tile order re-profiled and re-uploaded every launch (RRTE_TEST_RECYCLE=1) or
a fixed list re-uploaded every launch (RRTE_TILE_ORDER=2), both kernel kinds, and the kernel's own
index checks on (RRTE_DEBUG=4: every list slot, tile, frame and output row range-checked on the
device, rrte_hip_check_word).  Every frame must be the first frame's bytes and the check word 0."""
import ctypes as C
import mmap

import numpy as np
import pytest

import scenes_extra as se
from rrte_amd import LoweredScene, abi, scenes
from rrte_amd.renderer import Context

pytestmark = pytest.mark.gpu


class _Buf:
    """A caller buffer: a numpy heap array, or an anonymous mapping viewed as one that free() unmaps
    (the next mapping of the same size usually lands at the same address)."""

    def __init__(self, kind, n, dtype):
        self.mm = mmap.mmap(-1, n * np.dtype(dtype).itemsize) if kind == "mmap" else None
        self.a = np.frombuffer(self.mm, dtype=dtype) if self.mm is not None else np.empty(n, dtype=dtype)
        self.addr = self.a.ctypes.data

    def take(self):
        b = self.a.tobytes()
        self.a = None
        if self.mm is not None:
            self.mm.close()
        return b


def _render(ctx, sc, prm, addr8, addrf, linear):
    p = abi.RenderParams.from_buffer_copy(prm)
    if linear:
        p.flags |= abi.FLAG_F32_LINEAR
    ctx.check(ctx.lib.rrte_hip_render_f32(ctx.h, sc.ref(), C.byref(p), addr8, addrf))


def _check_word(ctx):
    w = C.c_uint64()
    ctx.check(ctx.lib.rrte_hip_check_word(ctx.h, C.byref(w)))
    return int(w.value)


@pytest.mark.parametrize("policy", ["recycle", "fixed_recycle"])
@pytest.mark.parametrize("jit", [abi.JIT_ON, abi.JIT_OFF])
def test_fresh_contexts_fresh_buffers(policy, jit, monkeypatch):
    monkeypatch.setenv("RRTE_DEBUG", "4")
    monkeypatch.setenv("RRTE_TEST_RECYCLE", "1")
    if policy == "fixed_recycle":
        monkeypatch.setenv("RRTE_TILE_ORDER", "2")
    ref = {}
    iters = 0
    for it in range(12):
        for (w, h) in [(641, 359), (240, 160), (333, 97)]:
            objs, lights, cam, cfg = se.convex_sdf_scene(w, h)
            sc = LoweredScene(objs, lights, cam)
            prm = cfg.lower()
            kind = "mmap" if it % 2 else "heap"
            ctx = Context(0, jit=jit)
            frames = []
            for linear in (False, True, False, True):
                out8, outf = _Buf(kind, w * h * 4, np.uint8), _Buf(kind, w * h * 4, np.float32)
                _render(ctx, sc, prm, out8.addr, outf.addr, linear)
                st = ctx.stats()
                frames.append((out8.take(), outf.take(), int(st.shadow_rays)))
            assert _check_word(ctx) == 0, (w, h, it)
            if jit == abi.JIT_ON:
                assert ctx.stats().jit_active == 1
            ctx.close()
            want = ref.setdefault((w, h), frames[:2])
            for i, f in enumerate(frames):
                assert f == want[i % 2], f"size {w}x{h} iteration {it} frame {i} ({kind} buffers)"
            iters += 1
    assert iters == 36


def test_check_word_reports_a_bad_slot(monkeypatch):
    """The device check itself: RRTE_FAULT_BAD_SLOT=1 (honoured only together with RRTE_DEBUG bit 2)
    makes slot 0 of every uploaded tile list name a tile far outside the frame; the wave that reads it
    must report code 2 and stop before touching memory, the rest of the frame renders, and the word
    clears after a read.  A clean context reads 0."""
    objs, lights, cam, cfg = se.convex_sdf_scene(97, 61)
    sc = LoweredScene(objs, lights, cam)
    prm = cfg.lower()
    monkeypatch.setenv("RRTE_DEBUG", "4")
    monkeypatch.setenv("RRTE_TILE_ORDER", "2")
    clean = Context(0, jit=abi.JIT_OFF)
    out8 = np.empty(97 * 61 * 4, np.uint8)
    clean.check(clean.lib.rrte_hip_render(clean.h, sc.ref(), C.byref(prm), out8.ctypes.data))
    assert _check_word(clean) == 0
    clean.close()
    monkeypatch.setenv("RRTE_FAULT_BAD_SLOT", "1")
    for jit in (abi.JIT_OFF, abi.JIT_ON):
        ctx = Context(0, jit=jit)
        ctx.check(ctx.lib.rrte_hip_render(ctx.h, sc.ref(), C.byref(prm), out8.ctypes.data))
        assert _check_word(ctx) == 2
        assert _check_word(ctx) == 0
        ctx.close()


def test_check_word_reports_a_bad_scene_record(monkeypatch):
    """The device check of the uploaded scene (rrte_hip.hip scene_records_check, RRTE_DEBUG bit 2):
    the uploaded objects' kinds, SDF node ranges and CSG-guard links are checked on the device copy the
    kernels read.  Clean uploads of SDF scenes with guards read 0; RRTE_FAULT_BAD_SLOT=2 puts an
    out-of-range kind into object 0 of the device copy only, which must report code 16 (the kernels skip
    an unknown kind, so the frame still completes)."""
    monkeypatch.setenv("RRTE_DEBUG", "4")
    out8 = None
    for name in ("sdf-showcase", "deformation-stress"):
        objs, lights, cam, cfg = scenes.SCENES[name](96, 54)
        sc = LoweredScene(objs, lights, cam)
        prm = cfg.lower()
        out8 = np.empty(96 * 54 * 4, np.uint8)
        ctx = Context(0, jit=abi.JIT_OFF)
        ctx.check(ctx.lib.rrte_hip_render(ctx.h, sc.ref(), C.byref(prm), out8.ctypes.data))
        assert _check_word(ctx) == 0, name
        ctx.close()
    objs, lights, cam, cfg = se.convex_sdf_scene(97, 61)
    sc = LoweredScene(objs, lights, cam)
    prm = cfg.lower()
    out8 = np.empty(97 * 61 * 4, np.uint8)
    monkeypatch.setenv("RRTE_FAULT_BAD_SLOT", "2")
    ctx = Context(0, jit=abi.JIT_OFF)
    ctx.check(ctx.lib.rrte_hip_render(ctx.h, sc.ref(), C.byref(prm), out8.ctypes.data))
    assert _check_word(ctx) == 16
    assert _check_word(ctx) == 0
    ctx.close()
