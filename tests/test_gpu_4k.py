"""BASELINE configs[3] -- sdf-showcase at 3840x2160, row-tiled across 2/4/8 GPUs -- against the oracle
(scene: examples/sdf-showcase/src/main.rs:168-381 layout with real SDFs).

At 4K the frame is wider than 2048 pixels, so camera-ray tile culling switches from 8x8 tiles to
16x16 blocks (rrte_hip.hip fill_tile_rects); every rank's share of a multi-GPU frame maps its packed
16-row bands to interleaved image rows (ray_kernels.hpp image_row).  Each rank of N = 2, 4, 8 is
rendered on this GPU exactly as it would be on its own (RRTE_EMULATE_RANK=N:R: that rank's bands,
packed) and its linear image rows must equal the ORACLE's rows bit for bit, with the oracle's
shadow-ray count for exactly those bands.  (The RCCL gather that composes the ranks is covered by
tests/test_gpu_gather.py and tests/test_dist.py.)"""
import ctypes as C

import numpy as np
import pytest

import oracle
from rrte_amd import LoweredScene, abi, scenes
from rrte_amd.renderer import Context
from test_gpu_parity import compare

pytestmark = pytest.mark.gpu

W, H, BAND = 3840, 2160, 16
NBANDS = (H + BAND - 1) // BAND


_oracle = {}


def oracle_4k(name="sdf_showcase"):
    """The oracle's linear 4K image and its shadow-ray count per 16-row band (one call per band into
    the same full-size buffers: the oracle writes rows [r0, r1) at their image positions)."""
    if name in _oracle:
        return _oracle[name]
    objs, lights, cam, cfg = getattr(scenes, name)(W, H)
    sc = LoweredScene(objs, lights, cam)
    prm = cfg.lower()
    prm.flags |= abi.FLAG_F32_LINEAR
    lib = oracle.load()
    lin = np.zeros(W * H * 4, np.float32)
    u8 = np.zeros(W * H * 4, np.uint8)
    band_shadow = []
    for b in range(NBANDS):
        sh = C.c_uint64(0)
        st = lib.rrte_oracle_render(C.byref(sc.ir), C.byref(prm), u8.ctypes.data, lin.ctypes.data, C.byref(sh), 16,
                                    b * BAND, min(H, (b + 1) * BAND))
        assert st == 0
        band_shadow.append(sh.value)
    _oracle[name] = (lin.reshape(H, W, 4), band_shadow)
    return _oracle[name]


@pytest.mark.parametrize("jit", [abi.JIT_OFF, abi.JIT_ON])
def test_sdf_showcase_4k_matches_oracle(jit):
    """The whole 4K frame on one GPU (16x16 culling blocks), generic and scene-specialised kernels."""
    compare(*scenes.sdf_showcase(W, H), threads=16, jit=jit)


def band_owner(b, n, sky, rb, pb):
    """The rank owning image band b (include/rrte_hip.h rrte_hip_band_layout)."""
    if b < sky or n == 1:
        return 0
    s = (b - sky) % (rb + (n - 1) * pb)
    return 0 if s < rb else 1 + (s - rb) % (n - 1)


@pytest.mark.parametrize("name,nranks,sky_on", [("sdf_showcase", n, sky) for n in (2, 4, 8) for sky in ("1", "0")]
                         + [("deformation_stress", 8, "1")])
def test_4k_rank_shares_match_oracle_rows(name, nranks, sky_on, monkeypatch):
    """Each rank's share under the frame's band partition (the sky bands on rank 0 and the rest round
    robin, rrte_hip_band_layout; RRTE_BAND_SKY=0: the plain interleave).  sdf-showcase is BASELINE
    configs[3]; the deformation-stress scene at N = 8 is configs[4] (VERDICT r04 missing #3)."""
    import torch
    lin, band_shadow = oracle_4k(name)
    objs, lights, cam, cfg = getattr(scenes, name)(W, H)
    cfg.band_rows = BAND
    sc = LoweredScene(objs, lights, cam)
    prm = cfg.lower()
    prm.flags |= abi.FLAG_F32_LINEAR
    lib = abi.load()
    monkeypatch.setenv("RRTE_BAND_SKY", sky_on)
    sky, rb, pb = abi.band_layout(sc.ref(), C.byref(prm), nranks)
    if name == "sdf_showcase":
        assert (sky > 0) == (sky_on == "1")  # the 4K showcase has sky rows above every object
    total = 0
    for rank in range(nranks):
        monkeypatch.setenv("RRTE_EMULATE_RANK", f"{nranks}:{rank}")
        ctx = Context(0, jit=abi.JIT_ON)
        rows = lib.rrte_hip_band_rows_for_rank_ex(H, BAND, nranks, rank, sky, rb, pb)
        img_rows = [y for y in range(H) if band_owner(y // BAND, nranks, sky, rb, pb) == rank]
        assert len(img_rows) == rows
        f32 = torch.zeros(rows * W * 4, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()  # the fill ran on torch's stream; the renders run on others
        ctx.check(ctx.lib.rrte_hip_render_async(ctx.h, sc.ref(), C.byref(prm), None, f32.data_ptr(), None))
        ctx.check(ctx.lib.rrte_hip_synchronize(ctx.h))
        st = ctx.stats()
        got = f32.cpu().numpy().view(np.uint32).reshape(rows, W, 4)
        want = lin[img_rows].view(np.uint32)
        bad = (got != want).any(-1)
        assert not bad.any(), f"rank {rank}/{nranks}: {int(bad.sum())} pixels differ from the oracle"
        assert st.jit_active == 1
        assert int(st.shadow_rays) == sum(band_shadow[b] for b in range(NBANDS) if band_owner(b, nranks, sky, rb, pb) == rank), rank
        total += int(st.shadow_rays)
        ctx.close()
    assert total == sum(band_shadow)
