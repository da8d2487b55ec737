"""Multi-rank row-band composition on CPU (gloo, world_size 2, 3 and 4), in the layout of the batched GPU
path (rrte_hip.hip render_batch / flush_batch): each rank renders the bands the frame's band partition
gives it (rrte_hip_band_layout: sky bands on the root, the rest round robin at the root:peer ratio;
the oracle stands in for the per-rank kernel); the ROOT writes its own bands straight into the frame at their
image rows (KParams::out_image_rows), every PEER packs its rows as ray_kernel does for a rank -- RGB24,
the alpha byte dropped, since LAMBERT_SHADOW proves it 255 -- and sends the slab to the root point to
point (ncclSend / ncclRecv there, dist.send / recv here), and the root expands only the peers' rows
with the mapping of deinterleave_batch_kernel (alpha 255 restored).  The result must equal the
single-process frame bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

BAND = 4
W, H = 64, 48  # (the showcase at this size: 2 sky bands, ratios 1:1 at N = 2 and 1:2 at N = 3)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _owner(b, n, sky, rb, pb):
    """The rank owning image band b (include/rrte_hip.h rrte_hip_band_layout)."""
    if b < sky or n == 1:
        return 0
    q = (b - sky) % (rb + (n - 1) * pb)
    return 0 if q < rb else 1 + (q - rb) % (n - 1)


def _rank_rows(sc, prm, rank, n):
    """A rank's image rows in packing order (image order) and the slab rows (the most any rank owns)."""
    import ctypes as C
    from rrte_amd import abi
    lib = abi.load()
    part = abi.band_layout(sc.ref(), C.byref(prm), n)
    rows = [lib.rrte_hip_band_rows_for_rank_ex(H, BAND, n, r, *part) for r in range(n)]
    img_rows = [[y for y in range(H) if _owner(y // BAND, n, *part) == r] for r in range(n)]
    assert [len(x) for x in img_rows] == rows
    return img_rows[rank], img_rows, max(rows), part


def _worker(rank, n, port, scene_name, q):
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=n)
    try:
        import oracle
        from rrte_amd import LoweredScene, scenes
        objs, lights, cam, cfg = scenes.SCENES[scene_name](W, H, mode="lambert_shadow")
        cfg.band_rows = BAND
        sc = LoweredScene(objs, lights, cam)
        img_rows, all_rows, cap, part = _rank_rows(sc, cfg.lower(), rank, n)
        packed = np.zeros((cap, W, 4), np.uint8)  # one gather slot per rank, cap rows
        shadow = 0
        for i, y in enumerate(img_rows):
            full, _, sh = oracle.render(sc, cfg.lower(), nthreads=1, rows=(y, y + 1), want_f32=False)
            packed[i] = full.reshape(H, W, 4)[y]
            shadow += sh
        tot = torch.tensor([shadow], dtype=torch.int64)
        dist.all_reduce(tot)
        if rank != 0:
            rgb24 = np.ascontiguousarray(packed[..., :3])  # the slab format (kFlagSlabRgb24)
            assert (packed[:len(img_rows), :, 3] == 255).all()  # alpha provably 255 (slab_rgb24)
            dist.send(torch.from_numpy(rgb24.reshape(-1)), dst=0)
        else:
            out = np.zeros((H, W, 4), np.uint8)
            for i, y in enumerate(img_rows):  # the root's own bands, in place
                out[y] = packed[i]
            slabs = {}
            for r in range(1, n):
                t = torch.zeros(cap * W * 3, dtype=torch.uint8)
                dist.recv(t, src=r)
                slabs[r] = t.numpy().reshape(cap, W, 3)
            for r in range(1, n):  # deinterleave_batch_kernel<RGB24>: peers' rows only (skip_rank = root)
                for i, y in enumerate(all_rows[r]):
                    out[y, :, :3] = slabs[r][i]
                    out[y, :, 3] = 255
            ref, _, ref_sh = oracle.render(sc, cfg.lower(), nthreads=2, want_f32=False)
            q.put((np.array_equal(out, ref.reshape(H, W, 4)), int(tot.item()), ref_sh, part))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [2, 3, 4])
def test_band_gather_composition_matches_single_frame(n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, n, port, "sdf-showcase", q)) for r in range(n)]
    for p in procs:
        p.start()
    ok, shadow_sum, ref_shadow, part = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok
    assert shadow_sum == ref_shadow  # shadow-ray counts add up across ranks
    assert part[0] > 0  # the partition in use has sky bands on the root
