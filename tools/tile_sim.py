"""List-scheduling model of one lone frame from tools/tile_dump.py's per-tile durations: the tiles are
dispatched in a given order onto S wave slots (S = the peak concurrency seen in the dump) and the
model's makespan is compared for image order and for the K slowest tiles first.  Durations are the
measured loaded ones, so the model ignores how a wave's speed depends on its SIMD's load; it ranks
orders, it does not predict microseconds.  usage: python tools/tile_sim.py gpurun_out/tiles_*.npz"""
import heapq
import sys

import numpy as np


def makespan(order, dur, slots):
    free = [0.0] * slots
    heapq.heapify(free)
    end = 0.0
    for i in order:
        t = heapq.heappop(free)
        e = t + dur[i]
        end = max(end, e)
        heapq.heappush(free, e)
    return end


z = np.load(sys.argv[1])
for key in ("lone0", "lone1", "stream0"):
    v = z[key]
    dur = v[:, 2].astype(np.float64) / 100.0
    st = (v[:, 0].astype(np.uint64) | (v[:, 1].astype(np.uint64) << 32))
    st = (st - st.min()).astype(np.float64) / 100.0
    ev = np.concatenate([np.stack([st, np.ones_like(st)], 1), np.stack([st + dur, -np.ones_like(st)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    slots = int(np.cumsum(ev[:, 1]).max())
    n = len(dur)
    img = np.arange(n)
    srt = np.argsort(-dur, kind="stable")
    print(f"{key}: {n} tiles, measured span {(st + dur).max():.1f} us, peak concurrency {slots}, "
          f"sum {dur.sum() / slots:.1f} us per slot, max tile {dur.max():.1f} us")
    print(f"  model image order {makespan(img, dur, slots):.1f} us")
    for k in (64, 128, 256, 512, 1024, 2048, n):
        hot = srt[:k]
        mask = np.ones(n, bool)
        mask[hot] = False
        order = np.concatenate([np.sort(hot), img[mask]])
        print(f"  model hot-first K={k}: {makespan(order, dur, slots):.1f} us, "
              f"K-th slowest tile {dur[srt[min(k, n) - 1]]:.1f} us")
