"""Kernel-trace summary of the last window of a run (rocprofv3 --kernel-trace csv): every kernel that
started inside the window of the last `n` ray-kernel launches, per kernel name (count, mean and total
duration), the GPU-busy union, the span, and the idle gaps between consecutive busy intervals.  Used for
the batched multi-GPU rank path (one launch renders up to 8 frames) where timeline2.py's one-launch-
per-frame view does not apply.
usage: python tools/trace_window.py <kernel_trace.csv> <n_ray_launches> <frames> <out.md> [title]"""
import csv
import sys
from collections import defaultdict

path, n, frames, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
title = sys.argv[5] if len(sys.argv) > 5 else "trace window"
rows = list(csv.DictReader(open(path)))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
ray = [r for r in rows if "rrte_jit_kernel" in r["Kernel_Name"] or "ray_kernel" in r["Kernel_Name"]]
# multi-frame launches: grid (tile columns, frames, hot rows + tile rows) -- frames in y since the hot-first
# tile order (round 3); in z before it
FR = "Grid_Size_Y"
if any(int(r.get(FR) or 1) > 1 for r in ray):
    ray = [r for r in ray if int(r.get(FR) or 1) > 1]  # batched path: the multi-frame launches only
w0 = ray[-n]["s"]
# the window: from the first of those launches to the end of the last kernel that follows the last one
# before the next launch of another kind of frame (the bench's later single-frame measurements)
after = [r for r in rows if r["s"] > ray[-1]["s"] and ("rrte_jit_kernel" in r["Kernel_Name"] or "ray_kernel" in r["Kernel_Name"])]
cut = after[0]["s"] if after else None
win = [r for r in rows if r["s"] >= w0 and (cut is None or r["s"] < cut)]
t1 = max(r["e"] for r in win)
per = defaultdict(list)
for r in win:
    name = r["Kernel_Name"].split("(")[0][:90]
    per[name].append((r["e"] - r["s"]) / 1e3)
iv = sorted(((r["s"] - w0) / 1e3, (r["e"] - w0) / 1e3) for r in win)
busy, gaps, cur = 0.0, [], None
for s, e in iv:
    if cur is None or s > cur[1]:
        if cur:
            busy += cur[1] - cur[0]
            gaps.append(s - cur[1])
        cur = [s, e]
    else:
        cur[1] = max(cur[1], e)
busy += cur[1] - cur[0]
span = (t1 - w0) / 1e3
lines = [f"# {title}", "", f"source: `rocprofv3 --kernel-trace`; window = the last {n} ray-kernel launches (multi-frame ones when the run has any) "
         f"({frames} frames) and every kernel started after the first of them", "",
         "| kernel | count | mean us | total us |", "|---|---|---|---|"]
for name, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    lines.append(f"| `{name}` | {len(d)} | {sum(d) / len(d):.1f} | {sum(d):.1f} |")
gaps.sort()
lines += ["", f"- span: **{span:.1f} us** = {span / frames:.2f} us per frame",
          f"- GPU busy (union): {busy:.1f} us ({busy / span * 100:.0f} % of the span); idle gaps: {len(gaps)}, "
          f"total {sum(gaps):.1f} us, largest {gaps[-1] if gaps else 0:.1f} us", ""]
open(out, "w").write("\n".join(lines))
print("\n".join(lines))
