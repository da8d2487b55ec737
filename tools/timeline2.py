"""Timeline summary of the timed frames of a bench.py run from a rocprofv3 kernel trace (csv): each
frame's ray-kernel start / end / duration relative to the first, frames running at once, the GPU-busy
union and the whole span -- written as a markdown profile.
usage: python tools/timeline2.py <kernel_trace.csv> <skip> <count> <out.md> [title]"""
import csv
import sys

path, skip, count, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
title = sys.argv[5] if len(sys.argv) > 5 else "timeline"
rows = [r for r in csv.DictReader(open(path)) if "rrte_jit_kernel" in r["Kernel_Name"] or "ray_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = rows[skip:skip + count]
t0 = int(ks[0]["Start_Timestamp"])
iv = [((int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3) for r in ks]
lines = [f"# {title}", "", f"source: `rocprofv3 --kernel-trace`, {len(rows)} ray-kernel launches in the trace; "
         f"timed frames = launches {skip}..{skip + count - 1}", "", "| frame | start us | end us | duration us | running at start |",
         "|---|---|---|---|---|"]
for i, (s, e) in enumerate(iv):
    conc = sum(1 for (a, b) in iv if a <= s < b)
    lines.append(f"| {i} | {s:.1f} | {e:.1f} | {e - s:.1f} | {conc} |")
span = max(e for _, e in iv)
# union of busy intervals
busy, cur = 0.0, None
for s, e in sorted(iv):
    if cur is None or s > cur[1]:
        if cur:
            busy += cur[1] - cur[0]
        cur = [s, e]
    else:
        cur[1] = max(cur[1], e)
busy += cur[1] - cur[0]
durs = sorted(e - s for s, e in iv)
maxc = max(sum(1 for (a, b) in iv if a <= t < b) for t, _ in iv)
lines += ["", f"- span of the {count} frames: **{span:.1f} us** = {span / count:.2f} us per frame",
          f"- GPU busy (union of kernel intervals): {busy:.1f} us",
          f"- per-frame kernel duration: median {durs[len(durs) // 2]:.1f} us, min {durs[0]:.1f}, max {durs[-1]:.1f} "
          f"(frames overlap: up to {maxc} running at once, so a frame's duration exceeds the per-frame rate)", ""]
open(out, "w").write("\n".join(lines))
print("\n".join(lines[-5:]))
