"""Timeline of bench.py's timed frames from a rocprofv3 kernel trace (csv): when each frame's ray
kernel started and ended relative to the first, how many ran at once, and the span against the sum
of the serialized launches.  usage: python tools/timeline.py <kernel_trace.csv> <skip> <count>
(skip = ray-kernel launches before the timed region: warm-up + the sequential roofline pass)."""
import csv
import sys

path, skip, count = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rows = [r for r in csv.DictReader(open(path)) if "rrte_jit_kernel" in r["Kernel_Name"] or "ray_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = rows[skip:skip + count]
t0 = int(ks[0]["Start_Timestamp"])
print(f"{len(rows)} ray kernels in the trace; timed region = launches {skip}..{skip + count - 1}")
ends = []
for i, r in enumerate(ks):
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    ends.append(e)
    print(f"frame {i:2d}: start {s / 1e3:8.1f} us  end {e / 1e3:8.1f} us  dur {(e - s) / 1e3:6.1f} us")
span = max(ends)
print(f"span {span / 1e3:.1f} us for {count} frames = {span / 1e3 / count:.2f} us/frame")
