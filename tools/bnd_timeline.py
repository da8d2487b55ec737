"""Per-frame timeline of the blocking drop-in path from a rocprofv3 kernel + memory-copy trace
(tools/bnd_trace.sh): for the last frames, each ray-kernel launch and D2H copy relative to the
frame's first kernel start.  usage: python tools/bnd_timeline.py <trace dir>"""
import csv
import glob
import sys

d = sys.argv[1]
kf = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
mf = glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True)
ev = []
for r in csv.DictReader(open(kf[0])):
    if "rrte_jit_kernel" in r["Kernel_Name"] or "ray_kernel" in r["Kernel_Name"]:
        ev.append(("K", int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", r.get("Stream_Id", ""))))
if mf:
    for r in csv.DictReader(open(mf[0])):
        kind = r.get("Direction", r.get("Operation", ""))
        size = r.get("Size", r.get("Bytes", ""))
        ev.append(("C" + str(kind)[:12] + ":" + str(size), int(r["Start_Timestamp"]), int(r["End_Timestamp"]), ""))
ev.sort(key=lambda e: e[1])
ks = [e for e in ev if e[0] == "K"]
nk = len(ks)
per = max(1, nk // 13)  # 13 frames (3 warm-up + 10)
start = ks[-per * 3][1]
print(f"{nk} kernels ({per} per frame); last 3 frames, us from the first kernel start")
for e in ev:
    if e[1] >= start:
        print(f"  {e[0]:24s} {((e[1] - start) / 1e3):9.1f} {((e[2] - start) / 1e3):9.1f}  dur {((e[2] - e[1]) / 1e3):7.1f}  q{e[3]}")
