"""Merged host/device timeline of the timed window of an emulated rank run (rocprofv3 --kernel-trace
--hip-runtime-trace csv): the window starts at the first host launch of the first multi-frame ray
kernel (grid y > 1) of the last `nb` such launches and ends at the last kernel of the run's batched
part; prints every kernel (start, end, duration, queue) and the host calls that enqueue work
(kernel launches, event records and waits, copies) relative to the window start.
usage: python tools/emu_timeline.py <out_dir> <nb_multiframe_launches>"""
import csv
import glob
import sys

d, nb = sys.argv[1], int(sys.argv[2])
kt = [r for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True) for r in csv.DictReader(open(f))]
ht = [r for f in glob.glob(f"{d}/**/*hip_api_trace.csv", recursive=True) for r in csv.DictReader(open(f))]
for r in kt + ht:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
kt.sort(key=lambda r: r["s"])
ht.sort(key=lambda r: r["s"])
multi = [r for r in kt if ("rrte_jit_kernel" in r["Kernel_Name"] or "ray_kernel" in r["Kernel_Name"])
         and int(r.get("Grid_Size_Y") or 1) > 1]
win = multi[-nb:]
corr = {r["Correlation_Id"]: r for r in ht}
first_api = corr.get(win[0]["Correlation_Id"])
t0 = first_api["s"] if first_api else win[0]["s"]
t_end = max(r["e"] for r in kt if r["s"] >= win[0]["s"] and r["s"] <= win[-1]["e"] + 200000)
events = []
for r in kt:
    if t0 <= r["s"] <= t_end:
        events.append((r["s"], f"K {(r['s'] - t0) / 1e3:8.1f} .. {(r['e'] - t0) / 1e3:8.1f} ({(r['e'] - r['s']) / 1e3:6.1f} us) "
                               f"q{r.get('Queue_Id', '?')} gy={r.get('Grid_Size_Y', '?')} {r['Kernel_Name'][:60]}"))
keep = ("Launch", "EventRecord", "StreamWaitEvent", "Memcpy", "Synchronize", "EventQuery", "StreamQuery")
for r in ht:
    if t0 - 5000 <= r["s"] <= t_end and any(k in r["Function"] for k in keep):
        events.append((r["s"], f"H {(r['s'] - t0) / 1e3:8.1f} +{(r['e'] - r['s']) / 1e3:5.1f} us  {r['Function']}"))
events.sort()
last_q = None
for _, line in events:
    if "Query" in line:  # collapse polling runs
        if last_q:
            continue
        last_q = True
    else:
        last_q = False
    print(line)
print(f"window: {(t_end - t0) / 1e3:.1f} us from the first multi-frame launch call to the last kernel end")
