"""Summarize a tools/prof.sh output dir into profiles/<name>.md and profiles/pmc_<name>.json.

usage: python tools/summarize_prof.py gpurun_out/prof_<tag> <name> <workload-key>
<workload-key> must be bench.py's key (e.g. sdf-showcase@1920x1080/lambert_shadow): bench.py takes the
newest summary with that key for the bench line's `roofline.traffic` and `valu` objects.
HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) under-reports wide coalesced reads
by 2x on gfx950 (doubled here, flagged as uncalibrated for this access pattern); WRITE_SIZE (KiB)
is exact for wide stores; both are per dispatch.
"""
import collections
import re
import csv
import json
import sys
import time
from pathlib import Path

src, name, workload = Path(sys.argv[1]), sys.argv[2], sys.argv[3]
KERNEL_RE = re.compile(r"ray_kernel|rrte_jit_kernel")
out_md = [f"# rocprofv3 summary: {name}", "", f"workload: `{workload}`", ""]
stats = src / "trace" / "run_kernel_stats.csv"
if stats.exists():
    out_md += ["## kernel trace (`rocprofv3 --kernel-trace --stats`)", "", "```", stats.read_text().strip(), "```", ""]
pmc = collections.defaultdict(list)
meta = {}
for f in sorted(src.glob("pmc*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if KERNEL_RE.search(r["Kernel_Name"]):
            pmc[r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta = {k: r[k] for k in ("Kernel_Name", "Grid_Size", "Workgroup_Size", "LDS_Block_Size",
                                      "Scratch_Size", "VGPR_Count", "SGPR_Count")}
avg = {k: sum(v) / len(v) for k, v in pmc.items()}
dur_ns = None
if stats.exists():
    for r in csv.DictReader(open(stats)):
        if KERNEL_RE.search(r["Name"]):
            dur_ns = float(r["AverageNs"])
bid = src / "build_id.txt"  # (tools/prof.sh: rrte_hip_build_id of the profiled build)
res = {"created": time.time(), "workload": workload, "build_id": bid.read_text().strip() if bid.exists() else None, "kernel": meta.get("Kernel_Name"), "dispatch": meta, "counters_per_dispatch": avg,
       "avg_kernel_ns": dur_ns}
if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
    fetch = avg["FETCH_SIZE"] * 1024 * 2  # gfx950: FETCH_SIZE reads 1/2 of wide coalesced reads
    write = avg["WRITE_SIZE"] * 1024
    res["hbm_bytes_per_launch"] = fetch + write
    res["hbm_note"] = "FETCH_SIZE*1024*2 + WRITE_SIZE*1024 per dispatch (MI355X_MICROARCH.md §HBM correction)"
if "SQ_INSTS_VALU" in avg and dur_ns:
    # wave64 VALU instruction = 64 lane-ops issued over 2 cycles on a SIMD32: chip peak
    # 256 CU * 4 SIMD / 2 cyc * 2.4 GHz = 1228.8 G wave-instr/s
    rate = avg["SQ_INSTS_VALU"] / (dur_ns * 1e-9)
    res["valu"] = {"wave_instr_per_s": rate, "peak_wave_instr_per_s": 1228.8e9, "issue_frac": rate / 1228.8e9,
                   "VALUBusy_pct": avg.get("VALUBusy"), "VALUUtilization_pct": avg.get("VALUUtilization"),
                   "OccupancyPercent": avg.get("OccupancyPercent")}
out_md += ["## PMC counters (mean per ray_kernel dispatch, separate --pmc passes)", "", "| counter | value |",
           "|---|---|"] + [f"| {k} | {v:.6g} |" for k, v in sorted(avg.items())] + ["", "dispatch: " + json.dumps(meta), ""]
out_md += ["## derived", "", "```json", json.dumps({k: v for k, v in res.items() if k in ("hbm_bytes_per_launch",
                                                                                         "valu", "avg_kernel_ns")},
                                                  indent=1), "```", ""]
# the driver's configuration traced (tools/prof.sh tl/: 5 warm-up frames, 20 sequential, 20 back to back,
# then the 20 timed frames with 4 in flight): the timed frames' spans and overlap (tools/timeline2.py)
tl = src / "tl" / "run_kernel_trace.csv"
if tl.exists():
    import subprocess
    tmp = src / "timeline.md"
    subprocess.run([sys.executable, str(Path(__file__).parent / "timeline2.py"), str(tl), "45", "20", str(tmp),
                    "the driver's 20 timed steps (4 frames in flight)"], check=False, capture_output=True)
    if tmp.exists():
        out_md += ["## in-flight timeline of the timed frames (`rocprofv3 --kernel-trace`, tools/timeline2.py)", ""]
        out_md += tmp.read_text().splitlines()[1:] + [""]
Path("profiles").mkdir(exist_ok=True)
Path(f"profiles/{name}.md").write_text("\n".join(out_md))
Path(f"profiles/pmc_{name}.json").write_text(json.dumps(res, indent=1))
print(json.dumps(res.get("valu"), indent=1), res.get("hbm_bytes_per_launch"))
