"""One-line summary of a bench.py JSON line (stdin) for GPU logs."""
import json
import sys

d = json.loads(sys.stdin.read())
r = d.get("roofline", {})
v = d.get("verified", {})
out = {"value": d["value"], "ms_per_step": d["ms_per_step"], "avg_launch_ms": r.get("avg_launch_ms"),
       "valu_frac": r.get("frac"), "latency_ms": d.get("frame_latency_ms"),
       "verified": {k: v.get(k) for k in ("u8_max_diff", "bytes_differing", "shadow_rays_match")} if v else None,
       "boundary": (d.get("boundary") or {}).get("ms_per_frame_reused_buffer"),
       "hot": d.get("tile_order", {}).get("hot_slots")}
if "kernel_kinds" in d:
    out["kinds"] = {k: v.get("ms_per_frame", v.get("generic_ms_per_frame")) for k, v in d["kernel_kinds"].items()
                    if isinstance(v, dict)}
print(json.dumps(out))
