"""Benchmark: Mray/s (primary + shadow) of the sdf-showcase scene at 1920x1080.

python bench.py --gpus N --steps K --warmup W
  N = 1: one rrte_hip_render_async frame per step on cuda:0.
  N > 1: launched by torch.distributed.run; every rank renders its interleaved
         16-row bands of the SAME 1080p frame (the frame's band partition) and the frame
         is composed on rank 0 over RCCL/xGMI send/recv (rrte_hip_render_gather_async) -> strong scaling.
A "step" is one frame.  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import shutil
import statistics
import sys
import time
from pathlib import Path

import numpy as np

# Frames in flight need their streams on distinct hardware queues.  HIP's default is 4 per process (the
# GPU box exports GPU_MAX_HW_QUEUES=4), shared with torch's and the library's own streams; one rank of
# an 8-GPU job then needs ~40 us for its share of a frame instead of ~24 us with 32 queues
# (tools/runs/r02_inflight.sh, 20 steps; the one-GPU frame is the same with 4 or 32).  The bench's own
# setting is RRTE_BENCH_HW_QUEUES (default 32), applied before HIP starts; the value in effect is
# recorded in the JSON line (config.hw_queues).  Under rocprofv3 the profiler starts HIP before this
# line runs, so the profiling scripts export GPU_MAX_HW_QUEUES themselves.
HW_QUEUES = os.environ.get("RRTE_BENCH_HW_QUEUES", "32")
os.environ["GPU_MAX_HW_QUEUES"] = HW_QUEUES

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from rrte_amd import LoweredScene, abi, scenes  # noqa: E402
from rrte_amd.renderer import Context  # noqa: E402

HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
VALU_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector peak (packed)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)  # 0.1 ms frames: 200 keep the ramp/drain under 5 %
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--scene", default="sdf-showcase", choices=sorted(scenes.SCENES))
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--mode", default="lambert_shadow", choices=["lambert_shadow", "refcompat"])
    ap.add_argument("--band-rows", type=int, default=16)
    ap.add_argument("--spp", type=int, default=None, help="override samples per pixel (profiling other configs)")
    ap.add_argument("--max-depth", type=int, default=None, help="override max_depth")
    ap.add_argument("--random", action="store_true", help="random jitter (and scatter) instead of pixel centres")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-stock", action="store_true", help="skip the stock-config secondary measurement")
    ap.add_argument("--no-boundary", action="store_true",
                    help="skip the blocking drop-in measurement (profiles: only the headline's launches in the trace)")
    ap.add_argument("--inflight", type=int, default=None,
                    help="frames in flight: consecutive frames rotate over this many streams + output buffers "
                         "so one frame's tail overlaps the next frame's start (1 = strictly one after another); "
                         "default 4 on one GPU (tools/runs/r02_inflight.sh); N > 1: frames per gather batch, default 8")
    ap.add_argument("--streams", type=int, default=1,
                    help="N > 1: caller streams the frames rotate over, independent of the gather batch "
                         "(--inflight); 1 with multi-frame batch launches (the library renders on its own streams), "
                         "e.g. 4 with RRTE_BATCH_LAUNCH=0 (each frame launched at its call on its caller's stream)")
    ap.add_argument("--flyby", type=int, default=0,
                    help="camera fly-by: frame i renders camera pose i %% K of K poses orbiting the scene's target "
                         "(0.6 degrees apart; pose 0 = the scene's own camera); 0 = static camera")
    ap.add_argument("--no-legs", action="store_true",
                    help="skip the secondary BASELINE configs (basic-demo 640x480, advanced-demo 1080p, "
                         "sdf-showcase 4K, deformation stress 4K) measured beside the headline at N = 1")
    ap.add_argument("--jit", default="on", choices=["on", "off", "auto"],
                    help="scene-specialised kernel (hiprtc, compiled during warm-up) or the generic kernel")
    return ap.parse_args()


def cpu_threads():
    threads = int(os.environ.get("RRTE_CPU_THREADS", os.cpu_count() or 1))
    # the GPU box shows the whole machine in os.cpu_count(); our share is what sched_getaffinity allows
    try:
        threads = min(threads, len(os.sched_getaffinity(0)))
    except AttributeError:
        pass
    return min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def physical_cores():
    """Physical cores of the host (distinct (physical id, core id) pairs in /proc/cpuinfo), or None."""
    try:
        cores, phys = set(), "0"
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                phys = line.split(":", 1)[1].strip()
            elif line.startswith("core id"):
                cores.add((phys, line.split(":", 1)[1].strip()))
        return len(cores) or None
    except OSError:
        return None


def cpu_baseline(scene, params, budget_s, stock=None):
    """The oracle (C restatement of Raytracer::render) on this host's cores:
    N threads: median of up to 5 whole frames after 1 warm-up; 1 thread: one whole frame (or a
    row band if the budget is short); plus the reference's stock config on a row band."""
    import oracle

    threads = cpu_threads()
    W, H = params.width, params.height
    frame8, _, _ = oracle.render(scene, params, nthreads=threads, want_f32=False)  # warm-up
    times, shadow = [], 0
    t_start = time.perf_counter()
    while len(times) < 5:
        t0 = time.perf_counter()
        frame8, _, shadow = oracle.render(scene, params, nthreads=threads, want_f32=False)
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_start > budget_s:
            break
    med = statistics.median(times)
    rays = W * H * params.samples_per_pixel + shadow
    out = {
        "value": rays / med / 1e6, "unit": "Mray/s", "cores": threads, "kind": "port",
        "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(),
        "sample": f"median of {len(times)} whole {W}x{H} frames (1 warm-up) of the same scene/mode, "
                  f"{med * 1e3:.1f} ms/frame, oracle/rrte_oracle.c -O3 -march=x86-64-v3, {threads} threads",
    }
    # 1 thread: whole frame if it fits the budget (estimated from the N-thread time), else a centre band
    est = med * threads
    rows = (0, H) if est <= budget_s else (H // 2 - max(8, int(H * budget_s / est)) // 2,
                                          H // 2 + max(8, int(H * budget_s / est)) // 2)
    t0 = time.perf_counter()
    _, _, sh1 = oracle.render(scene, params, nthreads=1, rows=rows, want_f32=False)
    t1 = time.perf_counter() - t0
    out["single_thread"] = {"value": (W * (rows[1] - rows[0]) * params.samples_per_pixel + sh1) / t1 / 1e6,
                            "unit": "Mray/s", "cores": 1, "rows": list(rows)}
    # the whole host, extrapolated: the job may use `threads` of the host's CPUs
    # (its affinity share); the measured per-thread rate at that thread count x the host's physical
    # cores is an upper estimate of the reference's rayon path on the whole machine (no SMT gain)
    phys = physical_cores()
    if phys:
        per_thread = out["value"] / threads
        out["whole_host_extrapolation"] = {
            "value": round(per_thread * phys, 1), "unit": "Mray/s", "physical_cores": phys,
            "note": f"{per_thread:.2f} Mray/s per thread at {threads} threads x {phys} physical cores "
                    "(linear scaling assumed: an upper estimate, not a measurement)"}
    if stock is not None:  # reference stock config (spp 4, depth 50, random jitter/scatter) on a row band
        sscene, sprm, band = stock
        t0 = time.perf_counter()
        oracle.render(sscene, sprm, nthreads=threads, rows=band, want_f32=False)
        ts = time.perf_counter() - t0
        out["stock_config"] = {"value": W * (band[1] - band[0]) * sprm.samples_per_pixel / ts / 1e6,
                               "unit": "Msample/s", "cores": threads, "rows": list(band)}
    return out, (frame8, shadow)


def oracle_frame(scene, params):
    """The oracle's RGBA8 frame and shadow-ray count (the verification reference when the CPU baseline
    leg does not run: N > 1, --no-cpu)."""
    import oracle

    out8, _, shadow = oracle.render(scene, params, nthreads=cpu_threads(), want_f32=False)
    return out8, shadow


def verify_frames(frames_u8, timed_shadow, steps, ref, refs=None, shadow_total=None):
    """The timed frames against the oracle: every buffer in flight holds the last
    timed frame rendered into it; compared byte for byte with the oracle's RGBA8 frame of the same
    scene and parameters (the device gamma byte is proven identical to its powf path; glibc's powf
    may differ by an ulp, hence u8 max diff <= 1 as the bar), and the timed frames' shadow-ray total
    with steps x the oracle's count (exact)."""
    if refs is None:
        refs = [ref] * len(frames_u8)
        shadow_total = steps * int(ref[1])
    diffs = [np.abs(f.astype(np.int16) - r8.astype(np.int16)) for f, (r8, _) in zip(frames_u8, refs)]
    return {"frames": len(frames_u8), "u8_max_diff": int(max(int(d.max()) for d in diffs)),
            "bytes_differing": int(sum(int((d != 0).sum()) for d in diffs)),
            "shadow_rays_match": int(timed_shadow) == int(shadow_total),
            "shadow_rays_per_frame": {"timed_mean": timed_shadow / steps, "oracle": shadow_total / steps},
            "reference": "oracle/rrte_oracle.c (C restatement of Raytracer::render), same scene and parameters"}


def flop_tally(scene, params):
    """Algorithmic FP32 ops of one frame from the oracle's instrumented counting build
    (oracle/rrte_oracle.c rrte_oracle_flops).  Not timed."""
    import oracle

    cnt, flops = oracle.count(scene, params, nthreads=cpu_threads())
    return flops, int(cnt.sdf_steps), int(cnt.samples + cnt.shadow_rays)


def pmc_traffic(workload_key, build_id):
    """The committed rocprofv3 PMC summary (profiles/pmc_*.json) of this workload AND this build
    (rrte_hip_build_id: device headers + hiprtc options), or None; plus a note naming the newest
    summary of the workload when none matches the build (its counters are then not reported)."""
    best, newest = None, None
    for p in sorted((ROOT / "profiles").glob("pmc_*.json")):
        try:
            d = json.loads(p.read_text())
        except Exception:
            continue
        if d.get("workload") != workload_key or d.get("hbm_bytes_per_launch") is None:
            continue
        d["file"] = f"profiles/{p.name}"
        if newest is None or d.get("created", 0) >= newest.get("created", 0):
            newest = d
        if d.get("build_id") == build_id and (best is None or d.get("created", 0) >= best.get("created", 0)):
            best = d
    note = {"build_id": build_id, "profile": best["file"] if best else None, "build_id_match": best is not None}
    if best is None and newest is not None:
        note["newest_profile_of_another_build"] = newest["file"]
    return best, note


def measured_valu_peak():
    """Wave64 VALU issue rates measured on MI355X by tools/valu_peak.hip (profiles/r01_valu_peak.json):
    FMA-class (v_fma/v_add/v_mul_f32) and compare/select-class (v_cmp, v_cndmask_e64, v_max_f32)."""
    f = ROOT / "profiles" / "r01_valu_peak.json"
    if not f.exists():
        return None
    ops = {o["op"]: o["wave_instr_per_s"] for o in json.loads(f.read_text())["ops"]}
    fma = statistics.mean(ops[k] for k in ("v_fma_f32", "v_add_f32", "v_mul_f32"))
    sel = statistics.mean(ops[k] for k in ("v_cmp_lt_f32(vcc)", "v_cndmask_b32_e64 s[20:21]", "v_max_f32"))
    return {"fma_add_mul": fma, "cmp_select_max": sel, "source": "profiles/r01_valu_peak.json"}


def auto_cold_start(scene, prm, fulls, sptrs, dev, rays_per_frame, limit_s=8.0):
    """The default JIT policy (RRTE_JIT_AUTO) from a cold start -- a new context and an empty code-object
    cache, as a drop-in user's first run: frames rendered back to back (frames in flight as the
    headline) on the generic kernel while the scene-specialised kernel compiles in the background,
    until it takes over.  Reports the time to the switch, the generic frames rendered meanwhile and
    their rate, and the hiprtc compile time (a cache miss)."""
    import tempfile

    import torch
    F = len(fulls)
    tmp = tempfile.mkdtemp(prefix="rrte_jit_cold_")
    old = os.environ.get("RRTE_JIT_CACHE_DIR")
    os.environ["RRTE_JIT_CACHE_DIR"] = tmp  # (read by the background compile too)
    try:
        c = Context(dev.index, jit=abi.JIT_AUTO)
        t0 = time.perf_counter()
        n, switch = 0, None
        while time.perf_counter() - t0 < limit_s:
            c.check(c.lib.rrte_hip_render_async(c.h, scene.ref(), C.byref(prm), fulls[n % F].data_ptr(), None,
                                                sptrs[n % F]))
            n += 1
            if n % F == 0:
                torch.cuda.synchronize(dev)
                if c.stats().jit_active:
                    switch = (time.perf_counter() - t0, n)
                    break
        torch.cuda.synchronize(dev)
        st = c.stats()
        c.close()
    finally:
        if old is None:
            os.environ.pop("RRTE_JIT_CACHE_DIR", None)
        else:
            os.environ["RRTE_JIT_CACHE_DIR"] = old
        shutil.rmtree(tmp, ignore_errors=True)
    if switch is None:
        return {"switched": False, "seconds": round(limit_s, 2), "generic_frames": n}
    gen = max(1, switch[1] - F)  # (the last in-flight group ran on the specialised kernel)
    return {"switched": True, "ms_to_specialised": round(switch[0] * 1e3, 1), "generic_frames": gen,
            "generic_ms_per_frame": round(switch[0] * 1e3 / gen, 4),
            "generic_Mray_s": round(rays_per_frame / (switch[0] / gen) / 1e6, 1),
            "jit_compile_ms": round(st.jit_compile_ms, 1),
            "note": "new context, empty code-object cache (RRTE_JIT_CACHE_DIR=fresh dir): frames on the generic "
                    "kernel until the background hiprtc compile lands (include/rrte_hip.h RRTE_JIT_AUTO)"}


def kernel_variants(scene, prm, fulls, sptrs, dev, rays_per_frame, anim=None, n=200):
    """Secondary throughput of the headline workload per kernel kind (rank 0, N=1; not the headline):
    the generic kernel, the TOPOLOGY specialisation (structure compiled in, values read from the
    uploaded scene: one compile serves every frame of an animation), the FULL specialisation (the
    headline's kernel), each on a context of its own, frames in flight as the headline runs them --
    and `topology_animated`: the topology kernel on an ANIMATION, every frame a new scene (objects,
    lights and materials changed; rrte_amd.scenes.animate_values), uploaded into the scene-version ring
    while the earlier frames are in flight."""
    import torch
    out = {}
    F = len(fulls)
    kinds = [("generic", abi.JIT_OFF, "0", None), ("topology", abi.JIT_ON, "1", None), ("full", abi.JIT_ON, "0", None)]
    if anim:
        kinds.append(("topology_animated", abi.JIT_ON, "1", anim))
    for kind, jit, topo, frames in kinds:
        old = os.environ.get("RRTE_JIT_TOPO")
        os.environ["RRTE_JIT_TOPO"] = topo  # read at context creation
        try:
            c = Context(dev.index, jit=jit)
        finally:
            if old is None:
                os.environ.pop("RRTE_JIT_TOPO", None)
            else:
                os.environ["RRTE_JIT_TOPO"] = old
        sc_of = (lambda i: frames[i % len(frames)]) if frames else (lambda i: scene)  # noqa: E731
        go = lambda i: c.check(c.lib.rrte_hip_render_async(c.h, sc_of(i).ref(), C.byref(prm),  # noqa: E731
                                                           fulls[i % F].data_ptr(), None, sptrs[i % F]))
        for i in range(max(F + 1, len(frames) if frames else 0)):
            go(i)
        torch.cuda.synchronize(dev)
        c.check(c.lib.rrte_hip_synchronize(c.h))
        a = time.perf_counter()
        for i in range(n):
            go(i)
        torch.cuda.synchronize(dev)
        ts = (time.perf_counter() - a) / n
        c.check(c.lib.rrte_hip_synchronize(c.h))
        st = c.stats()
        rays = rays_per_frame if not frames else prm.width * prm.height * prm.samples_per_pixel + int(st.shadow_rays) / n
        out[kind] = {"value": round(rays / ts / 1e6, 3), "unit": "Mray/s", "ms_per_frame": round(ts * 1e3, 4),
                     "jit_active": int(st.jit_active)}
        if frames:
            out[kind]["scenes"] = len(frames)
            out[kind]["upload_host_ms"] = round(st.upload_ms, 4)
        c.close()
    out["auto_cold_start"] = auto_cold_start(scene, prm, fulls, sptrs, dev, rays_per_frame)
    if "topology_animated" in out:
        out["topology_animated"]["vs_static_topology"] = round(
            out["topology_animated"]["ms_per_frame"] / out["topology"]["ms_per_frame"], 4)
    out["note"] = (f"{n} frames each, {F} in flight; jit_active 0 generic / 1 full / 2 topology "
                   "(include/rrte_hip.h rrte_hip_set_jit); topology_animated: a new scene every frame "
                   "(8-frame value animation, cycled)")
    return out


def stock_config(args):
    """The reference's own default workload on the same scene (SURVEY §8d secondary number):
    REFCOMPAT, spp 4, max_depth 50, random jitter and scatter (counter-based RNG)."""
    objs, lights, cam, cfg = scenes.SCENES[args.scene](args.width, args.height, mode="refcompat")
    cfg.samples_per_pixel, cfg.max_depth, cfg.jitter = 4, 50, "random"
    return LoweredScene(objs, lights, cam), cfg.lower()


# The other BASELINE.json configs at N = 1, measured the way the headline is: frames in
# flight on the scene-specialised kernel, HIP-event launch time for the VALU roofline, the oracle's flop
# tally, the oracle on the host's threads as the CPU baseline (the same frame doubles as the verification
# reference), and the PMC summary of the same workload and build when one is committed.
LEGS = [
    ("configs[0]", "basic-demo", 640, 480, "refcompat", "basic-demo 640x480 (ground + 3 spheres, the reference's 2 "
     "point lights), the reference CPU raytracer's formula (REFCOMPAT, max_depth 1)"),
    ("configs[2]", "advanced-demo", 1920, 1080, "lambert_shadow", "advanced-demo 1920x1080 (6 spheres, 5 point "
     "lights with shadow rays)"),
    ("configs[3]", "sdf-showcase", 3840, 2160, "lambert_shadow", "sdf-showcase 3840x2160, the 1-GPU point of the "
     "2/4/8-GPU row-tiled config"),
    ("configs[4]", "deformation-stress", 3840, 2160, "lambert_shadow", "deformation stress 3840x2160 (64-node CSG "
     "under bend -> twist -> 4-octave noise), the 1-GPU point of the 8-GPU config"),
]


def config_leg(name, W, H, mode, dev, cpu_budget_s, flight=4, target_s=0.5):
    import torch
    objs, lights, cam, cfg = scenes.SCENES[name](W, H, mode=mode)
    scene, prm = LoweredScene(objs, lights, cam), cfg.lower()
    c = Context(dev.index, jit=abi.JIT_ON)
    lib = c.lib
    streams = [torch.cuda.Stream(dev) for _ in range(flight)]
    sp = [C.c_void_p(s.cuda_stream) for s in streams]
    outs = [torch.empty(W * H, dtype=torch.int32, device=dev) for _ in range(flight)]
    go = lambda i: c.check(lib.rrte_hip_render_async(c.h, scene.ref(), C.byref(prm), outs[i % flight].data_ptr(),  # noqa: E731
                                                     None, sp[i % flight]))
    for i in range(3):  # compile + the first profiled frames
        go(i)
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    go(0)
    torch.cuda.synchronize(dev)
    one = max(time.perf_counter() - t, 1e-6)
    n = int(min(2000, max(20, target_s / one)))
    # per launch: frames back to back on one stream between two events
    n_seq = min(n, 20)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(streams[0])
    for _ in range(n_seq):
        go(0)
    e1.record(streams[0])
    torch.cuda.synchronize(dev)
    launch_ms = e0.elapsed_time(e1) / n_seq
    c.check(lib.rrte_hip_synchronize(c.h))  # fold earlier counts away
    c.stats()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(n):
        go(i)
    t_enq = time.perf_counter()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    c.check(lib.rrte_hip_synchronize(c.h))
    st = c.stats()
    frames = [o.cpu().numpy().view(np.uint8).copy() for o in outs[:min(flight, n)]]
    jit_active = int(st.jit_active)
    c.close()
    shadow = int(st.shadow_rays)
    rays = W * H * prm.samples_per_pixel * n + shadow
    value = rays / elapsed / 1e6
    # the oracle on the host's threads: whole frames (median of up to 3 within the budget); the last one is
    # the verification reference
    import oracle
    threads = cpu_threads()
    times, ref = [], None
    ts0 = time.perf_counter()
    while len(times) < 3 and (not times or time.perf_counter() - ts0 < cpu_budget_s):
        a = time.perf_counter()
        r8, _, rsh = oracle.render(scene, prm, nthreads=threads, want_f32=False)
        times.append(time.perf_counter() - a)
        ref = (r8, rsh)
    cpu_s = statistics.median(times)
    cpu_value = (W * H * prm.samples_per_pixel + ref[1]) / cpu_s / 1e6
    flops, _, _ = flop_tally(scene, prm)
    valu_tf = flops / (launch_ms * 1e-3) / 1e12
    wl = f"{name}@{W}x{H}/{mode}"
    pmc, pmc_note = pmc_traffic(wl, abi.build_id())
    leg = {"workload": None, "value": round(value, 3), "unit": "Mray/s", "ms_per_frame": round(elapsed / n * 1e3, 5),
           "frames": n, "frames_in_flight": flight,
           # host time of the issue loop alone: close to ms_per_frame = the frame rate is the call rate
           # (small frames: DESIGN.md §14 #2, tools/enqueue_rate.py)
           "enqueue_ms_per_frame": round((t_enq - t0) / n * 1e3, 5),
           "primary_rays_per_frame": W * H * prm.samples_per_pixel,
           "shadow_rays_per_frame": shadow / n, "kernel": "rrte_jit_kernel (scene-specialised)" if jit_active else
           "generic", "avg_launch_ms": round(launch_ms, 5),
           "roofline": {"bound": "valu", "achieved": round(valu_tf, 3), "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": valu_tf / VALU_PEAK_TFLOPS, "flops_per_launch": flops,
                        "achieved_at_frame_rate": round(flops / (elapsed / n) / 1e12, 3),
                        "traffic": pmc["hbm_bytes_per_launch"] if pmc else None, "profile": pmc_note,
                        "hbm": {"achieved": round(4 * W * H / (launch_ms * 1e-3) / 1e9, 3), "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": 4 * W * H / (launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}},
           "cpu_baseline": {"value": round(cpu_value, 3), "unit": "Mray/s", "cores": threads, "kind": "port",
                            "sample": f"median of {len(times)} whole {W}x{H} frames, {cpu_s * 1e3:.1f} ms/frame, "
                                      f"oracle/rrte_oracle.c, {threads} threads"},
           "verified": verify_frames(frames, shadow, n, ref, refs=None) if n >= len(frames) else None}
    leg["cpu_baseline"]["gpu_over_cpu"] = round(value / cpu_value, 2)
    if pmc and pmc.get("valu") is not None:
        leg["valu"] = {k: pmc["valu"].get(k) for k in ("VALUUtilization_pct", "VALUBusy_pct", "OccupancyPercent",
                                                        "issue_frac")}
        cpd = pmc.get("counters_per_dispatch", {})
        leg["valu"]["SQ_INSTS_VALU"] = cpd.get("SQ_INSTS_VALU")
        leg["valu"]["SQ_INSTS_SALU"] = cpd.get("SQ_INSTS_SALU")
    return leg


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    import torch.distributed as dist

    # rehearsal on a box with fewer GPUs than ranks: RRTE_BENCH_DEVICE pins every rank to one device
    if os.environ.get("RRTE_BENCH_DEVICE") is not None:
        local_rank = int(os.environ["RRTE_BENCH_DEVICE"])
    dist_on = world > 1
    # RRTE_BENCH_GATHER=1 (rehearsal on one GPU): the N > 1 frame path -- batched gathers through a
    # 1-rank communicator (RRTE_FORCE_GATHER) -- at N=1; not a headline configuration
    gath = dist_on or os.environ.get("RRTE_BENCH_GATHER") == "1"
    if gath and not dist_on:
        os.environ["RRTE_FORCE_GATHER"] = "1"
    F = max(1, args.inflight if args.inflight is not None else (8 if gath else 4))
    spin = os.environ.get("RRTE_BENCH_SPIN", "1") != "0"  # 0: close the timed region with the blocking sync only
    if dist_on:
        dist.init_process_group("gloo")  # control plane only; the frame gather is RCCL inside librrte_hip
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    objs, lights, cam, cfg = scenes.SCENES[args.scene](args.width, args.height, mode=args.mode)
    cfg.band_rows = args.band_rows
    if args.spp is not None:
        cfg.samples_per_pixel = args.spp
    if args.max_depth is not None:
        cfg.max_depth = args.max_depth
    if args.random:
        cfg.jitter = "random"
    scene = LoweredScene(objs, lights, cam)
    prm = cfg.lower()
    poses = [scene]
    if args.flyby > 1:  # an orbit about the target the examples aim at (rrte_amd.scenes: look_at (0, 2, 0))
        import copy
        import math
        from rrte_amd.math import vec3
        p0 = [float(v) for v in cam.transform.position]
        for k in range(1, args.flyby):
            c2 = copy.deepcopy(cam)
            a = 0.0105 * k
            dx, dz = p0[0], p0[2]
            c2.transform.position = vec3(dx * math.cos(a) - dz * math.sin(a), p0[1], dx * math.sin(a) + dz * math.cos(a))
            c2.look_at((0.0, 2.0, 0.0))
            poses.append(LoweredScene(objs, lights, c2))
    # N > 1: frames are exchanged in batches of F (rrte_hip_set_gather_batch): each batch renders in
    # multi-frame launches (8 frames per launch) on the library's render streams -- rank 0 writing its
    # own bands straight into the frame buffers -- and ONE grouped ncclSend / ncclRecv per batch on its
    # comm stream moves the peers' RGB24 rows to rank 0, which expands them.  Every
    # frame is still composed on rank 0 inside the timed region (the last batch is flushed before its end).
    ctx = Context(local_rank, jit={"off": abi.JIT_OFF, "on": abi.JIT_ON, "auto": abi.JIT_AUTO}[args.jit])
    lib = ctx.lib

    if gath:
        uid = torch.zeros(abi.UNIQUE_ID_BYTES, dtype=torch.uint8)
        if rank == 0:
            buf = (C.c_uint8 * abi.UNIQUE_ID_BYTES)()
            ctx.check(lib.rrte_hip_comm_unique_id(buf))
            uid.copy_(torch.tensor(list(buf), dtype=torch.uint8))
        if dist_on:
            dist.broadcast(uid, 0)
        idb = (C.c_uint8 * abi.UNIQUE_ID_BYTES)(*uid.tolist())
        ctx.check(lib.rrte_hip_comm_init(ctx.h, world, rank, idb))
        ctx.check(lib.rrte_hip_set_gather_batch(ctx.h, min(F, 16)))  # warm-up: the batched path

    W, H = args.width, args.height
    # dedicated (non-null) streams, one output buffer per frame in flight
    streams = [torch.cuda.Stream(dev) for _ in range(max(F, args.streams) if gath else F)]
    NS = max(1, min(args.streams, len(streams))) if gath else F  # caller streams the gather frames rotate over
    fulls = [torch.empty(W * H, dtype=torch.int32, device=dev) for _ in range(F)]
    full, stream = fulls[0], streams[0]
    torch.cuda.set_stream(stream)
    sptrs = [C.c_void_p(s.cuda_stream) for s in streams]
    assert all(p.value for p in sptrs), "need non-null HIP stream handles"

    # the call arguments are built once: the loop below is the library's host path plus one ctypes call
    h, sref, pref = ctx.h, scene.ref(), C.byref(prm)
    srefs = [ps.ref() for ps in poses]
    K = len(srefs)
    fptrs = [f.data_ptr() for f in fulls]
    render_gather, render_async = lib.rrte_hip_render_gather_async, lib.rrte_hip_render_async

    def step(i=0):
        j = i % F
        if gath:
            # batched frames render on the library's own streams (multi-frame launches at the batch's
            # close); one caller stream keeps the batch's dependency on its callers to one event
            st = render_gather(h, srefs[i % K], pref, 0, fptrs[j] if rank == 0 else None, sptrs[i % NS])
        else:
            st = render_async(h, srefs[i % K], pref, fptrs[j], None, sptrs[j])
        if st:
            ctx.check(st)

    for i in range(max(args.warmup, 2)):  # >= 2: the specialised kernel is compiled on warm-up frames
        step(i)
    torch.cuda.synchronize(dev)

    # per-launch kernel duration (roofline): frames strictly one after another on one stream
    # (N > 1: each frame rendered and gathered on its own)
    if gath:
        ctx.check(lib.rrte_hip_set_gather_batch(ctx.h, 1))
    n_seq = min(args.steps, 20)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_seq)]
    for i in range(n_seq):
        evs[i][0].record(stream)
        step(0)
        evs[i][1].record(stream)
    torch.cuda.synchronize(dev)
    launch_ms = [a.elapsed_time(b) for a, b in evs]
    # the same frames back to back between two events: an event pair around every launch also times the
    # stream's gap before and after it (~20 us), so the per-launch figure is the pair's span / frames
    b2b = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    b2b[0].record(stream)
    for i in range(n_seq):
        step(0)
    b2b[1].record(stream)
    torch.cuda.synchronize(dev)
    b2b_ms = b2b[0].elapsed_time(b2b[1]) / n_seq
    ctx.check(lib.rrte_hip_synchronize(ctx.h))  # folds warm-up and sequential-pass shadow counts away

    if gath:
        ctx.check(lib.rrte_hip_set_gather_batch(ctx.h, min(F, 16)))
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    t_enq = time.perf_counter()  # host time to enqueue the timed frames (diagnostic: host-bound if close to elapsed)
    if gath:
        ctx.check(lib.rrte_hip_flush(ctx.h))  # the last, partial gather batch
    if spin:
        # poll for the end of the work (events on every stream the frames and the library used)
        # before the closing synchronize: a blocking device synchronize wakes the host ~40 us after
        # the last kernel ends (tools/runs/r02_timeline2.sh); the work measured is the same
        # (the streams the timed frames were issued on: an event on a stream no frame used is the first
        # work that stream ever sees, and with every frame buffer's stream over HIP's hardware-queue
        # limit -- 16 in flight -- that first dispatch waited ~10 ms for a queue, inside the timed region)
        used = streams[:NS] if gath else streams
        ends = [torch.cuda.Event() for _ in used]
        for e, s in zip(ends, used):
            e.record(s)
        busy = C.c_uint32(1)
        while busy.value or not all(e.query() for e in ends):
            ctx.check(lib.rrte_hip_query(ctx.h, C.byref(busy)))
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if dist_on:
        dist.barrier()
    ctx.check(lib.rrte_hip_synchronize(ctx.h))
    st = ctx.stats()
    elapsed = t1 - t0
    # the timed frames themselves, for the verification against the oracle (outside the timed region)
    timed_frames = [f.cpu().numpy().view(np.uint8).copy() for f in fulls[:min(F, args.steps)]] if rank == 0 else []
    rows = H
    if dist_on:  # this rank's rows under the frame's band partition (sky bands on the root, the rest round robin)
        sky, rb, pb = C.c_uint32(), C.c_uint32(), C.c_uint32()
        ctx.check(lib.rrte_hip_band_layout(scene.ref(), C.byref(prm), world, 0, C.byref(sky), C.byref(rb),
                                           C.byref(pb)))
        rows = lib.rrte_hip_band_rows_for_rank_ex(H, args.band_rows, world, rank, sky.value, rb.value, pb.value)
    primary = W * rows * prm.samples_per_pixel * args.steps
    shadow = int(st.shadow_rays)
    jit_ranks = int(st.jit_active != 0)  # ranks whose timed frames ran the scene-specialised kernel
    if args.jit == "on" and not st.jit_active:
        print(f"rank {rank}: the scene-specialised kernel is not active (JIT failed?); timed on the generic kernel",
              file=sys.stderr)

    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        cnt = torch.tensor([primary, shadow, jit_ranks], dtype=torch.float64)
        dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
        primary, shadow, jit_ranks = int(cnt[0].item()), int(cnt[1].item()), int(cnt[2].item())

    # single-frame latency (enqueue -> frame complete on the device), D2H of the frame separately;
    # N > 1: each frame gathered on its own
    if gath:
        ctx.check(lib.rrte_hip_set_gather_batch(ctx.h, 1))
    lat = []
    for _ in range(5):
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize(dev)
        a = time.perf_counter()
        step()
        torch.cuda.synchronize(dev)
        lat.append(time.perf_counter() - a)
    latency_ms = statistics.median(lat) * 1e3
    host = torch.empty(W * H, dtype=torch.int32, pin_memory=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    host.copy_(full, non_blocking=True)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    d2h_ms = e0.elapsed_time(e1)

    # The drop-in boundary as Engine::render_frame uses it (engine.rs:280-312 -> raytracer.rs:45-89):
    # blocking rrte_hip_render into a host RGBA8 buffer, D2H included -- into a reused buffer, and
    # into a fresh zeroed buffer per frame as the reference allocates one (`vec![0u8; w*h*4]`,
    # raytracer.rs:54).  Not the headline (SURVEY §8d excludes D2H); rank 0, N = 1 only.
    boundary = None
    if world == 1 and not args.no_boundary:
        hbuf = np.zeros(W * H * 4, dtype=np.uint8)
        pout = lambda b: b.ctypes.data_as(C.POINTER(C.c_uint8))  # noqa: E731
        for _ in range(3):
            ctx.check(lib.rrte_hip_render(ctx.h, scene.ref(), C.byref(prm), pout(hbuf)))
        nb = 20
        a = time.perf_counter()
        for _ in range(nb):
            ctx.check(lib.rrte_hip_render(ctx.h, scene.ref(), C.byref(prm), pout(hbuf)))
        reused_ms = (time.perf_counter() - a) / nb * 1e3
        a = time.perf_counter()
        alloc_s = 0.0
        for _ in range(nb):
            a0 = time.perf_counter()
            fresh = np.zeros(W * H * 4, dtype=np.uint8)
            alloc_s += time.perf_counter() - a0
            ctx.check(lib.rrte_hip_render(ctx.h, scene.ref(), C.byref(prm), pout(fresh)))
        fresh_ms = (time.perf_counter() - a) / nb * 1e3
        # where a fresh buffer's time goes: the allocation (np.zeros: lazily zeroed pages), and the same
        # call into a fresh buffer whose pages were touched first (the copy no longer takes the page
        # faults of a never-touched buffer)
        touched_s = 0.0
        for _ in range(nb):
            fresh = np.zeros(W * H * 4, dtype=np.uint8)
            fresh[::4096] = 1  # first touch of every page, outside the timed call
            a0 = time.perf_counter()
            ctx.check(lib.rrte_hip_render(ctx.h, scene.ref(), C.byref(prm), pout(fresh)))
            touched_s += time.perf_counter() - a0
        # a pinned buffer (registered once with rrte_hip_host_register, as an engine reusing its frame
        # buffer would; or page-locked by the caller): the kernel writes the frame into it directly
        reg = np.zeros(W * H * 4, dtype=np.uint8)
        ctx.check(lib.rrte_hip_host_register(ctx.h, reg.ctypes.data, reg.nbytes))
        for _ in range(10):  # (past the zero-copy launch shape's first frames: its profile and list upload)
            ctx.check(lib.rrte_hip_render(ctx.h, scene.ref(), C.byref(prm), pout(reg)))
        a = time.perf_counter()
        for _ in range(nb):
            ctx.check(lib.rrte_hip_render(ctx.h, scene.ref(), C.byref(prm), pout(reg)))
        reg_ms = (time.perf_counter() - a) / nb * 1e3
        reg_ok = bool(np.array_equal(reg, hbuf))
        ctx.check(lib.rrte_hip_host_unregister(ctx.h, reg.ctypes.data))
        # a buffer the engine allocates page-locked (hipHostMalloc; torch's pinned memory is): zero copy too
        pin = torch.zeros(W * H * 4, dtype=torch.uint8, pin_memory=True)
        ppin = C.cast(C.c_void_p(pin.data_ptr()), C.POINTER(C.c_uint8))
        for _ in range(3):
            ctx.check(lib.rrte_hip_render(ctx.h, scene.ref(), C.byref(prm), ppin))
        a = time.perf_counter()
        for _ in range(nb):
            ctx.check(lib.rrte_hip_render(ctx.h, scene.ref(), C.byref(prm), ppin))
        pin_ms = (time.perf_counter() - a) / nb * 1e3
        pin_ok = bool(np.array_equal(pin.numpy(), hbuf))
        # Engine::render_frame's loop as rust/patches/0002 wires it, in the C++ mirror
        # (rrte_amd/cpp: Raytracer::render_into, the calls rrte-hip-sys's Context::render_engine_frame
        # makes): the engine's frame buffer reused every frame and pinned once through the C ABI, the
        # scene lowered from its objects every frame; every timed frame checked against render()
        import subprocess
        import tempfile
        eng_ms, eng_ok, eng_lower_ms = None, False, None
        tool = ROOT / "rrte_amd" / "lib" / "cpp_mirror_tool"
        if tool.exists():
            with tempfile.TemporaryDirectory() as td:
                r = subprocess.run([str(tool), "engine", args.scene, str(W), str(H), args.mode,
                                    str(Path(td) / "f.bin"), str(nb)], capture_output=True, text=True, timeout=300)
            for tok in r.stdout.split("\n"):
                if tok.startswith("engine_loop_ms_per_frame"):
                    eng_ms = float(tok.split()[1])
                    eng_lower_ms = float(tok.split()[5])
                    eng_ok = r.returncode == 0 and "mismatched 0" in tok
        boundary = {"entry": "rrte_hip_render (blocking; Raytracer::render's signature, host RGBA8 out, D2H included)",
                    "ms_per_frame_engine_loop": round(eng_ms, 4) if eng_ms is not None else None,
                    "engine_loop_equals_render": eng_ok,
                    "engine_loop_lowering_ms": eng_lower_ms,
                    "engine_loop_note": "Engine::render_frame through Raytracer::render_into (rust/patches/0002), run "
                                        "in the C++ mirror (cpp_mirror_tool engine, its own process): the engine's "
                                        "frame_buffer reused and pinned once, the scene lowered from its objects every "
                                        "frame, each timed frame compared with Raytracer::render",
                    "ms_per_frame_reused_buffer": round(reused_ms, 4),
                    "ms_per_frame_fresh_buffer": round(fresh_ms, 4),
                    "fresh_alloc_ms": round(alloc_s / nb * 1e3, 4),
                    "ms_per_frame_fresh_pretouched": round(touched_s / nb * 1e3, 4),
                    "ms_per_frame_registered_buffer": round(reg_ms, 4),
                    "registered_equals_copy_path": reg_ok,
                    "ms_per_frame_hostmalloc_buffer": round(pin_ms, 4),
                    "hostmalloc_equals_copy_path": pin_ok,
                    "frames": nb, "note": "fresh = a new zeroed W*H*4 buffer per frame, as raytracer.rs:54 allocates; "
                                          "registered = the reused buffer pinned once (rrte_hip_host_register): the "
                                          "kernel stores the frame into it directly, no D2H copy; hostmalloc = a "
                                          "frame buffer allocated page-locked (hipHostMalloc), zero copy as well"}

    kinds = None
    if world == 1 and not args.no_stock:
        anim = [scenes.animate_values(LoweredScene(objs, lights, cam), f) for f in range(8)]
        kinds = kernel_variants(scene, prm, fulls, sptrs, dev, W * H * prm.samples_per_pixel + shadow // args.steps,
                                anim=anim)

    # the reference's stock config (rank 0, N=1 only; not the headline) on the headline's context: its
    # own scene-specialised REFCOMPAT kernel (runtime sample / bounce loops), compiled on the warm-up frames
    stock = None
    if world == 1 and not args.no_stock:
        sscene, sprm = stock_config(args)
        for i in range(2):
            ctx.check(lib.rrte_hip_render_async(ctx.h, sscene.ref(), C.byref(sprm), fulls[i % F].data_ptr(), None,
                                                sptrs[i % F]))
        torch.cuda.synchronize(dev)
        n_stock = 6
        a = time.perf_counter()
        for i in range(n_stock):
            ctx.check(lib.rrte_hip_render_async(ctx.h, sscene.ref(), C.byref(sprm), fulls[i % F].data_ptr(), None,
                                                sptrs[i % F]))
        torch.cuda.synchronize(dev)
        ts = (time.perf_counter() - a) / n_stock
        stock = {"workload": f"{args.scene} {W}x{H} reference stock config: REFCOMPAT, spp=4, max_depth=50, "
                             "random jitter + scatter (counter-based RNG)",
                 "value": round(W * H * 4 / ts / 1e6, 3), "unit": "Msample/s", "ms_per_frame": round(ts * 1e3, 4)}

    legs = None
    if world == 1 and not args.no_legs:
        legs = {}
        for key, name, lw, lh, lmode, desc in LEGS:
            legs[key] = config_leg(name, lw, lh, lmode, dev, cpu_budget_s=args.cpu_seconds)
            legs[key]["workload"] = desc

    if rank == 0:
        rays = primary + shadow
        value = rays / elapsed / 1e6
        # per launch: the back-to-back span / frames (what rocprof's average kernel duration is compared
        # with); the per-frame event brackets' median and mean are reported beside it
        mean_launch_ms = float(np.mean(launch_ms))
        median_launch_ms = float(np.median(launch_ms))
        avg_launch_ms = b2b_ms
        # algorithmic HBM bytes per launch: the RGBA8 framebuffer store, 4 B per pixel;
        # the scene (<= a few KB) is served from the scalar cache and counts once.
        bytes_per_launch = 4 * W * rows
        achieved = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9
        flops_frame, _, _ = flop_tally(scene, prm)
        flops_launch = flops_frame * rows / H
        valu_tf = flops_launch / (avg_launch_ms * 1e-3) / 1e12
        wl = f"{args.scene}@{W}x{H}/{args.mode}"
        pmc, pmc_note = pmc_traffic(wl, abi.build_id())
        line = {
            "metric": "Mray/s (primary+shadow) at 1920x1080, sdf-showcase scene; 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",  # one 1080p frame per step whatever N: total work fixed
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": f"{args.scene} {W}x{H}, {args.mode}, spp={prm.samples_per_pixel}, max_depth={prm.max_depth}, "
                            + ("random jitter" if args.random else "pixel-centre jitter")
                            + (f", {args.band_rows}-row bands over {world} GPUs (sky bands on rank 0, the rest round robin) + RCCL send/recv to rank 0"
                               f" in batches of {min(F, 16)} frames" if world > 1 else "")
                            + (", REHEARSAL: gather path through a 1-rank communicator" if gath and not dist_on else ""),
                "scene": args.scene, "width": W, "height": H, "mode": args.mode,
                "primary_rays_per_frame": W * H * prm.samples_per_pixel,
                "shadow_rays_per_frame": shadow // args.steps,
                "frames_in_flight": F,
                "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                "parallelism": f"rows{world}" if world > 1 else "single",
            },
            # the binding roofline: VALU FP32 (no dense contraction, no MFMA).  achieved =
            # algorithmic FP32 ops of one launch (the oracle's instrumented counting build) / the
            # average launch duration; HBM beside it (4 B/pixel frame store, PMC traffic)
            "roofline": {
                "bound": "valu",
                "achieved": round(valu_tf, 3),
                "peak": VALU_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": valu_tf / VALU_PEAK_TFLOPS,
                "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
                "traffic_unit": "HBM bytes per launch (rocprofv3 PMC, profiles/pmc_*.json of this build)",
                "profile": pmc_note,
                "flops_per_launch": flops_launch,
                "frac_of_unpacked_peak": valu_tf / (VALU_PEAK_TFLOPS / 2),
                "achieved_at_frame_rate": round(flops_launch / (elapsed / args.steps) / 1e12, 3),
                "kernel": ("rrte_jit_kernel (scene-specialised, hiprtc)" if st.jit_active else
                           "rrte::ray_kernel<%s> (generic)" % ("LAMBERT_SHADOW" if args.mode == "lambert_shadow" else "REFCOMPAT")),
                "jit_compile_ms": round(st.jit_compile_ms, 1) if st.jit_active else None,
                "jit_active_ranks": f"{jit_ranks}/{world}",
                "avg_launch_ms": round(avg_launch_ms, 5),
                "bracket_median_ms": round(median_launch_ms, 5),
                "bracket_mean_ms": round(mean_launch_ms, 5),
                "avg_launch_note": f"HIP events around {n_seq} frames run back to back on one stream, span / {n_seq}; "
                                   "launch_ms_each: an event pair around each frame (includes the stream gap)",
                "launch_ms_each": [round(x, 4) for x in launch_ms],
                "note": "peak = packed-FP32 vector peak (MI355X_MICROARCH.md); the kernel issues unpacked FP32, one ray "
                        "per lane" + ("" if world == 1 else f"; N > 1: rank 0's share, flops scaled by its rows ({rows}/{H})"),
                "hbm": {"achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "bytes_per_launch": bytes_per_launch,
                        "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
                        "note": "algorithmic bytes = the 4 B/pixel RGBA8 frame store"},
            },
        }
        line["primary_only"] = {"value": round(primary / elapsed / 1e6, 3), "unit": "Mray/s"}
        line["frame_latency_ms"] = round(latency_ms, 4)
        line["host_enqueue_ms_per_step"] = round((t_enq - t0) / args.steps * 1e3, 4)
        # hot-first tile order: slots of the timed frames' launches dispatched first
        env_order = os.environ.get("RRTE_TILE_ORDER", "")
        line["tile_order"] = {"hot_slots": int(st.hot_tiles),
                              "tiles": ((W + 7) // 8) * ((rows + 7) // 8),
                              "mode": {"0": "image order", "2": "fixed permutation (tests)"}.get(
                                  env_order, "measured cost, slowest first (default)")}
        line["d2h_ms"] = round(d2h_ms, 4)  # frame to pinned host memory, excluded from `value`
        if pmc and pmc.get("valu") is not None:
            line["valu"] = dict(pmc["valu"])
            mp = measured_valu_peak()
            if mp:
                # the PMC issue rate against the MEASURED wave64 issue rates of this chip (tools/valu_peak.hip)
                r = line["valu"]["wave_instr_per_s"]
                line["valu"]["measured_peak"] = mp
                line["valu"]["frac_of_measured_fma_class_peak"] = r / mp["fma_add_mul"]
                line["valu"]["frac_of_measured_cmp_select_peak"] = r / mp["cmp_select_max"]
            # the same instructions issued at the frame rate of the timed stream (frames in flight): the
            # lone-launch rate above includes one frame's fill and drain, the stream rate does not
            insts = pmc.get("counters_per_dispatch", {}).get("SQ_INSTS_VALU")
            if insts:
                fr = insts / (elapsed / args.steps)
                line["valu"]["wave_instr_per_s_at_frame_rate"] = fr
                line["valu"]["issue_frac_at_frame_rate"] = fr / line["valu"]["peak_wave_instr_per_s"]
                if mp:
                    line["valu"]["frac_of_measured_fma_class_peak_at_frame_rate"] = fr / mp["fma_add_mul"]
        if boundary is not None:
            line["boundary"] = boundary
        if kinds is not None:
            line["kernel_kinds"] = kinds
        if legs is not None:
            line["configs"] = legs
        if stock is not None:
            line["stock_config"] = stock
        if world == 1 and not args.no_cpu:
            sband = (H // 2 - H // 8, H // 2 + H // 8)  # centre quarter of the frame
            line["cpu_baseline"], ref = cpu_baseline(scene, prm, args.cpu_seconds,
                                                     stock=(*stock_config(args), sband) if stock else None)
            line["cpu_baseline"]["gpu_over_cpu"] = round(value / line["cpu_baseline"]["value"], 2)
            if "whole_host_extrapolation" in line["cpu_baseline"]:
                wh = line["cpu_baseline"]["whole_host_extrapolation"]
                wh["gpu_over_whole_host"] = round(value / wh["value"], 2)
            if stock and "stock_config" in line["cpu_baseline"]:
                line["stock_config"]["gpu_over_cpu"] = round(stock["value"] / line["cpu_baseline"]["stock_config"]["value"], 2)
        else:
            ref = oracle_frame(scene, prm)
        if K > 1:  # fly-by: every buffer against the oracle frame of its last frame's pose
            refs = [oracle_frame(ps, prm) for ps in poses]
            last = [max(i for i in range(args.steps) if i % F == j) for j in range(len(timed_frames))]
            line["verified"] = verify_frames(timed_frames, shadow, args.steps, None,
                                             refs=[refs[i % K] for i in last],
                                             shadow_total=sum(refs[i % K][1] for i in range(args.steps)))
            line["config"]["flyby_poses"] = K
        else:
            line["verified"] = verify_frames(timed_frames, shadow, args.steps, ref)  # (shadow: summed over ranks)
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
