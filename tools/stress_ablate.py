"""Timing ablation of the deformation-stress scene (diagnostic only, not a parity path):
full scene vs. the noise deformer with fewer octaves, with the oracle's march-step count per pixel
(at 480x270) so the per-evaluation cost can be separated from the step count.
usage: python tools/stress_ablate.py [octaves ...]"""
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    octs = int(sys.argv[2])
    from rrte_amd import renderer, scenes
    orig = renderer.NoiseDeformer.with_octaves
    renderer.NoiseDeformer.with_octaves = lambda self, n: orig(self, octs)
    if len(sys.argv) > 3 and sys.argv[3] == "count":
        import oracle
        from rrte_amd import LoweredScene
        o, l, c, cfg = scenes.deformation_stress(480, 270)
        cnt, flops = oracle.count(LoweredScene(o, l, c), cfg.lower(), nthreads=8)
        print(json.dumps({"steps_px": cnt.sdf_steps / (480 * 270), "flops_px": flops / (480 * 270)}))
        sys.exit(0)
    import bench
    sys.argv = ["bench.py", "--scene", "deformation-stress", "--width", "3840", "--height", "2160",
                "--no-cpu", "--no-stock", "--steps", "6", "--warmup", "2"]
    bench.main()
    sys.exit(0)

for octs in [int(a) for a in sys.argv[1:]] or [4, 2, 0]:
    cnt = json.loads(subprocess.run([sys.executable, __file__, "--child", str(octs), "count"], check=True,
                                    capture_output=True, text=True).stdout.strip().splitlines()[-1])
    out = subprocess.run(["timeout", "-k", "10", "200", sys.executable, __file__, "--child", str(octs)], check=True,
                         capture_output=True, text=True).stdout.strip().splitlines()[-1]
    d = json.loads(out)
    print(f"octaves={octs} ms/frame={d['ms_per_step']:.3f} launch_ms={d['roofline']['avg_launch_ms']:.3f} "
          f"steps/px={cnt['steps_px']:.2f} flops/px={cnt['flops_px']:.0f} "
          f"ns/step-px={d['roofline']['avg_launch_ms'] * 1e6 / (3840 * 2160 * cnt['steps_px']):.4f}", flush=True)
