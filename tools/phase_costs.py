"""Per-phase cost of the render kernel on a BASELINE config (instrumented pass, crt_render_count):
wave iterations and wall-clock ticks per phase, ticks per iteration, lane utilization.
usage: python tools/phase_costs.py [config2|config3|config4] [ranks rank] (a rank's share of the
4-row deal over `ranks`, as the multi-GPU bench renders it)"""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import cpp_raytracer_amd as crt  # noqa: E402
from cpp_raytracer_amd import Tiling, camera_with  # noqa: E402

CONFIGS = {
    "config2": ("rtow_final", 42, dict(image_w=1200, image_h=800, samples_per_pixel=500, max_depth=50)),
    "config3": ("cornell", None, dict(image_w=600, image_h=600, samples_per_pixel=1000, max_depth=1000)),
    "config4": ("millions", 42, dict(image_w=1920, image_h=1080, samples_per_pixel=256, max_depth=50)),
}
name = sys.argv[1] if len(sys.argv) > 1 else "config2"
scene, seed, cam_kw = CONFIGS[name]
d = crt.SceneData.named(scene, seed)
d.camera = camera_with(d.camera, **cam_kw)
s = crt.GpuScene(d, build_device=0 if len(d.objects) > 100_000 else None)
s.upload(0)
tl = Tiling(4, int(sys.argv[2]), int(sys.argv[3]), 0) if len(sys.argv) > 3 else None
c = s.render_count(0, crt.resolve_camera(d.camera, 2024), tl)
print(f"{name}: rays {c.rays}, nodes {c.nodes_visited}, sphere tests {c.sphere_tests}, quad tests {c.parallelogram_tests}")
work = {"walk": c.nodes_visited, "leaf": c.sphere_tests + c.parallelogram_tests, "shade": c.rays}
for ph in ("walk", "leaf", "shade"):
    it = getattr(c, "wave_iters_" + ph)
    tk = getattr(c, "ticks_" + ph)
    print(f"  {ph:5s}: iterations {it:>12d}  ticks {tk:>14d} ({tk / c.ticks_total:.3f})  "
          f"ticks/iteration {tk / max(1, it):7.3f}  lane utilization {work[ph] / max(1, 64 * it):.3f}")
print(f"  tail ticks {c.ticks_tail} ({c.ticks_tail / c.ticks_total:.3f}), total {c.ticks_total}, kernel {c.kernel_ms:.1f} ms (instrumented)")
