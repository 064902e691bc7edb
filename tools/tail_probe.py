"""Where a rank's share of the config-2 frame loses time against 1/N of the whole frame: the
instrumented pass (render_count) of rank shares at N = 1 and 8, with the average wave's span
against the kernel's, the tail share (first idle lane to wave end) and the phase shares.
usage: python tools/tail_probe.py"""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import cpp_raytracer_amd as crt  # noqa: E402
from cpp_raytracer_amd import Tiling, camera_with  # noqa: E402

d = crt.SceneData.named("rtow_final", 42)
d.camera = camera_with(d.camera, image_w=1200, image_h=800, samples_per_pixel=500, max_depth=50)
s = crt.GpuScene(d)
s.upload(0)
cam = crt.resolve_camera(d.camera, 2024)
waves = int(os.environ.get("WAVES", "5120"))
for n, r in ((1, 0), (8, 7), (8, 0)):
    st = s.render_count(0, cam, Tiling(4, n, r, 0))
    avg_ms = st.ticks_total / waves / 1e5  # wall_clock64: 100 MHz
    print(f"N={n} rank {r}: kernel {st.kernel_ms:.2f} ms, average wave span {avg_ms:.2f} ms, "
          f"tail share {st.ticks_tail / st.ticks_total:.4f}, rays {st.rays}, "
          f"walk {st.ticks_walk / st.ticks_total:.3f} leaf {st.ticks_leaf / st.ticks_total:.3f} "
          f"shade {st.ticks_shade / st.ticks_total:.3f}", flush=True)
