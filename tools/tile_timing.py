"""Per-rank render time of a BASELINE frame when its rows are dealt over N ranks (4-row blocks,
crt_tiling{4, N, r}, what bench.py and crt_render do), measured on one GPU by rendering each rank's
share alone, packed (CRT_TILING_PACKED): estimates strong-scaling efficiency T(1) / (N * max_r
T_r(N)) without N GPUs. Also the per-rank setup a rank pays before its first frame: scene build
(host or GPU BVH build) and upload to HBM.
usage: python tools/tile_timing.py [--config 2|3|4|5] [--steps K] [--all] [--ns 1,2,4,8]
(--all: every rank of every N; default: ranks 0 and N - 1)"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import cpp_raytracer_amd as crt  # noqa: E402
from cpp_raytracer_amd import Tiling, camera_with  # noqa: E402
from cpp_raytracer_amd.tiles import owned_rows  # noqa: E402

CONFIGS = {
    "2": ("rtow_final", 42, dict(image_w=1200, image_h=800, samples_per_pixel=500, max_depth=50)),
    "3": ("cornell", None, dict(image_w=600, image_h=600, samples_per_pixel=1000, max_depth=1000)),
    "4": ("millions", 42, dict(image_w=1920, image_h=1080, samples_per_pixel=256, max_depth=50)),
    "5": ("rtow_final", 42, dict(image_w=3840, image_h=2160, samples_per_pixel=10000, max_depth=50)),
}
ap = argparse.ArgumentParser()
ap.add_argument("--config", default="2", choices=sorted(CONFIGS))
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--all", action="store_true")
ap.add_argument("--ns", default="1,2,4,8")
a = ap.parse_args()
scene, seed, kw = CONFIGS[a.config]
d = crt.SceneData.named(scene, seed)
d.camera = camera_with(d.camera, **kw)
h, w = kw["image_h"], kw["image_w"]
big = len(d.objects) > 100_000
# a rank's setup: build (GPU BVH build for the millions scene, as bench.py does) and upload
t0 = time.perf_counter()
s = crt.GpuScene(d, build_device=0 if big else None)
t_build = time.perf_counter() - t0
t0 = time.perf_counter()
s.upload(0)
torch.cuda.synchronize()
t_upload = time.perf_counter() - t0
info = s.info()
print(f"config {a.config} ({scene}, {w}x{h}, {kw['samples_per_pixel']} spp): {info.num_primitives} primitives, "
      f"{info.num_nodes} nodes; rank setup: scene build {t_build * 1e3:.1f} ms "
      f"({'GPU' if big else 'host'} BVH {info.build_ms:.1f} ms), upload {t_upload * 1e3:.1f} ms "
      f"({info.device_bytes / 2**20:.1f} MiB)", flush=True)
cam = crt.resolve_camera(d.camera, 2024)
st = torch.cuda.current_stream()
t1 = None
for n in (int(x) for x in a.ns.split(",")):
    worst, per = 0.0, []
    for r in (range(n) if a.all else sorted({0, n - 1})):
        rows = len(owned_rows(h, 4, n, r))
        frame = torch.empty(max(1, rows), w, 3, dtype=torch.float64, device="cuda")
        tl = Tiling(4, n, r, 1)
        s.render_async(0, cam, frame.data_ptr(), st.cuda_stream, tl)  # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            s.render_async(0, cam, frame.data_ptr(), st.cuda_stream, tl)
        torch.cuda.synchronize()
        per.append((time.perf_counter() - t0) / a.steps)
        worst = max(worst, per[-1])
        del frame
    if n == 1 or t1 is None:
        t1 = worst * n
    print(f"N={n}: slowest rank {worst * 1e3:.2f} ms, est. efficiency {t1 / (n * worst):.3f}"
          + (f" (ranks: {' '.join(f'{x * 1e3:.2f}' for x in per)} ms)" if a.all else ""), flush=True)
assert s.guard(0) == 0
