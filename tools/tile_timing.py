"""Per-rank render time of the config-2 frame when its rows are dealt over N ranks (4-row blocks),
measured on one GPU by rendering each rank's share alone: estimates strong-scaling efficiency
T(1) / (N * max_r T_r(N)) without N GPUs. usage: python tools/tile_timing.py [steps] [all]
(all: every rank of every N; default: ranks 0 and N - 1)"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import cpp_raytracer_amd as crt  # noqa: E402
from cpp_raytracer_amd import Tiling, camera_with  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
all_ranks = len(sys.argv) > 2 and sys.argv[2] == "all"
d = crt.SceneData.named("rtow_final", 42)
d.camera = camera_with(d.camera, image_w=1200, image_h=800, samples_per_pixel=500, max_depth=50)
s = crt.GpuScene(d)
s.upload(0)
cam = crt.resolve_camera(d.camera, 2024)
frame = torch.zeros(800, 1200, 3, dtype=torch.float64, device="cuda")
st = torch.cuda.current_stream()
t1 = None
for n in (1, 2, 4, 8):
    worst = 0.0
    per = []
    for r in (range(n) if all_ranks else (0, n - 1)):
        tl = Tiling(4, n, r, 0)
        s.render_async(0, cam, frame.data_ptr(), st.cuda_stream, tl)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            s.render_async(0, cam, frame.data_ptr(), st.cuda_stream, tl)
        torch.cuda.synchronize()
        per.append((time.perf_counter() - t0) / steps)
        worst = max(worst, per[-1])
    if n == 1:
        t1 = worst
    print(f"N={n}: slowest rank {worst * 1e3:.1f} ms, est. efficiency {t1 / (n * worst):.3f}"
          + (f" (ranks: {' '.join(f'{x * 1e3:.2f}' for x in per)} ms)" if all_ranks else ""), flush=True)
