"""A rank's share of the config-2 frame at N GPUs under grid-size / item-size settings (one GPU):
the slowest rank's render time for each (CRT_GRID_BLOCKS, CRT_ITEM_CHUNKS, CRT_TAIL_CHUNKS).
usage: N=8 python tools/grid_sweep.py "blocks:k:tail" ...   (x = the default)"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import cpp_raytracer_amd as crt  # noqa: E402
from cpp_raytracer_amd import Tiling, camera_with  # noqa: E402

n = int(os.environ.get("N", "8"))
d = crt.SceneData.named("rtow_final", 42)
d.camera = camera_with(d.camera, image_w=1200, image_h=800, samples_per_pixel=500, max_depth=50)
s = crt.GpuScene(d)
s.upload(0)
cam = crt.resolve_camera(d.camera, 2024)
frame = torch.zeros(800, 1200, 3, dtype=torch.float64, device="cuda")
st = torch.cuda.current_stream()


def share_ms(tl, steps=3):
    s.render_async(0, cam, frame.data_ptr(), st.cuda_stream, tl)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        s.render_async(0, cam, frame.data_ptr(), st.cuda_stream, tl)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


for spec in sys.argv[1:]:
    for name, v in zip(("CRT_GRID_BLOCKS", "CRT_ITEM_CHUNKS", "CRT_TAIL_CHUNKS"), spec.split(":")):
        if v == "x":
            os.environ.pop(name, None)
        else:
            os.environ[name] = v
    per = [share_ms(Tiling(4, n, r, 0)) for r in range(n)]
    print(f"N={n} {spec}: slowest {max(per):.2f} ms, mean {sum(per) / n:.2f} ms", flush=True)
