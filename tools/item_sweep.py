"""Item-size sweep for a rank's share of the config-2 frame (one GPU): for each N and each
(CRT_ITEM_CHUNKS, CRT_TAIL_CHUNKS) pair, the slowest rank's render time over all N ranks.
usage: [NS="4 8"] [KS="2 3 4"] [TS="13 25 40"] python tools/item_sweep.py"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import cpp_raytracer_amd as crt  # noqa: E402
from cpp_raytracer_amd import Tiling, camera_with  # noqa: E402

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


def env_list(name, default):
    v = os.environ.get(name)
    return [int(x) for x in v.split()] if v else default


combos = [(None, None)] + [(k, t) for k in env_list("KS", [2, 3, 4]) for t in env_list("TS", [13, 25, 40])]
for n in env_list("NS", [4, 8]):
    for k, t in combos:
        for name, v in (("CRT_ITEM_CHUNKS", k), ("CRT_TAIL_CHUNKS", t)):
            if v is None:
                os.environ.pop(name, None)
            else:
                os.environ[name] = str(v)
        per = [share_ms(Tiling(4, n, r, 0)) for r in range(n)]
        print(f"N={n} K={k or 'auto'} tail={t if t is not None else 'auto'}: slowest {max(per):.2f} ms, "
              f"mean {sum(per) / n:.2f} ms", flush=True)
