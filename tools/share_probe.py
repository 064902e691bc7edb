"""Why a rank's share of the config-2 frame at N GPUs takes more than 1/N of the whole frame:
per-share render time (5 renders after a warm-up, one GPU) for the default 4-row interleave, a
contiguous block of the same rows count, and item sizes forced to 1 or 7 chunks
(CRT_ITEM_CHUNKS / CRT_TAIL_CHUNKS), each x N against the whole frame.
usage: python tools/share_probe.py"""
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


def timed(tl, env=None, steps=5):
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        s.render_async(0, cam, frame.data_ptr(), st.cuda_stream, tl)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            s.render_async(0, cam, frame.data_ptr(), st.cuda_stream, tl)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


whole = timed(None)
print(f"whole frame: {whole:.2f} ms", flush=True)
for label, tl, n, env in [
    ("whole frame, 1-chunk items", None, 1, {"CRT_ITEM_CHUNKS": "1", "CRT_TAIL_CHUNKS": "0"}),
    ("N=8 rank 0, 4-row interleave (default)", Tiling(4, 8, 0, 0), 8, None),
    ("N=8 rank 0, 7-chunk items + tail", Tiling(4, 8, 0, 0), 8, {"CRT_ITEM_CHUNKS": "7", "CRT_TAIL_CHUNKS": "13"}),
    ("N=8 rank 0, 100 contiguous rows", Tiling(100, 8, 0, 0), 8, None),
    ("N=8 rank 3, 100 contiguous rows", Tiling(100, 8, 3, 0), 8, None),
    ("N=2 rank 0, 4-row interleave", Tiling(4, 2, 0, 0), 2, None),
    ("N=2 rank 0, 400 contiguous rows", Tiling(400, 2, 0, 0), 2, None),
]:
    ms = timed(tl, env)
    print(f"{label}: {ms:.2f} ms, x{n} = {ms * n:.1f} ms ({ms * n / whole:.3f} of the whole frame)", flush=True)
