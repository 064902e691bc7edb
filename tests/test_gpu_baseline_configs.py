"""BASELINE configs 3, 4 and 5 at their exact sizes on the GPU (BASELINE.json configs[2:5]):
  config 3  cornell_box_test(false), 600x600, 1000 spp, max_depth 1000
  config 4  millions_of_spheres (seed 42, 2,106,105 spheres), 1920x1080, 256 spp, max_depth 50
  config 5  rtweekend_final_image (seed 42), 3840x2160, 10,000 spp, max_depth 50
No oracle renders a whole frame at these sizes, so each test checks size-independent properties
of the full frame (finite, non-negative, bounded where the scene bounds radiance, the guard of
crt_schlick.h at 0, identical under the row tilings an 8-GPU job uses) and 8x8 windows against
the C oracle (pinned to the reference by tests/test_oracle.py) at the places a bug would show:
partial-sum band edges, tile-row edges, the most expensive rows and the last pixels.
Tolerance: north_star's 1e-4 per channel (the paths are identical; observed error ~1e-15)."""
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, str(ROOT / "oracle"))
import crt_oracle_py as orc  # noqa: E402

pytestmark = [pytest.mark.gpu, pytest.mark.slow]
TOL = 1e-4


def scene(crt, name, seed, **cam):
    from cpp_raytracer_amd import camera_with
    d = crt.SceneData.named(name, seed)
    d.camera = camera_with(d.camera, **cam)
    return d


def render_frame(crt, s, d, base, tiling=None, out=None):
    import torch
    cs = d.camera
    if out is None:
        out = torch.full((cs.image_h, cs.image_w, 3), float("nan"), dtype=torch.float64, device="cuda")
    s.render_async(0, crt.resolve_camera(cs, base), out.data_ptr(), torch.cuda.current_stream().cuda_stream, tiling)
    return out


def check_windows(d, frame, base, windows, threads=16):
    worst = 0.0
    for r0, r1, c0, c1 in windows:
        want = orc.render(d, base, threads=threads, crop=(r0, r1, c0, c1))
        err = np.abs(frame[r0:r1, c0:c1] - want)
        assert err.max() <= TOL, f"window {(r0, r1, c0, c1)}: max err {err.max()}"
        worst = max(worst, float(err.max()))
    return worst


def check_tiling(crt, s, d, base, whole, ranks, blocks):
    """The rows an N-rank job renders (Tiling(4, N, k), bench.py / crt_render) equal the
    whole-frame render bit for bit, for the given ranks k."""
    import torch
    from cpp_raytracer_amd import Tiling
    from cpp_raytracer_amd.tiles import owned_rows
    h = d.camera.image_h
    part = torch.full_like(whole, float("nan"))
    for k in blocks:
        render_frame(crt, s, d, base, Tiling(4, ranks, k, 0), part)
    torch.cuda.synchronize()
    for k in blocks:
        rows = torch.as_tensor(owned_rows(h, 4, ranks, k), device="cuda")
        assert torch.equal(part[rows], whole[rows]), (ranks, k)


def test_config3_cornell_full_size(crt):
    import torch
    d = scene(crt, "cornell", None, image_w=600, image_h=600, samples_per_pixel=1000, max_depth=1000)
    s = crt.GpuScene(d)
    s.upload(0)
    base = 303
    whole = render_frame(crt, s, d, base)
    again = render_frame(crt, s, d, base)
    torch.cuda.synchronize()
    assert torch.equal(whole, again)  # deterministic
    check_tiling(crt, s, d, base, whole, 8, range(8))
    f = whole.cpu().numpy()
    assert np.isfinite(f).all() and f.min() >= 0
    # the light (intensity 15) is seen directly; the room is lit (the black background shows
    # around the open front of the box)
    assert f.max() == 15 and (f.mean(axis=2) > 0).mean() > 0.85
    check_windows(d, f, base, [
        (0, 8, 0, 8),             # corner
        (296, 304, 296, 304),     # centre (between the boxes)
        (428, 436, 150, 158),     # the short box's face: long paths inside the room
        (4, 12, 252, 260),        # tile rows 1-2 edge under the light
        (592, 600, 592, 600),     # last pixels
    ])


def test_config4_millions_full_size(crt):
    import torch
    d = scene(crt, "millions", 42, image_w=1920, image_h=1080, samples_per_pixel=256, max_depth=50)
    s = crt.GpuScene(d, build_device=0)
    info = s.info()
    assert info.num_primitives == 2_106_105
    s.upload(0)
    base = 404
    whole = render_frame(crt, s, d, base)
    torch.cuda.synchronize()
    check_tiling(crt, s, d, base, whole, 8, (0, 3, 7))  # three ranks' shares of an 8-GPU job
    assert s.guard(0) == 0
    f = whole.cpu().numpy()
    assert np.isfinite(f).all() and f.min() >= 0
    check_windows(d, f, base, [
        (536, 544, 956, 964),     # centre: the deepest BVH walks
        (0, 8, 0, 8),             # sky corner
        (1072, 1080, 1912, 1920), # last pixels
        (700, 708, 300, 308),     # the sphere field, lower left
    ])


def test_config5_rtow_4k_10000spp(crt):
    """82.9 G samples (~12 s on one GPU): the partial sums of the 189 sample chunks per pixel
    take 37.6 GB, so the frame renders in bands of 244 rows (4 GiB budget); windows straddle the
    first band edge and a later one."""
    import torch
    d = scene(crt, "rtow_final", 42, image_w=3840, image_h=2160, samples_per_pixel=10000, max_depth=50)
    s = crt.GpuScene(d)
    s.upload(0)
    base = 505
    whole = render_frame(crt, s, d, base)
    torch.cuda.synchronize()
    assert s.guard(0) == 0
    f = whole.cpu().numpy()
    assert np.isfinite(f).all() and f.min() >= 0 and f.max() <= 1  # no lights, background <= 1
    check_windows(d, f, base, [
        (240, 248, 1916, 1924),   # first band edge (row 244)
        (1460, 1468, 2000, 2008), # band edge at row 1464
        (1076, 1084, 1916, 1924), # centre: the glass sphere
        (2152, 2160, 3832, 3840), # last pixels
    ])
    del f
    # rank 2's share of an 8-GPU split, rendered alone, equals those rows of the whole frame
    check_tiling(crt, s, d, base, whole, 8, (2,))
