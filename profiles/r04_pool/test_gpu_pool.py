"""The block-level ray exchange (render_pool_kernel, CRT_POOL=1; north_star's compaction of live
rays between bounces, camera.h:205-258 is the bounce boundary): rays move between the 16 waves of
a block through LDS rings, so which lane traces a ray changes, never a ray's operations. Frames
must be bit-identical to the per-wave kernel's (render_kernel) and match the reference goldens."""
import numpy as np
import pytest

from conftest import load_npz
from test_gpu_parity import TOL, render_full, scene_for

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", ["config1", "rtow_crop", "rtow_glass_crop", "cornell_crop", "cornell_empty_small",
                                  "parallelograms_small", "lights_crop", "christmas_crop"])
def test_pool_equals_wave_kernel_and_reference(crt, golden_meta, monkeypatch, case):
    meta = golden_meta["renders"][case]
    d = scene_for(crt, meta)
    want = render_full(crt, d, meta["base_seed"])
    monkeypatch.setenv("CRT_POOL", "1")
    got = render_full(crt, d, meta["base_seed"])
    assert np.array_equal(got, want)
    gold = load_npz(f"render_{case}.npz")["rgb"]
    if meta["crop"]:
        r0, r1, c0, c1 = meta["crop"]
        got = got[r0:r1, c0:c1]
    assert np.all(np.abs(got - gold) <= TOL * np.maximum(1, np.abs(gold)))


@pytest.mark.parametrize("grid", ["1", "3", "37"])
def test_pool_schedule_does_not_change_frames(crt, monkeypatch, grid):
    """Grids of 1, 3 and 37 blocks (CRT_GRID_BLOCKS): a different exchange pattern, the same frame."""
    from cpp_raytracer_amd import camera_with
    d = crt.SceneData.named("rtow_final", 42)
    d.camera = camera_with(d.camera, image_w=96, image_h=64, samples_per_pixel=12, max_depth=50)
    want = render_full(crt, d, 31)
    monkeypatch.setenv("CRT_POOL", "1")
    monkeypatch.setenv("CRT_GRID_BLOCKS", grid)
    assert np.array_equal(render_full(crt, d, 31), want)


@pytest.mark.parametrize("scene,w,h,spp,depth", [("rtow_final", 300, 200, 16, 50), ("cornell", 120, 120, 24, 1000)])
def test_pool_counts_equal_wave_kernel(crt, monkeypatch, scene, w, h, spp, depth):
    """The instrumented pass of the pool kernel traces the same rays, node and primitive tests."""
    from cpp_raytracer_amd import camera_with
    d = crt.SceneData.named(scene, 42 if scene == "rtow_final" else None)
    d.camera = camera_with(d.camera, image_w=w, image_h=h, samples_per_pixel=spp, max_depth=depth)
    s = crt.GpuScene(d)
    s.upload(0)
    cam = crt.resolve_camera(d.camera, 3)
    a = s.render_count(0, cam)
    monkeypatch.setenv("CRT_POOL", "1")
    b = s.render_count(0, cam)
    for f in ("samples", "rays", "nodes_visited", "sphere_tests", "parallelogram_tests", "candidate_tests"):
        assert getattr(a, f) == getattr(b, f), f


@pytest.mark.parametrize("seed", [0, 1, 4, 5, 8, 9, 12, 13])
def test_pool_random_worlds(crt, monkeypatch, seed):
    """Randomized sphere-only and axis-aligned-parallelogram worlds (test_gpu_fuzz_scenes.py's
    families 0 and 1): the pool kernel's frame equals the per-wave kernel's bit for bit."""
    from test_gpu_fuzz_scenes import random_world, render_gpu
    family, d = random_world(crt, seed)
    base = 9000 + seed
    want, _ = render_gpu(crt, d, base)
    monkeypatch.setenv("CRT_POOL", "1")
    got, guard = render_gpu(crt, d, base)
    assert guard == 0
    assert np.array_equal(got, want), family
