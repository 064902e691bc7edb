"""GPU kernel vs the C oracle at sizes beyond the golden fixtures, on every kernel variant
(LDS-staged scene, HBM scene + LDS stack, HBM stack), plus size-independent properties at the
BASELINE sizes. Tolerance: north_star's 1e-4 per channel; paths are expected bit-identical."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, str(ROOT / "oracle"))
import crt_oracle_py as orc  # noqa: E402

pytestmark = pytest.mark.gpu
TOL = 1e-4


def scene(crt, name, seed=None, **cam):
    from cpp_raytracer_amd import camera_with
    d = crt.SceneData.named(name, seed)
    d.camera = camera_with(d.camera, **cam)
    return d


def gpu(crt, d, base, **kw):
    s = crt.GpuScene(d, **kw)
    out, _ = s.render(crt.resolve_camera(d.camera, base), 1)
    return out


def check(got, want):
    err = np.abs(got - want)
    assert err.max() <= TOL, f"max err {err.max()} at {np.unravel_index(err.argmax(), err.shape)}"
    return err.max()


def test_rtow_full_frame_small(crt):
    d = scene(crt, "rtow_final", 42, image_w=200, image_h=134, samples_per_pixel=8, max_depth=50)
    check(gpu(crt, d, 31), orc.render(d, 31, threads=8))


def test_cornell_deep_paths(crt):
    d = scene(crt, "cornell", image_w=96, image_h=96, samples_per_pixel=8, max_depth=1000)
    check(gpu(crt, d, 32), orc.render(d, 32, threads=8))


def test_christmas_tree_hbm_scene(crt):
    # 4202 primitives: too big for the LDS budget -> scene in HBM, stack in LDS
    d = scene(crt, "christmas_tree", image_w=135, image_h=76, samples_per_pixel=8)
    check(gpu(crt, d, 33), orc.render(d, 33, threads=8))


def test_hbm_stack_variant(crt, monkeypatch):
    monkeypatch.setenv("CRT_FORCE_GSTACK", "1")
    d = scene(crt, "rtow_final", 42, image_w=80, image_h=54, samples_per_pixel=4, max_depth=50)
    check(gpu(crt, d, 34), orc.render(d, 34, threads=8))


def test_linear_mode_matches_bvh(crt):
    # a non-Scene Hittable renders through one always-entered leaf; same pixels as the BVH (the
    # reference-pinned linear cases are test_gpu_parity.py::test_linear_world_matches_reference)
    d = scene(crt, "cornell", image_w=48, image_h=48, samples_per_pixel=4, max_depth=50)
    check(gpu(crt, d, 35, linear=True), gpu(crt, d, 35))


def test_pathological_oversize_leaf(crt):
    d = scene(crt, "bvh_pathological", image_w=64, image_h=36, samples_per_pixel=2, max_depth=10)
    check(gpu(crt, d, 36), orc.render(d, 36, threads=8))


def test_lights_and_dielectrics(crt):
    d = scene(crt, "rtow_final_lights", image_w=160, image_h=90, samples_per_pixel=8)
    check(gpu(crt, d, 37), orc.render(d, 37, threads=8))


@pytest.mark.slow
def test_millions_crop_deep_bvh(crt):
    # 2.1M spheres, 504,893 nodes, depth 26: u32 stack, HBM scene; a crop of the BASELINE frame
    d = scene(crt, "millions", 42, image_w=1920, image_h=1080, samples_per_pixel=4, max_depth=50)
    full = gpu(crt, d, 38)
    want = orc.render(d, 38, threads=16, crop=(500, 532, 900, 964))
    check(full[500:532, 900:964], want)


@pytest.mark.slow
def test_baseline_config2_properties(crt):
    """Full BASELINE config 2 frame (1200x800x500 spp, depth 50): no oracle at this size, so
    size-independent properties: finite, in [0, 1] (no lights; background <= 1), deterministic
    across two renders, identical under a 3-way row tiling, and a checked 8x8 window equal to the
    oracle for the same pixels."""
    import torch
    from cpp_raytracer_amd import Tiling
    d = scene(crt, "rtow_final", 42, image_w=1200, image_h=800, samples_per_pixel=500, max_depth=50)
    s = crt.GpuScene(d)
    s.upload(0)
    cam = crt.resolve_camera(d.camera, 2024)
    a = torch.empty(800, 1200, 3, dtype=torch.float64, device="cuda")
    b = torch.empty_like(a)
    st = torch.cuda.current_stream().cuda_stream
    s.render_async(0, cam, a.data_ptr(), st)
    for t in range(3):
        s.render_async(0, cam, b.data_ptr(), st, Tiling(16, 3, t, 0))
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert s.guard(0) == 0  # no Dielectric branch of the 4 frames depends on glibc's pow rounding
    an = a.cpu().numpy()
    assert np.isfinite(an).all() and an.min() >= 0 and an.max() <= 1
    want = orc.render(d, 2024, threads=16, crop=(396, 404, 596, 604))
    check(an[396:404, 596:604], want)


@pytest.mark.parametrize("name,seed,kw", [
    ("rtow_final", 42, dict(image_w=120, image_h=80, samples_per_pixel=8)),
    ("cornell", None, dict(image_w=64, image_h=64, samples_per_pixel=8, max_depth=100)),
    ("christmas_tree", None, dict(image_w=96, image_h=54, samples_per_pixel=4)),
])
def test_minmax_slab_equals_reference_selects(crt, monkeypatch, name, seed, kw):
    """walk_step's min/max slab (NaN-free rays) against its EXACT variant (the reference's
    select sequence, forced for every ray by CRT_EXACT_SLAB): bit-identical frames."""
    d = scene(crt, name, seed, **kw)
    fast = gpu(crt, d, 40)
    monkeypatch.setenv("CRT_EXACT_SLAB", "1")
    exact = gpu(crt, d, 40)
    assert np.array_equal(fast, exact)


@pytest.mark.parametrize("name,seed,kw", [
    ("rtow_final", 42, dict(image_w=120, image_h=80, samples_per_pixel=16)),
    ("cornell", None, dict(image_w=64, image_h=64, samples_per_pixel=8, max_depth=100)),
    ("parallelograms", None, dict(image_w=64, image_h=64, samples_per_pixel=8)),
    ("christmas_tree", None, dict(image_w=96, image_h=54, samples_per_pixel=4)),
])
def test_f32_decisions_equal_f64(crt, monkeypatch, name, seed, kw):
    """The f32 node test and the packed-f32 sphere and parallelogram filters only prove outcomes
    of the f64 tests (walk(), sphere_pair_candidates(), quad_candidate()): frames with every node
    test and every primitive decided in f64 (CRT_F64_NODES, CRT_F64_SPHERES, CRT_F64_QUADS, read at
    upload) are bit-identical."""
    d = scene(crt, name, seed, **kw)
    fast = gpu(crt, d, 41)
    monkeypatch.setenv("CRT_F64_NODES", "1")
    monkeypatch.setenv("CRT_F64_SPHERES", "1")
    monkeypatch.setenv("CRT_F64_QUADS", "1")
    slow = gpu(crt, d, 41)
    assert np.array_equal(fast, slow)


@pytest.mark.parametrize("spp", [40, 2000])
def test_work_queue_schedule_does_not_change_frames(crt, monkeypatch, spp):
    """Which wave traces which (chunk, pixel) unit, and when, does not enter the result: the
    chunk length depends on spp only and each unit's sum lands in its own partial slot. Frames
    from persistent grids of 1, 3 and 37 blocks (CRT_GRID_BLOCKS) and the full grid are
    bit-identical, including a half-empty last tile row."""
    d = scene(crt, "rtow_final", 42, image_w=120, image_h=84, samples_per_pixel=spp, max_depth=20)
    base = gpu(crt, d, 43)
    for blocks in (1, 3, 37):
        monkeypatch.setenv("CRT_GRID_BLOCKS", str(blocks))
        assert np.array_equal(base, gpu(crt, d, 43)), blocks
    # eight XCD-local segment queues with stealing (the HBM-scene default) vs one queue
    for blocks in (3, 1000):
        monkeypatch.setenv("CRT_GRID_BLOCKS", str(blocks))
        monkeypatch.setenv("CRT_XCD_QUEUES", "1")
        assert np.array_equal(base, gpu(crt, d, 43)), ("xcd", blocks)


def test_xcd_queues_do_not_change_hbm_frames(crt, monkeypatch):
    """The HBM-scene kernels take work from eight segment queues (one per XCD); one queue gives the
    same frame bit for bit."""
    d = scene(crt, "christmas_tree", image_w=96, image_h=54, samples_per_pixel=8)
    base = gpu(crt, d, 46)
    monkeypatch.setenv("CRT_XCD_QUEUES", "0")
    assert np.array_equal(base, gpu(crt, d, 46))


@pytest.mark.parametrize("name,seed", [("rtow_final", 42), ("cornell", None), ("christmas_tree", None),
                                       ("dance_floor", None)])
def test_closest_hits_many_rays_bit_exact(crt, name, seed):
    """200k random rays (origins spread over and beyond the scene box, random directions, some
    axis-aligned) through crt_closest_hits vs the oracle: every t / point / normal bit-identical.
    Exercises the node test, the sphere coarse reject, the exact sqrt / division shortcuts and
    the parallelogram test far more densely than rendering does."""
    d = crt.SceneData.named(name, seed)
    s = crt.GpuScene(d)
    nodes, _ = s.export_bvh()
    rng = np.random.default_rng(7)
    lo = np.array([nodes[0]["bounds"][0], nodes[0]["bounds"][2], nodes[0]["bounds"][4]])
    hi = np.array([nodes[0]["bounds"][1], nodes[0]["bounds"][3], nodes[0]["bounds"][5]])
    lo, hi = np.maximum(lo, -1e3), np.minimum(hi, 1e3)
    span = hi - lo
    n = 200_000
    o = lo - 0.25 * span + rng.random((n, 3)) * 1.5 * span
    dirs = rng.normal(size=(n, 3))
    dirs[: n // 20, rng.integers(0, 3)] = 0.0          # zero direction components
    rays = np.concatenate([o, dirs], axis=1)
    got = s.closest_hits(rays, 1e-5, float("inf"))
    want = orc.hits(d, rays, 1e-5, float("inf"))
    assert np.array_equal(got["prim"], want["prim"])
    hit = got["prim"] != -1
    assert hit.mean() > 0.05
    for f in ("t", "point", "normal"):
        assert np.array_equal(got[f][hit].view(np.uint64), want[f][hit].view(np.uint64)), f


@pytest.mark.parametrize("spp,mb", [(40, 1), (2000, 1), (2000, 3)])
def test_partial_budget_bands_do_not_change_frames(crt, monkeypatch, spp, mb):
    """A launch renders the owned frame in bands whose partial sums fit a budget
    (CRT_PARTIAL_MB; default 4 GiB). A pixel's sample chunks are summed in the same order in any
    band, so a 1 MB budget (3 to 63 bands here, some a single tile wide) gives the same frame
    bit for bit, under a multi-GPU row tiling too."""
    from cpp_raytracer_amd import Tiling
    import torch
    d = scene(crt, "rtow_final", 42, image_w=120, image_h=84, samples_per_pixel=spp, max_depth=20)
    base = gpu(crt, d, 44)
    monkeypatch.setenv("CRT_PARTIAL_MB", str(mb))
    assert np.array_equal(base, gpu(crt, d, 44))
    s = crt.GpuScene(d)
    s.upload(0)
    cam = crt.resolve_camera(d.camera, 44)
    out = torch.zeros(84, 120, 3, dtype=torch.float64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for t in range(3):
        s.render_async(0, cam, out.data_ptr(), st, Tiling(4, 3, t, 0))
    torch.cuda.synchronize()
    assert np.array_equal(base, out.cpu().numpy())


@pytest.mark.parametrize("w,h,crops", [
    # 75,000 tile rows (> 65535): two row bands; rows around the band edge and the last rows
    (8, 300_000, [(262_130, 262_150, 0, 8), (299_990, 300_000, 0, 8)]),
    # 68,750 tile columns (> 65535): two column bands; columns around the edge and the last ones
    (1_100_000, 2, [(0, 2, 1_048_540, 1_048_580), (0, 2, 1_099_960, 1_100_000)]),
])
def test_tall_and_wide_frames(crt, w, h, crops):
    """Frames with more than 65535 tile rows or columns (a tile is 16 x 4 pixels) render every
    pixel: checked against the oracle on windows across the band edges and at the far end."""
    d = scene(crt, "config1", None, image_w=w, image_h=h, samples_per_pixel=1, max_depth=4)
    out = gpu(crt, d, 45)
    assert np.isfinite(out).all()
    for r0, r1, c0, c1 in crops:
        check(out[r0:r1, c0:c1], orc.render(d, 45, threads=8, crop=(r0, r1, c0, c1)))


def _box_room(crt, seed, n_boxes, **cam):
    """The Cornell room plus random axis-aligned boxes and wall-flush light panels on a coarse
    grid: coincident faces, boxes touching the walls and each other, rays grazing shared planes."""
    from cpp_raytracer_amd import OBJECT_DTYPE
    d = scene(crt, "cornell", **cam)
    rng = np.random.default_rng(seed)
    objs = [o for o in d.objects]
    for _ in range(n_boxes):
        a = rng.integers(0, 15, 3) * 37.0
        b = a + rng.integers(1, 5, 3) * 37.0
        o = np.zeros(1, OBJECT_DTYPE)[0]
        o["kind"], o["material"] = 3, rng.integers(0, len(d.materials))  # CRT_BOX
        o["v"][:6] = np.concatenate([a, np.minimum(b, 555.0)])
        objs.append(o)
    for _ in range(3):  # light panels lying on a wall plane
        o = np.zeros(1, OBJECT_DTYPE)[0]
        o["kind"], o["material"] = 2, int(np.flatnonzero(d.materials["kind"] == 4)[0])  # CRT_PARALLELOGRAM, the light
        ax = rng.integers(0, 3)
        v = rng.integers(1, 12, 3) * 37.0
        v[ax] = 555.0 * rng.integers(0, 2)
        s1, s2 = np.zeros(3), np.zeros(3)
        s1[(ax + 1) % 3], s2[(ax + 2) % 3] = 74.0, -74.0
        o["v"][:] = np.concatenate([v, s1, s2])
        objs.append(o)
    d.objects = np.array(objs, dtype=OBJECT_DTYPE)
    return d


@pytest.mark.parametrize("seed", [1, 2])
def test_flat_box_quad_filter(crt, monkeypatch, seed):
    """Axis-aligned parallelograms take the flat-box filter (the walk's f32 node test on each
    one's box, crt_quad_filter.h): frames equal the oracle's, and are bit-identical to the generic
    f32 filter (CRT_GENERIC_QUADS) and to every parallelogram decided in f64 (CRT_F64_QUADS)."""
    d = _box_room(crt, seed, 12, image_w=72, image_h=72, samples_per_pixel=6, max_depth=60)
    flat = gpu(crt, d, 50 + seed)
    check(flat, orc.render(d, 50 + seed, threads=8))
    monkeypatch.setenv("CRT_GENERIC_QUADS", "1")
    assert np.array_equal(flat, gpu(crt, d, 50 + seed))
    monkeypatch.delenv("CRT_GENERIC_QUADS")
    monkeypatch.setenv("CRT_F64_QUADS", "1")
    assert np.array_equal(flat, gpu(crt, d, 50 + seed))


@pytest.mark.parametrize("name,kw", [
    ("cornell", dict(image_w=48, image_h=48, samples_per_pixel=4, max_depth=100)),
    ("rtow_final_lights", dict(image_w=80, image_h=45, samples_per_pixel=4)),
    ("parallelograms", dict(image_w=48, image_h=48, samples_per_pixel=4)),
])
@pytest.mark.parametrize("gstack", [False, True])
def test_hbm_scene_kernels_with_parallelograms(crt, monkeypatch, name, kw, gstack):
    """The HBM-scene kernels (scene in HBM: CRT_NO_LDS_SCENE; stack in LDS or, CRT_FORCE_GSTACK,
    in HBM) on scenes with parallelograms, which launch the instances with the parallelogram
    paths (QF): frames equal the oracle's."""
    monkeypatch.setenv("CRT_NO_LDS_SCENE", "1")
    if gstack:
        monkeypatch.setenv("CRT_FORCE_GSTACK", "1")
    d = scene(crt, name, **kw)
    check(gpu(crt, d, 60), orc.render(d, 60, threads=8))


@pytest.mark.parametrize("name,seed,kw", [
    ("rtow_final", 42, dict(image_w=96, image_h=64, samples_per_pixel=8, max_depth=50)),
    ("cornell", None, dict(image_w=64, image_h=64, samples_per_pixel=8, max_depth=200)),
])
def test_five_wave_instance_equals_four_wave(crt, monkeypatch, name, seed, kw):
    """Small sphere-only and flat-parallelogram LDS scenes run the 5-wave instances (96 VGPRs,
    spills, no f64 spheres in LDS); the 4-wave instances (CRT_FOUR_WAVES) give the same frame bit
    for bit, and both the oracle's."""
    d = scene(crt, name, seed, **kw)
    five = gpu(crt, d, 70)
    check(five, orc.render(d, 70, threads=8))
    monkeypatch.setenv("CRT_FOUR_WAVES", "1")
    assert np.array_equal(five, gpu(crt, d, 70))


@pytest.mark.parametrize("name,seed,kw", [
    ("christmas_tree", None, dict(image_w=96, image_h=54, samples_per_pixel=6)),
    ("rtow_final", 42, dict(image_w=96, image_h=64, samples_per_pixel=4, max_depth=50)),
    ("cornell", None, dict(image_w=64, image_h=64, samples_per_pixel=4, max_depth=200)),
    ("millions", 42, dict(image_w=64, image_h=36, samples_per_pixel=4, max_depth=20)),
])
def test_pair_walk_equals_node_walk(crt, monkeypatch, name, seed, kw):
    """The HBM-scene kernels' sibling-pair walk (walk_pairs, round 6) against the one-node walk it
    replaced (CRT_NO_PAIR_WALK=1): the same primitive tests in the same order with the same t_max,
    so bit-identical frames, on scenes forced into HBM (CRT_NO_LDS_SCENE) and on millions (4202 to
    2.1 M primitives, sphere-only and parallelogram instances), and the GPU frame equals the oracle's."""
    monkeypatch.setenv("CRT_NO_LDS_SCENE", "1")
    d = scene(crt, name, seed, **kw)
    s = crt.GpuScene(d, build_device=0 if name == "millions" else None)
    cam = crt.resolve_camera(d.camera, 41)
    pair, _ = s.render(cam, 1)
    pair_f64 = f64_node_tests(s, cam, monkeypatch)
    monkeypatch.setenv("CRT_NO_PAIR_WALK", "1")
    node, _ = s.render(cam, 1)
    node_f64 = f64_node_tests(s, cam, monkeypatch)
    assert pair.tobytes() == node.tobytes()
    assert s.guard(0) == 0
    # the pair walk leaves no more node tests to f64 than the one-node walk (a threshold shared by
    # a pair's two nodes once left 16x as many, round 6)
    assert pair_f64 <= 1.1 * node_f64 + 64, (pair_f64, node_f64)
    if name != "millions":  # the oracle's millions build alone takes ~10 s
        check(pair, orc.render(d, 41, threads=8))


@pytest.mark.parametrize("name,seed,kw,limit", [
    ("rtow_final", 42, dict(image_w=120, image_h=80, samples_per_pixel=8, max_depth=50), 1e-3),
    ("millions", 42, dict(image_w=96, image_h=54, samples_per_pixel=4, max_depth=50), 1e-2),
])
def test_f32_walk_decides_almost_every_node(crt, monkeypatch, name, seed, kw, limit):
    """The f32 node test leaves few decisions to f64 (config 2: 8.6e-5 of node tests, config 4
    with the pair walk 1.9e-3). A change that keeps frames bit-identical but makes many gaps
    undecidable (round 6's med3 form of the slab clamp: 0.5% on config 2, 6-8% slower) fails here."""
    d = scene(crt, name, seed, **kw)
    s = crt.GpuScene(d, build_device=0 if name == "millions" else None)
    cam = crt.resolve_camera(d.camera, 44)
    s.upload(0)
    monkeypatch.setenv("CRT_COUNT_SPEC", "1")
    st = s.render_count(0, cam)
    assert st.nodes_visited > 0
    assert st.slow_node_tests <= limit * st.nodes_visited, (st.slow_node_tests, st.nodes_visited)


def f64_node_tests(s, cam, monkeypatch):
    """Node tests the instrumented pass decided in f64, walking like the timed kernel."""
    s.upload(0)
    with monkeypatch.context() as m:
        m.setenv("CRT_COUNT_SPEC", "1")
        return s.render_count(0, cam).slow_node_tests


@pytest.mark.parametrize("name,seed,view", [
    ("rtow_final", 42, dict(center=(0.0, 1.0, 14.0), lookat=(0.0, 1.0, 0.0))),
    ("christmas_tree", None, dict(center=(0.0, 10.0, 50.0), direction=(0.0, 0.0, -1.0))),
])
def test_pair_walk_axis_aligned_camera(crt, monkeypatch, name, seed, view):
    """Primary rays almost parallel to the z axis (camera on the axis, no defocus): their slab
    values on x and y are huge for boxes the ray misses there, which is what a threshold shared
    by both nodes of a pair step turned into undecidable f32 tests (round 6). The pair walk with
    per-node thresholds still gives the one-node walk's frame bit for bit, and the oracle's."""
    monkeypatch.setenv("CRT_NO_LDS_SCENE", "1")
    d = scene(crt, name, seed, image_w=64, image_h=48, samples_per_pixel=4, max_depth=20, defocus_angle=0.0,
              **view)
    s = crt.GpuScene(d)
    cam = crt.resolve_camera(d.camera, 43)
    pair, _ = s.render(cam, 1)
    pair_f64 = f64_node_tests(s, cam, monkeypatch)
    monkeypatch.setenv("CRT_NO_PAIR_WALK", "1")
    node, _ = s.render(cam, 1)
    node_f64 = f64_node_tests(s, cam, monkeypatch)
    assert pair.tobytes() == node.tobytes()
    assert pair_f64 <= 1.1 * node_f64 + 64, (pair_f64, node_f64)
    check(pair, orc.render(d, 43, threads=8))
