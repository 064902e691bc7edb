"""Scene set-up on the device (crt_stage_gpu.hip): a scene created with
crt_bvh_params.build_device is flattened, built and staged in HBM. Its device copy must be
byte-identical to the copy the host path stages and uploads (crt_host.cpp stage(), crt_device.hip
stage_image) from the host build of the same scene — which tests/test_host_abi.py pins to the
reference's BVH goldens — for every named scene, for primitive mixes (spheres, parallelograms,
boxes), tie-heavy scenes, extreme build parameters, scenes outside the f32 filters' ranges, and a
NaN scene (which must take the host path)."""
import numpy as np
import pytest

from test_gpu_bvh_build import SCENES, tie_scene
from test_gpu_fuzz_scenes import random_world

pytestmark = pytest.mark.gpu


def same_image(crt, data, **kw):
    host = crt.GpuScene(data, **kw)
    dev = crt.GpuScene(data, build_device=0, **kw)
    hi, di = host.info(), dev.info()
    for f in ("num_objects", "num_materials", "num_primitives", "num_spheres", "num_parallelograms",
              "num_nodes", "depth", "max_leaf_size", "device_bytes"):
        assert getattr(hi, f) == getattr(di, f), f
    hn, ho = host.export_bvh()
    dn, do = dev.export_bvh()
    assert hn.tobytes() == dn.tobytes()
    assert np.array_equal(ho, do)
    a, b = host.device_image(0), dev.device_image(0)
    if not np.array_equal(a, b):
        bad = np.flatnonzero(a != b)
        pytest.fail(f"device images differ in {len(bad)} bytes, first at {bad[0]} of {len(a)}")
    return host, dev


@pytest.mark.parametrize("name,seed", SCENES)
def test_named_scene_device_image_equals_host(crt, name, seed):
    same_image(crt, crt.SceneData.named(name, seed))


@pytest.mark.parametrize("seed", range(16))
def test_random_worlds(crt, seed):
    _, d = random_world(crt, seed)
    same_image(crt, d)


@pytest.mark.parametrize("seed,n", [(1, 1), (2, 2), (3, 7), (6, 40000)])
def test_tie_scenes(crt, seed, n):
    same_image(crt, tie_scene(seed, n))


@pytest.mark.parametrize("nb,ml", [(2, 12), (64, 1), (16, 200)])
def test_build_parameters(crt, nb, ml):
    same_image(crt, crt.SceneData.named("rtow_final", 42), num_buckets=nb, max_prims_in_node=ml)
    same_image(crt, crt.SceneData.named("cornell"), num_buckets=nb, max_prims_in_node=ml)


def test_boxes_and_spheres_many(crt):
    """Thousands of Boxes among spheres: the per-object primitive offsets and the sphere ranks are
    scans on the device."""
    from cpp_raytracer_amd import OBJECT_DTYPE
    rng = np.random.default_rng(11)
    d = crt.SceneData.named("rtow_final", 42)
    n = 5000
    boxes = np.zeros(n, OBJECT_DTYPE)
    boxes["kind"] = 3
    boxes["material"] = rng.integers(0, len(d.materials), n)
    a = rng.uniform(-20, 20, (n, 3))
    boxes["v"][:, :3] = a
    boxes["v"][:, 3:6] = a + rng.uniform(-1, 1, (n, 3))
    objs = np.concatenate([d.objects, boxes])
    d.objects = objs[rng.permutation(len(objs))]
    same_image(crt, d)


def test_out_of_f32_range(crt):
    """Coordinates beyond the f32 walk / filter ranges: the flags come out the same (f64 paths)."""
    d = crt.SceneData.named("rtow_final", 42)
    d.objects["v"][:5] *= 1e13
    same_image(crt, d)
    d = crt.SceneData.named("cornell")
    d.objects["v"][0] *= 1e13
    same_image(crt, d)


@pytest.mark.parametrize("value", [np.nan, np.inf])
def test_non_finite_scene_takes_host_path(crt, value):
    """A sphere with a NaN centre folds to the empty box [inf, -inf] (NaN centroid): such scenes
    build and stage on the host, whatever build_device asks."""
    d = crt.SceneData.named("rtow_final", 42)
    d.objects["v"][3, 0] = value
    same_image(crt, d)


def test_errors_match_host(crt):
    d = crt.SceneData.named("rtow_final", 42)
    d.objects["material"][7] = len(d.materials) + 3
    msgs = []
    for kw in ({}, {"build_device": 0}):
        with pytest.raises(crt.CrtError) as e:
            crt.GpuScene(d, **kw)
        msgs.append(str(e.value))
    assert msgs[0] == msgs[1]
    assert "object 7 references material" in msgs[0]


def test_closest_hits_and_render_on_device_staged_scene(crt):
    """The per-slot refs come back from HBM for closest-hit queries; a frame renders identically."""
    d = crt.SceneData.named("christmas_tree")
    host, dev = same_image(crt, d)
    rng = np.random.default_rng(5)
    rays = np.concatenate([rng.uniform(-10, 10, (4096, 3)), rng.normal(size=(4096, 3))], axis=1)
    assert host.closest_hits(rays).tobytes() == dev.closest_hits(rays).tobytes()
    cam = crt.resolve_camera(crt.camera_with(d.camera, image_w=48, image_h=32, samples_per_pixel=4,
                                             max_depth=10), 7)
    assert host.render(cam)[0].tobytes() == dev.render(cam)[0].tobytes()


@pytest.mark.slow
def test_millions_device_image(crt):
    same_image(crt, crt.SceneData.named("millions", 42))


@pytest.mark.slow
def test_millions_with_boxes_and_parallelograms(crt):
    """2.1 M spheres with Boxes and parallelograms mixed in: both device scans span many tiles
    (over a thousand 2048-element tiles, so the tile sums are scanned in several chunks)."""
    from cpp_raytracer_amd import OBJECT_DTYPE
    rng = np.random.default_rng(3)
    d = crt.SceneData.named("millions", 42)
    n = 3000
    extra = np.zeros(2 * n, OBJECT_DTYPE)
    extra["kind"][:n] = 3
    extra["kind"][n:] = 2
    extra["material"] = rng.integers(0, len(d.materials), 2 * n)
    a = rng.uniform(-300, 300, (2 * n, 3))
    extra["v"][:n, :3] = a[:n]
    extra["v"][:n, 3:6] = a[:n] + rng.uniform(0.2, 3, (n, 3))
    extra["v"][n:, :3] = a[n:]
    extra["v"][n:, 3:9] = rng.uniform(-2, 2, (n, 6))
    objs = np.concatenate([d.objects, extra])
    d.objects = objs[rng.permutation(len(objs))]
    same_image(crt, d)


def test_device_set_up_frees_its_temporaries(crt):
    """Creating and destroying a device-staged scene returns the device memory it took: the
    temporaries of the set-up (objects, boxes, tree, scans) are freed at once, the copy at destroy."""
    import torch
    d = crt.SceneData.named("rtow_final", 42)
    objs = np.concatenate([d.objects] * 400)  # 194k spheres: the device route
    objs["v"][:, :3] += np.repeat(np.arange(400), len(d.objects))[:, None] * 30.0
    d.objects = objs
    crt.GpuScene(d, build_device=0).close()  # warm: runtime pools, module load
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    for _ in range(3):
        g = crt.GpuScene(d, build_device=0)
        assert g.info().device_bytes > 0
        g.close()
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info()
    assert free0 - free1 < 64 << 20, (free0, free1)


def test_peer_copy_to_second_device(crt):
    """A device-staged scene reaches GPUs other than its build device by a peer copy of its HBM
    image (device_upload). That copy must equal the host-staged image byte for byte — guard words
    included: they start at zero, not at the source copy's running Schlick count — and a frame
    rendered over two devices must equal the one-device frame. Needs two visible GPUs."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two visible GPUs")
    d = crt.SceneData.named("rtow_final", 42)
    host = crt.GpuScene(d)
    dev = crt.GpuScene(d, build_device=0)
    cam = crt.resolve_camera(crt.camera_with(d.camera, image_w=64, image_h=40, samples_per_pixel=4,
                                             max_depth=10), 7)
    one = dev.render(cam)[0]  # counts into device 0's guard word before device 1 gets its copy
    assert np.array_equal(host.device_image(1), dev.device_image(1))
    two = dev.render(cam, num_devices=2)[0]
    assert one.tobytes() == two.tobytes()
    assert dev.guard(1) == 0
