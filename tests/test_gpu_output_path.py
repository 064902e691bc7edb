"""Output path across devices (SURVEY §8 row f2, §8 row e): packed per-device row buffers
(CRT_TILING_PACKED), the fused tone-map before the gather (crt_render_ppm: every device converts its
rows to 8-bit Image::send_as_ppm values, image.h:38-56 / rgb.h:90-115, so 3 B a pixel cross xGMI
and PCIe), and repeated multi-device renders in one process. Multi-device cases run on logical
devices of GPU 0 (CRT_EMULATE_DEVICES), through the same tiling and gather code."""
import numpy as np
import pytest

from conftest import load_npz

pytestmark = pytest.mark.gpu
INT_MIN = -2**31


def small(crt, w=160, h=97, spp=4):
    from cpp_raytracer_amd import camera_with
    d = crt.SceneData.named("rtow_final", 42)
    d.camera = camera_with(d.camera, image_w=w, image_h=h, samples_per_pixel=spp, max_depth=50)
    return d


def test_packed_tiling_equals_owned_rows(crt):
    """crt_render_async with CRT_TILING_PACKED writes the owned rows in order and nothing else."""
    import torch
    from cpp_raytracer_amd import Tiling
    from cpp_raytracer_amd.tiles import owned_rows
    d = small(crt)
    s = crt.GpuScene(d)
    s.upload(0)
    cam = crt.resolve_camera(d.camera, 77)
    full, _ = s.render(cam, 1)
    st = torch.cuda.current_stream().cuda_stream
    for n, rank in [(3, 0), (3, 2), (8, 5)]:
        rows = owned_rows(97, 4, n, rank)
        buf = torch.full((len(rows) + 1, 160, 3), 7.0, dtype=torch.float64, device="cuda")
        s.render_async(0, cam, buf.data_ptr(), st, Tiling(4, n, rank, 1))
        torch.cuda.synchronize()
        got = buf.cpu().numpy()
        assert np.array_equal(got[: len(rows)], full[rows])
        assert np.all(got[len(rows):] == 7.0)  # nothing past the owned rows


def test_unknown_tiling_flags_rejected(crt):
    import torch
    from cpp_raytracer_amd import Tiling
    d = small(crt, 16, 8, 1)
    s = crt.GpuScene(d)
    s.upload(0)
    buf = torch.zeros(8, 16, 3, dtype=torch.float64, device="cuda")
    with pytest.raises(crt.CrtError):
        s.render_async(0, crt.resolve_camera(d.camera, 1), buf.data_ptr(), 0, Tiling(4, 2, 0, 6))


@pytest.mark.parametrize("devices", [1, 3, 8])
def test_render_ppm_matches_reference_config1(crt, monkeypatch, devices):
    """crt_render_ppm of BASELINE config 1 at base seed 7: every integer equals the reference's
    Image::send_as_ppm output (tests/golden/ppm_cases.npz, from oracle/_ref)."""
    want = load_npz("ppm_cases.npz")["config1_values"]
    d = crt.SceneData.named("config1")
    if devices > 1:
        monkeypatch.setenv("CRT_EMULATE_DEVICES", str(devices))
    s = crt.GpuScene(d)
    got, _ = s.render_ppm(crt.resolve_camera(d.camera, 7), devices)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("devices,height", [(2, 97), (5, 3), (8, 90)])
def test_render_ppm_equals_ppm_of_frame(crt, monkeypatch, devices, height):
    """The fused path gives the integers crt_ppm_values gives for crt_render's f64 frame."""
    import torch
    d = small(crt, h=height)
    s = crt.GpuScene(d)
    cam = crt.resolve_camera(d.camera, 77)
    frame, _ = s.render(cam, 1)
    t = torch.from_numpy(frame).cuda()
    torch.cuda.synchronize()
    want = crt.ppm_values(0, t.data_ptr(), height, 160, torch.cuda.current_stream().cuda_stream)
    monkeypatch.setenv("CRT_EMULATE_DEVICES", str(devices))
    got, _ = s.render_ppm(cam, devices)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("w,h,devices", [(40, 10, 3), (300, 300, 1)])
def test_render_ppm_host_redo_path(crt, monkeypatch, w, h, devices):
    """0 spp makes every pixel NaN (the reference's 0 * inf), which no 8-bit value holds: the kernel
    lists the pixels for the host (40 x 10 over 3 devices), or, past the list's 65,536 entries
    (300 x 300), the host redoes the whole device share; both print INT_MIN like send_as_ppm."""
    d = small(crt, w, h, 0)
    if devices > 1:
        monkeypatch.setenv("CRT_EMULATE_DEVICES", str(devices))
    s = crt.GpuScene(d)
    got, _ = s.render_ppm(crt.resolve_camera(d.camera, 5), devices)
    assert got.shape == (h, w, 3) and np.all(got == INT_MIN)


def test_render_multi_twice_in_one_process(crt, monkeypatch):
    """Repeat calls of the multi-device render in one process (peer access is enabled once per
    device pair; a repeat must not leave an error behind for the next launch check)."""
    d = small(crt, h=41)
    s = crt.GpuScene(d)
    cam = crt.resolve_camera(d.camera, 9)
    one, _ = s.render(cam, 1)
    monkeypatch.setenv("CRT_EMULATE_DEVICES", "4")
    for _ in range(3):
        again, _ = s.render(cam, 4)
        assert np.array_equal(again, one)
        p, _ = s.render_ppm(cam, 4)
        assert p.shape == (41, 160, 3)
