"""The C++ drop-in API (cpp_raytracer_amd/include, same paths and names as the reference's
include/): the reference's own src/main.cpp compiles UNCHANGED against it, and every scene it
builds reaches the GPU path identical to the library's named-scene builders (which the parity
fixtures use). Needs /root/reference (this container); skipped on the GPU box."""
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

from conftest import ROOT

REF_MAIN = Path("/root/reference/src/main.cpp")
INC = ROOT / "cpp_raytracer_amd" / "include"
LIBDIR = ROOT / "cpp_raytracer_amd" / "lib"

pytestmark = pytest.mark.skipif(not REF_MAIN.exists(), reason="reference sources not present")


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    d = tmp_path_factory.mktemp("cppapi")
    exe = d / "main_scenes"
    obj = d / "main.o"
    subprocess.run(["g++", "-std=c++20", "-O2", "-w", f"-I{INC}", "-Dmain=crt_reference_main", "-c",
                    str(REF_MAIN), "-o", str(obj)], check=True)
    subprocess.run(["g++", "-std=c++20", "-O2", f"-I{INC}", str(ROOT / "tests/cpp/main_scene_driver.cpp"),
                    str(obj), "-o", str(exe), f"-L{LIBDIR}", "-lcrt_hip", f"-Wl,-rpath,{LIBDIR}"], check=True)
    return exe


def test_reference_main_compiles_unchanged(tmp_path):
    exe = tmp_path / "main_amd"
    r = subprocess.run(["g++", "-std=c++20", "-O2", f"-I{INC}", str(REF_MAIN), "-o", str(exe),
                        f"-L{LIBDIR}", "-lcrt_hip", f"-Wl,-rpath,{LIBDIR}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]


def dump(driver, tmp_path, name, seed=None):
    out = tmp_path / f"{name}.crts"
    env = dict(os.environ, CRT_DUMP_SCENE=str(out))
    args = [str(driver), name] + ([str(seed)] if seed is not None else [])
    r = subprocess.run(args, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return out


def same_camera(crt, a, b):
    ca, cb = crt.resolve_camera(a), crt.resolve_camera(b)
    for k in ("origin", "pixel00", "pixel_delta_x", "pixel_delta_y", "defocus_disk_x", "defocus_disk_y",
              "background"):
        assert list(getattr(ca, k)) == list(getattr(cb, k)), k
    assert (ca.image_w, ca.image_h, ca.samples_per_pixel, ca.max_depth) == \
           (cb.image_w, cb.image_h, cb.samples_per_pixel, cb.max_depth)


@pytest.mark.parametrize("name,seed", [("rtow_final", 42), ("rtow_final_lights", None), ("parallelograms", None),
                                       ("cornell", None), ("cornell_empty", None), ("christmas_tree", None)])
def test_main_cpp_scene_equals_library_scene(crt, driver, tmp_path, name, seed):
    got = crt.SceneData.load(dump(driver, tmp_path, name, seed))
    want = crt.SceneData.named(name, seed)
    if name == "cornell":  # main.cpp's Boxes reach the ABI as their six faces
        gn, go = crt.GpuScene(got).export_bvh()
        wn, wo = crt.GpuScene(want).export_bvh()
        assert gn.tobytes() == wn.tobytes() and np.array_equal(go, wo)
        # per-primitive materials: expand the library's boxes the same way
        wmat = np.concatenate([np.repeat(o["material"], 6 if o["kind"] == crt.CRT_BOX else 1)
                               for o in want.objects])
        assert want.materials[wmat].tobytes() == got.materials[got.objects["material"]].tobytes()
    else:
        assert got.objects["v"].tobytes() == want.objects["v"].tobytes()
        assert np.array_equal(got.objects["kind"], want.objects["kind"])
        assert got.materials[got.objects["material"]].tobytes() == \
            want.materials[want.objects["material"]].tobytes()
    same_camera(crt, got.camera, want.camera)


@pytest.mark.slow
def test_main_cpp_millions_scene_equals_library_scene(crt, driver, tmp_path):
    got = crt.SceneData.load(dump(driver, tmp_path, "millions", 42))
    want = crt.SceneData.named("millions", 42)
    assert len(got.objects) == len(want.objects) == 2106105
    assert got.objects["v"].tobytes() == want.objects["v"].tobytes()
    assert got.materials[got.objects["material"]].tobytes() == \
        want.materials[want.objects["material"]].tobytes()
    same_camera(crt, got.camera, want.camera)


def test_api_program_without_gpu_exits_loudly(crt, tmp_path):
    if crt.device_count() > 0:
        pytest.skip("a GPU is visible")
    src = tmp_path / "p.cpp"
    src.write_text('#include "base/camera.h"\n#include "shapes/shapes.h"\n'
                   'int main(){Scene w; w.add(std::make_shared<Sphere>(Point3D(0,0,-1),0.5,'
                   'std::make_shared<Lambertian>(RGB::from_mag(0.5))));'
                   'SeedSeqGenerator::get_instance().set_seed(1);'
                   'Camera().set_image_dimensions(8,8).render(w); return 0;}\n')
    exe = tmp_path / "p"
    subprocess.run(["g++", "-std=c++20", f"-I{INC}", str(src), "-o", str(exe), f"-L{LIBDIR}", "-lcrt_hip",
                    f"-Wl,-rpath,{LIBDIR}"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode != 0 and "Error: Camera::render" in r.stdout
