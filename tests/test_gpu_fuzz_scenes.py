"""Randomized worlds rendered on the GPU against the C oracle (itself pinned to the reference's
code by tests/test_oracle.py): each seed draws a world of one family — spheres only (the
five-wave sphere instance), axis-aligned parallelograms and boxes only (the flat-box instance),
rotated parallelograms only (the generic parallelogram filter), or a mix (the general instance)
— with every material kind (Metal fuzz 0 and > 0, Dielectrics with index above and below 1,
lights), hollow spheres (negative radius), a random camera (field of view, defocus, odd image
sizes, background), depths from 1 to 50 and, for some seeds, the whole world scaled by 1e3 or
1e-2; and renders it again with the scene kept in HBM
(CRT_NO_LDS_SCENE). Bar: the paths are bit-identical, so each channel is within 1e-12 x max(1,
|want|) (the colour's forward vs recursive accumulation moves a few ulps, as in test_gpu_parity.py;
north_star's 1e-4 holds a fortiori), and the Schlick guard (crt_schlick.h) at 0."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, str(ROOT / "oracle"))
import crt_oracle_py as orc  # noqa: E402

pytestmark = pytest.mark.gpu
TOL = 1e-12  # relative to max(1, |want|)
FAMILIES = ("spheres", "flat", "rotated", "mixed")


def random_world(crt, seed):
    from cpp_raytracer_amd import MATERIAL_DTYPE, OBJECT_DTYPE, camera_with
    from cpp_raytracer_amd._capi import D3
    rng = np.random.default_rng(seed)
    family = FAMILIES[seed % len(FAMILIES)]
    # materials: one of each kind, then random extras
    mats = []

    def mat(kind, color, param):
        m = np.zeros(1, MATERIAL_DTYPE)[0]
        m["kind"], m["color"], m["param"] = kind, color, param
        mats.append(m)

    mat(1, rng.uniform(0.05, 0.95, 3), 0.0)                            # Lambertian
    mat(2, rng.uniform(0.3, 1.0, 3), 0.0)                              # Metal, mirror
    mat(2, rng.uniform(0.3, 1.0, 3), rng.uniform(0.05, 1.0))           # Metal, fuzzed (<= 1)
    mat(3, np.zeros(3), rng.choice([1.5, 1.0 / 1.33, 2.4, 1.0]))      # Dielectric
    mat(4, rng.uniform(0.5, 1.0, 3), rng.uniform(1.0, 8.0))            # DiffuseLight
    for _ in range(rng.integers(0, 4)):
        k = int(rng.integers(1, 5))
        mat(k, rng.uniform(0.05, 1.0, 3), {1: 0.0, 2: rng.uniform(0, 1), 3: rng.uniform(1.1, 2.0),
                                           4: rng.uniform(1, 5)}[k])
    nm = len(mats)
    objs = []

    def obj(kind, material, v):
        o = np.zeros(1, OBJECT_DTYPE)[0]
        o["kind"], o["material"] = kind, material
        o["v"][:len(v)] = v
        objs.append(o)

    if family in ("spheres", "mixed"):
        if rng.random() < 0.5:  # the ground
            obj(1, 0, [0.0, -1000.0, 0.0, 1000.0])
        for _ in range(rng.integers(3, 30)):
            r = rng.uniform(0.15, 1.4) * (-1 if rng.random() < 0.12 else 1)  # hollow glass
            obj(1, int(rng.integers(0, nm)), [*rng.uniform(-4, 4, 3), r])
    if family in ("flat", "mixed"):
        for _ in range(rng.integers(4, 11)):  # axis-aligned parallelograms
            ax = rng.permutation(3)
            s1, s2 = np.zeros(3), np.zeros(3)
            s1[ax[0]] = rng.uniform(0.5, 4) * rng.choice([-1, 1])
            s2[ax[1]] = rng.uniform(0.5, 4) * rng.choice([-1, 1])
            obj(2, int(rng.integers(0, nm)), [*rng.uniform(-4, 4, 3), *s1, *s2])
        for _ in range(rng.integers(1, 4)):  # boxes
            a = rng.uniform(-4, 3, 3)
            obj(3, int(rng.integers(0, nm)), [*a, *(a + rng.uniform(0.3, 2.5, 3))])
    if family in ("rotated", "mixed"):
        for _ in range(rng.integers(2, 8)):
            obj(2, int(rng.integers(0, nm)), [*rng.uniform(-4, 4, 3), *rng.uniform(-3, 3, 3), *rng.uniform(-3, 3, 3)])
    dark = rng.random() < 0.25  # a black background, lit by a light sphere overhead
    if dark:
        obj(1, 4, [0.0, 9.0, 0.0, 3.0])
    # the whole world at another scale now and then (f32 filter margins relative to the scene)
    scale = {3: 1e3, 5: 1e-2}.get(seed % 8, 1.0)
    d = crt.SceneData.named("config1")
    d.materials = np.array(mats, dtype=MATERIAL_DTYPE)
    d.objects = np.array(objs, dtype=OBJECT_DTYPE)
    d.objects["v"] *= scale
    w, h = [(40, 30), (33, 17), (16, 48), (64, 36)][seed % 4]
    direction = rng.normal(size=3)
    center = -direction / np.linalg.norm(direction) * rng.uniform(9, 16) * scale
    defocus = 0.0 if rng.random() < 0.5 else rng.uniform(0.2, 2.5)
    d.camera = camera_with(d.camera, image_w=w, image_h=h, samples_per_pixel=int(rng.choice([3, 4, 5, 8])),
                           max_depth=int(rng.choice([1, 5, 20, 50] if family != "flat" else [5, 20, 50])), center=D3(*center),
                           lookat=D3(*(rng.uniform(-1, 1, 3) * scale)), has_lookat=1, up=D3(0.0, 1.0, 0.0),
                           fov=float(rng.uniform(20, 80)), fov_is_vertical=1, defocus_angle=defocus,
                           focus_dist=float(rng.uniform(6, 16) * scale), has_focus_dist=1,
                           background=D3(*(np.zeros(3) if dark else rng.uniform(0, 1, 3))))
    return family, d


def render_gpu(crt, d, base):
    s = crt.GpuScene(d)
    out, _ = s.render(crt.resolve_camera(d.camera, base), 1)
    guard = s.guard(0)
    s.close()
    return out, guard


# CRT_FUZZ_WORLDS widens the sweep for a one-off run (profiles/r04_final/fuzz_*.log)
@pytest.mark.parametrize("seed", range(int(os.environ.get("CRT_FUZZ_WORLDS", "48"))))
def test_random_world_matches_oracle(crt, monkeypatch, seed):
    family, d = random_world(crt, seed)
    base = 9000 + seed
    want = orc.render(d, base, threads=16)
    got, guard = render_gpu(crt, d, base)
    assert guard == 0
    err = np.abs(got - want) / np.maximum(1.0, np.abs(want))
    assert np.isfinite(got).all() and err.max() <= TOL, \
        f"{family}: max rel err {err.max()} at {np.unravel_index(err.argmax(), err.shape)}"
    # the same world from HBM (the HBM-scene kernels: another instance of every phase)
    monkeypatch.setenv("CRT_NO_LDS_SCENE", "1")
    hbm, _ = render_gpu(crt, d, base)
    assert np.array_equal(got, hbm), family
