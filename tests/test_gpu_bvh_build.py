"""GPU BVH build (crt_bvh_params.build_device) against the host build, which
tests/test_host_abi.py pins to the reference's own BVH goldens: node arrays (bounds bit for bit,
index / count / axis) and the primitive order must be identical, for every named scene, for
non-default bucket / leaf-size parameters, and for random scenes with duplicate and signed-zero
coordinates (ties in the bounds folds and the partition)."""
import sys
import time

import numpy as np
import pytest

from conftest import ROOT, load_npz

SCENES = [("config1", None), ("rtow_final", 42), ("rtow_final_lights", None), ("cornell", None),
          ("cornell_empty", None), ("parallelograms", None), ("dance_floor", None),
          ("christmas_tree", None), ("bvh_pathological", None)]


def same_tree(crt, data, **kw):
    host = crt.GpuScene(data, **kw)
    gpu = crt.GpuScene(data, build_device=0, **kw)
    hn, ho = host.export_bvh()
    gn, go = gpu.export_bvh()
    assert len(hn) == len(gn)
    assert np.array_equal(hn["bounds"].view(np.uint64), gn["bounds"].view(np.uint64))
    for f in ("index", "count", "axis", "flags"):
        assert np.array_equal(hn[f], gn[f]), f
    assert np.array_equal(ho, go)
    hi, gi = host.info(), gpu.info()
    assert (hi.depth, hi.max_leaf_size) == (gi.depth, gi.max_leaf_size)


def tie_scene(seed, n):
    sys.path.insert(0, str(ROOT / "tests" / "golden"))
    from gen_golden import tie_scene as make
    return make(seed, n)


pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,seed", SCENES)
def test_named_scene_gpu_build_equals_host(crt, name, seed):
    same_tree(crt, crt.SceneData.named(name, seed))


@pytest.mark.parametrize("nb,ml", [(2, 12), (8, 4), (64, 1), (32, 32), (16, 200)])
def test_build_parameters(crt, nb, ml):
    same_tree(crt, crt.SceneData.named("rtow_final", 42), num_buckets=nb, max_prims_in_node=ml)


@pytest.mark.parametrize("seed,n", [(1, 1), (2, 2), (3, 7), (6, 40000), (8, 150000)])
def test_random_scenes_with_ties(crt, seed, n):
    same_tree(crt, tie_scene(seed, n))


@pytest.mark.parametrize("seed", [4, 5, 7])
def test_tie_scenes_equal_reference_bvh(crt, seed):
    """GPU build against the reference's own BVH of tie-heavy scenes (tests/golden/bvh_ties.npz)."""
    g = load_npz("bvh_ties.npz")
    k = f"s{seed}_"
    d = crt.SceneData.named("config1")
    d.materials, d.objects = g[k + "materials"], g[k + "objects"]
    nodes, order = crt.GpuScene(d, build_device=0).export_bvh()
    assert np.array_equal(nodes["bounds"].view(np.uint64), g[k + "bounds"].view(np.uint64))
    for f in ("index", "count", "axis"):
        assert np.array_equal(nodes[f], g[k + f])
    assert np.array_equal(order, g[k + "order"])


@pytest.mark.slow
def test_millions_gpu_build(crt):
    d = crt.SceneData.named("millions", 42)
    t0 = time.perf_counter()
    crt.GpuScene(d, build_device=0).close()
    t_gpu = time.perf_counter() - t0
    t0 = time.perf_counter()
    crt.GpuScene(d).close()
    t_host = time.perf_counter() - t0
    print(f"millions BVH build: host {t_host * 1e3:.0f} ms, GPU {t_gpu * 1e3:.0f} ms")
    same_tree(crt, d)
