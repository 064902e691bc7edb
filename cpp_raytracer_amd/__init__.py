"""MI355X-native render path for DeltaPavonis/cpp_raytracer.

The hot path (Camera::render -> BVH traversal -> primitive hits -> material scatter) runs as a
gfx950 HIP kernel in lib/libcrt_hip.so behind the C ABI of include/crt_render.h. This module is
the Python host side of that ABI: scene description I/O, the reference's named scenes, camera
resolution, scene upload and render launches. It never computes a pixel itself.
"""
from __future__ import annotations

import ctypes as C
import struct
from dataclasses import dataclass
from pathlib import Path
from typing import Optional

import numpy as np

from . import _capi
from ._capi import (CRT_BOX, CRT_DIELECTRIC, CRT_DIFFUSE_LIGHT, CRT_LAMBERTIAN, CRT_METAL,
                    CRT_PARALLELOGRAM, CRT_SPHERE, HIT_DTYPE, MATERIAL_DTYPE, NODE_DTYPE,
                    OBJECT_DTYPE, BVHParams, Camera, CameraSettings, CrtError, RenderStats,
                    SceneInfo, Tiling, check, lib)

__all__ = [
    "SceneData", "GpuScene", "CameraSettings", "Camera", "Tiling", "RenderStats", "CrtError",
    "resolve_camera", "sample_seed", "rand_double", "device_count", "lib", "ppm_values", "write_ppm",
    "CRT_LAMBERTIAN", "CRT_METAL", "CRT_DIELECTRIC", "CRT_DIFFUSE_LIGHT",
    "CRT_SPHERE", "CRT_PARALLELOGRAM", "CRT_BOX",
]

SCENE_MAGIC = b"CRTS"
SCENE_VERSION = 1


def sample_seed(base: int, pixel: int, sample: int) -> int:
    return int(lib().crt_sample_seed(base & 0xFFFFFFFF, pixel & 0xFFFFFFFF, sample & 0xFFFFFFFF))


def rand_double(state: int, lo: float = 0.0, hi: float = 1.0) -> tuple[int, float]:
    """One draw of the reference LCG (rand_util.h:85-117); returns (new_state, value)."""
    s = C.c_uint32(state & 0xFFFFFFFF)
    v = lib().crt_rand_double(C.byref(s), lo, hi)
    return s.value, v


def device_count() -> int:
    n = C.c_int(0)
    rc = lib().crt_device_count(C.byref(n))
    return n.value if rc == 0 else 0


def ppm_values(device: int, frame_ptr: int, height: int, width: int, stream: int = 0) -> np.ndarray:
    """Image::send_as_ppm's integers (h, w, 3 int32) for a device frame of h*w RGB f64 pixels
    (crt_ppm_values: computed on the GPU)."""
    out = np.zeros((height, width, 3), np.int32)
    check(lib().crt_ppm_values(device, C.c_void_p(frame_ptr), height * width, out.ctypes.data,
                               C.c_void_p(stream)), "crt_ppm_values")
    return out


def write_ppm(path, values: np.ndarray) -> None:
    """Writes (h, w, 3) integers as Image::send_as_ppm does (crt_ppm_write)."""
    v = np.ascontiguousarray(values, np.int32)
    h, w, _ = v.shape
    check(lib().crt_ppm_write(str(path).encode(), w, h, v.ctypes.data), "crt_ppm_write")


def _settings_bytes(cs: CameraSettings) -> bytes:
    return C.string_at(C.addressof(cs), C.sizeof(cs))


@dataclass
class SceneData:
    """Host description of a world: materials + objects (+ the scene's camera settings)."""
    materials: np.ndarray
    objects: np.ndarray
    camera: CameraSettings

    @classmethod
    def named(cls, name: str, seed: Optional[int] = None) -> "SceneData":
        """A scene of the reference's src/main.cpp, built with the reference's RNG semantics."""
        mp = C.POINTER(_capi.Material)()
        op = C.POINTER(_capi.Object)()
        nm, no = C.c_size_t(0), C.c_size_t(0)
        cs = CameraSettings()
        rc = lib().crt_scene_build_named(name.encode(), (seed or 0) & 0xFFFFFFFF, int(seed is not None),
                                         C.byref(mp), C.byref(nm), C.byref(op), C.byref(no),
                                         C.byref(cs))
        check(rc, f"crt_scene_build_named({name!r})")
        try:
            mats = np.frombuffer(C.string_at(mp, nm.value * MATERIAL_DTYPE.itemsize),
                                 dtype=MATERIAL_DTYPE).copy()
            objs = np.frombuffer(C.string_at(op, no.value * OBJECT_DTYPE.itemsize),
                                 dtype=OBJECT_DTYPE).copy()
        finally:
            lib().crt_free(C.cast(mp, C.c_void_p))
            lib().crt_free(C.cast(op, C.c_void_p))
        return cls(mats, objs, cs)

    # --- the CRTS serialization format (header, camera settings, materials, objects) ---
    def to_bytes(self) -> bytes:
        head = SCENE_MAGIC + struct.pack("<IQQ", SCENE_VERSION, len(self.materials), len(self.objects))
        return (head + _settings_bytes(self.camera) + self.materials.astype(MATERIAL_DTYPE).tobytes()
                + self.objects.astype(OBJECT_DTYPE).tobytes())

    def save(self, path) -> None:
        Path(path).write_bytes(self.to_bytes())

    @classmethod
    def from_bytes(cls, b: bytes) -> "SceneData":
        if b[:4] != SCENE_MAGIC:
            raise CrtError("not a CRTS scene file")
        ver, nm, no = struct.unpack_from("<IQQ", b, 4)
        if ver != SCENE_VERSION:
            raise CrtError(f"CRTS version {ver} unsupported")
        off = 4 + struct.calcsize("<IQQ")
        cs = CameraSettings.from_buffer_copy(b[off:off + C.sizeof(CameraSettings)])
        off += C.sizeof(CameraSettings)
        mats = np.frombuffer(b, MATERIAL_DTYPE, nm, off).copy()
        off += nm * MATERIAL_DTYPE.itemsize
        objs = np.frombuffer(b, OBJECT_DTYPE, no, off).copy()
        return cls(mats, objs, cs)

    @classmethod
    def load(cls, path) -> "SceneData":
        return cls.from_bytes(Path(path).read_bytes())


def resolve_camera(settings: CameraSettings, base_seed: int = 0) -> Camera:
    """Camera::init (camera.h:87-157) -> the per-sample loop's constants."""
    cam = Camera()
    check(lib().crt_camera_resolve(C.byref(settings), C.byref(cam)), "crt_camera_resolve")
    cam.base_seed = base_seed & 0xFFFFFFFF
    return cam


def camera_with(settings: CameraSettings, **kw) -> CameraSettings:
    """A copy of `settings` with fields replaced (image_w=..., samples_per_pixel=..., ...)."""
    cs = CameraSettings.from_buffer_copy(_settings_bytes(settings))
    for k, v in kw.items():
        setattr(cs, k, v)
    return cs


class GpuScene:
    """A flattened scene + reference-order BVH with per-device HBM copies. The BVH is built on
    the host, or on GPU `build_device` (the same tree, crt_bvh_params.build_device)."""

    def __init__(self, data: SceneData, num_buckets: int = 32, max_prims_in_node: int = 12,
                 linear: bool = False, build_device: Optional[int] = None):
        self.data = data
        self._h = C.c_void_p()
        mats = np.ascontiguousarray(data.materials, dtype=MATERIAL_DTYPE)
        objs = np.ascontiguousarray(data.objects, dtype=OBJECT_DTYPE)
        prm = BVHParams(num_buckets, max_prims_in_node, int(linear),
                        0 if build_device is None else build_device + 1)
        check(lib().crt_scene_create(mats.ctypes.data, len(mats), objs.ctypes.data, len(objs),
                                     C.byref(prm), C.byref(self._h)), "crt_scene_create")

    def close(self) -> None:
        if self._h:
            lib().crt_scene_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def info(self) -> SceneInfo:
        si = SceneInfo()
        check(lib().crt_scene_info_get(self._h, C.byref(si)), "crt_scene_info_get")
        return si

    def export_bvh(self) -> tuple[np.ndarray, np.ndarray]:
        si = self.info()
        nodes = np.zeros(si.num_nodes, NODE_DTYPE)
        order = np.zeros(si.num_primitives, np.uint32)
        check(lib().crt_scene_export_bvh(self._h, nodes.ctypes.data, order.ctypes.data),
              "crt_scene_export_bvh")
        return nodes, order

    def upload(self, device: int = 0) -> None:
        check(lib().crt_scene_upload(self._h, device), f"crt_scene_upload(device={device})")

    def device_image(self, device: int = 0) -> np.ndarray:
        """The bytes of the scene's copy in HBM of `device` (crt_scene_image)."""
        out = np.zeros(self.info().device_bytes, np.uint8)
        check(lib().crt_scene_image(self._h, device, out.ctypes.data, out.nbytes),
              f"crt_scene_image(device={device})")
        return out

    def render_async(self, device: int, cam: Camera, out_ptr: int, stream: int = 0,
                     tiling: Optional[Tiling] = None) -> None:
        """Enqueue a render of the owned rows into the device buffer at out_ptr."""
        t = C.byref(tiling) if tiling is not None else None
        check(lib().crt_render_async(self._h, device, C.byref(cam), t, C.c_void_p(out_ptr),
                                     C.c_void_p(stream)), "crt_render_async")

    def render_count(self, device: int, cam: Camera, tiling: Optional[Tiling] = None) -> RenderStats:
        st = RenderStats()
        t = C.byref(tiling) if tiling is not None else None
        check(lib().crt_render_count(self._h, device, C.byref(cam), t, C.byref(st)), "crt_render_count")
        return st

    def render(self, cam: Camera, num_devices: int = 1) -> tuple[np.ndarray, RenderStats]:
        """Blocking whole-frame render gathered into host memory: (h, w, 3) float64."""
        out = np.empty((cam.image_h, cam.image_w, 3), np.float64)
        st = RenderStats()
        check(lib().crt_render(self._h, C.byref(cam), num_devices, out.ctypes.data, C.byref(st)),
              "crt_render")
        return out, st

    def render_ppm(self, cam: Camera, num_devices: int = 1) -> tuple[np.ndarray, RenderStats]:
        """Blocking whole-frame render fused with Image::send_as_ppm's integers (crt_render_ppm:
        each device tone-maps its rows to 8-bit values before the gather): (h, w, 3) int32."""
        out = np.empty((cam.image_h, cam.image_w, 3), np.int32)
        st = RenderStats()
        check(lib().crt_render_ppm(self._h, C.byref(cam), num_devices, out.ctypes.data, C.byref(st)),
              "crt_render_ppm")
        return out, st

    def guard(self, device: int = 0, reset: bool = False) -> int:
        """Dielectric decisions since upload (or the last reset) that a one-ulp different
        pow(1 - cos, 5) could have flipped (crt_render_guard; 0 = every branch as the reference's)."""
        v = C.c_uint64()
        check(lib().crt_render_guard(self._h, device, C.byref(v), int(reset)), "crt_render_guard")
        return int(v.value)

    def closest_hits(self, rays: np.ndarray, t_min: float = 1e-5, t_max: float = float("inf"),
                     device: int = 0) -> np.ndarray:
        rays = np.ascontiguousarray(rays, np.float64).reshape(-1, 6)
        out = np.zeros(len(rays), HIT_DTYPE)
        check(lib().crt_closest_hits(self._h, device, rays.ctypes.data, len(rays), t_min, t_max,
                                     out.ctypes.data), "crt_closest_hits")
        return out
