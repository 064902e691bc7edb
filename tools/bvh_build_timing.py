"""Where the millions-of-spheres scene's set-up time goes (BASELINE config 4: 2,106,105 spheres):
scene creation with the GPU BVH build (crt_scene_create with build_device, which sets the scene up
on the device: crt_stage_gpu.hip) and the upload (free on the build device), against the host
staging of the same GPU-built tree (CRT_HOST_STAGE=1: host flattening, host stage() and
stage_image, then the copy to HBM). build_ms = the BVH build alone. CRT_DEBUG_BUILD=1 also
prints the phases. usage: python tools/bvh_build_timing.py [reps]"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import cpp_raytracer_amd as crt  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
d = crt.SceneData.named("millions", 42)
crt.GpuScene(crt.SceneData.named("config1"), build_device=0).upload(0)  # warm up HIP
for route in ("device", "host"):
    for r in range(reps):
        if route == "host":
            os.environ["CRT_HOST_STAGE"] = "1"
        t0 = time.perf_counter()
        g = crt.GpuScene(d, build_device=0)
        t1 = time.perf_counter()
        g.upload(0)
        t2 = time.perf_counter()
        os.environ.pop("CRT_HOST_STAGE", None)
        print(f"rep {r} {route:6s} staging: scene create {(t1 - t0) * 1e3:.1f} ms (build_ms {g.info().build_ms:.1f}), "
              f"upload {(t2 - t1) * 1e3:.1f} ms, total {(t2 - t0) * 1e3:.1f} ms", flush=True)
        g.close()
