import time, os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import cpp_raytracer_amd as crt
d = crt.SceneData.named("millions", 42)
crt.GpuScene(crt.SceneData.named("config1"), build_device=0)  # warm up HIP
t = time.perf_counter(); g = crt.GpuScene(d, build_device=0); t1 = time.perf_counter()
print("gpu build total ms", (t1 - t) * 1e3, "reported", g.info().build_ms)
