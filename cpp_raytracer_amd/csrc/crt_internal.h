// Internal layout shared by the host side (crt_host.cpp) and the gfx950 kernels
// (crt_device.hip). Not part of the ABI; include/crt_render.h is.
#pragma once

#include <cstddef>
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/crt_render.h"

namespace crt {

constexpr int kMaxDevices = 16;

// ---- HBM layout (one copy per device) ------------------------------------------------------
// BVH node: the LinearBVHNode of bvh.h:117-161 packed into one 64-byte line (4 x dwordx4 loads).
struct alignas(16) DevNode {
    double b[6];        // x.min x.max y.min y.max z.min z.max
    uint32_t index;     // first primitive slot (leaf) / right child (interior)
    uint32_t count;     // primitives in the leaf, 0 for interior
    uint32_t axis;      // split axis (interior)
    uint32_t flags;     // leaf: kNodeAlways = skip the AABB test (linear leaf); interior: left child
};
// The device copy lists the nodes breadth-first (crt_host.cpp stage()), children explicit.
static_assert(sizeof(DevNode) == 64, "node must be one 64-byte line");
constexpr uint32_t kNodeAlways = 1u;
// The device node array ends with a sentinel node (index = node count): box [-inf, inf]^3, count
// kSentinelCount, both children itself. The render kernel keeps a reference to it in a guard
// level below each lane's stack, so popping an empty stack lands on the sentinel, and the walk
// loop's only exit test is "entered a node with a primitive count" (crt_device.hip walk()).
constexpr uint32_t kSentinelCount = 0xffffffffu;

// Sphere (sphere.h:16-18): centre + radius in one 32-byte record.
struct alignas(16) DevSphere {
    double c[3];
    double r;
};

// Parallelogram (parallelogram.h:138-170) with the ctor's precomputed normals.
struct alignas(16) DevQuad {
    double v[3], s1[3], s2[3], n[3], sn[3];
    double pad;
};
static_assert(sizeof(DevQuad) == 128, "quad record");

// Material (material.h): kind, albedo/colour, fuzz | refractive index | intensity, emit colour.
struct alignas(16) DevMaterial {
    uint32_t kind, pad;
    double color[3];
    double param;
    double emit[3];     // DiffuseLight::emit() = intensity * colour (material.h:261-263), else 0
};

// Primitive reference per BVH slot: high bit = parallelogram, low 31 bits = index into the
// kind's array. Spheres/quads are stored in slot order, so for a sphere-only scene ref == slot.
constexpr uint32_t kRefQuad = 0x80000000u;

struct DeviceCopy {
    bool valid = false;
    void* base = nullptr;
    size_t bytes = 0;
    DevNode* nodes = nullptr;
    uint32_t* refs = nullptr;
    DevSphere* spheres = nullptr;
    uint32_t* sphere_mat = nullptr;
    DevQuad* quads = nullptr;
    uint32_t* quad_mat = nullptr;
    DevMaterial* mats = nullptr;
    // per-device scratch reused across renders (partial sums of sample chunks)
    double* partial = nullptr;
    size_t partial_bytes = 0;
    unsigned long long* counters = nullptr;   // instrumented pass
};

// A flattened primitive (Scene::get_primitive_components order) with the derived data the
// reference ctors compute.
struct Prim {
    uint32_t kind;      // CRT_SPHERE / CRT_PARALLELOGRAM
    uint32_t material;
    double v[15];       // sphere: c[3], r | quad: v, s1, s2, unit n, scaled n
    double box[6];      // get_aabb()
};

}  // namespace crt

struct crt_scene {
    std::vector<crt_material> materials;
    std::vector<crt_object> objects;
    std::vector<crt::Prim> prims;
    std::vector<crt_bvh_node> nodes;
    std::vector<uint32_t> order;           // slot -> primitive index
    // device-layout staging (host)
    std::vector<crt::DevNode> dnodes;
    std::vector<uint32_t> refs;
    std::vector<crt::DevSphere> spheres;
    std::vector<uint32_t> sphere_mat;
    std::vector<crt::DevQuad> quads;
    std::vector<uint32_t> quad_mat;
    std::vector<crt::DevMaterial> dmats;
    uint32_t depth = 0;
    uint32_t max_leaf = 0;
    double build_ms = 0;
    bool linear = false;
    bool exact_slab = false;  // some node box is inverted / NaN on an axis: walk_step EXACT only
    crt::DeviceCopy dev[crt::kMaxDevices];
    std::mutex mu;
};

namespace crt {
// error plumbing (crt_host.cpp)
int fail(int code, const std::string& msg);
void clear_error();

// device side (crt_device.hip)
int device_upload(crt_scene* s, int device);
void device_release(crt_scene* s);
int device_render(const crt_scene* s, int device, const crt_camera* cam, const crt_tiling* t,
                  double* d_rgb, void* stream, crt_render_stats* count_stats);
int device_closest_hits(crt_scene* s, int device, const double* rays, size_t n, double t_min,
                        double t_max, crt_hit* out);
int device_count(int* n);
int device_build_bvh(crt_scene* s, uint32_t num_buckets, uint32_t max_leaf, int device,
                     const std::vector<double>& boxes, const std::vector<double>& cents);
int device_ppm_values(int device, const double* d_rgb, size_t n, int32_t* h_values, void* stream);
// host: RGB::as_string's three integers for one pixel (std::pow, x86 int conversion)
void ppm_pixel_host(const double rgb[3], int32_t out[3]);
int render_multi(crt_scene* s, const crt_camera* cam, int num_devices, double* h_rgb,
                 crt_render_stats* stats);
}  // namespace crt
