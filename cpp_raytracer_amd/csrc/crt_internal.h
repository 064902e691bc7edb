// Internal layout shared by the host side (crt_host.cpp) and the gfx950 kernels
// (crt_device.hip). Not part of the ABI; include/crt_render.h is.
#pragma once

#include <cstddef>
#include <algorithm>
#include <cstdint>
#include <memory>
#include <mutex>
#include <type_traits>
#include <utility>
#include <string>
#include <thread>
#include <vector>

#include "../../include/crt_render.h"
#include "crt_quad_filter.h"

namespace crt {

constexpr int kMaxDevices = 16;

// Allocator whose resize() leaves trivially constructible elements uninitialized: the host staging
// arrays of multi-million-primitive scenes are written in full right after they are sized, and
// zero-filling them first cost a serial pass over hundreds of MB.
// Blocks of 32 MB and more are 2 MB aligned and advised as transparent huge pages: first-touch
// page faults of 4 KB pages (90k for the millions scene's primitive array alone) dominated its
// preparation.
void* big_alloc(size_t bytes);
void big_free(void* p, size_t bytes) noexcept;
template <typename T>
struct NoInitAlloc : std::allocator<T> {
    using value_type = T;
    template <typename U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <typename U>
    NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
    T* allocate(size_t n) { return static_cast<T*>(big_alloc(n * sizeof(T))); }
    void deallocate(T* p, size_t n) noexcept { big_free(p, n * sizeof(T)); }
    template <typename U>
    void construct(U* p) noexcept(std::is_nothrow_default_constructible_v<U>) {
        ::new (static_cast<void*>(p)) U;
    }
    template <typename U, typename... Args>
    void construct(U* p, Args&&... args) {
        ::new (static_cast<void*>(p)) U(std::forward<Args>(args)...);
    }
};
template <typename T>
using BigVec = std::vector<T, NoInitAlloc<T>>;

// f(begin, end) over [0, n) in contiguous chunks on up to 16 threads (scene preparation of
// multi-million-primitive scenes; every element is written by exactly one thread).
template <typename F>
inline void parallel_for(size_t n, size_t min_chunk, F&& f) {
    const size_t hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t nt = std::min<size_t>(std::min<size_t>(hw, 16), (n + min_chunk - 1) / min_chunk);
    if (nt <= 1) {
        f(size_t(0), n);
        return;
    }
    const size_t per = (n + nt - 1) / nt;
    std::vector<std::thread> th;
    for (size_t t = 0; t < nt; ++t) {
        const size_t a = t * per, b = std::min(n, a + per);
        if (a < b) th.emplace_back([&f, a, b] { f(a, b); });
    }
    for (auto& x : th) x.join();
}

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

// The render kernel's walk reads a compact single-precision copy of the same node array
// (32 bytes, two 16-byte loads) and decides most node tests in f32 with a proven error margin,
// falling back to the f64 node above only where the margin cannot decide (crt_device.hip walk()).
// Node references are byte offsets into this array (index * 32), in LDS and in HBM alike; an
// interior node's right child carries the split axis in its (always zero) low five bits.
//   interior: w0 = right_ref | axis, w1 = left_ref (< 2^31)
//   leaf:     w0 = first primitive slot, w1 = 0x80000000 | count
//   sentinel: w0 = its own ref | 3, w1 = 0xffffffff
// Bounds are the f64 bounds rounded to nearest; the f32 decisions need every finite bound within
// [-2^40, 2^40] (infinite bounds are exact), else the kernel decides every node in f64.
struct alignas(16) DevNodeF {
    float b[6];         // x.min x.max y.min y.max z.min z.max
    uint32_t w0, w1;
};
static_assert(sizeof(DevNodeF) == 32, "f32 node is 32 bytes");
constexpr uint32_t kNodeFShift = 5;            // ref = index << 5
constexpr uint32_t kLeafFlagF = 0x80000000u;   // w1 of a leaf / the sentinel
constexpr uint32_t kSentinelW1 = 0xffffffffu;
constexpr double kF32BoundMax = 0x1p40;

// Sphere (sphere.h:16-18): centre + radius in one 32-byte record.
struct alignas(16) DevSphere {
    double c[3];
    double r;
};

// The sphere candidate filter of the render kernel's two-pass leaves (crt_device.hip
// sphere_pair_candidates) reads spheres two at a time in packed f32: record i holds slots i and
// i + 1 (the last record's second half is zero). r2e = RN32(r^2 (1 + 2^-14) + 2^22 |c - c32|^2)
// folds the rounding of the centre into the radius. Needs |c_k|, |r| <= 2^30 for every sphere.
struct alignas(16) DevSpherePair {
    float cx[2], cy[2], cz[2], r2e[2];
};
static_assert(sizeof(DevSpherePair) == 32, "sphere pair record");
constexpr double kF32SphereMax = 0x1p30;

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
// The render kernel's per-slot copies (device_upload) also carry shading constants: emit[0] of a
// non-emitting sphere slot = 1 / r, a Dielectric's colour = (1. / ri, r0 front, r0 back).

// Primitive reference per BVH slot: high bit = parallelogram, low 31 bits = index into the
// kind's array. Spheres/quads are stored in slot order, so for a sphere-only scene ref == slot.
constexpr uint32_t kRefQuad = 0x80000000u;

// ---- the records of the device image, one definition for the host staging (crt_host.cpp
// stage(), crt_device.hip stage_image) and the device scene set-up (crt_stage_gpu.hip) -------

// A material as the render kernel reads it: DiffuseLight::emit() = intensity * colour
// (material.h:261-263) precomputed, each channel * intensity.
CRT_HD DevMaterial material_record(const crt_material& m) {
    DevMaterial d{};
    d.kind = m.kind;
    d.color[0] = m.color[0];
    d.color[1] = m.color[1];
    d.color[2] = m.color[2];
    d.param = m.param;
    if (m.kind == CRT_DIFFUSE_LIGHT)
        for (int k = 0; k < 3; ++k) d.emit[k] = m.color[k] * m.param;
    return d;
}

// Shading constants of a per-slot material record, with the reference's own operations (IEEE
// f64, no contraction), so shade reads the values its divisions would give:
//   emit[0] of a non-emitting sphere slot = 1 / r (the normal's (p - c) / r, vec3d.h:34);
//   a Dielectric's colour (unused: attenuation 1) = the front-face ratio 1. / ri
//   (material.h:191) and reflectance's r0 (material.h:178-179) for the front and back ratio.
CRT_HD void shading_consts(DevMaterial& m, const DevSphere* sp) {
    if (m.kind == CRT_DIELECTRIC) {
        double r = (1 - 1. / m.param) / (1 + 1. / m.param);
        const double front = r * r;
        r = (1 - m.param / 1.) / (1 + m.param / 1.);
        m.color[0] = 1. / m.param;
        m.color[1] = front;
        m.color[2] = r * r;
    }
    if (sp && m.kind != CRT_DIFFUSE_LIGHT) m.emit[0] = 1 / sp->r;
}

// Half of a sphere pair record (DevSpherePair) from one sphere; true when the sphere is outside
// the f32 filter's range.
CRT_HD bool sphere_pair_half(const DevSphere& sp, float& cx, float& cy, float& cz, float& r2e) {
    double dc2 = 0;
    bool bad = false;
    for (int k = 0; k < 3; ++k) {
        if (!(std::fabs(sp.c[k]) <= kF32SphereMax)) bad = true;
        const double e = sp.c[k] - static_cast<double>(static_cast<float>(sp.c[k]));
        dc2 += e * e;
    }
    if (!(std::fabs(sp.r) <= kF32SphereMax)) bad = true;
    cx = static_cast<float>(sp.c[0]);
    cy = static_cast<float>(sp.c[1]);
    cz = static_cast<float>(sp.c[2]);
    r2e = static_cast<float>(sp.r * sp.r * (1 + 0x1p-14) + dc2 * 0x1p22);
    return bad;
}

// The f32 walk record of device node i (DevNodeF); true when a finite bound is beyond the f32
// walk's range.
CRT_HD bool node_record(const DevNode& n, uint32_t i, DevNodeF& f) {
    bool bad = false;
    for (int k = 0; k < 6; ++k) {
        f.b[k] = static_cast<float>(n.b[k]);  // round to nearest
        if (!std::isinf(n.b[k]) && !(std::fabs(n.b[k]) <= kF32BoundMax)) bad = true;
    }
    if (n.count == 0 && n.index == n.flags + 1 && !(n.flags & 1u)) {
        // interior: children side by side, the left one at an even index (stage()); the walk
        // takes the right child as left | 32
        f.w0 = n.axis;
        f.w1 = n.flags << kNodeFShift;
    } else if (n.count == 0) {
        // the root of an empty tree (empty box, no children): an empty leaf
        f.w0 = 0;
        f.w1 = kLeafFlagF;
    } else if (n.count == kSentinelCount) {
        // "axis" 3: R.neg bit 3 (kZeroDir) is clear in the f32 walk, so the far child the
        // walk stores at the sentinel (into the guard level) is w0 & ~31, the sentinel itself
        f.w0 = (i << kNodeFShift) | 3u;
        f.w1 = kSentinelW1;
    } else {
        f.w0 = n.index;
        f.w1 = kLeafFlagF | n.count;
    }
    return bad;
}

// Parallelogram-only scenes of axis-aligned parallelograms (slot = parallelogram): the leaf's
// flat boxes grouped by the axis their box is flat on (x, then y, then z; slot order inside a
// group), each record keeping its slot's offset in the leaf (pad[0]) and the leaf's first record
// the group sizes (pad[1] = nx | ny << 8), so the filter runs one loop per axis with the flat
// axis' two slab values folded into one (leaf_step, flat_axis_candidate). The records' order only
// changes which iteration computes a candidate bit, not the bit. A record flat on no axis cannot
// occur (quad_flat_box accepted every parallelogram, so each box is flat on one axis); should one
// appear, this returns true and the scene leaves the flat-box filter rather than have
// flat_axis_candidate read a wrong axis. k = the node's device index.
CRT_HD bool regroup_leaf(const DevNode& nd, size_t k, DevQuadBox* quadbox) {
    if (nd.count == 0 || nd.count > 32 || nd.count == kSentinelCount) return false;
    // the pad (node 1, crt_host.cpp stage()): an empty-box leaf over slot 0 that no node refers
    // to; regrouping it too would race with the real leaf of slot 0
    if (k == 1 && !(nd.b[0] <= nd.b[1])) return false;
    DevQuadBox tmp[32];
    uint32_t n = 0, groups[3] = {0, 0, 0};
    bool bad = false;
    for (uint32_t axis = 0; axis < 3; ++axis)
        for (uint32_t j = 0; j < nd.count; ++j) {
            const DevQuadBox& r = quadbox[nd.index + j];
            uint32_t flat = 3;
            for (uint32_t q = 0; q < 3 && flat == 3; ++q)
                if (r.b[2 * q] == r.b[2 * q + 1]) flat = q;
            if (flat == 3) bad = true;
            if (flat == axis) {
                tmp[n] = r;
                tmp[n].pad[0] = j;
                ++n;
                ++groups[axis];
            }
        }
    if (n != nd.count) return bad;
    tmp[0].pad[1] = groups[0] | groups[1] << 8;
    for (uint32_t j = 0; j < n; ++j) quadbox[nd.index + j] = tmp[j];
    return bad;
}

struct DeviceCopy {
    bool valid = false;
    void* base = nullptr;
    size_t bytes = 0;
    DevNode* nodes = nullptr;
    DevNodeF* fnodes = nullptr;   // f32 walk copy (refs = byte offsets)
    bool f32_ok = false;          // every finite node bound within +-kF32BoundMax
    uint32_t* refs = nullptr;
    DevSphere* spheres = nullptr;
    DevSpherePair* spair = nullptr;  // f32 filter records (slot i, i + 1)
    bool spheres_f32_ok = false;     // every sphere within +-kF32SphereMax
    uint32_t* sphere_mat = nullptr;
    DevQuad* quads = nullptr;
    DevQuadF* quadf = nullptr;       // f32 filter records (crt_quad_filter.h)
    bool quads_f32_ok = false;       // every parallelogram within the filter's range
    DevQuadBox* quadbox = nullptr;   // flat boxes of axis-aligned parallelograms (crt_quad_filter.h)
    bool quads_flat_ok = false;      // every parallelogram axis-aligned: the flat-box filter applies
    uint32_t* quad_mat = nullptr;
    DevMaterial* mats = nullptr;
    // the material of every sphere / parallelogram slot (the render kernel's shading reads one
    // record by the hit's slot instead of an index and then the material)
    DevMaterial* sphere_mrec = nullptr;
    DevMaterial* quad_mrec = nullptr;
    // per-device scratch reused across renders (partial sums of sample chunks)
    double* partial = nullptr;
    size_t partial_bytes = 0;
    unsigned long long* counters = nullptr;   // instrumented pass
    // parity guard words (zeroed at upload): [0] Dielectric reflect-or-refract decisions that a
    // 1-ulp difference of pow(1 - cos, 5) could have flipped (shade(), crt_render_guard)
    unsigned long long* guard = nullptr;
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
    crt::BigVec<crt_material> materials;
    crt::BigVec<crt_object> objects;
    crt::BigVec<crt::Prim> prims;
    crt::BigVec<double> pbox;              // primitive boxes, 6 doubles each (GPU BVH build only)
    crt::BigVec<crt_bvh_node> nodes;
    crt::BigVec<uint32_t> order;           // slot -> primitive index
    // device-layout staging (host)
    crt::BigVec<crt::DevNode> dnodes;
    crt::BigVec<uint32_t> refs;
    crt::BigVec<crt::DevSphere> spheres;
    crt::BigVec<uint32_t> sphere_mat;
    crt::BigVec<crt::DevQuad> quads;
    crt::BigVec<uint32_t> quad_mat;
    crt::BigVec<crt::DevMaterial> dmats;
    // element counts of the device layout (device_layout), set by the host staging (stage()) or
    // by the device scene set-up (crt_stage_gpu.hip), which leaves the host arrays above empty
    size_t num_objects = 0, num_materials = 0, num_prims = 0;
    size_t num_dnodes = 0, num_spheres = 0, num_quads = 0, num_dmats = 0;
    // >= 0: the scene was staged on that device (its image is s->dev[image_device]'s allocation;
    // other devices copy it from there); -1: staged on the host (s->image)
    int image_device = -1;
    uint32_t depth = 0;
    uint32_t max_leaf = 0;
    double build_ms = 0;
    bool linear = false;
    bool exact_slab = false;  // some node box is inverted / NaN on an axis: walk_step EXACT only
    crt::DeviceCopy dev[crt::kMaxDevices];
    std::mutex dev_mu[crt::kMaxDevices];  // one upload per device at a time (device_upload)
    // the device image (device_layout arrays at their offsets), staged by the first upload
    crt::BigVec<char> image;
    bool staged = false;
    bool image_f32_ok = false, image_spheres_f32_ok = false, image_quads_f32_ok = false, image_quads_flat_ok = false;
    std::mutex mu;  // staging
};

namespace crt {
// The one device allocation of a scene copy (device_upload): 256-byte aligned sub-arrays in this
// order; crt_scene_info reports its total as device_bytes.
enum DevArray { kArrNodes, kArrFNodes, kArrRefs, kArrSpheres, kArrSpherePairs, kArrSphereMat, kArrQuads,
                kArrQuadF, kArrQuadBox, kArrQuadMat, kArrMats, kArrSphereMrec, kArrQuadMrec, kArrGuard,
                kArrCount };
inline size_t device_layout(const crt_scene* s, size_t off[kArrCount + 1]) {
    const size_t n_nodes = s->num_dnodes, n_sp = s->num_spheres, n_q = s->num_quads;
    const size_t bytes[kArrCount] = {
        n_nodes * sizeof(DevNode), n_nodes * sizeof(DevNodeF), s->num_prims * 4, n_sp * sizeof(DevSphere),
        n_sp * sizeof(DevSpherePair), n_sp * 4, n_q * sizeof(DevQuad), n_q * sizeof(DevQuadF),
        n_q * sizeof(DevQuadBox), n_q * 4, std::max<size_t>(1, s->num_dmats) * sizeof(DevMaterial),
        n_sp * sizeof(DevMaterial), n_q * sizeof(DevMaterial), 64};
    size_t o = 0;
    for (int i = 0; i < kArrCount; ++i) {
        off[i] = o;
        o = (o + bytes[i] + 255) & ~size_t(255);
    }
    off[kArrCount] = o;
    return o;
}

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
const char* device_build_info();
int device_guard(crt_scene* s, int device, uint64_t* schlick_undecided, bool reset);
int device_build_bvh(crt_scene* s, uint32_t num_buckets, uint32_t max_leaf, int device,
                     const BigVec<double>& boxes);
void device_bind_copy(crt_scene* s, int device, void* base, size_t total);
int device_image(crt_scene* s, int device, void* host, size_t bytes);
// A tree built on the current device (crt_bvh_gpu.hip): the preorder node array (bvh.h:468-550)
// and the slot order in HBM.
struct DeviceTree {
    crt_bvh_node* nodes = nullptr;
    uint32_t* order = nullptr;   // slot -> primitive
    uint32_t nnodes = 0, depth = 0, max_leaf = 0;
};
int device_build_tree(size_t n, const double* d_pb, uint32_t num_buckets, uint32_t max_leaf, DeviceTree& out);
void device_tree_free(DeviceTree& t);
// The scene set up on `device` from the caller's objects and materials (crt_stage_gpu.hip): the
// primitives, the GPU BVH build and the device image, which becomes the scene's copy on that
// device. *host_path = true (nothing done) when the scene must take the host path instead.
int device_create_scene(crt_scene* s, const crt_material* materials, size_t num_materials,
                        const crt_object* objects, size_t num_objects, const crt_bvh_params& prm, int device,
                        bool* host_path);
// the host's validation of objects and materials (crt_host.cpp): CRT_OK or the error of the first
// bad one, with the primitive / sphere counts and whether any object is a Box
int validate_scene(const crt_material* materials, size_t nm, const crt_object* objects, size_t no,
                   size_t* nprims, size_t* nspheres, bool* boxes);
int device_ppm_values(int device, const double* d_rgb, size_t n, int32_t* h_values, void* stream);
// host: RGB::as_string's three integers for one pixel (std::pow, x86 int conversion)
void ppm_pixel_host(const double rgb[3], int32_t out[3]);
int render_multi(crt_scene* s, const crt_camera* cam, int num_devices, double* h_rgb,
                 crt_render_stats* stats);
int render_multi_ppm(crt_scene* s, const crt_camera* cam, int num_devices, int32_t* h_values,
                     crt_render_stats* stats);
}  // namespace crt
