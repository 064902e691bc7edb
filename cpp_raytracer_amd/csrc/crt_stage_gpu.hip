// Scene set-up on the device, for scenes whose BVH is built on the GPU (crt_bvh_params.build_device):
// the caller's objects and materials go to HBM once, and everything the host staging computes
// from them — the primitives and their boxes (Scene::get_primitive_components, scene.h:85-106),
// the tree (crt_bvh_gpu.hip), the device node order, the per-slot arrays, the f32 filter records
// and the per-slot material records (crt_host.cpp stage(), crt_device.hip stage_image) — is
// computed there, into the scene's copy on that device. The records come from the same
// definitions as the host's (crt_prims.h, crt_internal.h, crt_quad_filter.h), compiled with
// -ffp-contract=off, so the image is byte-identical to the host-staged one
// (tests/test_gpu_stage.py compares them array by array).
//
// Node order (stage()): the first kTopBfs nodes breadth-first, then each remaining subtree
// depth-first with the two children of a node side by side. The breadth-first top is a few
// hundred nodes and is computed on the host from the preorder array it downloads anyway; the
// position of every other node follows from its path below the top: a node expanded depth-first
// at child-base c puts its children at c and c + 1, the left child's descendants from c + 2 on and
// the right child's after them, from c + 1 + size(left) (in preorder, size(left) = right - left).
#include <hip/hip_runtime.h>

#define CRT_HD __host__ __device__ __forceinline__

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "crt_internal.h"
#include "crt_prims.h"

#pragma clang fp contract(off)

namespace crt {
namespace stagegpu {

constexpr uint32_t kT = 256;
constexpr uint32_t kNone = 0xffffffffu;
constexpr size_t kTopBfs = 1024;  // stage(): the breadth-first top of the device node order

// flag word bits (an atomicOr by each lane that sees the condition; all are rare)
enum : uint32_t {
    kNanBox = 1u,       // a primitive box with a NaN / infinite bound: the host path (flatten())
    kExactSlab = 2u,    // a node box inverted / NaN on an axis (crt_scene::exact_slab)
    kF32Bad = 4u,       // a node bound beyond the f32 walk's range
    kSphBad = 8u,       // a sphere beyond the f32 filter's range
    kQuadsBad = 16u,    // a parallelogram beyond its f32 filter's range
    kFlatBad = 32u,     // a parallelogram that is not axis-aligned
    kRegroupBad = 64u,  // a flat box flat on no axis (regroup_leaf)
    kWalkBad = 128u,    // a node position walk that did not end (a malformed tree)
};

__device__ __forceinline__ void raise_flag(uint32_t* flags, uint32_t bit, bool cond) {
    if (cond) atomicOr(flags, bit);
}

static dim3 grid_of(size_t n) { return dim3(static_cast<uint32_t>((n + kT - 1) / kT)); }

// ---- exclusive scan of u32 counts (n + 1 outputs, the last = the total) ----------------------
constexpr uint32_t kScanItems = 8, kScanTile = kT * kScanItems;

__device__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* lds, uint32_t& total) {
    const uint32_t t = threadIdx.x;
    lds[t] = v;
    __syncthreads();
    for (uint32_t d = 1; d < kT; d <<= 1) {
        const uint32_t x = t >= d ? lds[t - d] : 0u;
        __syncthreads();
        lds[t] += x;
        __syncthreads();
    }
    total = lds[kT - 1];
    const uint32_t incl = lds[t];
    __syncthreads();
    return incl - v;
}

__global__ __launch_bounds__(kT) void scan_tiles(const uint32_t* __restrict__ in, size_t n,
                                                 uint32_t* __restrict__ out, uint32_t* __restrict__ tile_sum) {
    __shared__ uint32_t lds[kT];
    const size_t base = static_cast<size_t>(blockIdx.x) * kScanTile + threadIdx.x * kScanItems;
    uint32_t v[kScanItems], sum = 0;
    for (uint32_t k = 0; k < kScanItems; ++k) {
        v[k] = base + k < n ? in[base + k] : 0u;
        sum += v[k];
    }
    uint32_t total;
    uint32_t run = block_exclusive_scan(sum, lds, total);
    for (uint32_t k = 0; k < kScanItems; ++k) {
        if (base + k < n) out[base + k] = run;
        run += v[k];
    }
    if (threadIdx.x == 0) tile_sum[blockIdx.x] = total;
}

// one block: the tiles' sums scanned in place, the grand total into out[n]
__global__ __launch_bounds__(kT) void scan_tile_sums(uint32_t* __restrict__ tile_sum, uint32_t ntiles,
                                                     uint32_t* __restrict__ out, size_t n) {
    __shared__ uint32_t lds[kT];
    uint32_t carry = 0;
    for (uint32_t a = 0; a < ntiles; a += kT) {
        const uint32_t i = a + threadIdx.x;
        const uint32_t v = i < ntiles ? tile_sum[i] : 0u;
        uint32_t total;
        const uint32_t ex = block_exclusive_scan(v, lds, total);
        if (i < ntiles) tile_sum[i] = carry + ex;
        carry += total;
    }
    if (threadIdx.x == 0) out[n] = carry;
}

__global__ __launch_bounds__(kT) void scan_add(uint32_t* __restrict__ out, size_t n,
                                               const uint32_t* __restrict__ tile_sum) {
    const size_t i = static_cast<size_t>(blockIdx.x) * kT + threadIdx.x;
    if (i < n) out[i] += tile_sum[i / kScanTile];
}

// ---- validation (crt_host.cpp validate_scene, on the device) ------------------------------------
// stat[0] = first bad object, stat[1] = first bad material (~0u: none), stat[3] = spheres,
// stat[4] = Boxes (sums over the objects, valid when no object is bad; stat[2] unused)
__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t* lds) {
    uint32_t total;
    (void)block_exclusive_scan(v, lds, total);
    return total;
}

__global__ __launch_bounds__(kT) void validate_objects(const crt_object* __restrict__ obj, size_t no, size_t nm,
                                                       uint32_t* __restrict__ stat) {
    __shared__ uint32_t lds[kT];
    const size_t i = static_cast<size_t>(blockIdx.x) * kT + threadIdx.x;
    uint32_t ns = 0, nb = 0;
    if (i < no) {
        const uint32_t kind = obj[i].kind, mat = obj[i].material;
        if (mat >= nm || (kind != CRT_SPHERE && kind != CRT_PARALLELOGRAM && kind != CRT_BOX))
            atomicMin(&stat[0], static_cast<uint32_t>(i));
        ns = kind == CRT_SPHERE ? 1u : 0u;
        nb = kind == CRT_BOX ? 1u : 0u;
    }
    ns = block_sum(ns, lds);
    nb = block_sum(nb, lds);
    if (threadIdx.x == 0) {
        atomicAdd(&stat[3], ns);
        atomicAdd(&stat[4], nb);
    }
}

__global__ __launch_bounds__(kT) void validate_materials(const crt_material* __restrict__ mat, size_t nm,
                                                         uint32_t* __restrict__ stat) {
    const size_t i = static_cast<size_t>(blockIdx.x) * kT + threadIdx.x;
    if (i < nm && (mat[i].kind < CRT_LAMBERTIAN || mat[i].kind > CRT_DIFFUSE_LIGHT))
        atomicMin(&stat[1], static_cast<uint32_t>(i));
}

// ---- primitives ------------------------------------------------------------------------------
__global__ __launch_bounds__(kT) void object_counts(const crt_object* __restrict__ obj, size_t no,
                                                    uint32_t* __restrict__ cnt) {
    const size_t i = static_cast<size_t>(blockIdx.x) * kT + threadIdx.x;
    if (i < no) cnt[i] = prim::object_prims(obj[i]);
}

// each object's primitives' boxes (the build's input) and, for scenes with Boxes, the primitive's
// object (off = first primitive of each object)
__global__ __launch_bounds__(kT) void emit_boxes(const crt_object* __restrict__ obj, size_t no,
                                                 const uint32_t* __restrict__ off, double* __restrict__ pb,
                                                 uint32_t* __restrict__ pobj, uint32_t* __restrict__ flags) {
    const size_t i = static_cast<size_t>(blockIdx.x) * kT + threadIdx.x;
    bool nan = false;
    if (i < no) {
        const crt_object o = obj[i];
        const size_t p0 = off ? off[i] : i;
        const uint32_t np = prim::object_prims(o);
        for (uint32_t j = 0; j < np; ++j) {
            double v[15], box[6];
            (void)prim::object_prim(o, j, v, box);
            for (int k = 0; k < 6; ++k) {
                pb[6 * (p0 + j) + k] = box[k];
                nan = nan || !std::isfinite(box[k]);
            }
            if (pobj) pobj[p0 + j] = static_cast<uint32_t>(i);
        }
    }
    raise_flag(flags, kNanBox, nan);
}

// ---- device node order -----------------------------------------------------------------------
// top[j] = {preorder node, device position, child-base (kNone unless expanded depth-first)}
__global__ __launch_bounds__(kT) void scatter_top(const uint32_t* __restrict__ top, uint32_t ntop,
                                                  uint32_t* __restrict__ tpos, uint32_t* __restrict__ tbase) {
    const uint32_t j = blockIdx.x * kT + threadIdx.x;
    if (j >= ntop) return;
    tpos[top[3 * j]] = top[3 * j + 1];
    tbase[top[3 * j]] = top[3 * j + 2];
}

// the device position of every preorder node (stage()'s breadth-first top, then sibling-pair
// depth-first subtrees): from the root through the top to the node's frontier ancestor, then
// down its depth-first expansion. A path of a well-formed tree has at most depth + 1 nodes, so
// max_steps = the build's depth + 2 bounds both walks together; only a malformed tree exceeds it
__global__ __launch_bounds__(kT) void node_positions(const crt_bvh_node* __restrict__ nd, uint32_t nn,
                                                     const uint32_t* __restrict__ tpos,
                                                     const uint32_t* __restrict__ tbase, uint32_t max_steps,
                                                     uint32_t* __restrict__ pos, uint32_t* __restrict__ flags) {
    const uint32_t i = blockIdx.x * kT + threadIdx.x;
    bool bad = false;
    if (i < nn) {
        uint32_t at = tpos[i];
        if (at == kNone) {
            uint32_t p = 0, steps = 0;
            for (;; ++steps) {  // the frontier ancestor: the last top node on the path
                const uint32_t c = i < nd[p].index ? p + 1 : nd[p].index;
                if (tpos[c] == kNone || steps > max_steps) break;
                p = c;
            }
            uint32_t base = tbase[p];  // breadth-first index of p's first child
            for (;; ++steps) {
                const uint32_t l = p + 1, r = nd[p].index;
                if (i == l || i == r || steps > max_steps || base == kNone || r <= l) {
                    bad = !(i == l || i == r);
                    at = (i == r ? base + 1 : base) + 1;  // place(k) = k + 1 for k >= 1
                    break;
                }
                if (i < r) {
                    p = l;
                    base += 2;
                } else {
                    p = r;
                    base += 1 + (r - l);
                }
            }
        }
        pos[i] = bad ? 1u : at;  // a malformed tree is reported (kWalkBad), never written out of range
    }
    raise_flag(flags, kWalkBad, bad);
}

// the device node (children explicit) and its f32 walk record at the node's position; thread 0
// also writes the pad (position 1) and the sentinel (position nn + 1)
__global__ __launch_bounds__(kT) void emit_nodes(const crt_bvh_node* __restrict__ nd, uint32_t nn,
                                                 const uint32_t* __restrict__ pos, DevNode* __restrict__ dn,
                                                 DevNodeF* __restrict__ fn, uint32_t* __restrict__ flags) {
    const uint32_t i = blockIdx.x * kT + threadIdx.x;
    bool exact = false, bad = false;
    if (i < nn) {
        const crt_bvh_node n = nd[i];
        DevNode d;
        for (int k = 0; k < 6; ++k) d.b[k] = n.bounds[k];
        for (int k = 0; k < 3; ++k)
            if (!(n.bounds[2 * k] <= n.bounds[2 * k + 1])) exact = true;
        const bool inner = n.count == 0 && i + 1 < nn;
        d.index = inner ? pos[n.index] : n.index;
        d.count = n.count;
        d.axis = n.axis;
        d.flags = inner ? pos[i + 1] : n.flags;
        const uint32_t at = pos[i];
        dn[at] = d;
        DevNodeF f;
        bad = node_record(d, at, f);
        fn[at] = f;
    }
    if (i == 0) {
        const uint32_t nd_end = nn + 1;
        DevNode pad, sen;
        for (int k = 0; k < 3; ++k) {
            pad.b[2 * k] = INFINITY;
            pad.b[2 * k + 1] = -INFINITY;
            sen.b[2 * k] = -INFINITY;
            sen.b[2 * k + 1] = INFINITY;
        }
        pad.index = pad.flags = 0;
        pad.count = 1;
        pad.axis = 0;
        sen.index = sen.flags = nd_end;
        sen.count = kSentinelCount;
        sen.axis = 0;
        dn[1] = pad;
        dn[nd_end] = sen;
        DevNodeF f;
        (void)node_record(pad, 1, f);
        fn[1] = f;
        (void)node_record(sen, nd_end, f);
        fn[nd_end] = f;
    }
    raise_flag(flags, kExactSlab, exact);
    raise_flag(flags, kF32Bad, bad);
}

// ---- per-slot arrays -------------------------------------------------------------------------
__global__ __launch_bounds__(kT) void slot_is_sphere(const crt_object* __restrict__ obj, const uint32_t* __restrict__ order,
                                                     size_t n, const uint32_t* __restrict__ pobj,
                                                     uint32_t* __restrict__ out) {
    const size_t s = static_cast<size_t>(blockIdx.x) * kT + threadIdx.x;
    if (s >= n) return;
    const uint32_t p = order[s];
    out[s] = obj[pobj ? pobj[p] : p].kind == CRT_SPHERE ? 1u : 0u;
}

struct SlotOut {
    uint32_t* refs;
    DevSphere* spheres;
    uint32_t* sphere_mat;
    DevMaterial* smrec;
    DevQuad* quads;
    uint32_t* quad_mat;
    DevMaterial* qmrec;
    DevQuadF* quadf;
    DevQuadBox* quadbox;
};

// slot s: its primitive recomputed from its object (prim::object_prim), stored at its rank among
// the slots of its kind (sidx = exclusive count of sphere slots; null when every slot is a sphere
// or every slot a parallelogram), with its material record and filter records
__global__ __launch_bounds__(kT) void emit_slots(const crt_object* __restrict__ obj, const crt_material* __restrict__ mat,
                                                 const uint32_t* __restrict__ order, size_t n,
                                                 const uint32_t* __restrict__ off, const uint32_t* __restrict__ pobj,
                                                 const uint32_t* __restrict__ sidx, uint32_t all_spheres, SlotOut O,
                                                 uint32_t* __restrict__ flags) {
    const size_t s = static_cast<size_t>(blockIdx.x) * kT + threadIdx.x;
    bool qbad = false, fbad = false;
    if (s < n) {
        const uint32_t p = order[s];
        const uint32_t o = pobj ? pobj[p] : p;
        const uint32_t j = off ? p - off[o] : 0u;
        const crt_object ob = obj[o];
        double v[15], box[6];
        const uint32_t kind = prim::object_prim(ob, j, v, box);
        const size_t is = sidx ? sidx[s] : (all_spheres ? s : 0);
        DevMaterial m = material_record(mat[ob.material]);
        if (kind == CRT_SPHERE) {
            DevSphere d;
            d.c[0] = v[0];
            d.c[1] = v[1];
            d.c[2] = v[2];
            d.r = v[3];
            O.refs[s] = static_cast<uint32_t>(is);
            O.spheres[is] = d;
            O.sphere_mat[is] = ob.material;
            shading_consts(m, &d);
            O.smrec[is] = m;
        } else {
            const size_t iq = s - is;
            DevQuad q{};
            for (int k = 0; k < 3; ++k) {
                q.v[k] = v[k];
                q.s1[k] = v[3 + k];
                q.s2[k] = v[6 + k];
                q.n[k] = v[9 + k];
                q.sn[k] = v[12 + k];
            }
            O.refs[s] = kRefQuad | static_cast<uint32_t>(iq);
            O.quads[iq] = q;
            O.quad_mat[iq] = ob.material;
            shading_consts(m, nullptr);
            O.qmrec[iq] = m;
            DevQuadF qf;
            qbad = !quad_record(q.v, q.s1, q.s2, q.sn, qf);
            O.quadf[iq] = qf;
            DevQuadBox qb{};
            fbad = !quad_flat_box(q.v, q.s1, q.s2, qb);
            O.quadbox[iq] = qb;
        }
    }
    raise_flag(flags, kQuadsBad, qbad);
    raise_flag(flags, kFlatBad, fbad);
}

__global__ __launch_bounds__(kT) void emit_materials(const crt_material* __restrict__ mat, size_t nm,
                                                     DevMaterial* __restrict__ out) {
    const size_t i = static_cast<size_t>(blockIdx.x) * kT + threadIdx.x;
    if (i < nm) out[i] = material_record(mat[i]);
}

__global__ __launch_bounds__(kT) void emit_sphere_pairs(const DevSphere* __restrict__ sp, size_t nsp,
                                                        DevSpherePair* __restrict__ out, uint32_t* __restrict__ flags) {
    const size_t i = static_cast<size_t>(blockIdx.x) * kT + threadIdx.x;
    bool bad = false;
    if (i < nsp) {
        DevSpherePair r;
        bad = sphere_pair_half(sp[i], r.cx[0], r.cy[0], r.cz[0], r.r2e[0]);
        if (i + 1 < nsp) (void)sphere_pair_half(sp[i + 1], r.cx[1], r.cy[1], r.cz[1], r.r2e[1]);
        else r.cx[1] = r.cy[1] = r.cz[1] = r.r2e[1] = 0;
        out[i] = r;
    }
    raise_flag(flags, kSphBad, bad);
}

// parallelogram-only scenes whose parallelograms are all axis-aligned (no kFlatBad): each leaf's
// flat boxes grouped by flat axis (regroup_leaf)
__global__ __launch_bounds__(kT) void regroup_leaves(const DevNode* __restrict__ dn, size_t nd,
                                                     DevQuadBox* __restrict__ quadbox, uint32_t* __restrict__ flags) {
    const size_t k = static_cast<size_t>(blockIdx.x) * kT + threadIdx.x;
    if (*flags & kFlatBad) return;  // uniform: the filter does not apply, nothing to group
    bool bad = false;
    if (k < nd) bad = regroup_leaf(dn[k], k, quadbox);
    raise_flag(flags, kRegroupBad, bad);
}

}  // namespace stagegpu

#define SG_TRY(expr)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) {                                                             \
            rc = fail(CRT_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));       \
            goto done;                                                                      \
        }                                                                                   \
    } while (0)

int device_create_scene(crt_scene* s, const crt_material* materials, size_t num_materials,
                        const crt_object* objects, size_t num_objects, const crt_bvh_params& prm, int device,
                        bool* host_path) {
    using namespace stagegpu;
    *host_path = false;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev || device >= kMaxDevices)
        return fail(CRT_E_NODEVICE, "GPU BVH build: device " + std::to_string(device) + " not visible");
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    const bool dbg = std::getenv("CRT_DEBUG_BUILD") != nullptr;
    auto tp = std::chrono::steady_clock::now();
    auto phase = [&](const char* what) {  // CRT_DEBUG_BUILD: where the set-up's time goes
        if (!dbg) return;
        (void)hipDeviceSynchronize();
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "device scene %-12s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(now - tp).count());
        tp = now;
    };
    const size_t no = num_objects, nm = num_materials;
    size_t n = 0, nq = 0, num_spheres = 0;
    bool boxes = false;
    int rc = CRT_OK;
    crt_object* d_obj = nullptr;
    crt_material* d_mat = nullptr;
    uint32_t *d_cnt = nullptr, *d_off = nullptr, *d_pobj = nullptr, *d_flags = nullptr, *d_tiles = nullptr;
    uint32_t *d_tpos = nullptr, *d_tbase = nullptr, *d_pos = nullptr, *d_top = nullptr, *d_sidx = nullptr, *d_sflag = nullptr;
    double* d_pb = nullptr;
    void* base = nullptr;
    DeviceTree t;
    uint32_t flags = 0;
    uint32_t stat[5] = {~0u, ~0u, 0, 0, 0};
    std::vector<uint32_t> top;  // (node, position, child-base) triples
    size_t total = 0;
    // exclusive scan of in[0, m) into out[0, m]
    auto scan = [&](const uint32_t* in, size_t m, uint32_t* out) {
        const uint32_t tiles = static_cast<uint32_t>((m + kScanTile - 1) / kScanTile);
        hipLaunchKernelGGL(scan_tiles, dim3(std::max(1u, tiles)), dim3(kT), 0, 0, in, m, out, d_tiles);
        hipLaunchKernelGGL(scan_tile_sums, dim3(1), dim3(kT), 0, 0, d_tiles, std::max(1u, tiles), out, m);
        hipLaunchKernelGGL(scan_add, grid_of(m), dim3(kT), 0, 0, out, m, d_tiles);
    };
    {
        if (no >= 0x7fffffffu) {
            rc = fail(CRT_E_INVALID, "too many primitives");
            goto done;
        }
        SG_TRY(hipMalloc(&d_obj, no * sizeof(crt_object)));
        SG_TRY(hipMalloc(&d_mat, std::max<size_t>(1, nm) * sizeof(crt_material)));
        SG_TRY(hipMalloc(&d_flags, 5 * 4));
        SG_TRY(hipMemcpy(d_flags, stat, sizeof stat, hipMemcpyHostToDevice));
        SG_TRY(hipMemcpy(d_obj, objects, no * sizeof(crt_object), hipMemcpyHostToDevice));
        if (nm) SG_TRY(hipMemcpy(d_mat, materials, nm * sizeof(crt_material), hipMemcpyHostToDevice));
        phase("upload");
        // validation on the device; the host's own pass words the error of a bad input
        hipLaunchKernelGGL(validate_objects, grid_of(no), dim3(kT), 0, 0, d_obj, no, nm, d_flags);
        if (nm) hipLaunchKernelGGL(validate_materials, grid_of(nm), dim3(kT), 0, 0, d_mat, nm, d_flags);
        SG_TRY(hipGetLastError());
        SG_TRY(hipMemcpy(stat, d_flags, sizeof stat, hipMemcpyDeviceToHost));
        if (stat[0] != ~0u || stat[1] != ~0u) {
            size_t np_h = 0, ns_h = 0;
            bool bx_h = false;
            rc = validate_scene(materials, nm, objects, no, &np_h, &ns_h, &bx_h);
            if (rc == CRT_OK) rc = fail(CRT_E_INVALID, "device scene set-up: validation disagrees with the host's");
            goto done;
        }
        n = no + 5 * static_cast<size_t>(stat[4]);  // a Box is six primitives
        num_spheres = stat[3];
        nq = n - num_spheres;
        boxes = stat[4] != 0;
        if (n >= 0x7fffffffu) {
            rc = fail(CRT_E_INVALID, "too many primitives");
            goto done;
        }
        SG_TRY(hipMemset(d_flags, 0, 4));
        SG_TRY(hipMalloc(&d_tiles, (std::max(n, no) / kScanTile + 2) * 4));
        SG_TRY(hipMalloc(&d_pb, n * 6 * sizeof(double)));
        phase("validate");
        if (boxes) {  // primitive offsets per object and primitive -> object
            SG_TRY(hipMalloc(&d_cnt, no * 4));
            SG_TRY(hipMalloc(&d_off, (no + 1) * 4));
            SG_TRY(hipMalloc(&d_pobj, n * 4));
            hipLaunchKernelGGL(object_counts, grid_of(no), dim3(kT), 0, 0, d_obj, no, d_cnt);
            scan(d_cnt, no, d_off);
        }
        hipLaunchKernelGGL(emit_boxes, grid_of(no), dim3(kT), 0, 0, d_obj, no, d_off, d_pb, d_pobj, d_flags);
        SG_TRY(hipGetLastError());
        SG_TRY(hipMemcpy(&flags, d_flags, 4, hipMemcpyDeviceToHost));
        phase("primitives");
        if (flags & kNanBox) {  // the host build handles non-finite boxes
            *host_path = true;
            goto done;
        }
        const auto tb = std::chrono::steady_clock::now();
        rc = device_build_tree(n, d_pb, prm.num_buckets, prm.max_prims_in_node, t);
        if (rc) goto done;
        s->build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb).count();
        (void)hipFree(d_pb);
        d_pb = nullptr;
        // the preorder array and the order stay on the host too (crt_scene_export_bvh, closest hits)
        s->nodes.resize(t.nnodes);
        s->order.resize(n);
        SG_TRY(hipMemcpy(s->nodes.data(), t.nodes, t.nnodes * sizeof(crt_bvh_node), hipMemcpyDeviceToHost));
        SG_TRY(hipMemcpy(s->order.data(), t.order, n * 4, hipMemcpyDeviceToHost));
        s->depth = t.depth;
        s->max_leaf = t.max_leaf;
        phase("build");
        // the breadth-first top (stage()) and the child-bases of its unexpanded nodes
        const uint32_t nn = t.nnodes;
        if (static_cast<size_t>(nn) + 2 >= (size_t{1} << (31 - kNodeFShift))) {  // device_upload's limit
            rc = fail(CRT_E_INVALID, "BVH too large for the device node layout");
            goto done;
        }
        const auto& N = s->nodes;
        auto interior = [&](uint32_t i) { return N[i].count == 0 && i + 1 < nn; };
        std::vector<uint32_t> bfs{0};
        size_t q = 0;
        for (; q < bfs.size() && bfs.size() < kTopBfs; ++q)
            if (interior(bfs[q])) {
                bfs.push_back(bfs[q] + 1);
                bfs.push_back(N[bfs[q]].index);
            }
        top.reserve(3 * bfs.size());
        uint32_t c = static_cast<uint32_t>(bfs.size());  // the depth-first expansions start here
        for (size_t k = 0; k < bfs.size(); ++k) {
            const uint32_t i = bfs[k];
            uint32_t cb = kNone;
            if (k >= q && interior(i)) {  // placed, unexpanded: its subtree is expanded depth-first next
                cb = c;
                uint32_t e = i;  // size of i's subtree: its rightmost descendant + 1 - i
                while (interior(e)) e = N[e].index;
                c += e - i;      // size - 1 descendants
            }
            top.push_back(i);
            top.push_back(k == 0 ? 0u : static_cast<uint32_t>(k + 1));
            top.push_back(cb);
        }
        // the device layout's counts, then the image, zeroed (padding and guard words)
        s->num_objects = no;
        s->num_materials = nm;
        s->num_prims = n;
        s->num_dnodes = static_cast<size_t>(nn) + 2;  // tree, pad, sentinel
        s->num_spheres = num_spheres;
        s->num_quads = nq;
        s->num_dmats = nm;
        size_t off[kArrCount + 1];
        total = device_layout(s, off);
        SG_TRY(hipMalloc(&base, total));
        SG_TRY(hipMemset(base, 0, total));
        char* b = static_cast<char*>(base);
        SG_TRY(hipMalloc(&d_tpos, nn * 4));
        SG_TRY(hipMalloc(&d_tbase, nn * 4));
        SG_TRY(hipMalloc(&d_pos, nn * 4));
        SG_TRY(hipMalloc(&d_top, top.size() * 4));
        SG_TRY(hipMemset(d_tpos, 0xff, nn * 4));
        SG_TRY(hipMemset(d_tbase, 0xff, nn * 4));
        SG_TRY(hipMemcpy(d_top, top.data(), top.size() * 4, hipMemcpyHostToDevice));
        const uint32_t ntop = static_cast<uint32_t>(top.size() / 3);
        hipLaunchKernelGGL(scatter_top, grid_of(ntop), dim3(kT), 0, 0, d_top, ntop, d_tpos, d_tbase);
        hipLaunchKernelGGL(node_positions, grid_of(nn), dim3(kT), 0, 0, t.nodes, nn, d_tpos, d_tbase,
                           static_cast<uint32_t>(t.depth) + 2u, d_pos, d_flags);
        auto* dn = reinterpret_cast<DevNode*>(b + off[kArrNodes]);
        hipLaunchKernelGGL(emit_nodes, grid_of(nn), dim3(kT), 0, 0, t.nodes, nn, d_pos, dn,
                           reinterpret_cast<DevNodeF*>(b + off[kArrFNodes]), d_flags);
        SG_TRY(hipGetLastError());
        // slots: sphere ranks by a scan when both kinds occur
        if (num_spheres != 0 && nq != 0) {
            SG_TRY(hipMalloc(&d_sidx, (n + 1) * 4));
            SG_TRY(hipMalloc(&d_sflag, n * 4));
            hipLaunchKernelGGL(slot_is_sphere, grid_of(n), dim3(kT), 0, 0, d_obj, t.order, n, d_pobj, d_sflag);
            scan(d_sflag, n, d_sidx);
        }
        const SlotOut O{reinterpret_cast<uint32_t*>(b + off[kArrRefs]),
                        reinterpret_cast<DevSphere*>(b + off[kArrSpheres]),
                        reinterpret_cast<uint32_t*>(b + off[kArrSphereMat]),
                        reinterpret_cast<DevMaterial*>(b + off[kArrSphereMrec]),
                        reinterpret_cast<DevQuad*>(b + off[kArrQuads]),
                        reinterpret_cast<uint32_t*>(b + off[kArrQuadMat]),
                        reinterpret_cast<DevMaterial*>(b + off[kArrQuadMrec]),
                        reinterpret_cast<DevQuadF*>(b + off[kArrQuadF]),
                        reinterpret_cast<DevQuadBox*>(b + off[kArrQuadBox])};
        hipLaunchKernelGGL(emit_slots, grid_of(n), dim3(kT), 0, 0, d_obj, d_mat, t.order, n, d_off, d_pobj, d_sidx,
                           nq == 0 ? 1u : 0u, O, d_flags);
        hipLaunchKernelGGL(emit_materials, grid_of(nm), dim3(kT), 0, 0, d_mat, nm,
                           reinterpret_cast<DevMaterial*>(b + off[kArrMats]));
        if (num_spheres)
            hipLaunchKernelGGL(emit_sphere_pairs, grid_of(num_spheres), dim3(kT), 0, 0, O.spheres, num_spheres,
                               reinterpret_cast<DevSpherePair*>(b + off[kArrSpherePairs]), d_flags);
        if (num_spheres == 0 && nq != 0)
            hipLaunchKernelGGL(regroup_leaves, grid_of(s->num_dnodes), dim3(kT), 0, 0, dn, s->num_dnodes, O.quadbox, d_flags);
        SG_TRY(hipGetLastError());
        SG_TRY(hipMemcpy(&flags, d_flags, 4, hipMemcpyDeviceToHost));
        phase("image");
        if (flags & kWalkBad) {
            rc = fail(CRT_E_INVALID, "device scene set-up: node placement did not end (malformed tree)");
            goto done;
        }
        s->exact_slab = (flags & kExactSlab) != 0;
        s->image_f32_ok = !(flags & kF32Bad);
        s->image_spheres_f32_ok = !(flags & kSphBad);
        s->image_quads_f32_ok = !(flags & kQuadsBad);
        s->image_quads_flat_ok = !(flags & (kFlatBad | kRegroupBad));
        s->image_device = device;
        device_bind_copy(s, device, base, total);
        base = nullptr;  // the scene's copy on `device` owns it now
    }
done:
    (void)hipFree(d_obj);
    (void)hipFree(d_mat);
    (void)hipFree(d_cnt);
    (void)hipFree(d_off);
    (void)hipFree(d_pobj);
    (void)hipFree(d_flags);
    (void)hipFree(d_tiles);
    (void)hipFree(d_tpos);
    (void)hipFree(d_tbase);
    (void)hipFree(d_pos);
    (void)hipFree(d_top);
    (void)hipFree(d_sidx);
    (void)hipFree(d_sflag);
    (void)hipFree(d_pb);
    (void)hipFree(base);
    device_tree_free(t);
    (void)hipSetDevice(prev);
    return rc;
}

}  // namespace crt
