// Host side of the render path: scene flattening, the reference's binned-SAH BVH build,
// Camera::init, the reference RNG, and the named scenes of the reference's src/main.cpp.
//
// Every floating-point expression here keeps the reference's operation order (the file is
// compiled with -ffp-contract=off) so the BVH node arrays and camera vectors are bit-identical
// to the ones the reference computes. Citations are paths in DeltaPavonis/cpp_raytracer.
#include <algorithm>
#include <atomic>
#include <sys/mman.h>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <numbers>
#include <numeric>
#include <optional>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "crt_internal.h"
#include "crt_prims.h"

namespace crt {

// ---------------------------------------------------------------------------------------------
// errors
void* big_alloc(size_t bytes) {
    constexpr size_t kHuge = size_t{2} << 20, kMin = size_t{32} << 20;
    static const bool off = std::getenv("CRT_NO_HUGEPAGES") != nullptr;
    if (bytes < kMin || off) {
        void* p = std::malloc(std::max<size_t>(bytes, 1));
        if (!p) throw std::bad_alloc();
        return p;
    }
    const size_t rounded = (bytes + kHuge - 1) / kHuge * kHuge;
    void* p = std::aligned_alloc(kHuge, rounded);
    if (!p) throw std::bad_alloc();
    (void)madvise(p, rounded, MADV_HUGEPAGE);
    return p;
}
void big_free(void* p, size_t) noexcept { std::free(p); }

static thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}
void clear_error() { g_last_error.clear(); }

// ---------------------------------------------------------------------------------------------
// minimal double vector with the reference's operator semantics (math/vec3d.h)
struct V3 {
    double x = 0, y = 0, z = 0;
    double operator[](int a) const { return a == 0 ? x : (a == 1 ? y : z); }
};
static inline V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline V3 neg(V3 a) { return {-a.x, -a.y, -a.z}; }
static inline V3 mul(V3 a, double d) { return {a.x * d, a.y * d, a.z * d}; }      // vec3d.h:32,102
static inline V3 divv(V3 a, double d) { return mul(a, 1 / d); }                  // vec3d.h:34
static inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; } // vec3d.h:114
static inline V3 cross(V3 a, V3 b) {                                              // vec3d.h:116
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
static inline double mag2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
static inline double mag(V3 a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
static inline V3 unit(V3 a) { return divv(a, mag(a)); }                           // vec3d.h:127
static inline V3 v3(const double* p) { return {p[0], p[1], p[2]}; }
static inline void put(double* p, V3 a) { p[0] = a.x; p[1] = a.y; p[2] = a.z; }

// std::fmin / std::fmax with glibc's semantics (crt_prims.h)
using prim::gfmax;
using prim::gfmin;

// ---- intervals / AABB (math/interval.h, acceleration/aabb.h) --------------------------------
struct Iv {
    double min, max;
    double size() const { return max - min; }
    void merge(const Iv& o) { min = gfmin(min, o.min); max = gfmax(max, o.max); }   // interval.h:45-54
    void merge(double d) { min = gfmin(min, d); max = gfmax(max, d); }
    double mid() const { return std::midpoint(min, max); }                         // interval.h:31
};
constexpr double kInf = std::numeric_limits<double>::infinity();
struct Box3 {
    Iv a[3] = {{kInf, -kInf}, {kInf, -kInf}, {kInf, -kInf}};                    // AABB::empty
    void merge(const Box3& o) { for (int i = 0; i < 3; ++i) a[i].merge(o.a[i]); }
    void merge(V3 p) { a[0].merge(p.x); a[1].merge(p.y); a[2].merge(p.z); }
    V3 centroid() const { return {a[0].mid(), a[1].mid(), a[2].mid()}; }         // aabb.h:27
    double area() const {                                                          // aabb.h:29-31
        return 2 * (a[0].size() * a[0].size() + a[1].size() * a[1].size() +
                    a[2].size() * a[2].size());
    }
};
static Box3 box_of(const double* b) {
    Box3 r;
    for (int i = 0; i < 3; ++i) r.a[i] = {b[2 * i], b[2 * i + 1]};
    return r;
}
static void box_put(double* b, const Box3& r) {
    for (int i = 0; i < 3; ++i) { b[2 * i] = r.a[i].min; b[2 * i + 1] = r.a[i].max; }
}

// ---------------------------------------------------------------------------------------------
// flattening: objects -> primitives (Scene::get_primitive_components, scene.h:85-106)

// One object's primitives (crt_prims.h, shared with the device scene set-up)
static void emit_object(const crt_object& o, Prim* out) {
    const uint32_t np = prim::object_prims(o);
    for (uint32_t j = 0; j < np; ++j) {
        out[j].kind = prim::object_prim(o, j, out[j].v, out[j].box);
        out[j].material = o.material;
    }
}

// The objects' and materials' validation, in object order (first error wins): the primitive
// count, the sphere count and whether any object is a Box (six primitives).
int validate_scene(const crt_material* materials, size_t nm, const crt_object* objects, size_t no,
                   size_t* nprims, size_t* nspheres, bool* boxes) {
    // in parallel chunks: each chunk's counts and its first bad object / material; the first bad
    // one overall is reported (objects before materials), as a sequential pass would
    constexpr size_t kChunk = 1 << 16;
    const size_t nco = (no + kChunk - 1) / kChunk, ncm = (nm + kChunk - 1) / kChunk;
    std::vector<size_t> cnp(nco, 0), cns(nco, 0), cbad(nco, SIZE_MAX), mbad(ncm, SIZE_MAX);
    std::vector<char> cbx(nco, 0);
    // (counts in locals, stored once per chunk: the per-chunk slots of neighbouring threads share
    // cache lines)
    parallel_for(nco, 1, [&](size_t a, size_t b) {
        for (size_t c = a; c < b; ++c) {
            size_t np_c = 0, ns_c = 0, bad = SIZE_MAX;
            bool bx_c = false;
            for (size_t i = c * kChunk; i < std::min(no, (c + 1) * kChunk); ++i) {
                const uint32_t kind = objects[i].kind, mat = objects[i].material;
                if (mat >= nm || (kind != CRT_SPHERE && kind != CRT_PARALLELOGRAM && kind != CRT_BOX)) {
                    bad = i;
                    break;
                }
                np_c += kind == CRT_BOX ? 6 : 1;
                ns_c += kind == CRT_SPHERE;
                bx_c = bx_c || kind == CRT_BOX;
            }
            cnp[c] = np_c;
            cns[c] = ns_c;
            cbx[c] = bx_c;
            cbad[c] = bad;
        }
    });
    parallel_for(ncm, 1, [&](size_t a, size_t b) {
        for (size_t c = a; c < b; ++c) {
            size_t bad = SIZE_MAX;
            for (size_t i = c * kChunk; i < std::min(nm, (c + 1) * kChunk); ++i)
                if (materials[i].kind < CRT_LAMBERTIAN || materials[i].kind > CRT_DIFFUSE_LIGHT) {
                    bad = i;
                    break;
                }
            mbad[c] = bad;
        }
    });
    size_t np = 0, ns = 0;
    bool bx = false;
    for (size_t c = 0; c < nco; ++c) {
        if (cbad[c] != SIZE_MAX) {
            const size_t i = cbad[c];
            const crt_object& o = objects[i];
            if (o.material >= nm)
                return fail(CRT_E_INVALID, "object " + std::to_string(i) + " references material " +
                                               std::to_string(o.material) + " out of range");
            return fail(CRT_E_INVALID, "object " + std::to_string(i) + " has unknown kind " +
                                           std::to_string(o.kind));
        }
        np += cnp[c];
        ns += cns[c];
        bx = bx || cbx[c];
    }
    for (size_t c = 0; c < ncm; ++c)
        if (mbad[c] != SIZE_MAX) return fail(CRT_E_INVALID, "material " + std::to_string(mbad[c]) + " has unknown kind");
    *nprims = np;
    *nspheres = ns;
    *boxes = bx;
    return CRT_OK;
}

static int flatten(crt_scene* s, bool boxes) {
    // validate in object order (first error wins), then emit in parallel at prefix offsets
    const size_t no = s->objects.size();
    size_t np = 0, ns = 0;
    bool bx = false;
    if (int rc = validate_scene(s->materials.data(), s->materials.size(), s->objects.data(), no, &np, &ns, &bx)) return rc;
    std::vector<size_t> off(no + 1, 0);
    for (size_t i = 0; i < no; ++i) off[i + 1] = off[i] + prim::object_prims(s->objects[i]);
    const auto tv = std::chrono::steady_clock::now();
    s->prims.resize(off[no]);
    // boxes: the GPU BVH build's input, written while the primitives are hot in cache
    if (boxes) s->pbox.resize(off[no] * 6);
    std::atomic<bool> nan_box{false};
    parallel_for(no, 4096, [&](size_t a, size_t b) {
        bool nan = false;
        for (size_t i = a; i < b; ++i) {
            Prim* p = s->prims.data() + off[i];
            emit_object(s->objects[i], p);
            if (boxes)
                for (size_t j = off[i]; j < off[i + 1]; ++j, ++p) {
                    std::memcpy(&s->pbox[6 * j], p->box, 6 * sizeof(double));
                    for (int k = 0; k < 6; ++k) nan = nan || !std::isfinite(p->box[k]);
                }
        }
        if (nan) nan_box = true;
    });
    // the GPU build reproduces the host build only for finite boxes (with a NaN, fmin/fmax pick by
    // operand order in ways its order-preserving keys do not model; an infinite bound makes NaN
    // centroids and areas, e.g. a sphere with a NaN centre folds to the empty box [inf, -inf]):
    // such scenes build on the host
    if (nan_box) BigVec<double>().swap(s->pbox);
    if (std::getenv("CRT_DEBUG_BUILD"))
        std::fprintf(stderr, "flatten: emit %.3f ms\n", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tv).count());
    return CRT_OK;
}

// ---------------------------------------------------------------------------------------------
// BVH build: binned SAH exactly as bvh.h:183-461, preorder flattening bvh.h:468-550.

namespace {
struct TreeNode {
    Box3 box;
    std::unique_ptr<TreeNode> left, right;
    size_t first = 0, count = 0;  // leaf span in `order`
    uint32_t axis = 0;
};

struct Builder {
    const BigVec<Prim>& prims;
    BigVec<uint32_t>& order;
    size_t nb, max_leaf;
    size_t total = 0;
    std::vector<Box3> boxes;
    std::vector<V3> cents;

    Builder(const BigVec<Prim>& p, BigVec<uint32_t>& o, size_t nb_, size_t ml)
        : prims(p), order(o), nb(nb_), max_leaf(ml) {
        boxes.resize(p.size());
        cents.resize(p.size());
        for (size_t i = 0; i < p.size(); ++i) {
            boxes[i] = box_of(p[i].box);
            cents[i] = boxes[i].centroid();
        }
    }

    size_t bucket_of(uint32_t prim, int axis, const Box3& cb) const {
        // bvh.h:275-292 (and the identical predicate of the partition, :418-433)
        double offset = (cents[prim][axis] - cb.a[axis].min) / cb.a[axis].size();
        size_t b = static_cast<size_t>(static_cast<double>(nb) * offset);
        if (b == nb) --b;
        return b;
    }

    std::unique_ptr<TreeNode> leaf(size_t lo, size_t hi, const Box3& box) {
        auto n = std::make_unique<TreeNode>();
        n->box = box;
        n->first = lo;
        n->count = hi - lo;
        return n;
    }

    std::unique_ptr<TreeNode> build(size_t lo, size_t hi) {
        ++total;
        Box3 bounds;
        for (size_t i = lo; i < hi; ++i) bounds.merge(boxes[order[i]]);
        if (hi - lo == 1) return leaf(lo, hi, bounds);
        Box3 cb;
        for (size_t i = lo; i < hi; ++i) cb.merge(cents[order[i]]);

        double min_cost = kInf;
        int best_axis = 0;
        size_t best_bucket = 0;
        std::vector<size_t> bn(nb);
        std::vector<Box3> bb(nb);
        std::vector<double> costs(nb - 1);
        for (int axis = 0; axis < 3; ++axis) {
            if (cb.a[axis].size() <= 0) continue;  // is_empty_exclusive, bvh.h:244
            std::fill(bn.begin(), bn.end(), 0);
            std::fill(bb.begin(), bb.end(), Box3{});
            for (size_t i = lo; i < hi; ++i) {
                size_t b = bucket_of(order[i], axis, cb);
                bn[b]++;
                bb[b].merge(boxes[order[i]]);
            }
            Box3 before;
            size_t nbef = 0;
            for (size_t k = 0; k + 1 < nb; ++k) {  // bvh.h:348-356
                before.merge(bb[k]);
                nbef += bn[k];
                costs[k] = before.area() * static_cast<double>(nbef);
            }
            Box3 after;
            size_t naft = 0;
            // bvh.h:360-369: the reference merges bucket i itself into the "after" side
            for (int k = static_cast<int>(nb) - 2; k >= 0; --k) {
                after.merge(bb[k]);
                naft += bn[k];
                costs[k] += after.area() * static_cast<double>(naft);
            }
            for (size_t k = 0; k + 1 < nb; ++k) {
                if (costs[k] < min_cost) {
                    min_cost = costs[k];
                    best_axis = axis;
                    best_bucket = k;
                }
            }
        }
        if (std::isinf(min_cost)) return leaf(lo, hi, bounds);  // bvh.h:395-397
        double leaf_cost = static_cast<double>(hi - lo);
        if (hi - lo > max_leaf || min_cost < leaf_cost) {
            // std::partition of libstdc++ (the reference's bvh.h:417): same algorithm, so the
            // same permutation.
            auto mid = std::partition(order.begin() + lo, order.begin() + hi, [&](uint32_t p) {
                           return bucket_of(p, best_axis, cb) <= best_bucket;
                       }) - order.begin();
            auto l = build(lo, mid);
            auto r = build(mid, hi);
            auto n = std::make_unique<TreeNode>();
            n->box = bounds;
            n->left = std::move(l);
            n->right = std::move(r);
            n->axis = best_axis;
            return n;
        }
        return leaf(lo, hi, bounds);
    }
};

void flatten_tree(const TreeNode* t, BigVec<crt_bvh_node>& out, size_t& next, uint32_t lvl,
                  uint32_t& depth, uint32_t& max_leaf) {
    size_t me = next++;
    depth = std::max(depth, lvl);
    crt_bvh_node n{};
    box_put(n.bounds, t->box);
    if (!t->left) {
        n.index = static_cast<uint32_t>(t->first);
        n.count = static_cast<uint32_t>(t->count);
        n.axis = 0;
        max_leaf = std::max<uint32_t>(max_leaf, n.count);
        out[me] = n;
    } else {
        flatten_tree(t->left.get(), out, next, lvl + 1, depth, max_leaf);
        n.index = static_cast<uint32_t>(next);
        n.count = 0;
        n.axis = t->axis;
        out[me] = n;
        flatten_tree(t->right.get(), out, next, lvl + 1, depth, max_leaf);
    }
}
}  // namespace

static int build_bvh(crt_scene* s, const crt_bvh_params& prm) {
    auto t0 = std::chrono::steady_clock::now();
    const size_t n = s->prims.size();
    s->order.resize(n);
    std::iota(s->order.begin(), s->order.end(), 0u);
    s->nodes.clear();
    s->depth = 0;
    s->max_leaf = 0;
    if (n == 0) {
        // an empty world: one empty leaf (never hit)
        crt_bvh_node e{};
        box_put(e.bounds, Box3{});
        s->nodes.push_back(e);
        s->depth = 1;
    } else if (prm.linear) {
        Box3 b;
        for (auto& p : s->prims) b.merge(box_of(p.box));
        crt_bvh_node e{};
        box_put(e.bounds, b);
        e.index = 0;
        e.count = static_cast<uint32_t>(n);
        e.flags = kNodeAlways;
        s->nodes.push_back(e);
        s->depth = 1;
        s->max_leaf = static_cast<uint32_t>(n);
    } else if (prm.build_device != 0 && !s->pbox.empty()) {
        // the same tree built on a GPU (crt_bvh_gpu.hip) from the boxes flatten() wrote; the
        // centroids are computed there (Builder's box_of(...).centroid())
        int rc = device_build_bvh(s, prm.num_buckets, prm.max_prims_in_node,
                                  static_cast<int>(prm.build_device) - 1, s->pbox);
        BigVec<double>().swap(s->pbox);
        if (rc) return rc;
    } else {
        if (prm.num_buckets < 2) return fail(CRT_E_INVALID, "num_buckets must be >= 2");
        Builder b(s->prims, s->order, prm.num_buckets, prm.max_prims_in_node);
        auto root = b.build(0, n);
        s->nodes.resize(b.total);
        size_t next = 0;
        flatten_tree(root.get(), s->nodes, next, 1, s->depth, s->max_leaf);
    }
    BigVec<double>().swap(s->pbox);
    s->build_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return CRT_OK;
}

// RGB::as_string (rgb.h:99-115) with its defaults as the x86-64 reference build computes it:
// std::pow(x, 1 / gamma) with gamma = 2 taken at run time (a libm pow, as in the reference),
// static_cast<int> as cvttsd2si (NaN / out of range -> INT_MIN).
static volatile double g_ppm_gamma = 2;

void ppm_pixel_host(const double rgb[3], int32_t out[3]) {
    const double gamma = g_ppm_gamma, scale = 255 + 0.999999;
    const double L = 0.2126 * rgb[0] + 0.7152 * rgb[1] + 0.0722 * rgb[2];
    for (int k = 0; k < 3; ++k) {
        const double v = scale * std::pow(rgb[k] / (1 + L), 1 / gamma);
        out[k] = (v > -2147483649.0 && v < 2147483648.0) ? static_cast<int32_t>(v) : INT32_MIN;
    }
}

// device-layout staging arrays
static void stage(crt_scene* s) {
    // Device node array, children explicit: an interior node's left child in `flags`, its right
    // child in `index`; a leaf keeps its primitive range and flags. The traversal visits the same
    // nodes in the same order as over the preorder array. Order: breadth-first for the first
    // kTopBfs nodes (the top levels, so any prefix of them is a top treelet the render kernel can
    // keep in LDS), then each remaining subtree depth-first with siblings side by side (a node's
    // two children share a 128-byte line, and a subtree is contiguous: cache locality for trees
    // that live in HBM).
    constexpr size_t kTopBfs = 1024;
    const size_t nn = s->nodes.size();
    const bool dbg = std::getenv("CRT_DEBUG_BUILD") != nullptr;
    auto t0 = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!dbg) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "stage: %-8s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(now - t0).count());
        t0 = now;
    };
    auto interior = [&](uint32_t i) {
        return s->nodes[i].count == 0 && !(s->nodes[i].flags & kNodeAlways) && i + 1 < nn;
    };
    std::vector<uint32_t> bfs, pos(nn, 0);
    bfs.reserve(nn);
    if (nn) bfs.push_back(0);
    size_t q = 0;
    for (; q < bfs.size() && bfs.size() < kTopBfs; ++q) {
        const uint32_t i = bfs[q];
        if (interior(i)) {
            bfs.push_back(i + 1);                  // preorder: the left child follows its parent
            bfs.push_back(s->nodes[i].index);      // the right child
        }
    }
    {  // placed but not yet expanded: bfs[q, size0); expand each subtree in sibling-pair DFS
        const size_t size0 = bfs.size();
        std::vector<uint32_t> todo;
        for (size_t r = size0; r-- > q;) todo.push_back(bfs[r]);  // so bfs[q] is expanded first
        while (!todo.empty()) {
            const uint32_t i = todo.back();
            todo.pop_back();
            if (!interior(i)) continue;
            const uint32_t l = i + 1, rr = s->nodes[i].index;
            bfs.push_back(l);
            bfs.push_back(rr);
            todo.push_back(rr);
            todo.push_back(l);
        }
    }
    // Device position of bfs[k]: the root at 0, an unused pad node at 1, bfs[k] at k + 1 for
    // k >= 1, so that every sibling pair (pushed together above) starts at an even position: a
    // right child is its left sibling + 1 and the pair fills one aligned 64-byte line of f32
    // nodes (the render walk derives both children from the left one).
    auto place = [](size_t k) { return static_cast<uint32_t>(k == 0 ? 0 : k + 1); };
    for (size_t k = 0; k < bfs.size(); ++k) pos[bfs[k]] = place(k);
    const size_t nd = nn ? nn + 1 : 0;  // tree + pad
    s->dnodes.resize(nd + 1);
    s->exact_slab = false;
    {  // the sentinel (kSentinelCount) after the tree's nodes
        DevNode& z = s->dnodes[nd];
        for (int k = 0; k < 3; ++k) {
            z.b[2 * k] = -std::numeric_limits<double>::infinity();
            z.b[2 * k + 1] = std::numeric_limits<double>::infinity();
        }
        z.index = z.flags = static_cast<uint32_t>(nd);
        z.count = kSentinelCount;
        z.axis = 0;
    }
    if (nn) {  // the pad: an empty one-primitive leaf no node refers to
        DevNode& z = s->dnodes[1];
        for (int k = 0; k < 3; ++k) {
            z.b[2 * k] = std::numeric_limits<double>::infinity();
            z.b[2 * k + 1] = -std::numeric_limits<double>::infinity();
        }
        z.index = z.flags = 0;
        z.count = 1;
        z.axis = 0;
    }
    for (size_t q = 0; q < bfs.size(); ++q) {
        const crt_bvh_node& n = s->nodes[bfs[q]];
        DevNode& d = s->dnodes[place(q)];
        for (int k = 0; k < 3; ++k)
            if (!(n.bounds[2 * k] <= n.bounds[2 * k + 1]) && !(n.flags & kNodeAlways)) s->exact_slab = true;
        std::memcpy(d.b, n.bounds, sizeof d.b);
        if (n.flags & kNodeAlways)  // the render walk's min/max slab enters [-inf, inf] unconditionally
            for (int k = 0; k < 3; ++k) {
                d.b[2 * k] = -std::numeric_limits<double>::infinity();
                d.b[2 * k + 1] = std::numeric_limits<double>::infinity();
            }
        const bool inner = n.count == 0 && !(n.flags & kNodeAlways) && bfs[q] + 1 < nn;
        d.index = inner ? pos[n.index] : n.index;
        d.count = n.count;
        d.axis = n.axis;
        d.flags = inner ? pos[bfs[q] + 1] : n.flags;
    }
    lap("nodes");
    // slot arrays: per chunk of slots count the spheres, then fill at prefix offsets (the sphere /
    // parallelogram arrays are in slot order either way)
    const size_t ns = s->order.size();
    s->refs.resize(ns);
    constexpr size_t kChunk = 1 << 16;
    const size_t nchunks = (ns + kChunk - 1) / kChunk;
    std::vector<size_t> csph(nchunks + 1, 0), cquad(nchunks + 1, 0);
    parallel_for(nchunks, 1, [&](size_t a, size_t b) {
        for (size_t c = a; c < b; ++c) {
            size_t k = 0;
            for (size_t slot = c * kChunk; slot < std::min(ns, (c + 1) * kChunk); ++slot)
                k += s->prims[s->order[slot]].kind == CRT_SPHERE;
            csph[c + 1] = k;
            cquad[c + 1] = std::min(ns, (c + 1) * kChunk) - c * kChunk - k;
        }
    });
    for (size_t c = 0; c < nchunks; ++c) {
        csph[c + 1] += csph[c];
        cquad[c + 1] += cquad[c];
    }
    s->spheres.resize(csph[nchunks]);
    s->sphere_mat.resize(csph[nchunks]);
    s->quads.resize(cquad[nchunks]);
    s->quad_mat.resize(cquad[nchunks]);
    parallel_for(nchunks, 1, [&](size_t a, size_t b) {
        for (size_t c = a; c < b; ++c) {
            size_t is = csph[c], iq = cquad[c];
            for (size_t slot = c * kChunk; slot < std::min(ns, (c + 1) * kChunk); ++slot) {
                const Prim& p = s->prims[s->order[slot]];
                if (p.kind == CRT_SPHERE) {
                    s->refs[slot] = static_cast<uint32_t>(is);
                    DevSphere& d = s->spheres[is];
                    d.c[0] = p.v[0]; d.c[1] = p.v[1]; d.c[2] = p.v[2]; d.r = p.v[3];
                    s->sphere_mat[is++] = p.material;
                } else {
                    s->refs[slot] = kRefQuad | static_cast<uint32_t>(iq);
                    DevQuad& q = s->quads[iq];
                    q = DevQuad{};
                    std::memcpy(q.v, p.v + 0, 3 * sizeof(double));
                    std::memcpy(q.s1, p.v + 3, 3 * sizeof(double));
                    std::memcpy(q.s2, p.v + 6, 3 * sizeof(double));
                    std::memcpy(q.n, p.v + 9, 3 * sizeof(double));
                    std::memcpy(q.sn, p.v + 12, 3 * sizeof(double));
                    s->quad_mat[iq++] = p.material;
                }
            }
        }
    });
    lap("slots");
    s->dmats.resize(s->materials.size());
    parallel_for(s->materials.size(), 1 << 14, [&](size_t a, size_t b) {
        for (size_t i = a; i < b; ++i) s->dmats[i] = material_record(s->materials[i]);
    });
    lap("materials");
    s->num_dnodes = s->dnodes.size();
    s->num_spheres = s->spheres.size();
    s->num_quads = s->quads.size();
    s->num_dmats = s->dmats.size();
}

// ---------------------------------------------------------------------------------------------
// Camera::init, camera.h:87-157
static void resolve_camera(const crt_camera_settings& st, crt_camera& c) {
    c = crt_camera{};
    c.image_w = st.image_w;
    c.image_h = st.image_h;
    c.samples_per_pixel = st.samples_per_pixel;
    c.max_depth = st.max_depth;
    double aspect = static_cast<double>(st.image_w) / static_cast<double>(st.image_h);
    V3 center = v3(st.center);
    V3 dir = st.has_lookat ? sub(v3(st.lookat), center) : v3(st.direction);
    double focal = st.has_focus_dist ? st.focus_dist : mag(dir);
    double vw, vh;
    if (st.fov_is_vertical) {
        vh = 2 * focal * std::tan(st.fov / 2);
        vw = vh * aspect;
    } else {
        vw = 2 * focal * std::tan(st.fov / 2);
        vh = vw / aspect;
    }
    V3 bz = neg(unit(dir));
    V3 bx = unit(cross(v3(st.up), bz));
    V3 by = cross(bz, bx);
    V3 xv = mul(bx, vw);
    V3 yv = mul(by, -vh);
    V3 pdx = divv(xv, static_cast<double>(st.image_w));
    V3 pdy = divv(yv, static_cast<double>(st.image_h));
    V3 ulc = sub(sub(sub(center, mul(bz, focal)), divv(xv, 2)), divv(yv, 2));
    V3 p00 = add(add(ulc, divv(pdx, 2)), divv(pdy, 2));
    double rad = focal * std::tan(st.defocus_angle / 2);
    put(c.origin, center);
    put(c.pixel00, p00);
    put(c.pixel_delta_x, pdx);
    put(c.pixel_delta_y, pdy);
    put(c.defocus_disk_x, mul(bx, rad));
    put(c.defocus_disk_y, mul(by, rad));
    c.defocus_angle = st.defocus_angle;
    c.background[0] = st.background[0];
    c.background[1] = st.background[1];
    c.background[2] = st.background[2];
    c.t_min = 0.00001;
}

// ---------------------------------------------------------------------------------------------
// The reference RNG (util/rand_util.h:51-127), one "thread" worth of state.
struct RefRng {
    std::optional<uint32_t> custom;
    bool d_init = false;
    uint32_t d_state = 0;
    bool i_init = false;
    std::mt19937 gen;
    std::uniform_int_distribution<> dist;

    uint32_t next_seed() {  // rand_util.h:51-72 (a random_device seed is never used here)
        custom = static_cast<uint32_t>(2'483'477u * (*custom) + 2'987'434'823u);
        return *custom;
    }
    double rd(double lo = 0, double hi = 1) {  // rand_util.h:85-117
        if (!d_init) { d_state = next_seed(); d_init = true; }
        d_state = 1'664'525u * d_state + 1'013'904'223u;
        constexpr double kScale =
            1 / static_cast<double>(std::numeric_limits<uint32_t>::max() - 1);
        return lo + (hi - lo) * static_cast<double>(d_state) * kScale;
    }
    int ri(int lo, int hi) {  // rand_util.h:120-127
        if (!i_init) { gen.seed(next_seed()); i_init = true; }
        dist.param(std::uniform_int_distribution<>::param_type{lo, hi});
        return dist(gen);
    }
    // RGB::random (rgb.h:64-66): from_mag(rand, rand, rand); a g++ build evaluates the three
    // arguments right to left, so the blue draw comes first.
    V3 rgb(double lo = 0, double hi = 1) {
        double b = rd(lo, hi);
        double g = rd(lo, hi);
        double r = rd(lo, hi);
        return {r, g, b};
    }
};

// Scene assembly helpers
struct SceneOut {
    std::vector<crt_material> mats;
    std::vector<crt_object> objs;
    crt_camera_settings cam{};
    uint32_t mat(uint32_t kind, V3 c, double param) {
        crt_material m{};
        m.kind = kind;
        m.color[0] = c.x; m.color[1] = c.y; m.color[2] = c.z;
        m.param = param;
        mats.push_back(m);
        return static_cast<uint32_t>(mats.size() - 1);
    }
    uint32_t lambertian(V3 c) { return mat(CRT_LAMBERTIAN, c, 0); }
    uint32_t metal(V3 c, double fuzz) { return mat(CRT_METAL, c, gfmin(fuzz, 1.)); }
    uint32_t dielectric(double ri) { return mat(CRT_DIELECTRIC, {0, 0, 0}, ri); }
    uint32_t light(V3 c, double k) { return mat(CRT_DIFFUSE_LIGHT, c, k); }
    void sphere(V3 c, double r, uint32_t m) {
        crt_object o{};
        o.kind = CRT_SPHERE;
        o.material = m;
        put(o.v, c);
        o.v[3] = r;
        objs.push_back(o);
    }
    void quad(V3 v, V3 a, V3 b, uint32_t m) {
        crt_object o{};
        o.kind = CRT_PARALLELOGRAM;
        o.material = m;
        put(o.v, v);
        put(o.v + 3, a);
        put(o.v + 6, b);
        objs.push_back(o);
    }
    void box(V3 a, V3 b, uint32_t m) {
        crt_object o{};
        o.kind = CRT_BOX;
        o.material = m;
        put(o.v, a);
        put(o.v + 3, b);
        objs.push_back(o);
    }
};

// camera defaults of camera.h:16-82, then setter helpers (camera.h:308-406)
static crt_camera_settings default_cam() {
    crt_camera_settings c{};
    c.image_w = 1280;
    c.image_h = 720;
    c.samples_per_pixel = 1;
    c.max_depth = 10;
    c.direction[2] = -1;
    c.up[1] = 1;
    c.fov = 90;  // the reference's default stores 90 as radians (camera.h:78)
    c.fov_is_vertical = 1;
    c.background[0] = c.background[1] = c.background[2] = 0.5;
    return c;
}
static double deg(double d) { return d * std::numbers::pi / 180; }
static void width_aspect(crt_camera_settings& c, size_t w, double aspect) {
    auto h = static_cast<size_t>(std::round(static_cast<double>(w) / aspect));
    c.image_w = static_cast<uint32_t>(w);
    c.image_h = static_cast<uint32_t>(std::max(size_t{1}, h));
}
static void look(crt_camera_settings& c, V3 center, V3 lookat) {
    put(c.center, center);
    put(c.lookat, lookat);
    c.has_lookat = 1;
}
static void towards(crt_camera_settings& c, V3 center, V3 p) {
    put(c.center, center);
    put(c.direction, sub(p, center));
    c.has_lookat = 0;
}
static void bg(crt_camera_settings& c, V3 b) { put(c.background, b); }

// src/main.cpp:13-75 rtow_final_image / :154-216 millions_of_spheres share this loop shape;
// lights variants (:77-152, :218-292) add DiffuseLight spheres.
static void spheres_field(RefRng& R, SceneOut& S, int a0, int a1, int b0, int b1,
                          double p_light, double light_lo, double light_hi, double p_diffuse,
                          double p_metal) {
    for (int a = a0; a < a1; a++) {
        for (int b = b0; b < b1; b++) {
            double choose = R.rd();
            double cx = a + 0.9 * R.rd();  // Point3D(x, 0.2, z): parenthesized aggregate init,
            double cz = b + 0.9 * R.rd();  // sequenced left to right
            V3 c{cx, 0.2, cz};
            if (mag(sub(c, V3{4, 0.2, 0})) > 0.9) {
                if (choose < p_light) {
                    V3 albedo = R.rgb();
                    double k = R.rd(light_lo, light_hi);
                    S.sphere(c, 0.2, S.light(albedo, k));
                } else if (choose < p_diffuse) {
                    V3 x = R.rgb();
                    V3 y = R.rgb();
                    S.sphere(c, 0.2, S.lambertian({x.x * y.x, x.y * y.y, x.z * y.z}));
                } else if (choose < p_metal) {
                    V3 albedo = R.rgb(0.5, 1);
                    double fuzz = R.rd(0, 0.5);
                    S.sphere(c, 0.2, S.metal(albedo, fuzz));
                } else {
                    S.sphere(c, 0.2, S.dielectric(1.5));
                }
            }
        }
    }
}

static void three_big_spheres(SceneOut& S) {
    S.sphere({0, 1, 0}, 1.0, S.dielectric(1.5));
    S.sphere({-4, 1, 0}, 1.0, S.lambertian({0.4, 0.2, 0.1}));
    S.sphere({4, 1, 0}, 1.0, S.metal({0.7, 0.6, 0.5}, 0.0));
}

static bool build_named(const std::string& name, RefRng& R, SceneOut& S) {
    crt_camera_settings& c = S.cam;
    c = default_cam();
    if (name == "config1") {
        // BASELINE config 1: ground + one Lambertian sphere, 400x225, 1 spp, depth 50
        S.sphere({0, -1000, 0}, 1000, S.lambertian({0.5, 0.5, 0.5}));
        S.sphere({0, 1, 0}, 1, S.lambertian({0.4, 0.2, 0.1}));
        width_aspect(c, 400, 16. / 9.);
        c.fov = deg(20);
        look(c, {13, 2, 3}, {0, 0, 0});
        c.samples_per_pixel = 1;
        c.max_depth = 50;
        bg(c, {0.7, 0.8, 1});
        return true;
    }
    if (name == "rtow_final") {  // src/main.cpp:13-75
        S.sphere({0, -1000, 0}, 1000, S.lambertian({0.5, 0.5, 0.5}));
        spheres_field(R, S, -11, 11, -11, 11, -1, 0, 0, 0.8, 0.95);
        three_big_spheres(S);
        width_aspect(c, 1200, 16. / 9.);
        c.fov = deg(20);
        look(c, {13, 2, 3}, {0, 0, 0});
        c.defocus_angle = deg(0.6);
        c.focus_dist = 10;
        c.has_focus_dist = 1;
        c.samples_per_pixel = 500;
        c.max_depth = 20;
        bg(c, {0.7, 0.8, 1});
        return true;
    }
    if (name == "rtow_final_lights") {  // src/main.cpp:77-152
        S.sphere({0, -1000000, 0}, 1000000, S.lambertian({0.5, 0.5, 0.5}));
        spheres_field(R, S, -11, 11, -11, 11, 0.035, 30, 100, 0.8, 0.9);
        three_big_spheres(S);
        S.sphere({0, 2.5, 2.5}, 0.2, S.light({0.380205, 0.680817, 0.385431}, 150));
        width_aspect(c, 1080, 16. / 9.);
        c.fov = deg(25);
        look(c, {13, 2, 3}, {0, 0, 0});
        c.defocus_angle = deg(0.48);
        c.focus_dist = 10;
        c.has_focus_dist = 1;
        c.samples_per_pixel = 2000;
        c.max_depth = 20;
        bg(c, {0, 0, 0});
        return true;
    }
    if (name == "millions") {  // src/main.cpp:154-216
        S.sphere({0, -1000000, 0}, 1000000, S.lambertian({0.5, 0.5, 0.5}));
        spheres_field(R, S, -1001, 1001, -1001, 51, -1, 0, 0, 0.8, 0.95);
        three_big_spheres(S);
        width_aspect(c, 2160, 16. / 9.);
        c.fov = deg(40);
        look(c, {0, 10, 50}, {0, 0, 0});
        c.defocus_angle = deg(0.1);
        c.focus_dist = 51;
        c.has_focus_dist = 1;
        c.samples_per_pixel = 500;
        c.max_depth = 50;
        return true;
    }
    if (name == "millions_lights") {  // src/main.cpp:218-292
        S.sphere({0, -1000000, 0}, 1000000, S.lambertian({0.5, 0.5, 0.5}));
        spheres_field(R, S, -1001, 1001, -1501, 51, 0.035, 5, 15, 0.8, 0.9);
        three_big_spheres(S);
        S.sphere({0, 12, 0}, 3, S.light({0.380205, 0.680817, 0.385431}, 150));
        width_aspect(c, 1080, 16. / 9.);
        c.fov = deg(40);
        look(c, {0, 12.5, 50}, {0, 0, 0});
        c.defocus_angle = deg(0.1);
        c.focus_dist = 51;
        c.has_focus_dist = 1;
        c.samples_per_pixel = 1000;
        c.max_depth = 20;
        bg(c, {0, 0, 0});
        return true;
    }
    if (name == "parallelograms") {  // src/main.cpp:294-324
        uint32_t lr = S.lambertian({1.0, 0.2, 0.2}), bgm = S.lambertian({0.2, 1.0, 0.2}),
                 rb = S.lambertian({0.2, 0.2, 1.0}), uo = S.lambertian({1.0, 0.5, 0.0}),
                 lt = S.lambertian({0.2, 0.8, 0.8});
        S.quad({-3, -2, 5}, {0, 0, -4}, {0, 4, 0}, lr);
        S.quad({-2, -2, 0}, {4, 0, 0}, {0, 4, 0}, bgm);
        S.quad({3, -2, 1}, {0, 0, 4}, {0, 4, 0}, rb);
        S.quad({-2, 3, 1}, {4, 0, 0}, {0, 0, 4}, uo);
        S.quad({-2, -3, 5}, {4, 0, 0}, {0, 0, -4}, lt);
        width_aspect(c, 1000, 1.);
        c.samples_per_pixel = 100;
        c.max_depth = 50;
        c.fov = deg(80);
        towards(c, {0, 0, 9}, {0, 0, 0});
        c.defocus_angle = 0;
        bg(c, {0.7, 0.8, 1});
        return true;
    }
    if (name == "cornell" || name == "cornell_empty") {  // src/main.cpp:326-363
        uint32_t red = S.lambertian({.65, .05, .05}), white = S.lambertian({.73, .73, .73}),
                 green = S.lambertian({.12, .45, .15}), light = S.light({1, 1, 1}, 15);
        S.quad({555, 0, 0}, {0, 555, 0}, {0, 0, 555}, green);
        S.quad({0, 0, 0}, {0, 555, 0}, {0, 0, 555}, red);
        S.quad({343, 554, 332}, {-130, 0, 0}, {0, 0, -105}, light);
        S.quad({0, 0, 0}, {555, 0, 0}, {0, 0, 555}, white);
        S.quad({555, 555, 555}, {-555, 0, 0}, {0, 0, -555}, white);
        S.quad({0, 0, 555}, {555, 0, 0}, {0, 555, 0}, white);
        if (name == "cornell") {
            S.box({130, 0, 65}, {295, 165, 230}, white);
            S.box({265, 0, 295}, {430, 330, 460}, white);
        }
        width_aspect(c, 1000, 1.);
        c.samples_per_pixel = 10;
        c.max_depth = 1000;
        c.fov = deg(40);
        towards(c, {278, 278, -800}, {278, 278, 0});
        c.defocus_angle = 0;
        bg(c, {0, 0, 0});
        return true;
    }
    if (name == "dance_floor") {  // src/main.cpp:365-412 raining_on_the_dance_floor
        for (int x = -1000; x <= 1000; ++x) {
            for (int z = -1000; z <= 100; ++z) {
                // ms<DiffuseLight>(RGB::random(), rand_double(0.5, 2)): g++ evaluates the
                // intensity argument first
                double k = R.rd(0.5, 2);
                V3 col = R.rgb();
                S.quad({x + 0.1, 0, z + 0.1}, {0.8, 0, 0}, {0, 0, 0.8}, S.light(col, k));
            }
        }
        for (size_t i = 0; i < 25000; ++i) {
            double choose = R.rd();
            uint32_t m = S.dielectric(R.rd(1.25, 2.5));
            if (choose < 0.05) m = S.metal(R.rgb(), 0);
            double r = R.rd(0.25, 0.8);  // radius argument first, then the braced centre
            double px = R.rd(-1000, 1000), py = R.rd(2, 40), pz = R.rd(-1000, 50);
            S.sphere({px, py, pz}, r, m);
        }
        for (size_t i = 0; i < 50; ++i) {
            uint32_t m = S.dielectric(1.5);
            double r = R.rd(0.25, 0.5);
            double px = R.rd(-20, 20), py = R.rd(1, 8), pz = R.rd(-50, 50);
            S.sphere({px, py, pz}, r, m);
        }
        width_aspect(c, 2160, 16. / 9.);
        c.samples_per_pixel = 50;
        c.max_depth = 50;
        c.fov = deg(40);
        towards(c, {0, 10, 50}, {0, 0, 0});
        c.defocus_angle = 0;
        bg(c, {0, 0, 0});
        return true;
    }
    if (name == "christmas_tree") {  // src/main.cpp:414-583
        S.quad({-1000000, 0, -1000000}, {2000000, 0, 0}, {0, 0, 2000000},
               S.lambertian({0.25, 0.25, 0.25}));
        S.sphere({20, 25, -25}, 2.5, S.light({0.8, 0.8, 0.8}, 500));
        const double apex = 20;
        const double ratio = 1. / 3.;
        const V3 colors[6] = {{156 / 255., 10 / 255., 72 / 255.},
                              {66 / 255., 106 / 255., 33 / 255.},
                              {41 / 255., 119 / 255., 133 / 255.},
                              {0.5, 0.5, 0.5},
                              {0.5, 0.5, 0.5},
                              {0.5, 0.5, 0.5}};
        auto too_close = [&](V3 c, double r) {
            for (auto& o : S.objs) {
                if (o.kind != CRT_SPHERE) continue;
                if (mag(sub(c, v3(o.v))) <= r + o.v[3] + 0.1) return true;
            }
            return false;
        };
        for (int i = 0; i < 200; ++i) {
            while (true) {
                double ry = R.rd(0, apex);
                if (ry > 17) ry = R.rd(0, apex);
                if (i == 0) ry = apex;
                double rad = (20 - ry) * ratio;
                double ang = R.rd(0, 2 * std::numbers::pi);
                // a g++ -O2/-O3 build fuses std::sin + std::cos of one angle into glibc's
                // sincos(), which can differ from sin() in the last bit: call it explicitly
                double sn, cs;
                ::sincos(ang, &sn, &cs);
                V3 cc{rad * sn, ry, rad * cs};
                double sr = R.rd(0.25, 0.45);
                if (too_close(cc, sr)) continue;
                // ms<Metal>(colors[rand_int(0, 5)], rand_double(0, 0.1)): fuzz drawn first
                double fz = R.rd(0, 0.1);
                int ci = R.ri(0, 5);
                uint32_t m = S.metal(colors[ci], fz);
                if (i == 0) m = S.light({1, 1, 1}, 10);
                S.sphere(cc, sr, m);
                break;
            }
        }
        uint32_t snow = S.lambertian({1, 1, 1});
        std::vector<std::pair<V3, double>> flakes;
        for (int i = 0; i < 4000; ++i) {
            while (true) {
                double x = R.rd(-30, 30), y = R.rd(0, 30), z = R.rd(-50, 50);
                V3 sc{x, y, z};
                double sr = (sc.z > 35 ? 0.015 : (sc.z > 20 ? 0.03 : 0.05));
                if (too_close(sc, sr)) continue;
                flakes.push_back({sc, sr});
                break;
            }
        }
        for (auto& f : flakes) S.sphere(f.first, f.second, snow);
        width_aspect(c, 1080, 16. / 9.);
        bg(c, {0, 0, 0});
        towards(c, {0, 17.5, 50}, {0, 10, 0});
        c.fov = deg(35);
        c.samples_per_pixel = 10000;
        c.max_depth = 50;
        return true;
    }
    if (name == "bvh_pathological") {  // src/main.cpp:585-650
        for (int i = 0; i < 135; ++i)
            S.sphere({std::pow(10.7, i), 0, 0}, std::pow(17.3, i), S.lambertian({0, 0, 0}));
        return true;
    }
    return false;
}

// ---------------------------------------------------------------------------------------------
// per-sample seeding (the framework's replacement of the per-thread seed)
uint32_t sample_seed(uint32_t base, uint32_t pixel, uint32_t sample) {
    uint64_t z = (static_cast<uint64_t>(pixel) << 32) | sample;
    z += static_cast<uint64_t>(base) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return static_cast<uint32_t>(z ^ (z >> 32));
}

}  // namespace crt

// =============================================================================================
// C ABI
using namespace crt;

extern "C" {

int crt_abi_version(void) { return CRT_ABI_VERSION; }

const char* crt_last_error(void) { return g_last_error.c_str(); }

// the kernels' compile-time switches plus the build stamp (Makefile: the sha256 of the sources as
// compiled and their git commit, "+dirty" when they differ from it)
#ifndef CRT_SOURCE_SHA
#define CRT_SOURCE_SHA "unknown"
#endif
#ifndef CRT_GIT
#define CRT_GIT "none"
#endif
const char* crt_build_info(void) {
    static const std::string info = std::string(device_build_info()) + " src=" CRT_SOURCE_SHA " git=" CRT_GIT;
    return info.c_str();
}

void crt_free(void* p) { std::free(p); }

uint32_t crt_sample_seed(uint32_t base_seed, uint32_t pixel, uint32_t sample) {
    return sample_seed(base_seed, pixel, sample);
}

double crt_rand_double(uint32_t* state, double min, double max) {
    *state = 1'664'525u * *state + 1'013'904'223u;
    constexpr double kScale = 1 / static_cast<double>(std::numeric_limits<uint32_t>::max() - 1);
    return min + (max - min) * static_cast<double>(*state) * kScale;
}

int crt_scene_build_named(const char* name, uint32_t seed, int has_seed,
                          crt_material** materials, size_t* num_materials,
                          crt_object** objects, size_t* num_objects, crt_camera_settings* cam) {
    clear_error();
    if (!name || !materials || !num_materials || !objects || !num_objects)
        return fail(CRT_E_INVALID, "crt_scene_build_named: null argument");
    std::string n(name);
    // scenes that seed themselves (src/main.cpp:79, :220, :367, :416)
    std::optional<uint32_t> own;
    if (n == "rtow_final_lights") own = 2286021279u;
    if (n == "millions_lights") own = 473654968u;
    if (n == "dance_floor") own = 5987634u;
    if (n == "christmas_tree") own = 20231225u;
    RefRng R;
    if (own) R.custom = *own;
    if (has_seed) R.custom = seed;
    if (!R.custom && !(n == "config1" || n == "parallelograms" || n == "cornell" ||
                       n == "cornell_empty" || n == "bvh_pathological"))
        return fail(CRT_E_INVALID, "scene '" + n + "' draws random numbers: give a seed");
    SceneOut S;
    if (!build_named(n, R, S)) return fail(CRT_E_INVALID, "unknown scene '" + n + "'");
    auto* m = static_cast<crt_material*>(std::malloc(sizeof(crt_material) * std::max<size_t>(1, S.mats.size())));
    auto* o = static_cast<crt_object*>(std::malloc(sizeof(crt_object) * std::max<size_t>(1, S.objs.size())));
    if (!m || !o) { std::free(m); std::free(o); return fail(CRT_E_ALLOC, "out of host memory"); }
    if (!S.mats.empty()) std::memcpy(m, S.mats.data(), sizeof(crt_material) * S.mats.size());
    if (!S.objs.empty()) std::memcpy(o, S.objs.data(), sizeof(crt_object) * S.objs.size());
    *materials = m;
    *num_materials = S.mats.size();
    *objects = o;
    *num_objects = S.objs.size();
    if (cam) *cam = S.cam;
    return CRT_OK;
}

int crt_scene_create(const crt_material* materials, size_t num_materials,
                     const crt_object* objects, size_t num_objects,
                     const crt_bvh_params* params, crt_scene** out) {
    clear_error();
    if (!out) return fail(CRT_E_INVALID, "crt_scene_create: out is null");
    if ((num_materials && !materials) || (num_objects && !objects))
        return fail(CRT_E_INVALID, "crt_scene_create: null array with nonzero count");
    crt_bvh_params prm{32, 12, 0, 0};
    if (params) prm = *params;
    std::unique_ptr<crt_scene> s;
    try {
        s = std::make_unique<crt_scene>();
        const bool dbg = std::getenv("CRT_DEBUG_BUILD") != nullptr;
        auto t0 = std::chrono::steady_clock::now();
        auto lap = [&](const char* what) {  // CRT_DEBUG_BUILD: scene creation phases
            if (!dbg) return;
            const auto now = std::chrono::steady_clock::now();
            std::fprintf(stderr, "scene phase %-8s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(now - t0).count());
            t0 = now;
        };
        // A GPU build sets the scene up on its device (crt_stage_gpu.hip): the objects and
        // materials go straight to HBM and the device image is computed there (CRT_HOST_STAGE=1:
        // the host path, which stages the same image on the host)
        if (prm.build_device != 0 && prm.linear == 0 && num_objects != 0 && std::getenv("CRT_HOST_STAGE") == nullptr) {
            bool host_path = false;
            int rc = device_create_scene(s.get(), materials, num_materials, objects, num_objects, prm,
                                         static_cast<int>(prm.build_device) - 1, &host_path);
            if (rc) return rc;
            lap("device");
            if (!host_path) {
                *out = s.release();
                return CRT_OK;
            }
        }
        // copied in parallel chunks into huge-page backed arrays (millions: 2.1 M objects and materials)
        s->materials.resize(num_materials);
        s->objects.resize(num_objects);
        parallel_for(num_materials, 1 << 15, [&](size_t a, size_t b) {
            std::memcpy(s->materials.data() + a, materials + a, (b - a) * sizeof(crt_material));
        });
        parallel_for(num_objects, 1 << 15, [&](size_t a, size_t b) {
            std::memcpy(s->objects.data() + a, objects + a, (b - a) * sizeof(crt_object));
        });
        lap("copy");
        int rc = flatten(s.get(), prm.build_device != 0 && prm.linear == 0);
        if (rc) return rc;
        lap("flatten");
        if (s->prims.size() >= 0x7fffffffu) return fail(CRT_E_INVALID, "too many primitives");
        s->num_objects = num_objects;
        s->num_materials = num_materials;
        s->num_prims = s->prims.size();
        s->linear = prm.linear != 0;
        rc = build_bvh(s.get(), prm);
        if (rc) return rc;
        lap("build");
        stage(s.get());
        lap("stage");
    } catch (const std::bad_alloc&) {
        return fail(CRT_E_ALLOC, "out of host memory building the scene");
    }
    *out = s.release();
    return CRT_OK;
}

int crt_scene_info_get(const crt_scene* s, crt_scene_info* info) {
    clear_error();
    if (!s || !info) return fail(CRT_E_INVALID, "crt_scene_info_get: null argument");
    crt_scene_info r{};
    r.num_objects = s->num_objects;
    r.num_materials = s->num_materials;
    r.num_primitives = s->num_prims;
    r.num_spheres = s->num_spheres;
    r.num_parallelograms = s->num_quads;
    r.num_nodes = s->nodes.size();
    r.depth = s->depth;
    r.max_leaf_size = s->max_leaf;
    size_t off[kArrCount + 1];
    r.device_bytes = device_layout(s, off);  // the allocation device_upload makes
    r.build_ms = s->build_ms;
    *info = r;
    return CRT_OK;
}

int crt_scene_export_bvh(const crt_scene* s, crt_bvh_node* nodes, uint32_t* prim_order) {
    clear_error();
    if (!s) return fail(CRT_E_INVALID, "crt_scene_export_bvh: null scene");
    if (nodes) std::memcpy(nodes, s->nodes.data(), s->nodes.size() * sizeof(crt_bvh_node));
    if (prim_order) std::memcpy(prim_order, s->order.data(), s->order.size() * sizeof(uint32_t));
    return CRT_OK;
}

int crt_scene_upload(crt_scene* s, int device) {
    clear_error();
    if (!s) return fail(CRT_E_INVALID, "crt_scene_upload: null scene");
    return device_upload(s, device);
}

int crt_scene_image(crt_scene* s, int device, void* host, size_t bytes) {
    clear_error();
    if (!s || !host) return fail(CRT_E_INVALID, "crt_scene_image: null argument");
    return device_image(s, device, host, bytes);
}

void crt_scene_destroy(crt_scene* s) {
    if (!s) return;
    device_release(s);
    delete s;
}

int crt_camera_resolve(const crt_camera_settings* st, crt_camera* out) {
    clear_error();
    if (!st || !out) return fail(CRT_E_INVALID, "crt_camera_resolve: null argument");
    if (st->image_w == 0 || st->image_h == 0)
        return fail(CRT_E_INVALID, "crt_camera_resolve: empty image");
    resolve_camera(*st, *out);
    return CRT_OK;
}

int crt_device_count(int* count) {
    clear_error();
    if (!count) return fail(CRT_E_INVALID, "crt_device_count: null argument");
    return device_count(count);
}

int crt_render_async(const crt_scene* s, int device, const crt_camera* cam,
                     const crt_tiling* tiling, double* d_rgb, void* stream) {
    clear_error();
    if (!s || !cam || !d_rgb) return fail(CRT_E_INVALID, "crt_render_async: null argument");
    return device_render(s, device, cam, tiling, d_rgb, stream, nullptr);
}

int crt_render_count(const crt_scene* s, int device, const crt_camera* cam,
                     const crt_tiling* tiling, crt_render_stats* stats) {
    clear_error();
    if (!s || !cam || !stats) return fail(CRT_E_INVALID, "crt_render_count: null argument");
    return device_render(s, device, cam, tiling, nullptr, nullptr, stats);
}

int crt_render(crt_scene* s, const crt_camera* cam, int num_devices, double* h_rgb,
               crt_render_stats* stats) {
    clear_error();
    if (!s || !cam || !h_rgb) return fail(CRT_E_INVALID, "crt_render: null argument");
    return render_multi(s, cam, num_devices, h_rgb, stats);
}

int crt_render_ppm(crt_scene* s, const crt_camera* cam, int num_devices, int32_t* h_values,
                   crt_render_stats* stats) {
    clear_error();
    if (!s || !cam || !h_values) return fail(CRT_E_INVALID, "crt_render_ppm: null argument");
    return render_multi_ppm(s, cam, num_devices, h_values, stats);
}

int crt_ppm_values(int device, const double* d_rgb, size_t n, int32_t* h_values, void* stream) {
    clear_error();
    if (n && (!d_rgb || !h_values)) return fail(CRT_E_INVALID, "crt_ppm_values: null argument");
    return device_ppm_values(device, d_rgb, n, h_values, stream);
}

int crt_ppm_write(const char* path, uint32_t w, uint32_t h, const int32_t* values) {
    clear_error();
    if (!path || (static_cast<uint64_t>(w) * h && !values)) return fail(CRT_E_INVALID, "crt_ppm_write: null argument");
    std::FILE* f = std::fopen(path, "wb");
    if (!f) return fail(CRT_E_INVALID, std::string("crt_ppm_write: could not open the file \"") + path + "\"");
    std::string buf = "P3\n" + std::to_string(w) + " " + std::to_string(h) + "\n255\n";
    const uint64_t n = static_cast<uint64_t>(w) * h;
    bool ok = true;
    for (uint64_t p = 0; p < n && ok; ++p) {
        for (int k = 0; k < 3; ++k) {
            buf += std::to_string(values[3 * p + k]);
            buf += k < 2 ? ' ' : '\n';
        }
        if (buf.size() > (1u << 20)) {
            ok = std::fwrite(buf.data(), 1, buf.size(), f) == buf.size();
            buf.clear();
        }
    }
    if (ok && !buf.empty()) ok = std::fwrite(buf.data(), 1, buf.size(), f) == buf.size();
    ok = (std::fclose(f) == 0) && ok;
    return ok ? CRT_OK : fail(CRT_E_INVALID, std::string("crt_ppm_write: write failed: ") + path);
}

int crt_closest_hits(crt_scene* s, int device, const double* rays, size_t n, double t_min,
                     double t_max, crt_hit* out) {
    clear_error();
    if (!s || (n && (!rays || !out))) return fail(CRT_E_INVALID, "crt_closest_hits: null argument");
    return device_closest_hits(s, device, rays, n, t_min, t_max, out);
}

int crt_render_guard(crt_scene* s, int device, uint64_t* schlick_undecided, int reset) {
    clear_error();
    if (!s || !schlick_undecided) return fail(CRT_E_INVALID, "crt_render_guard: null argument");
    return device_guard(s, device, schlick_undecided, reset != 0);
}

}  // extern "C"
