// gfx950 render path: the reference's per-pixel/per-sample loop (camera.h:264-297), recursive
// integrator (camera.h:205-258), BVH traversal (bvh.h:585-715), primitive tests (sphere.h:45-96,
// parallelogram.h:177-240) and material scatter (material.h:64-263) as ONE kernel.
//
// Numerics: IEEE double throughout, compiled with -ffp-contract=off, every expression in the
// reference's operation order, so the geometry of each path (hit points, directions, RNG
// decisions) is bit-identical to the reference's for the same per-sample RNG stream. Radiance is
// accumulated forward (throughput) instead of by recursion; that re-association moves a
// sample's colour by a few ulps and never changes a path.
#include <hip/hip_runtime.h>

#define CRT_HD __host__ __device__ __forceinline__

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <string>
#include <mutex>
#include <thread>
#include <type_traits>
#include <vector>

#include "crt_internal.h"
#include "crt_schlick.h"

#pragma clang fp contract(off)

namespace crt {

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(CRT_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));    \
    } while (0)

namespace dev {

#ifndef CRT_BLOCK
#define CRT_BLOCK 256
#endif
constexpr int kBlock = CRT_BLOCK;
// pixel tile of one work item's 64 units (kTileW x kTileH owned rows): 16 x 4 matches the
// multi-GPU bench's 4-row blocks, so a tile is contiguous on the image at any GPU count
// (per-rank share at 8 GPUs 13.0 vs 13.2 ms for 8 x 8; one GPU 87.5 vs 87.0)
#ifndef CRT_TILE_W
#define CRT_TILE_W 16
#endif
constexpr uint32_t kTileW = CRT_TILE_W, kTileH = 64 / CRT_TILE_W;
// waves per SIMD of the W5 instances (the "five-wave" ones)
constexpr int kManyWaves = 5;
// the HBM-scene instances' sibling-pair walk (walk_pairs; 0 builds the one-node walk for A/B)
#ifndef CRT_PAIR_WALK
#define CRT_PAIR_WALK 1
#endif
constexpr double kScale = 1 / static_cast<double>(4294967295u - 1);  // rand_util.h:110-112

typedef double Dvec2 __attribute__((ext_vector_type(2)));
typedef uint32_t Uvec4 __attribute__((ext_vector_type(4)));

struct SceneView {
    const DevNode* nodes;      // f64 nodes (HBM): trace(), the walk's EXACT variant and fallback
    const DevNodeF* fnodes;    // f32 walk nodes (HBM), refs = byte offsets
    uint32_t ntop;             // HBM-scene kernels: f32 refs below ntop are read from the LDS copy
    const uint32_t* refs;
    const DevSphere* spheres;
    const DevSpherePair* spair;  // f32 filter records (HBM)
    uint32_t spair_lds;          // LSCENE kernels: LDS byte offset of the staged copy
    const uint32_t* sphere_mat;
    const DevQuad* quads;
    const uint32_t* quad_mat;
    const DevMaterial* mats;
    const DevQuadF* quadf;       // f32 filter records of the parallelograms (HBM)
    const DevMaterial* sphere_mrec;  // per-slot material records (shade)
    const DevMaterial* quad_mrec;
    uint32_t quadf_lds;          // LSCENE kernels: LDS byte offset of the staged copy
    const DevQuadBox* quadbox;   // flat boxes of axis-aligned parallelograms (HBM)
    // LSCENE kernels: LDS byte offsets of the staged refs / f64 spheres / parallelograms, read
    // through typed LDS pointers (ds_read, not flat); spheres_lds = ~0u when the spheres stay in HBM
    uint32_t refs_lds, spheres_lds, quads_lds;
    uint32_t inv64_lds;          // flat-parallelogram LDS kernels: the lanes' 1 / d ([k][lane] doubles)
    unsigned long long* guard;   // parity guard words (DeviceCopy::guard)
};

struct CamView {
    double o[3], p00[3], pdx[3], pdy[3], ddx[3], ddy[3];
    double defocus_angle;
    double bg[3];
    double t_min;
    double inv_spp;
    uint32_t w, h, spp, max_depth, base_seed;
};

struct Work {
    uint32_t owned_rows;   // rows of this tiling
    uint32_t row_block, tile_count, tile_index;
    // one launch renders a band of the owned frame: owned rows [k0, k0 + bh) x columns
    // [col0, col0 + bw), in kTileW x kTileH pixel tiles (launch_render: a band has at most 65535
    // tiles either way, so a tile's coordinates pack into 16 bits each, and its partial sums
    // stay within the partial-sum budget)
    uint32_t col0, k0, bw, bh;
    uint32_t tiles_x, tiles_y, tiles;
    uint32_t chunks, chunk_len;        // sample chunks per pixel
    // work queue, taken in order by the waves of a persistent grid (render_kernel): bulk items
    // (tile i / groups, chunks [(i % groups) * item_chunks, + item_chunks)), then tail items
    // (tile j / tail_chunks, chunk bulk_chunks + j % tail_chunks); 64 units per chunk
    // XCD-local queues (v12): the band's tiles (tile-major) are cut into `segments` contiguous
    // ranges, segment x = tiles [tiles * x / segments, tiles * (x + 1) / segments), each with its own
    // counter queue[x] (zeroed before the launch) over its items: its tiles' bulk items, then its
    // tiles' tail items. A wave starts on segment blockIdx % segments (blocks b and b + 8 share an
    // XCD and its L2) and moves on to the next segments when its own is dry.
    uint32_t* queue;
    uint32_t segments;      // 8, or 1 (CRT_XCD_QUEUES=0)
    uint32_t n_items, bulk_items;
    uint32_t item_chunks, groups, bulk_chunks, tail_chunks;
    uint32_t rb_shift;      // log2(row_block) when it is a power of two, else 32
    // LDS layout of the scene-staging kernels (byte offsets / 16-byte padded sizes)
    uint32_t lds_nodes, lds_refs, lds_spheres, lds_quads, lds_quadf, lds_stack;
    uint32_t bytes_nodes, bytes_refs, bytes_spheres, bytes_quads, bytes_quadf;
    uint32_t lds_sph64, bytes_sph64;  // sphere-only LDS scenes: the f64 spheres too, when they fit
    uint32_t sphere_only;   // every primitive is a sphere: refs[slot] == slot
    uint32_t exact_slab;    // the scene needs walk_step's EXACT variant for every ray
    uint32_t ntop;          // HBM-scene kernels: f32 nodes [0, ntop) bytes staged in LDS at offset 0
    uint32_t sentinel;      // the sentinel node's reference (byte offset into the f32 nodes)
    uint32_t lds_cam;       // LDS copy of the CamView (read where used: keeps it out of SGPRs)
    uint32_t lds_acc;       // five-wave instances: the lanes' pixel sums (3 x kBlock doubles)
    uint32_t lds_inv64;     // flat-parallelogram LDS instances: the lanes' 1 / d (3 x kBlock doubles)
    uint32_t packed;        // the output holds only the owned rows (CRT_TILING_PACKED)
    // instrumented pass only (COUNT): walk speculatively like the timed kernel (CRT_COUNT_SPEC=1),
    // count per-round lane numbers (CRT_ROUND_COUNTERS=1; their atomics shift the phase timings)
    uint32_t count_spec, round_counters;
    uint32_t f32_ok;        // node bounds fit the f32 walk's error analysis (else f64 decides)
    uint32_t pair_walk;     // HBM-scene kernels built with CRT_PAIR_WALK: walk_pairs for NaN-free rays
    uint32_t spheres_f32;   // sphere-only scene within the f32 filter's range (two-pass leaves)
    uint32_t quads_f32;     // parallelogram-only scene within its f32 filter's range (two-pass leaves)
    uint32_t quads_flat;    // ... and every parallelogram axis-aligned: pass 1 is the flat-box node test
    float tmin32;           // RN32(camera t_min)
};

struct Counters {
    unsigned long long rays, nodes, sphere_tests, quad_tests;
    unsigned long long cyc_walk, cyc_leaf, cyc_shade, cyc_total;  // wave cycles (instrumented pass)
    unsigned long long cyc_tail;  // from the wave's first idle lane (chunk done) to its end
    unsigned long long it_walk, it_leaf, it_shade;  // wave iterations (lane utilization)
    unsigned long long slow_nodes, it_slow;  // node tests decided in f64 (lanes / wave iterations)
    unsigned long long cand, it_cand;        // two-pass leaves: exact tests of candidates (lanes / wave iterations)
    // per traversal round (walk + leaf): rounds, lanes walking at its start, lanes holding a leaf
    // after the walk, lanes with a finished ray after the leaf step (CRT_DEBUG_COUNTERS)
    unsigned long long rounds, round_walkers, round_leaves, round_done, shade_rounds;
    unsigned long long cyc_draw, cyc_init;  // wave ticks drawing units / starting paths + traversal set-up
};

// one lane's counts in the instrumented pass, added to the 64-bit Counters when the lane ends, and
// before then whenever one of them passes 2^31 (flush_counts, once per shade round): a lane of the
// persistent grid traces units for the whole launch, and a small grid on a large frame would wrap
// 32-bit counts (64-bit lane counts would cost the instrumented kernel spills)
struct LaneCounters {
    uint32_t rays, nodes, sphere_tests, quad_tests;
    uint32_t it_walk, it_leaf, it_shade;
    uint32_t slow_nodes, it_slow;
    uint32_t cand, it_cand;
};

// adds a lane's counts to the launch's totals and clears them (iteration counters are incremented
// by whichever lane led that iteration)
__device__ __forceinline__ void flush_counts(LaneCounters& c, Counters* t) {
    using ull = unsigned long long;
    atomicAdd(&t->rays, static_cast<ull>(c.rays));
    atomicAdd(&t->nodes, static_cast<ull>(c.nodes));
    atomicAdd(&t->sphere_tests, static_cast<ull>(c.sphere_tests));
    atomicAdd(&t->quad_tests, static_cast<ull>(c.quad_tests));
    atomicAdd(&t->it_walk, static_cast<ull>(c.it_walk));
    atomicAdd(&t->it_leaf, static_cast<ull>(c.it_leaf));
    atomicAdd(&t->it_shade, static_cast<ull>(c.it_shade));
    atomicAdd(&t->slow_nodes, static_cast<ull>(c.slow_nodes));
    atomicAdd(&t->it_slow, static_cast<ull>(c.it_slow));
    atomicAdd(&t->cand, static_cast<ull>(c.cand));
    atomicAdd(&t->it_cand, static_cast<ull>(c.it_cand));
    c = LaneCounters{};
}

// counts one per wave: only the lowest active lane increments
__device__ __forceinline__ bool wave_leader() {
    const uint64_t m = __ballot(1);
    return (threadIdx.x & 63) == static_cast<uint32_t>(__ffsll(static_cast<long long>(m)) - 1);
}

// Debug builds only (-DCRT_WATCHDOG=1, never the library's default): every wave-level loop of
// the render kernel checks a deadline (3 s after the launch's first wave started) and, past it,
// the wave prints where it was and ends (s_endpgm), so a kernel that would spin forever finishes
// with a report instead of hanging the device (tools/gpu_watchdog.sh).
#ifndef CRT_WATCHDOG
#define CRT_WATCHDOG 0
#endif
#if CRT_WATCHDOG
__device__ unsigned long long crt_wd_deadline;
#define CRT_WD(id, a, b)                                                                                   \
    do {                                                                                                   \
        if (wall_clock64() > *(volatile unsigned long long*)&crt_wd_deadline) {                            \
            if (wave_leader())                                                                             \
                printf("crt watchdog: block %u wave %u loop %d a %u b %u\n", blockIdx.x, threadIdx.x >> 6,  \
                       (int)(id), (unsigned)(a), (unsigned)(b));                                            \
            __builtin_amdgcn_endpgm();                                                                     \
        }                                                                                                  \
    } while (0)
#else
#define CRT_WD(id, a, b) do {} while (0)
#endif

// ---- reference RNG (rand_util.h:85-117) with per-sample state ------------------------------
__device__ __forceinline__ double rnd(uint32_t& s, double lo, double hi) {
    s = 1664525u * s + 1013904223u;
    return lo + (hi - lo) * static_cast<double>(s) * kScale;
}
// rnd(s, -1, 1) and rnd(s, 0, 1) with one f64 operation fewer, bit for bit: (1 - -1) * x = 2x is
// exact (x < 2^32), and RN(2x * kScale) = RN(x * (2 kScale)) with 2 kScale exact; 0 + y = y for
// the y = RN(x * kScale) >= 0 here (+0 included)
__device__ __forceinline__ double rnd_pm1(uint32_t& s) {
    s = 1664525u * s + 1013904223u;
    return static_cast<double>(s) * (2 * kScale) + -1.0;
}
__device__ __forceinline__ double rnd_01(uint32_t& s) {
    s = 1664525u * s + 1013904223u;
    return static_cast<double>(s) * kScale;
}

__device__ __forceinline__ uint32_t sample_seed(uint32_t base, uint32_t pixel, uint32_t sample) {
    uint64_t z = (static_cast<uint64_t>(pixel) << 32) | sample;
    z += static_cast<uint64_t>(base) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return static_cast<uint32_t>(z ^ (z >> 32));
}

// sqrt(x) bit for bit for x in [2^-767, inf), given r = v_rsq_f64(x): hipcc's own gfx950
// expansion of the IEEE sqrt (Goldschmidt + two Newton corrections) without its small-x scaling
// and 0/inf fix-up, which are identities there. Outside that range: sqrt() itself.
__device__ __forceinline__ double sqrt_from_rsq(double x, double r) {
    if (__builtin_expect(!(x >= 0x1p-767 && x < __builtin_inf()), 0)) return sqrt(x);
    double g = x * r, h = r * 0.5;
    const double e = fma(-h, g, 0.5);
    g = fma(g, e, g);
    h = fma(h, e, h);
    double d = fma(-g, g, x);
    g = fma(d, h, g);
    d = fma(-g, g, x);
    return fma(d, h, g);
}

// The shading code's square roots and reciprocals (unit vectors, the Dielectric's sin and
// refraction) without the range scaling and special-case fix-ups of hipcc's IEEE expansions, in
// the five-wave sphere-only kernel instances (FAST; config 2 73.7 -> 73.1-73.4 ms); the others
// keep sqrt() and the division (config 3 90.0 -> 91.3 ms, config 4 139.1 -> 140.2 ms with them).
template <bool FAST>
__device__ __forceinline__ double sqrt_exact(double x) {
    if (FAST) return sqrt_from_rsq(x, __builtin_amdgcn_rsq(x));
    return sqrt(x);
}
// 1 / s bit for bit: hipcc's gfx950 division 1 / s is div_scale, v_rcp_f64, two Newton steps
// y = fma(y, fma(-s, y, 1), y), q = 1 * y, r = fma(-s, q, 1), div_fmas = fma(r, y, q), div_fixup.
// For |s| in [2^-500, 2^500] div_scale scales nothing (it returns its operand), div_fmas adds no
// scale and div_fixup returns its first operand (no NaN, inf, zero or denormal arises), so the
// same operations without those three are that division's result; outside the range: 1 / s.
__device__ __forceinline__ double recip_core(double s) {  // |s| in [2^-500, 2^500]
    double y = __builtin_amdgcn_rcp(s);
    y = fma(y, fma(-s, y, 1.0), y);
    y = fma(y, fma(-s, y, 1.0), y);
    return fma(fma(-s, y, 1.0), y, y);
}
template <bool FAST>
__device__ __forceinline__ double recip_exact(double s) {
    if (!FAST) return 1 / s;
    if (__builtin_expect(!(fabs(s) >= 0x1p-500 && fabs(s) <= 0x1p500), 0)) return 1 / s;
    return recip_core(s);
}

// Vec3D::random_unit_vector (vec3d.h:64-75): rejection in the cube, then * (1 / |v|)
template <bool FAST = false>
__device__ __forceinline__ void random_unit_vector(uint32_t& s, double& x, double& y, double& z) {
    double m2;
    do {
        x = rnd_pm1(s);
        y = rnd_pm1(s);
        z = rnd_pm1(s);
        m2 = x * x + y * y + z * z;
    } while (!(m2 < 1));
    double inv = recip_exact<FAST>(sqrt_exact<FAST>(x * x + y * y + z * z));
    x = x * inv;
    y = y * inv;
    z = z * inv;
}

// AABB::is_hit_by_optimized (aabb.h:132-174). The early returns of the reference are folded into
// one boolean (the tests have no side effects), so the whole node is loaded up front (four
// 16-byte loads) and the test runs without branches.
struct NodeRegs {
    double b[6];
    uint32_t index, count, axis, flags;
};

__device__ __forceinline__ NodeRegs load_node(const DevNode* nodes, uint32_t i) {
    const uint4* p = reinterpret_cast<const uint4*>(nodes + i);
    const uint4 q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
    NodeRegs n;
    n.b[0] = __hiloint2double(q0.y, q0.x);
    n.b[1] = __hiloint2double(q0.w, q0.z);
    n.b[2] = __hiloint2double(q1.y, q1.x);
    n.b[3] = __hiloint2double(q1.w, q1.z);
    n.b[4] = __hiloint2double(q2.y, q2.x);
    n.b[5] = __hiloint2double(q2.w, q2.z);
    n.index = q3.x;
    n.count = q3.y;
    n.axis = q3.z;
    n.flags = q3.w;
    return n;
}

__device__ __forceinline__ bool slab(const NodeRegs& n, const double o[3], const double inv[3],
                                     uint32_t neg, double tmin, double tmax) {
    // x[neg] / x[!neg]: neg bit k selects max as the entry bound on axis k
    const double bx0 = (neg & 1u) ? n.b[1] : n.b[0], bx1 = (neg & 1u) ? n.b[0] : n.b[1];
    const double by0 = (neg & 2u) ? n.b[3] : n.b[2], by1 = (neg & 2u) ? n.b[2] : n.b[3];
    const double bz0 = (neg & 4u) ? n.b[5] : n.b[4], bz1 = (neg & 4u) ? n.b[4] : n.b[5];
    double xtmin = (bx0 - o[0]) * inv[0];
    double xtmax = (bx1 - o[0]) * inv[0];
    const double ytmin = (by0 - o[1]) * inv[1];
    const double ytmax = (by1 - o[1]) * inv[1];
    const double ztmin = (bz0 - o[2]) * inv[2];
    const double ztmax = (bz1 - o[2]) * inv[2];
    const bool c1 = !(xtmin > ytmax || ytmin > xtmax);
    if (ytmin > xtmin) xtmin = ytmin;
    if (ytmax < xtmax) xtmax = ytmax;
    const bool c2 = !(xtmin > ztmax || ztmin > xtmax);
    if (ztmin > xtmin) xtmin = ztmin;
    if (ztmax < xtmax) xtmax = ztmax;
    return c1 & c2 & (xtmin < tmax) & (xtmax > tmin);
}

// Reciprocal of a ray's dot(d, d) for div_a: ia = RN(1 / a), or NaN when a is outside the range
// where div_a's corrections are exact (then div_a divides).
template <bool FAST = false>
__device__ __forceinline__ double recip_a(double a) {
    return (a >= 0x1p-500 && a <= 0x1p500) ? (FAST ? recip_core(a) : 1 / a) : __builtin_nan("");
}

// n / a correctly rounded from ia = RN(1/a): q0 = n * ia, then two residual corrections
// q += fma(-a, q, n) * ia (Markstein's theorem: with ia = RN(1/a) and q within 1 ulp, the
// corrected q is RN(n / a); the first correction makes q faithful). No over/underflow for
// |n|, a in [2^-500, 2^500]; anything else divides.
__device__ __forceinline__ double div_a(double n, double a, double ia) {
    const double an = fabs(n);
    if (__builtin_expect(!(an >= 0x1p-500 && an <= 0x1p500 && ia == ia), 0)) return n / a;
    double q = n * ia;
    q = fma(fma(-a, q, n), ia, q);
    return fma(fma(-a, q, n), ia, q);
}

// Sphere::hit_by (sphere.h:45-96) returning the accepted root through t.
// Before the exact sqrt and divisions, a coarse bound (hardware rsq, error <= 2^-23 relative;
// margins of 2^-12 on every term) proves "both roots >= t_max" or "both roots <= t_min" for
// spheres that cannot be accepted; only those are skipped, so the accepted roots are exactly the
// reference's. NaN/inf anywhere makes the bound inconclusive and falls through to the exact test.
// The sqrt and the two divisions by a are the correctly rounded ones (sqrt_from_rsq, div_a with
// ia = recip_a(a)); lo / hi are lim_tmin / lim_tmax of the current t_min / t_max.
// Coarse-reject limits of hit_sphere: t * a scaled outward by 2^-30 (tmin side: inward).
__device__ __forceinline__ double lim_tmax(double tmax, double a) { return tmax * a * (1 + 0x1p-30); }
__device__ __forceinline__ double lim_tmin(double tmin, double a) { return tmin * a * (1 - 0x1p-30); }

// COARSE = false skips the coarse reject (the candidates of two-pass leaves passed a filter).
template <bool COARSE = true>
__device__ __forceinline__ bool hit_sphere(const DevSphere& sp, const double o[3], const double d[3],
                                           double a, double ia, double tmin, double tmax, double lo,
                                           double hi, double& t) {
    double ocx = o[0] - sp.c[0], ocy = o[1] - sp.c[1], ocz = o[2] - sp.c[2];
    double b = d[0] * ocx + d[1] * ocy + d[2] * ocz;
    double c = (ocx * ocx + ocy * ocy + ocz * ocz) - sp.r * sp.r;
    double disc = b * b - a * c;
    if (disc < 0) return false;
    const double rs = __builtin_amdgcn_rsq(disc);
    if (COARSE) {
        const double sqa = disc * rs;                              // ~sqrt(disc)
        const double m = (fabs(b) + sqa) * 0x1p-12;                // covers every rounding error
        const bool beyond = (-b - sqa) - m > hi;   // r1 > tmax, so r2 too  (hi = lim_tmax)
        const bool before = (-b + sqa) + m < lo;   // r2 < tmin, so r1 too  (lo = lim_tmin)
        if (beyond || before) return false;
    }
    double sq = sqrt_from_rsq(disc, rs);
    double root = div_a(-b - sq, a, ia);
    if (!(tmin < root && root < tmax)) {
        root = div_a(-b + sq, a, ia);
        if (!(tmin < root && root < tmax)) return false;
    }
    t = root;
    return true;
}

// v_min/v_max(3)_f32 of non-NaN operands. Written out because fminf/fmaxf make the compiler
// quieten possible signalling NaNs of operands it cannot prove canonical (tmin', tmax') with an
// extra v_max each, in every walk step.
__device__ __forceinline__ float vmin(float a, float b) { float r; asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
__device__ __forceinline__ float vmax(float a, float b) { float r; asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
__device__ __forceinline__ float vmin3(float a, float b, float c) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// b wave-uniform, in an SGPR
__device__ __forceinline__ float vmax_s(float a, float b) { float r; asm("v_max_f32 %0, %2, %1" : "=v"(r) : "v"(a), "s"(b)); return r; }
__device__ __forceinline__ float vmax_abs(float a, float b) {
    float r;
    asm("v_max_f32 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float vmax3_0(float a, float b) {  // max(a, b, 0)
    float r;
    asm("v_max3_f32 %0, %1, %2, 0" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float vmax3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// the kernel's min / max for crt_quad_filter.h flat_box_candidate
struct DevMinMax {
    static __device__ __forceinline__ float min(float a, float b) { return vmin(a, b); }
    static __device__ __forceinline__ float max(float a, float b) { return vmax(a, b); }
    static __device__ __forceinline__ float min3(float a, float b, float c) { return vmin3(a, b, c); }
    static __device__ __forceinline__ float max3(float a, float b, float c) { return vmax3(a, b, c); }
    static __device__ __forceinline__ float max_s(float a, float b) { return vmax_s(a, b); }
    static __device__ __forceinline__ float max_abs(float a, float b) { return vmax_abs(a, b); }
};

// The candidate filter of two-pass sphere leaves, two spheres per step in packed f32
// (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: one instruction for both spheres). It returns two
// bits, false only where the exact test (hit_sphere, i.e. Sphere::hit_by) provably rejects the
// sphere for every t_max' <= t_max. No square root: with y = -b - hi and w = b + lo,
//   no real root          <=  D < 0
//   both roots >= t_max   <=  y > 0 and y^2 > D
//   both roots <= t_min   <=  w > 0 and w^2 > D
// i.e. reject <=> max(y|y|, w|w|, 0) > D, where D bounds the exact test's discriminant from above
// with room to spare:
//   D = b'^2 - a' (q' (1 - 2^-15) - r2e - kap),  b' = d32 . X, q' = X . X, X = o32 - c32,
//   r2e = RN32(r^2 (1 + 2^-14) + 2^22 |c - c32|^2)  (per sphere, DevSpherePair),
//   kap = RN32(2^22 |o - o32|^2 + 2^-50)           (per ray),
// and hi = RN32(t_max a (1 + 2^-20)), lo = RN32(t_min a (1 - 2^-20)). Error budget: with
// S = a (|oc|^2 + r^2) >= b^2, |disc|, and Delta = |o - o32| + |c - c32| (the rounding of the
// inputs), every f32 rounding error is below 2^-19 S, and the terms in Delta are at most
// 4 a |oc| Delta + 2 a Delta^2 <= 2^-17 a |oc|^2 + 2^20 a Delta^2 (AM-GM); the slack of D,
// 2^-15 a q' + 2^-14 a r^2 + 2^22 a (|o - o32|^2 + |c - c32|^2) >= those, also covers the error of
// b' inside y and w (2 |y| |b' - b| <= 2^-18 a q + 2^18 a Delta^2), and hi / lo carry a 2^-20
// relative slack for the rounding of the exact roots (the f64 analysis: 2^-30). A sphere the
// filter rejects is rejected by the exact test for this t_max and any smaller one, so hits and
// the tie order are the sequential loop's. Valid for |o_k|, |d_k|, |c_k|, |r| <= 2^30 and
// a in [2^-60, 2^60] (leaf_step checks; W.spheres_f32 for the scene).
// tools/fuzz_sphere_filter.c checks the filter (this exact f32 sequence) against the exact test.
typedef float F2 __attribute__((ext_vector_type(2)));
// The ray in f32 for the packed filter (per entered leaf), two scalars per register pair; the
// packed instructions broadcast one half with op_sel / op_sel_hi (no splatted copies: 10 VGPRs
// instead of 20 while the leaf phase runs).
struct LeafRay32 {
    F2 oxy, ozdx, dydz, akap, hilo;  // (ox, oy) (oz, dx) (dy, dz) (a, kap) (hi, lo)
};
__device__ __forceinline__ void leaf_ray32(const double o[3], const double d[3], double a, double tmin,
                                           double tmax, LeafRay32& L) {
    float o32[3];
    double e2 = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        o32[k] = static_cast<float>(o[k]);
        const double e = o[k] - static_cast<double>(o32[k]);
        e2 = e2 + e * e;
    }
    L.oxy = F2{o32[0], o32[1]};
    L.ozdx = F2{o32[2], static_cast<float>(d[0])};
    L.dydz = F2{static_cast<float>(d[1]), static_cast<float>(d[2])};
    L.akap = F2{static_cast<float>(a), static_cast<float>(e2 * 0x1p22 + 0x1p-50)};
    L.hilo = F2{static_cast<float>(tmax * a * (1 + 0x1p-20)), static_cast<float>(tmin * a * (1 - 0x1p-20))};
}
__device__ __forceinline__ bool leaf_ray32_ok(const double o[3], const double d[3], double a) {
    bool ok = a >= 0x1p-60 && a <= 0x1p60;
#pragma unroll
    for (int k = 0; k < 3; ++k) ok = ok && fabs(o[k]) <= 0x1p30 && fabs(d[k]) <= 0x1p30;
    return ok;
}
__device__ __forceinline__ float vmul_abs(float a, float b) {  // a * |b|
    float r;
    asm("v_mul_f32 %0, %1, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// packed f32 with one operand broadcast from the low (_L) or high (_H) half of a ray pair p
__device__ __forceinline__ F2 sub_pL(F2 p, F2 c) {  // (p.x, p.x) - c
    F2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel_hi:[0,1] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(p), "v"(c));
    return r;
}
__device__ __forceinline__ F2 sub_pH(F2 p, F2 c) {  // (p.y, p.y) - c
    F2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(p), "v"(c));
    return r;
}
__device__ __forceinline__ F2 add_pH(F2 p, F2 c) {  // (p.y, p.y) + c
    F2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(r) : "v"(p), "v"(c));
    return r;
}
__device__ __forceinline__ F2 mul_pL(F2 p, F2 c) {  // (p.x, p.x) * c
    F2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(r) : "v"(p), "v"(c));
    return r;
}
__device__ __forceinline__ F2 mul_pH(F2 p, F2 c) {  // (p.y, p.y) * c
    F2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(r) : "v"(p), "v"(c));
    return r;
}
__device__ __forceinline__ F2 fma_pL(F2 p, F2 c, F2 e) {  // fma((p.x, p.x), c, e)
    F2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(r) : "v"(p), "v"(c), "v"(e));
    return r;
}
__device__ __forceinline__ F2 fma_pH(F2 p, F2 c, F2 e) {  // fma((p.y, p.y), c, e)
    F2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "=v"(r) : "v"(p), "v"(c), "v"(e));
    return r;
}
__device__ __forceinline__ F2 nsub_pL(F2 b, F2 p) {  // -b - (p.x, p.x)
    F2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel_hi:[1,0] neg_lo:[1,1] neg_hi:[1,1]" : "=v"(r) : "v"(b), "v"(p));
    return r;
}
__device__ __forceinline__ F2 add_bH(F2 b, F2 p) {  // b + (p.y, p.y)
    F2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(r) : "v"(b), "v"(p));
    return r;
}
// records read through explicitly typed LDS / global pointers (a generic pointer would make the
// compiler emit flat loads), as 16-byte vectors
typedef float Fvec4 __attribute__((ext_vector_type(4)));
struct PairLines {
    Fvec4 c;   // cx0 cx1 cy0 cy1
    Fvec4 zr;  // cz0 cz1 r2e0 r2e1
};
typedef __attribute__((address_space(3))) const PairLines LdsPair;
typedef __attribute__((address_space(1))) const PairLines GlobalPair;
template <typename P>
__device__ __forceinline__ DevSpherePair pair_at(P p) {
    const Fvec4 c = p->c, zr = p->zr;
    DevSpherePair r;
    r.cx[0] = c.x; r.cx[1] = c.y; r.cy[0] = c.z; r.cy[1] = c.w;
    r.cz[0] = zr.x; r.cz[1] = zr.y; r.r2e[0] = zr.z; r.r2e[1] = zr.w;
    return r;
}
struct SphereLines {
    Dvec2 a, b;  // (cx, cy), (cz, r)
};
typedef __attribute__((address_space(1))) const SphereLines GlobalSphere;
__device__ __forceinline__ DevSphere sphere_global(const DevSphere* p) {
    const GlobalSphere* q = (GlobalSphere*)p;
    const Dvec2 a = q->a, b = q->b;
    DevSphere r;
    r.c[0] = a.x; r.c[1] = a.y; r.c[2] = b.x; r.r = b.y;
    return r;
}
// an f32 parallelogram record in HBM through a typed global pointer (4 x 16-byte loads)
typedef __attribute__((address_space(1))) const Fvec4 GlobalFvec4;
__device__ __forceinline__ DevQuadF quadf_global(const DevQuadF* p) {
    const GlobalFvec4* q = (GlobalFvec4*)p;
    DevQuadF r;
    Fvec4* dst = reinterpret_cast<Fvec4*>(&r);
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[k] = q[k];
    return r;
}
// a 16-byte aligned record (DevSphere, DevQuad, u32) at an LDS byte offset, read as ds_read
typedef __attribute__((address_space(3))) const Dvec2 LdsDvec2;
template <typename T>
__device__ __forceinline__ T lds_rec(uint32_t off) {
    static_assert(sizeof(T) % 16 == 0, "16-byte lines");
    T r;
    Dvec2* dst = reinterpret_cast<Dvec2*>(&r);
    const LdsDvec2* src = (LdsDvec2*)static_cast<uintptr_t>(off);
#pragma unroll
    for (uint32_t k = 0; k < sizeof(T) / 16; ++k) dst[k] = src[k];
    return r;
}
__device__ __forceinline__ uint32_t lds_u32(uint32_t off) {
    return *(__attribute__((address_space(3))) const uint32_t*)static_cast<uintptr_t>(off);
}
// the verdicts of the record's two spheres shifted into cand: bit 1 = first, bit 0 = second
// (1 = candidate); cand = cand + cand + verdict by v_addc_co_u32 with the compare's VCC as the
// carry (written out: the compiler turns the C form into a shift, two selects and an or); the
// s_nop 1 is the VALU-writes-VCC -> VALU-reads-VCC hazard the compiler pads the same way
__device__ __forceinline__ uint32_t sphere_pair_candidates(uint32_t cand, const DevSpherePair& sp, const LeafRay32& L) {
    const F2 cx = {sp.cx[0], sp.cx[1]}, cy = {sp.cy[0], sp.cy[1]}, cz = {sp.cz[0], sp.cz[1]};
    const F2 r2e = {sp.r2e[0], sp.r2e[1]};
    const F2 xx = sub_pL(L.oxy, cx), xy = sub_pH(L.oxy, cy), xz = sub_pL(L.ozdx, cz);
    const F2 b = fma_pH(L.dydz, xz, fma_pL(L.dydz, xy, mul_pH(L.ozdx, xx)));
    const F2 q = __builtin_elementwise_fma(xz, xz, __builtin_elementwise_fma(xy, xy, xx * xx));
    const F2 g = __builtin_elementwise_fma(q, F2{1 - 0x1p-15f, 1 - 0x1p-15f}, -add_pH(L.akap, r2e));
    const F2 D = __builtin_elementwise_fma(b, b, -mul_pL(L.akap, g));
    const F2 y = nsub_pL(b, L.hilo), w = add_bH(b, L.hilo);
    const float m0 = vmax3_0(vmul_abs(y.x, y.x), vmul_abs(w.x, w.x));
    const float m1 = vmax3_0(vmul_abs(y.y, y.y), vmul_abs(w.y, w.y));
    asm volatile("v_cmp_ngt_f32 vcc, %1, %2\n\ts_nop 1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc"
                 : "+v"(cand) : "v"(m0), "v"(D.x) : "vcc");
    asm volatile("v_cmp_ngt_f32 vcc, %1, %2\n\ts_nop 1\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc"
                 : "+v"(cand) : "v"(m1), "v"(D.y) : "vcc");
    return cand;
}

// Parallelogram::hit_by (parallelogram.h:177-240)
__device__ __forceinline__ bool hit_quad(const DevQuad& q, const double o[3], const double d[3],
                                         double tmin, double tmax, double& t) {
    double den = q.n[0] * d[0] + q.n[1] * d[1] + q.n[2] * d[2];
    if (fabs(den) < 1e-9) return false;
    double vx = q.v[0] - o[0], vy = q.v[1] - o[1], vz = q.v[2] - o[2];
    double ht = (q.n[0] * vx + q.n[1] * vy + q.n[2] * vz) / den;
    if (!(tmin < ht && ht < tmax)) return false;
    double px = o[0] + d[0] * ht, py = o[1] + d[1] * ht, pz = o[2] + d[2] * ht;
    double wx = px - q.v[0], wy = py - q.v[1], wz = pz - q.v[2];
    // alpha = dot(sn, cross(w, s2)); beta = dot(sn, cross(s1, w))
    double c1x = wy * q.s2[2] - wz * q.s2[1];
    double c1y = wz * q.s2[0] - wx * q.s2[2];
    double c1z = wx * q.s2[1] - wy * q.s2[0];
    double alpha = q.sn[0] * c1x + q.sn[1] * c1y + q.sn[2] * c1z;
    double c2x = q.s1[1] * wz - q.s1[2] * wy;
    double c2y = q.s1[2] * wx - q.s1[0] * wz;
    double c2z = q.s1[0] * wy - q.s1[1] * wx;
    double beta = q.sn[0] * c2x + q.sn[1] * c2y + q.sn[2] * c2z;
    if (0 <= alpha && alpha <= 1 && 0 <= beta && beta <= 1) {
        t = ht;
        return true;
    }
    return false;
}

// sphere i: LS kernels read the LDS copy or, in the f32-filter mode, HBM through a typed pointer
template <bool LS>
__device__ __forceinline__ DevSphere sphere_at(const SceneView& S, uint32_t i) {
    if (!LS) return S.spheres[i];
    return S.spheres_lds != ~0u ? lds_rec<DevSphere>(S.spheres_lds + (i << 5)) : sphere_global(S.spheres + i);
}

// Resolve the hit record (hittable.h:46-71): hit point ray(t), outward normal, front face.
// IR: the sphere's 1/r comes in as ir (shade: the slot's material record holds RN(1/r), the
// same value the division gives); otherwise it is divided here.
template <bool LS, bool IR = false, bool SPH = false, bool QONLY = false>
__device__ __forceinline__ uint32_t hit_record(const SceneView& S, uint32_t ref, const double o[3],
                                               const double d[3], double t, double p[3],
                                               double nrm[3], bool& front, double ir_in = 0) {
    p[0] = o[0] + d[0] * t;
    p[1] = o[1] + d[1] * t;
    p[2] = o[2] + d[2] * t;
    double nx, ny, nz;
    uint32_t m;
    if (QONLY || (!SPH && (ref & kRefQuad))) {
        if constexpr (LS) {
            const DevQuad q = lds_rec<DevQuad>(S.quads_lds + ((ref & ~kRefQuad) << 7));
            nx = q.n[0]; ny = q.n[1]; nz = q.n[2];
        } else {
            const DevQuad& q = S.quads[ref & ~kRefQuad];
            nx = q.n[0]; ny = q.n[1]; nz = q.n[2];
        }
        m = S.quad_mat[ref & ~kRefQuad];
    } else {
        const auto normal = [&](const DevSphere& sp) {
            const double ir = IR ? ir_in : 1 / sp.r;  // (hit_point - center) / radius
            nx = (p[0] - sp.c[0]) * ir;
            ny = (p[1] - sp.c[1]) * ir;
            nz = (p[2] - sp.c[2]) * ir;
        };
        if constexpr (LS) normal(sphere_at<LS>(S, ref));
        else normal(S.spheres[ref]);
        m = S.sphere_mat[ref];
    }
    if (d[0] * nx + d[1] * ny + d[2] * nz > 0) {
        nrm[0] = -nx; nrm[1] = -ny; nrm[2] = -nz;
        front = false;
    } else {
        nrm[0] = nx; nrm[1] = ny; nrm[2] = nz;
        front = true;
    }
    return m;
}

// Per-lane traversal stack, interleaved [level][lane] so a wave's pushes hit distinct banks
// (LDS) or whole lines (HBM fallback for trees deeper than the LDS budget). Entries are u16 when
// the BVH has < 65536 nodes.
template <typename SE>
struct Stack {
    SE* base;
    uint32_t stride;
    __device__ __forceinline__ void put(int i, uint32_t v) { base[static_cast<size_t>(i) * stride] = static_cast<SE>(v); }
    __device__ __forceinline__ uint32_t get(int i) const { return base[static_cast<size_t>(i) * stride]; }
};

// BVH::hit_by (bvh.h:585-715): iterative DFS over the preorder nodes, near child first by the
// sign of the ray direction on the split axis, leaf primitives in order shrinking t_max.
// Control flow is "while-while" (Aila & Laine 2009): a lane walks interior nodes until it enters
// a leaf (or finishes), and the wave then tests all lanes' leaves together, so the primitive loop
// runs with most lanes active. Per lane, the sequence of node tests and primitive tests is
// exactly the reference's.
template <typename SE, bool COUNT>
__device__ __forceinline__ bool trace(const SceneView& S, Stack<SE>& st, const double o[3],
                                      const double d[3], double tmin, double& tmax,
                                      uint32_t& hit_ref, LaneCounters& ctr) {
    const double inv[3] = {1 / d[0], 1 / d[1], 1 / d[2]};
    const uint32_t neg = (d[0] < 0 ? 1u : 0u) | (d[1] < 0 ? 2u : 0u) | (d[2] < 0 ? 4u : 0u);
    const double a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];  // dot(ray.dir, ray.dir)
    const double ia = recip_a(a), lo = lim_tmin(tmin, a);
    double hi = lim_tmax(tmax, a);
    bool found = false;
    int sp = 0;
    uint32_t cur = 0;
    bool done = false;
    while (!done) {
        uint32_t first = 0, count = 0;
        while (true) {  // interior walk until a leaf is entered
            const NodeRegs n = load_node(S.nodes, cur);
            if (COUNT) ctr.nodes++;
            const bool enter = slab(n, o, inv, neg, tmin, tmax) | (n.count > 0 && (n.flags & kNodeAlways) != 0);
            if (enter) {
                if (n.count > 0) {
                    first = n.index;
                    count = n.count;
                    break;
                }
                if ((neg >> n.axis) & 1u) {  // children: left = flags, right = index
                    st.put(sp++, n.flags);
                    cur = n.index;
                } else {
                    st.put(sp++, n.index);
                    cur = n.flags;
                }
            } else {
                if (sp == 0) {
                    done = true;
                    break;
                }
                cur = st.get(--sp);
            }
        }
        for (uint32_t i = first; i < first + count; ++i) {  // the entered leaf's primitives
            const uint32_t ref = S.refs[i];
            double t;
            bool h;
            if (ref & kRefQuad) {
                if (COUNT) ctr.quad_tests++;
                h = hit_quad(S.quads[ref & ~kRefQuad], o, d, tmin, tmax, t);
            } else {
                if (COUNT) ctr.sphere_tests++;
                h = hit_sphere(S.spheres[ref], o, d, a, ia, tmin, tmax, lo, hi, t);
            }
            if (h) {
                tmax = t;
                hi = lim_tmax(t, a);
                hit_ref = ref;
                found = true;
            }
        }
        if (count > 0) {
            if (sp == 0) done = true;
            else cur = st.get(--sp);
        }
    }
    return found;
}

// Per-lane traversal state of the render kernel's current ray. The kernel advances it one BVH
// node per iteration (walk) and tests an entered leaf's primitives in a separate, batched phase;
// per lane the sequence of node tests and primitive tests is exactly trace()'s, i.e. the
// reference's BVH::hit_by.
enum : uint32_t { kWalk = 0, kLeaf = 1, kDone = 2, kIdle = 3 };

constexpr uint32_t kZeroDir = 8u;

struct Trav {
    // f32 copies for the walk's node test (walk()): inv32 = RN32(1/d), oinv32 = RN32(o * (1/d)),
    // marg = the per-ray part of the decision margin (inf: every node test is decided in f64)
    float inv32[3], oinv32[3];
    float marg;
    float tmax32;    // RN32(min(tmax, 2^100))
    double a;        // dot(d, d)
    double tmax;
    uint32_t cur, ref;
    int32_t sp;      // stack levels in use; -1 after the pop that follows the last leaf
    uint32_t first, count;  // the entered leaf's primitive range (walk -> leaf_step)
    uint32_t neg;    // bit k: d[k] < 0; kZeroDir: a slab value may be NaN (walk_step EXACT)
    uint32_t state;
    bool found;
};

__device__ __forceinline__ bool finite_nonzero(double x) { return fabs(x) < __builtin_inf() && x != 0; }
__device__ __forceinline__ bool finite(double x) { return fabs(x) < __builtin_inf(); }
__device__ __forceinline__ float tmax_f32(double t) { return static_cast<float>(fmin(t, 0x1p100)); }

__device__ __forceinline__ bool dir_ok(double x) { return fabs(x) >= 0x1p-1000 && fabs(x) <= 0x1p1000; }

// f32_ok: the scene's node bounds fit the f32 error analysis (Work::f32_ok)
__device__ __forceinline__ void trav_init(const double o[3], const double d[3], bool f32_ok, Trav& R) {
    R.a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
    R.tmax = __builtin_inf();
    R.tmax32 = 0x1p100f;
    R.cur = 0;
    R.sp = 0;
    R.ref = 0;
    // NaN-free slab values (the min/max and f32 walks): 1/d finite and non-zero, o finite. Rays
    // with a direction component outside [2^-1000, 2^1000] (zero, tiny, huge, NaN) take the EXACT
    // walk, which is the reference's select sequence for any ray.
    const bool fast = dir_ok(d[0]) && dir_ok(d[1]) && dir_ok(d[2]) &&
                      finite(o[0]) && finite(o[1]) && finite(o[2]);
    R.neg = (d[0] < 0 ? 1u : 0u) | (d[1] < 0 ? 2u : 0u) | (d[2] < 0 ? 4u : 0u) | (fast ? 0u : kZeroDir);
    // The f32 walk's ray constants, in f32 (v12): inv32 = v_rcp_f32(RN32(d)) (within 1 ulp of
    // 1/RN32(d), so within 3.01u of 1/d), oinv32 = RN32(RN32(o) * inv32) (within 5.02u of o/d);
    // walk() bounds the resulting slab values for these. The analysis holds for
    // 2^-40 <= |1/d_k| <= 2^40 and |o_k| <= 2^40, here ensured by 2^-39 <= |RN32(d_k)| <= 2^39;
    // other rays get marg = inf, i.e. every node test decided in f64.
    bool f32 = f32_ok;
    float A = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float d32 = static_cast<float>(d[k]), o32 = static_cast<float>(o[k]);
        R.inv32[k] = __builtin_amdgcn_rcpf(d32);
        R.oinv32[k] = o32 * R.inv32[k];
        A = __builtin_fmaxf(A, __builtin_fabsf(R.oinv32[k]));
        f32 = f32 && __builtin_fabsf(d32) <= 0x1p39f && __builtin_fabsf(d32) >= 0x1p-39f &&
              __builtin_fabsf(o32) <= 0x1p40f;
    }
    R.marg = f32 ? __builtin_fmaxf(A * 0x1p-19f, 0x1p-60f) : __builtin_inff();
    R.state = kWalk;
    R.found = false;
}

// ---- the render kernel's BVH walk ------------------------------------------------------------
// One node of the DFS (bvh.h:617-712 loop body without the leaf's primitive loop), branch-free:
// the node and the stack top are loaded in one batch, and the push / pop / leaf / done outcomes
// are selected rather than branched to (only the push is a masked store).
//
// Node test (AABB::is_hit_by_optimized, aabb.h:132-174). The reference swaps each axis' (t0, t1)
// by the sign of d and then narrows with "if (y > x) x = y"-style selects; for NaN-free slab
// values that is exactly
//   near = max_k min(t0_k, t1_k), far = min_k max(t0_k, t1_k),
//   enter = near <= far && near < tmax && far > tmin
// (c1 && c2 of the reference <=> every near_i <= far_j; +-0 ties only meet comparisons), with
// t_jk = RN(RN(b_jk - o_k) * inv_k) in f64. A slab value is NaN only for 0 * inf or inf - inf:
// rays whose 1/d is not finite and non-zero or whose origin is not finite (R.neg & kZeroDir), and
// scenes with an inverted / NaN node box (Work::exact_slab, where min/max would reorder the axis)
// take the EXACT variant: the reference's select sequence verbatim on the f64 node.
//
// The other rays decide the test in f32 first (Trav::inv32 / oinv32 / marg, DevNodeF):
//   t'_jk = fma(b32_jk, inv32_k, -oinv32_k),  b32 = RN32(b), inv32 = v_rcp_f32(RN32(d)) within
//   3.01u of inv = 1/d, oinv32 = RN32(RN32(o) * inv32) within 5.02u of o inv (trav_init; u =
//   2^-24). With A = max_k |o_k inv_k| and |b| <= |b - o| + |o|:
//   |t' - t| <= 4.01u |b||inv| + 5.02u |o||inv| + u |t'| + 2.01 u64 |t|
//            <= 5.02u |t'| + 9.04u A + 2^-85 = 2^-21.7 |t'| + 2^-20.8 A + 2^-85
// (2^-85: f32 underflow at |inv| <= 2^40). min / max are 1-Lipschitz, so lo' = max(near', tmin')
// and hi' = min(far', tmax') are within that bound of lo = max(near, tmin), hi = min(far, tmax)
// with |t'| <= M = max(|lo'|, |hi'|) (tmin', tmax' are RN32 of tmin, tmax, within u M; tmax' =
// 2^100 for larger tmax never binds, as |t'| < 2^82 here), and gap' = RN32(hi' - lo') is within
// 14.1u M + 18.1u A + 2^-84 <= 2^-20.1 M + 2^-19.8 A + 2^-84 of gap = hi - lo. So with
// th = 2^-19 M + marg, marg = max(2^-19 A', 2^-60), A' = max_k |oinv32_k| >= A (1 - 5.1u):
//   gap' >  th  =>  gap > 0: far > near, near < tmax, far > tmin  (enter)
//   gap' < -th  =>  gap < 0: far < near, far < tmin or tmax < near (no entry)
// and only lanes with |gap'| <= th (grazing rays, ties, rays with marg = inf) run the f64 test on
// the f64 node. Every decision is the f64 test's, so each ray visits the reference's node
// sequence. The f32 test is 18 single-rate instructions where the f64 one is 25 half-rate ones.
typedef __attribute__((address_space(3))) const unsigned char LdsByte;
struct NodeLines {
    Dvec2 b[3];  // (x.min, x.max), (y.min, y.max), (z.min, z.max)
    Uvec4 meta;  // index count axis flags
};
template <typename P>
__device__ __forceinline__ void node_lines(P p, NodeLines& n) {
    n.b[0] = p->b[0];
    n.b[1] = p->b[1];
    n.b[2] = p->b[2];
    n.meta = p->meta;
}
typedef __attribute__((address_space(1))) const NodeLines GlobalNode;
// the f64 node behind f32 ref `cur`
__device__ __forceinline__ GlobalNode* node64(const SceneView& S, uint32_t cur) {
    return (GlobalNode*)(S.nodes + (cur >> kNodeFShift));
}

// the f64 min/max test of a NaN-free ray (the f32 test's fallback)
__device__ __forceinline__ bool slab64(GlobalNode* p, const double o[3], const double d[3], double tmin,
                                       double tmax) {
    NodeLines nd;
    node_lines(p, nd);
    // divided here, in the rare branch: hoisted out of the walk loop, 1/d would hold 6 VGPRs
    double dx = d[0], dy = d[1], dz = d[2];
    asm volatile("" : "+v"(dx), "+v"(dy), "+v"(dz));
    const double inv[3] = {1 / dx, 1 / dy, 1 / dz};
    const Dvec2 bx = nd.b[0], by = nd.b[1], bz = nd.b[2];
    const double x0 = (bx.x - o[0]) * inv[0], x1 = (bx.y - o[0]) * inv[0];
    const double y0 = (by.x - o[1]) * inv[1], y1 = (by.y - o[1]) * inv[1];
    const double z0 = (bz.x - o[2]) * inv[2], z1 = (bz.y - o[2]) * inv[2];
    const double near = fmax(fmax(fmin(x0, x1), fmin(y0, y1)), fmin(z0, z1));
    const double far = fmin(fmin(fmax(x0, x1), fmax(y0, y1)), fmax(z0, z1));
    return (near <= far) & (near < tmax) & (far > tmin);
}

// the same test with the lane's 1 / d read from LDS (S.inv64_lds, written by the traversal set-up
// with the same division): the flat-parallelogram instances, whose walk decides ~28% of its
// iterations in f64 (Cornell's box faces lie on node bounds)
__device__ __forceinline__ bool slab64_inv(GlobalNode* p, const double o[3], uint32_t inv_lds, double tmin,
                                           double tmax) {
    NodeLines nd;
    node_lines(p, nd);
    typedef __attribute__((address_space(3))) const double LdsDoubleC;
    uint32_t t = threadIdx.x;
    asm volatile("" : "+v"(t));  // recomputed here, not held live across the walk
    LdsDoubleC* q = (LdsDoubleC*)static_cast<uintptr_t>(inv_lds + t * 8);
    const double inv[3] = {q[0], q[kBlock], q[2 * kBlock]};
    const Dvec2 bx = nd.b[0], by = nd.b[1], bz = nd.b[2];
    const double x0 = (bx.x - o[0]) * inv[0], x1 = (bx.y - o[0]) * inv[0];
    const double y0 = (by.x - o[1]) * inv[1], y1 = (by.y - o[1]) * inv[1];
    const double z0 = (bz.x - o[2]) * inv[2], z1 = (bz.y - o[2]) * inv[2];
    const double near = fmax(fmax(fmin(x0, x1), fmin(y0, y1)), fmin(z0, z1));
    const double far = fmin(fmin(fmax(x0, x1), fmax(y0, y1)), fmax(z0, z1));
    return (near <= far) & (near < tmax) & (far > tmin);
}

// The 32-byte f32 node at ref `cur`: LS kernels hold all nodes in LDS at offset 0 (the LDS
// pointer is the ref itself: render_kernel checks that its dynamic LDS starts at address 0),
// TOP kernels the first S.ntop bytes of them; the rest is read from HBM, with a separate masked
// load into the same registers (no per-lane pointer select, no flat loads).
struct NodeF {
    Uvec4 q0;  // x.min x.max y.min y.max (f32 bits)
    Uvec4 q1;  // z.min z.max w0 w1
};
typedef __attribute__((address_space(3))) const NodeF LdsNodeF;
typedef __attribute__((address_space(1))) const NodeF GlobalNodeF;
template <bool TOP, bool LS>
__device__ __forceinline__ void fetch_nodef(const SceneView& S, uint32_t cur, Uvec4& q0, Uvec4& q1) {
    if (LS) {
        LdsNodeF* p = (LdsNodeF*)static_cast<uintptr_t>(cur);
        q0 = p->q0;
        q1 = p->q1;
    } else if (TOP) {
        // Lanes below the treelet read HBM, the others LDS, into the same registers. Written as C,
        // the compiler waits for the HBM loads before it issues the LDS reads (it cannot know that
        // the two exec masks are disjoint, so it orders the register writes), which puts the LDS
        // latency behind the HBM latency in every step of a wave with lanes on both sides. Here
        // both are in flight together, and the statement waits for both (its loads are outside
        // the compiler's counters).
        // A side whose mask is empty is branched over: a vector-memory instruction issued with
        // EXEC = 0 still takes its slot in the address / data units (TA / TD, config 4's
        // binding resource), and a wave whose lanes are all in the treelet (or all below it)
        // is common at the start (end) of its rays' traversals.
        const uint64_t hbm = __ballot(cur >= S.ntop);
        uint64_t save;
        asm volatile(
            "s_and_saveexec_b64 %[save], %[hbm]\n\t"
            "s_cbranch_execz 1f\n\t"
            "global_load_dwordx4 %[q0], %[cur], %[base]\n\t"
            "global_load_dwordx4 %[q1], %[cur], %[base] offset:16\n"
            "1:\n\t"
            "s_andn2_b64 exec, %[save], %[hbm]\n\t"
            "s_cbranch_execz 2f\n\t"
            "ds_read_b128 %[q0], %[cur]\n\t"
            "ds_read_b128 %[q1], %[cur] offset:16\n"
            "2:\n\t"
            "s_mov_b64 exec, %[save]\n\t"
            "s_waitcnt vmcnt(0) lgkmcnt(0)"
            : [q0] "=&v"(q0), [q1] "=&v"(q1), [save] "=&s"(save)
            : [cur] "v"(cur), [hbm] "s"(hbm), [base] "s"(S.fnodes)
            : "memory");
    } else {
        GlobalNodeF* p = (GlobalNodeF*)(reinterpret_cast<const char*>(S.fnodes) + cur);
        q0 = p->q0;
        q1 = p->q1;
    }
}

// The node's two words (w0, w1: bytes 24-31) alone, the same way
typedef uint32_t Uvec2 __attribute__((ext_vector_type(2)));
template <bool TOP, bool LS>
__device__ __forceinline__ Uvec2 fetch_nodef_words(const SceneView& S, uint32_t cur) {
    typedef __attribute__((address_space(3))) const Uvec2 LdsU2;
    typedef __attribute__((address_space(1))) const Uvec2 GlobalU2;
    if (LS) return *(LdsU2*)static_cast<uintptr_t>(cur + 24);
    if (!TOP) return *(GlobalU2*)(reinterpret_cast<const char*>(S.fnodes) + cur + 24);
    const uint64_t hbm = __ballot(cur >= S.ntop);
    uint64_t save;
    Uvec2 w;
    asm volatile(
        "s_and_saveexec_b64 %[save], %[hbm]\n\t"
        "s_cbranch_execz 1f\n\t"
        "global_load_dwordx2 %[w], %[cur], %[base] offset:24\n"
        "1:\n\t"
        "s_andn2_b64 exec, %[save], %[hbm]\n\t"
        "s_cbranch_execz 2f\n\t"
        "ds_read_b64 %[w], %[cur] offset:24\n"
        "2:\n\t"
        "s_mov_b64 exec, %[save]\n\t"
        "s_waitcnt vmcnt(0) lgkmcnt(0)"
        : [w] "=&v"(w), [save] "=&s"(save)
        : [cur] "v"(cur), [hbm] "s"(hbm), [base] "s"(S.fnodes)
        : "memory");
    return w;
}

template <typename SE, bool COUNT, bool EXACT, bool TOP, bool LS, bool GS, bool SPEC, bool INVL = false, bool G2 = true>
__device__ __forceinline__ void walk(const SceneView& S, Stack<SE>& st, const double o[3], const double d[3],
                                     double tmin, float tmin32, Trav& R, LaneCounters& ctr) {
    // Every step ends with the next node in `cur`: the near child of an entered interior node,
    // else the stack top, popped. The level below the stack holds the sentinel node, entered by
    // every ray, so popping an empty stack leads to the sentinel and the only exit is "entered a
    // node with primitives" (a leaf, or the sentinel: traversal over). An entered leaf ends the
    // walk already popped (the reference pops right after the leaf's primitive loop, which leaves
    // the stack unchanged); its primitive range goes to leaf_step in R.first / R.count. So the
    // loop body has no branch but that exit (and the rare f64 decision), and every lane makes
    // the same updates.
    // The stack is walked with a pointer to its top level (level sp - 1). The far child is stored
    // at level sp whatever the outcome (above the live stack unless it is pushed; the stack has
    // depth + 1 levels); at the sentinel that store rewrites the guard level with the sentinel's
    // own reference, and the speculative read of the top reads the level below the guard (in
    // bounds: the host keeps it inside the allocation).
    const ptrdiff_t stride = static_cast<ptrdiff_t>(st.stride);
    SE* const empty = st.base - stride;
    SE* tp = st.base + (static_cast<ptrdiff_t>(R.sp) - 1) * stride;
    uint32_t cur = R.cur;
    uint32_t w0, w1;  // the last node's DevNodeF words (leaf / sentinel at the exit)
    bool stop;
    if (EXACT) {
        // divided here: without the barrier the compiler hoists these three divisions out of
        // the traversal rounds into every shade round, although the EXACT walk is rare
        double dx = d[0], dy = d[1], dz = d[2];
        asm volatile("" : "+v"(dx), "+v"(dy), "+v"(dz));
        const double inv[3] = {1 / dx, 1 / dy, 1 / dz};
        do {
            NodeLines nd;
            node_lines(node64(S, cur), nd);
            const Uvec4 meta = nd.meta;  // index count axis flags
            const uint32_t top = *tp;    // speculative pop
            if (COUNT) {
                if (meta.y != kSentinelCount) ctr.nodes++;
                if (wave_leader()) ctr.it_walk++;
            }
            // x[neg] / x[!neg]
            const bool nx = R.neg & 1u, ny = (R.neg >> 1) & 1u, nz = (R.neg >> 2) & 1u;
            const double bx0 = nx ? nd.b[0].y : nd.b[0].x, bx1 = nx ? nd.b[0].x : nd.b[0].y;
            const double by0 = ny ? nd.b[1].y : nd.b[1].x, by1 = ny ? nd.b[1].x : nd.b[1].y;
            const double bz0 = nz ? nd.b[2].y : nd.b[2].x, bz1 = nz ? nd.b[2].x : nd.b[2].y;
            double xtmin = (bx0 - o[0]) * inv[0];
            double xtmax = (bx1 - o[0]) * inv[0];
            const double ytmin = (by0 - o[1]) * inv[1];
            const double ytmax = (by1 - o[1]) * inv[1];
            const double ztmin = (bz0 - o[2]) * inv[2];
            const double ztmax = (bz1 - o[2]) * inv[2];
            const bool c1 = !(xtmin > ytmax || ytmin > xtmax);
            if (ytmin > xtmin) xtmin = ytmin;
            if (ytmax < xtmax) xtmax = ytmax;
            const bool c2 = !(xtmin > ztmax || ztmin > xtmax);
            if (ztmin > xtmin) xtmin = ztmin;
            if (ztmax < xtmax) xtmax = ztmax;
            const bool enter = (c1 & c2 & (xtmin < R.tmax) & (xtmax > tmin)) |
                               (meta.y != 0 && (meta.w & kNodeAlways) != 0) | (meta.y == kSentinelCount);
            const bool inner = enter & (meta.y == 0);
            const bool far_first = (R.neg >> meta.z) & 1u;
            const uint32_t left = meta.w << kNodeFShift, right = meta.x << kNodeFShift;
            tp[stride] = static_cast<SE>(far_first ? left : right);
            stop = enter ^ inner;  // entered, not interior: a leaf or the sentinel
            cur = inner ? (far_first ? right : left) : top;
            tp += inner ? stride : -stride;
            w0 = meta.x;
            w1 = meta.y == kSentinelCount ? kSentinelW1 : (kLeafFlagF | meta.y);
        } while (!stop);
    } else if (SPEC) {
        // Speculative walk (Aila & Laine's postponed leaves): a lane that enters its first leaf
        // records it and walks on, with its t_max of now, until it enters a second leaf (or
        // the sentinel), where it parks without moving: that node is the next round's first
        // step and is tested again then. The wave's loop runs while some lane still walks to
        // its first leaf, so lanes that find theirs early keep doing DFS steps instead of idling.
        // The primitive tests are the reference's, in its order: the DFS order does not depend
        // on t_max; a node entered here with the t_max of before the recorded leaf's tests is
        // either entered under the smaller t_max too, or the reference culls it, and then it
        // also culls (i) the parked node, tested again, and (ii) every far child pushed below
        // it, tested at its pop — their boxes lie inside the culled one, and the rounded slab
        // values are monotone in the bounds (near(child) >= near(parent), far(child) <=
        // far(parent)), so the test fails for them at any t_max the culled one failed at.
        // Only node visits are added. The stack stays within depth + 1 levels: it is the same DFS.
        // The loop is the wave's; parked lanes leave it through the exec mask (`run`). A lane
        // parks by popping like at any entered leaf and remembering the node (`pcur`); after the
        // loop its pop is undone. The recorded node is `pref` (~0u: none yet; the sentinel when
        // the lane entered it with no leaf recorded: traversal over), so the loop's exit test is
        // one compare.
        bool run = true, nopend = true;
        uint32_t pref = ~0u, pcur = 0;
        do {
            CRT_WD(4, cur, static_cast<uint32_t>(tp - empty));
            if (run) {
                Uvec4 q0, q1;
                fetch_nodef<TOP, LS>(S, cur, q0, q1);
                w0 = q1.z;
                w1 = q1.w;
                const uint32_t top = *tp;  // speculative pop
                if (COUNT) {
                    if (w1 != kSentinelW1) ctr.nodes++;
                    if (wave_leader()) ctr.it_walk++;
                }
                const float x0 = __builtin_fmaf(__uint_as_float(q0.x), R.inv32[0], -R.oinv32[0]);
                const float x1 = __builtin_fmaf(__uint_as_float(q0.y), R.inv32[0], -R.oinv32[0]);
                const float y0 = __builtin_fmaf(__uint_as_float(q0.z), R.inv32[1], -R.oinv32[1]);
                const float y1 = __builtin_fmaf(__uint_as_float(q0.w), R.inv32[1], -R.oinv32[1]);
                const float z0 = __builtin_fmaf(__uint_as_float(q1.x), R.inv32[2], -R.oinv32[2]);
                const float z1 = __builtin_fmaf(__uint_as_float(q1.y), R.inv32[2], -R.oinv32[2]);
                const float lo = vmax3(vmin(x0, x1), vmin(y0, y1), vmax_s(vmin(z0, z1), tmin32));
                const float hi = vmin3(vmax(x0, x1), vmax(y0, y1), vmin(vmax(z0, z1), R.tmax32));
                const float gap = hi - lo;
                const float th = __builtin_fmaf(vmax_abs(lo, hi), 0x1p-19f, R.marg);
                bool enter = gap > 0.f;
                const bool unc = !(fabsf(gap) > th);
                if (__builtin_expect(__ballot(unc) != 0, 0)) {
                    if (COUNT && wave_leader()) ctr.it_slow++;
                    if (unc) {
                        if (COUNT) ctr.slow_nodes++;
                        enter = INVL ? slab64_inv(node64(S, cur), o, S.inv64_lds, tmin, R.tmax)
                                     : slab64(node64(S, cur), o, d, tmin, R.tmax);
                    }
                }
                const bool inner = enter & (w1 < kLeafFlagF);
                const uint32_t near = w1 | (__builtin_amdgcn_ubfe(R.neg, w0, 1) << kNodeFShift);
                tp[stride] = static_cast<SE>(near ^ (1u << kNodeFShift));
                const bool reached = enter & !inner;  // a leaf or the sentinel
                // a lane that reaches the sentinel with no leaf recorded records it and pops the
                // second guard level, which holds the sentinel too: it parks there, with a leaf
                // recorded (one compare fewer a step than testing for the sentinel here; G2 =
                // false: the compare, for the flat-parallelogram instances, whose five-wave
                // register allocation spilled 14 VGPRs instead of 8 without it)
                const bool park = reached & (!nopend | (!G2 && w1 == kSentinelW1));
                pref = (reached & nopend) ? cur : pref;  // the first leaf (or the sentinel)
                pcur = park ? cur : pcur;
                run = !park;
                cur = inner ? near : top;
                tp += inner ? stride : -stride;
            }
            nopend = pref == ~0u;
        } while (__ballot(nopend) != 0);
        if (!run) {  // parked: back at the node, its pop undone
            cur = pcur;
            tp += stride;
        }
        // the recorded node's words (a leaf's primitive range, or the sentinel: traversal over)
        {
            const Uvec2 w = fetch_nodef_words<TOP, LS>(S, pref);
            w0 = w.x;
            w1 = w.y;
        }
        R.state = w1 == kSentinelW1 ? kDone : kLeaf;
        R.first = w0;
        R.count = w1 & ~kLeafFlagF;
        R.cur = cur;
        R.sp = static_cast<int32_t>(static_cast<uint32_t>(tp - empty)) / static_cast<int32_t>(st.stride);
        return;
    } else {
        do {
            CRT_WD(5, cur, static_cast<uint32_t>(tp - empty));
            Uvec4 q0, q1;
            fetch_nodef<TOP, LS>(S, cur, q0, q1);
            w0 = q1.z;
            w1 = q1.w;
            const uint32_t top = *tp;  // speculative pop
            if (COUNT) {
                if (w1 != kSentinelW1) ctr.nodes++;
                if (wave_leader()) ctr.it_walk++;
            }
            // the sentinel and linear-mode leaves carry [-inf, inf] boxes: entered (lo' = tmin',
            // hi' = tmax')
            const float x0 = __builtin_fmaf(__uint_as_float(q0.x), R.inv32[0], -R.oinv32[0]);
            const float x1 = __builtin_fmaf(__uint_as_float(q0.y), R.inv32[0], -R.oinv32[0]);
            const float y0 = __builtin_fmaf(__uint_as_float(q0.z), R.inv32[1], -R.oinv32[1]);
            const float y1 = __builtin_fmaf(__uint_as_float(q0.w), R.inv32[1], -R.oinv32[1]);
            const float z0 = __builtin_fmaf(__uint_as_float(q1.x), R.inv32[2], -R.oinv32[2]);
            const float z1 = __builtin_fmaf(__uint_as_float(q1.y), R.inv32[2], -R.oinv32[2]);
            const float lo = vmax3(vmin(x0, x1), vmin(y0, y1), vmax_s(vmin(z0, z1), tmin32));
            const float hi = vmin3(vmax(x0, x1), vmax(y0, y1), vmin(vmax(z0, z1), R.tmax32));
            const float gap = hi - lo;
            const float th = __builtin_fmaf(vmax_abs(lo, hi), 0x1p-19f, R.marg);
            bool enter = gap > 0.f;
            const bool unc = !(fabsf(gap) > th);
            if (__builtin_expect(__ballot(unc) != 0, 0)) {
                if (COUNT && wave_leader()) ctr.it_slow++;
                if (unc) {
                    if (COUNT) ctr.slow_nodes++;
                    enter = INVL ? slab64_inv(node64(S, cur), o, S.inv64_lds, tmin, R.tmax)
                                 : slab64(node64(S, cur), o, d, tmin, R.tmax);
                }
            }
            const bool inner = enter & (w1 < kLeafFlagF);
            // siblings are side by side, the left one 64-byte aligned: near = left | 32 when the
            // right child comes first (v_bfe_u32 takes the offset from w0's low five bits: the
            // split axis), far = near ^ 32. At a leaf the store lands above the live stack; at the
            // sentinel it overwrites the guard level, which every traversal start rewrites.
            const uint32_t near = w1 | (__builtin_amdgcn_ubfe(R.neg, w0, 1) << kNodeFShift);
            tp[stride] = static_cast<SE>(near ^ (1u << kNodeFShift));
            stop = enter ^ inner;  // entered, not interior: a leaf or the sentinel
            cur = inner ? near : top;
            tp += inner ? stride : -stride;
        } while (!stop);
    }
    R.state = w1 == kSentinelW1 ? kDone : kLeaf;
    R.first = w0;
    R.count = w1 & ~kLeafFlagF;
    R.cur = cur;
    // levels in use after the pop; -1 when the leaf was entered with an empty stack
    R.sp = static_cast<int32_t>(static_cast<uint32_t>(tp - empty)) / static_cast<int32_t>(st.stride);
}

// ---- the sibling-pair walk of the HBM-scene kernels (CRT_PAIR_WALK) ----------------------------
// A step tests BOTH children of an entered interior node: one 64-byte read (siblings are side by
// side, the left one 64-byte aligned, so a pair is one half of a 128-byte line) and two f32 node
// tests. Deep trees in HBM walk a dependent chain of node reads; testing a pair per step halves
// its length (config 4: ~38 node tests a ray, each an L1 / L2 latency).
// The lane's position is a token: the byte offset of the first node to test, | 1 when it is to be
// tested alone. Without the bit the step tests that node and its sibling (offset ^ 32: siblings
// are side by side, 64-byte aligned), the first one being the near child of their parent in the
// ray's order. An entered interior child X continues as token(X) = X.left | (the ray's sign on
// X's split axis) << 5 = X's near child (the old walk's `near`); an entered leaf that cannot be
// processed now (a far child) continues as its own offset | 1, i.e. a re-test of its box alone.
// Exactness (the primitive tests are the reference's, in its order, with its t_max):
// - the DFS order of the children does not depend on t_max, and is the reference's
//   (bvh.h:684-698: near child first by the sign of d on the parent's split axis);
// - the node test is monotone in t_max and in the box: a child box lies inside its parent's
//   (node boxes are unions of their primitives' boxes), and the rounded slab values satisfy
//   near(child) >= near(parent), far(child) <= far(parent), so "child entered at t" implies
//   "parent entered at t" and at any larger t_max;
// - so testing a node at a t_max at least the reference's (children before their elder sibling's
//   subtree has shrunk it) only adds node visits: a node the pair walk culls, the reference culls
//   too, at its own (smaller or equal) t_max;
// - and a leaf's primitives run only right after its box was entered at the current t_max: the
//   first leaf a step enters (tested at the current t_max) exits to the leaf phase at once; every
//   other leaf is re-tested (its offset | 1) when the walk comes back to it. The reference tests a
//   leaf's box iff every ancestor was entered at its (larger) t_max, which the entry of the leaf
//   at the current t_max implies, so both test the same leaves at the same t_max.
// - A popped interior token is not re-tested itself: its children are tested at the current
//   t_max, and by monotonicity they all fail where the reference would cull it.
// The speculative form (SPEC: Aila & Laine's postponed leaves, walk()): a lane that has recorded
// its first leaf walks on with the t_max of now and parks at its second leaf as a re-test token,
// so the leaf is tested again at the then-current t_max in the next round.
// Stack: tokens, the far token stored at level sp unconditionally (pushed when both children are
// entered and the near one is interior); the guard level holds the sentinel's token (its offset
// | 1: its "sibling", past the node array, is never tested). The root's token is 0 | 1 (the pad
// node beside it is never tested). tests/test_pair_walk_model.py runs this state machine against
// the reference's DFS on random trees.

constexpr uint32_t kTokAlone = 1u;  // token bit 0: the first node alone (root, sentinel, re-tests)

// v_cndmask_b32 with a lane mask from a ballot (scalar registers): m ? a : b per lane
__device__ __forceinline__ uint32_t vsel(uint64_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(m));
    return r;
}

// The step's two f32 nodes: f (the first) and g = f ^ 32, read from the LDS treelet or from HBM
// (the treelet holds whole sibling pairs, dispatch_render, so f and g are on the same side),
// both sides in flight together as in fetch_nodef.
template <bool TOP>
__device__ __forceinline__ void fetch_two(const SceneView& S, uint32_t f, uint32_t g, Uvec4& a0, Uvec4& a1, Uvec4& b0,
                                          Uvec4& b1) {
    if (TOP) {
        const uint64_t hbm = __ballot(f >= S.ntop);
        uint64_t save;
        asm volatile(
            "s_and_saveexec_b64 %[save], %[hbm]\n\t"
            "s_cbranch_execz 1f\n\t"
            "global_load_dwordx4 %[a0], %[f], %[base]\n\t"
            "global_load_dwordx4 %[a1], %[f], %[base] offset:16\n\t"
            "global_load_dwordx4 %[b0], %[g], %[base]\n\t"
            "global_load_dwordx4 %[b1], %[g], %[base] offset:16\n"
            "1:\n\t"
            "s_andn2_b64 exec, %[save], %[hbm]\n\t"
            "s_cbranch_execz 2f\n\t"
            "ds_read_b128 %[a0], %[f]\n\t"
            "ds_read_b128 %[a1], %[f] offset:16\n\t"
            "ds_read_b128 %[b0], %[g]\n\t"
            "ds_read_b128 %[b1], %[g] offset:16\n"
            "2:\n\t"
            "s_mov_b64 exec, %[save]\n\t"
            "s_waitcnt vmcnt(0) lgkmcnt(0)"
            : [a0] "=&v"(a0), [a1] "=&v"(a1), [b0] "=&v"(b0), [b1] "=&v"(b1), [save] "=&s"(save)
            : [f] "v"(f), [g] "v"(g), [hbm] "s"(hbm), [base] "s"(S.fnodes)
            : "memory");
    } else {
        GlobalNodeF* qa = (GlobalNodeF*)(reinterpret_cast<const char*>(S.fnodes) + f);
        GlobalNodeF* qb = (GlobalNodeF*)(reinterpret_cast<const char*>(S.fnodes) + g);
        a0 = qa->q0;
        a1 = qa->q1;
        b0 = qb->q0;
        b1 = qb->q1;
    }
}

// the f32 node test of walk() on one node: lo' = max(near', tmin'), hi' = min(far', tmax')
__device__ __forceinline__ void node_lohi(const Uvec4& q0, const Uvec4& q1, const Trav& R, float tmin32, float& lo,
                                          float& hi) {
    const float x0 = __builtin_fmaf(__uint_as_float(q0.x), R.inv32[0], -R.oinv32[0]);
    const float x1 = __builtin_fmaf(__uint_as_float(q0.y), R.inv32[0], -R.oinv32[0]);
    const float y0 = __builtin_fmaf(__uint_as_float(q0.z), R.inv32[1], -R.oinv32[1]);
    const float y1 = __builtin_fmaf(__uint_as_float(q0.w), R.inv32[1], -R.oinv32[1]);
    const float z0 = __builtin_fmaf(__uint_as_float(q1.x), R.inv32[2], -R.oinv32[2]);
    const float z1 = __builtin_fmaf(__uint_as_float(q1.y), R.inv32[2], -R.oinv32[2]);
    lo = vmax3(vmin(x0, x1), vmin(y0, y1), vmax_s(vmin(z0, z1), tmin32));
    hi = vmin3(vmax(x0, x1), vmax(y0, y1), vmin(vmax(z0, z1), R.tmax32));
}

template <typename SE, bool COUNT, bool TOP, bool INVL>
__device__ __forceinline__ void walk_pairs(const SceneView& S, Stack<SE>& st, const double o[3], const double d[3],
                                           double tmin, float tmin32, Trav& R, LaneCounters& ctr) {
    const ptrdiff_t stride = static_cast<ptrdiff_t>(st.stride);
    SE* const empty = st.base - stride;
    SE* tp = st.base + (static_cast<ptrdiff_t>(R.sp) - 1) * stride;
    uint32_t cur = R.cur;
    uint32_t run = 1;
    uint32_t pref = ~0u;  // the first leaf's re-test token (or the sentinel's), ~0u: none yet
    // The per-lane logic is written on lane masks (uint64_t ballots: scalar ALU) with v_cndmask
    // selects (vsel); as bools across the rare f64 branch, the compiler materialises the
    // conditions as 0 / 1 in VGPRs and spends ~40 VALU a step on them. (The loop state as masks
    // too, with a wave-uniform body and masked updates: 65 VALU a step instead of 69, but config 4
    // 128.9-129.4 vs 127.7-127.8 ms, profiles/r06_pair_tuning.)
    uint64_t nop = __ballot(true);  // lanes with no leaf recorded yet
    do {
        CRT_WD(7, cur, static_cast<uint32_t>(tp - empty));
        if (run) {
            const uint32_t f = cur & ~kTokAlone, g = f ^ 32u;  // the first node and its sibling
            Uvec4 a0, a1, b0, b1;
            fetch_two<TOP>(S, f, g, a0, a1, b0, b1);
            const uint32_t top = *tp;  // speculative pop
            float lo1, hi1, lo2, hi2;
            node_lohi(a0, a1, R, tmin32, lo1, hi1);
            node_lohi(b0, b1, R, tmin32, lo2, hi2);
            const float g1 = hi1 - lo1, g2 = hi2 - lo2;
            // each node its own threshold (walk()'s bound, M = max(|lo'|, |hi'|) of that node).
            // One shared threshold (the larger M) would save a VALU a step but leaves 16x as many
            // node tests to f64: a sibling missed on an axis the ray runs almost parallel to has
            // |lo'| ~ |inv|, and its M made the other node's gap undecidable (config 4: 1.49e9
            // f64 node tests a frame, 13% of walk iterations with one)
            const float t1 = __builtin_fmaf(vmax_abs(lo1, hi1), 0x1p-19f, R.marg);
            const float t2 = __builtin_fmaf(vmax_abs(lo2, hi2), 0x1p-19f, R.marg);
            const uint64_t two = __ballot(cur == f);  // the sibling is tested too
            uint64_t e1 = __ballot(g1 > 0.f), e2 = __ballot(g2 > 0.f) & two;
            const uint64_t u1 = __ballot(!(fabsf(g1) > t1)), u2 = two & __ballot(!(fabsf(g2) > t2));
            if (COUNT) {
                if (a1.w != kSentinelW1) ctr.nodes++;
                ctr.nodes += cur == f ? 1 : 0;
                if (wave_leader()) ctr.it_walk++;
            }
            if (__builtin_expect((u1 | u2) != 0, 0)) {  // lanes the f32 margin cannot decide: f64
                if (COUNT && wave_leader()) ctr.it_slow++;
                const uint64_t me = 1ull << (threadIdx.x & 63);
                bool f1 = false, f2 = false;
                if (u1 & me) {
                    if (COUNT) ctr.slow_nodes++;
                    f1 = INVL ? slab64_inv(node64(S, f), o, S.inv64_lds, tmin, R.tmax) : slab64(node64(S, f), o, d, tmin, R.tmax);
                }
                if (u2 & me) {
                    if (COUNT) ctr.slow_nodes++;
                    f2 = INVL ? slab64_inv(node64(S, g), o, S.inv64_lds, tmin, R.tmax) : slab64(node64(S, g), o, d, tmin, R.tmax);
                }
                e1 = (e1 & ~u1) | __ballot(f1);
                e2 = (e2 & ~u2) | __ballot(f2);
            }
            const uint64_t i1 = __ballot(a1.w < kLeafFlagF), i2 = __ballot(b1.w < kLeafFlagF);
            // X: the first entered node in the reference's order (the first one, else its sibling)
            const uint64_t both = e1 & e2, any = e1 | e2;
            const uint64_t xi = (e1 & i1) | (~e1 & i2);
            // an entered leaf: the first one is recorded and the walk goes on with its
            // continuation (the sibling's token, or the stack top); the second one parks as its
            // re-test token (the sibling's token pushed when both were entered). The sentinel is
            // recorded like a leaf and met again on the second guard level, where the lane parks.
            const uint64_t leaf = any & ~xi;
            const uint64_t park = leaf & ~nop;  // the sentinel: recorded, then met again below the guard
            const uint64_t dp = (any & xi) | park;  // cur = X's token
            // the nodes' tokens: an interior node's near child, a leaf's re-test
            const uint32_t tok1 = vsel(i1, (__builtin_amdgcn_ubfe(R.neg, a1.z, 1) << kNodeFShift) | a1.w, cur | kTokAlone);
            const uint32_t tok2 = vsel(i2, (__builtin_amdgcn_ubfe(R.neg, b1.z, 1) << kNodeFShift) | b1.w, g | kTokAlone);
            const uint32_t tx = vsel(e1, tok1, tok2);
            pref = vsel(leaf & nop, tx, pref);
            tp[stride] = static_cast<SE>(tok2);
            cur = vsel(dp, tx, vsel(both, tok2, top));
            // one level up when the walk descends with both entered, one down when it pops
            tp += static_cast<int32_t>(vsel(dp & both, 1u, vsel(~dp & ~both, ~0u, 0u))) * stride;
            run = vsel(park, 0u, 1u);
        }
        nop = __ballot(pref == ~0u);
    } while (nop != 0);
    {
        const Uvec2 w = fetch_nodef_words<TOP, false>(S, pref & ~kTokAlone);  // the recorded leaf
        R.state = w.y == kSentinelW1 ? kDone : kLeaf;
        R.first = w.x;
        R.count = w.y & ~kLeafFlagF;
    }
    R.cur = cur;
    R.sp = static_cast<int32_t>(static_cast<uint32_t>(tp - empty)) / static_cast<int32_t>(st.stride);
}

// the entered leaf's primitives in order (bvh.h:635-652), then "return" to the DFS.
// Sphere-only scenes store spheres in slot order, so the slot indexes them directly and the next
// sphere is loaded while the current one is tested.
// QONLY: every primitive is a parallelogram (the flat-parallelogram instances): the sphere paths,
// and with them the ray's sphere constants (dot(d, d), its reciprocal, the coarse-reject limits),
// are compiled out
template <typename SE, bool COUNT, bool TOP, bool LS, bool FAST = false, bool QONLY = false>
__device__ __forceinline__ void leaf_step(const SceneView& S, Stack<SE>& st, const double o[3],
                                              const double d[3], double tmin, float tmin32, bool sphere_only, bool pairs,
                                              bool qfilter, bool qflat, Trav& R, LaneCounters& ctr) {
    const uint2 range = make_uint2(R.first, R.count);  // index, count
    const uint32_t end = range.x + range.y;
    const double ia = recip_a<FAST>(R.a), lo = lim_tmin(tmin, R.a);
    double hi = lim_tmax(R.tmax, R.a);
    if (!QONLY && pairs && range.y <= 32 && leaf_ray32_ok(o, d, R.a)) {
        // two passes: the packed f32 candidate filter over every sphere against the leaf-entry
        // t_max, then the full test of the candidates in slot order with the shrinking t_max. A
        // sphere the first pass rejects is rejected by the full test for any smaller t_max too,
        // so the hits and the tie order are the sequential loop's; the full-test pass runs only
        // as often as the lane with most candidates needs (typically 1-3 of 6-12).
        // Pass 1 reads pair records (slots first + i, first + i + 1) and shifts both verdicts
        // into `cand`: after the pass, bit nbits - 1 - i stands for sphere i (nbits = count
        // rounded up to even; an odd count's extra verdict, for the slot after the leaf, is
        // masked off).
        LeafRay32 L;
        leaf_ray32(o, d, R.a, tmin, R.tmax, L);
        uint32_t cand = 0;
        const uint32_t nbits = (range.y + 1) & ~1u;
        if constexpr (LS) {
            for (uint32_t i = 0; i < range.y; i += 2) {
                if (COUNT) {
                    ctr.sphere_tests += i + 1 < range.y ? 2 : 1;
                    if (wave_leader()) ctr.it_leaf += 2;
                }
                cand = sphere_pair_candidates(cand, pair_at((LdsPair*)static_cast<uintptr_t>(S.spair_lds + ((range.x + i) << 5))), L);
            }
        } else {
            for (uint32_t i = 0; i < range.y; i += 2) {
                if (COUNT) {
                    ctr.sphere_tests += i + 1 < range.y ? 2 : 1;
                    if (wave_leader()) ctr.it_leaf += 2;
                }
                cand = sphere_pair_candidates(cand, pair_at((GlobalPair*)(S.spair + range.x + i)), L);
            }
        }
        cand &= ~(range.y & 1u);  // an odd count's last verdict is the slot after the leaf
        while (cand) {
            CRT_WD(6, cand, range.y);
            if (COUNT) {
                ctr.cand++;
                if (wave_leader()) ctr.it_cand++;
            }
            const uint32_t b = 31 - __builtin_clz(cand);
            cand ^= 1u << b;
            const uint32_t i = range.x + (nbits - 1 - b);
            double t;
            // the f64 spheres are in HBM (L1) in this mode
            if (hit_sphere<false>(sphere_at<LS>(S, i), o, d, R.a, ia, tmin, R.tmax, lo, hi, t)) {
                R.tmax = t;
                R.tmax32 = tmax_f32(t);
                hi = lim_tmax(t, R.a);
                R.ref = i;
                R.found = true;
            }
        }
    } else if (LS && qfilter && qflat && range.y <= 32) {
        // axis-aligned parallelograms (every Box face, the Cornell walls): pass 1 is the walk's
        // f32 node test on each one's flat box (crt_quad_filter.h: a rejection is a proven miss of
        // the reference's Parallelogram::hit_by for this t_max and any smaller one); rays outside
        // the walk's range have marg = inf and keep every parallelogram. Pass 2 as below.
        // one loop per flat axis over the leaf's records grouped by it (stage_image), each record
        // setting the bit of its slot
        uint32_t cand = 0;
        const uint32_t base = S.quadf_lds + (range.x << 5);
        const uint32_t g = lds_u32(base + 28);  // the group sizes, in the leaf's first record
        const uint32_t e0 = g & 0xffu, e1 = e0 + ((g >> 8) & 0xffu);
        uint32_t i = 0;
        const auto filter = [&](auto axis) {
            if (COUNT) {
                ctr.quad_tests++;
                if (wave_leader()) ctr.it_leaf++;
            }
            LdsNodeF* p = (LdsNodeF*)static_cast<uintptr_t>(base + (i << 5));
            const Uvec4 q0 = p->q0, q1 = p->q1;
            const float b[6] = {__uint_as_float(q0.x), __uint_as_float(q0.y), __uint_as_float(q0.z),
                                __uint_as_float(q0.w), __uint_as_float(q1.x), __uint_as_float(q1.y)};
            cand |= static_cast<uint32_t>(flat_axis_candidate<decltype(axis)::value, DevMinMax>(b, R.inv32, R.oinv32, tmin32, R.tmax32, R.marg)) << q1.z;
        };
        for (; i < e0; ++i) filter(std::integral_constant<int, 0>{});
        for (; i < e1; ++i) filter(std::integral_constant<int, 1>{});
        for (; i < range.y; ++i) filter(std::integral_constant<int, 2>{});
        while (cand) {
            CRT_WD(6, cand, range.y);
            if (COUNT) {
                ctr.cand++;
                if (wave_leader()) ctr.it_cand++;
            }
            const uint32_t i = range.x + static_cast<uint32_t>(__builtin_ctz(cand));
            cand &= cand - 1;
            double t;
            if (hit_quad(lds_rec<DevQuad>(S.quads_lds + (i << 7)), o, d, tmin, R.tmax, t)) {
                R.tmax = t;
                R.tmax32 = tmax_f32(t);
                R.ref = kRefQuad | i;
                R.found = true;
            }
        }
    } else if (LS && qfilter && !qflat && range.y <= 32 && quad_ray32_ok(o, d)) {
        // parallelogram-only scenes (a slot is its parallelogram's index): the same two passes,
        // with the f32 filter of crt_quad_filter.h (quad_candidate) in pass 1. LDS-scene kernels
        // only: in the HBM-scene kernels its registers cost spills (none of the reference's
        // parallelogram-only scenes is that large)
        QuadRay32 L;
        quad_ray32(o, d, tmin, R.tmax, L);
        uint32_t cand = 0;
        for (uint32_t i = 0; i < range.y; ++i) {
            if (COUNT) {
                ctr.quad_tests++;
                if (wave_leader()) ctr.it_leaf++;
            }
            const DevQuadF q = LS ? lds_rec<DevQuadF>(S.quadf_lds + ((range.x + i) << 6)) : quadf_global(S.quadf + range.x + i);
            cand |= static_cast<uint32_t>(quad_candidate(q, L, [](float x) { return __builtin_amdgcn_rcpf(x); })) << i;
        }
        while (cand) {
            CRT_WD(6, cand, range.y);
            if (COUNT) {
                ctr.cand++;
                if (wave_leader()) ctr.it_cand++;
            }
            const uint32_t i = range.x + static_cast<uint32_t>(__builtin_ctz(cand));
            cand &= cand - 1;
            double t;
            bool h;
            if constexpr (LS) h = hit_quad(lds_rec<DevQuad>(S.quads_lds + (i << 7)), o, d, tmin, R.tmax, t);
            else h = hit_quad(S.quads[i], o, d, tmin, R.tmax, t);
            if (h) {
                R.tmax = t;
                R.tmax32 = tmax_f32(t);
                R.ref = kRefQuad | i;
                R.found = true;
            }
        }
    } else if (!QONLY && sphere_only) {
        DevSphere cur = sphere_at<LS>(S, range.x);
        for (uint32_t i = range.x; i < end; ++i) {
            // one past the leaf's last sphere is still inside the scene copy (sphere_mat follows
            // the spheres in HBM, the parallelogram / stack regions in LDS); it is never tested
            const DevSphere nxt = sphere_at<LS>(S, i + 1);
            if (COUNT) {
                ctr.sphere_tests++;
                if (wave_leader()) ctr.it_leaf++;
            }
            double t;
            if (hit_sphere(cur, o, d, R.a, ia, tmin, R.tmax, lo, hi, t)) {
                R.tmax = t;
                R.tmax32 = tmax_f32(t);
                hi = lim_tmax(t, R.a);
                R.ref = i;
                R.found = true;
            }
            cur = nxt;
        }
    } else {
        for (uint32_t i = range.x; i < end; ++i) {
            // LS: refs, spheres and parallelograms are all staged (spheres_f32 is off here)
            const uint32_t ref = LS ? lds_u32(S.refs_lds + (i << 2)) : S.refs[i];
            double t;
            bool h;
            if (COUNT && wave_leader()) ctr.it_leaf++;
            if (QONLY || (ref & kRefQuad)) {
                if (COUNT) ctr.quad_tests++;
                if constexpr (LS) h = hit_quad(lds_rec<DevQuad>(S.quads_lds + ((ref & ~kRefQuad) << 7)), o, d, tmin, R.tmax, t);
                else h = hit_quad(S.quads[ref & ~kRefQuad], o, d, tmin, R.tmax, t);
            } else {
                if (COUNT) ctr.sphere_tests++;
                if constexpr (LS) h = hit_sphere(lds_rec<DevSphere>(S.spheres_lds + (ref << 5)), o, d, R.a, ia, tmin, R.tmax, lo, hi, t);
                else h = hit_sphere(S.spheres[ref], o, d, R.a, ia, tmin, R.tmax, lo, hi, t);
            }
            if (h) {
                R.tmax = t;
                R.tmax32 = tmax_f32(t);
                hi = lim_tmax(t, R.a);
                R.ref = ref;
                R.found = true;
            }
        }
    }
    // the pop after the leaf was made by walk (R.cur is the next node, unless the stack was empty)
    R.state = R.sp < 0 ? kDone : kWalk;
}

__device__ __forceinline__ uint32_t owned_row(const Work& w, uint32_t k) {
    if (w.rb_shift < 32) {  // power-of-two row blocks: no division
        const uint32_t blk = k >> w.rb_shift, in = k & ((1u << w.rb_shift) - 1);
        return ((blk * w.tile_count + w.tile_index) << w.rb_shift) | in;
    }
    const uint32_t blk = k / w.row_block, in = k % w.row_block;
    return (blk * w.tile_count + w.tile_index) * w.row_block + in;
}

// State of one lane's current path: the ray, the throughput and the bounces left (ray_color's
// depth_left, camera.h:207-213). Emission enters a path only where it ends (a DiffuseLight never
// scatters, a miss returns the background), so no running radiance is kept: the terminal
// T * (emit | background) goes straight into the pixel's sum.
struct Path {
    double o[3], d[3];
    double T[3];
    uint32_t depth;
    uint32_t rng;
};

// random_ray_through_pixel (camera.h:184-200) for a fresh sample
__device__ __forceinline__ void start_path(const CamView& C, uint32_t row, uint32_t col, uint32_t rng, Path& P) {
    if (C.defocus_angle <= 0) {
        P.o[0] = C.o[0]; P.o[1] = C.o[1]; P.o[2] = C.o[2];
    } else {  // random_point_in_defocus_disk (camera.h:160-168, vec3d.h:79-85)
        double vx, vy;
        do {
            vx = rnd_pm1(rng);
            vy = rnd_pm1(rng);
        } while (!(vx * vx + vy * vy + 0.0 * 0.0 < 1));
        P.o[0] = (C.o[0] + C.ddx[0] * vx) + C.ddy[0] * vy;
        P.o[1] = (C.o[1] + C.ddx[1] * vx) + C.ddy[1] * vy;
        P.o[2] = (C.o[2] + C.ddx[2] * vx) + C.ddy[2] * vy;
    }
    // converted here at every call: hoisted out of the kernel's loop, the two doubles would
    // stay live (and spill) across all phases
    uint32_t ir = row, ic = col;
    asm volatile("" : "+v"(ir), "+v"(ic));
    const double fr = static_cast<double>(ir), fc = static_cast<double>(ic);
    // a g++ build evaluates the second jitter draw (the pixel_delta_y one) first
    const double uy = rnd(rng, -0.5, 0.5);
    const double ux = rnd(rng, -0.5, 0.5);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double center = (C.p00[k] + C.pdy[k] * fr) + C.pdx[k] * fc;
        const double sample = (center + C.pdx[k] * ux) + C.pdy[k] * uy;
        P.d[k] = sample - P.o[k];
        P.T[k] = 1;
    }
    P.depth = C.max_depth;
    P.rng = rng;
}

// One level of ray_color (camera.h:205-258) after the closest-hit query: scatters
// (material.h:64-263) into the next ray, or ends the path adding T * (background | emission) to
// acc. Returns true when the path has ended (miss, light, absorption).
template <bool LS, bool SPH = false, bool QONLY = false, bool FAST = false>
__device__ __forceinline__ bool shade(const SceneView& S, const CamView& C, Path& P, bool hit,
                                      uint32_t ref, double t, double acc[3]) {
    if (!hit) {
        acc[0] = acc[0] + P.T[0] * C.bg[0];
        acc[1] = acc[1] + P.T[1] * C.bg[1];
        acc[2] = acc[2] + P.T[2] * C.bg[2];
        return true;
    }
    // the slot's material record, loaded first (its address needs only the slot)
    const DevMaterial& M = (QONLY || (!SPH && (ref & kRefQuad))) ? S.quad_mrec[ref & ~kRefQuad] : S.sphere_mrec[ref];
    double p[3], n[3];
    bool front;
    (void)hit_record<LS, true, SPH, QONLY>(S, ref, P.o, P.d, t, p, n, front, M.emit[0]);
    const uint32_t kind = M.kind;
    const bool lam = kind == CRT_LAMBERTIAN, met = kind == CRT_METAL, die = kind == CRT_DIELECTRIC;
    if (!(lam || met || die)) {  // DiffuseLight: emits, never scatters (material.h:248-263)
        acc[0] = acc[0] + P.T[0] * M.emit[0];
        acc[1] = acc[1] + P.T[1] * M.emit[1];
        acc[2] = acc[2] + P.T[2] * M.emit[2];
        return true;
    }
    // The scatter functions are interleaved by their common steps, so a wave with several
    // materials runs each step once: unit(d) (Metal material.h:120, Dielectric :191), the
    // Dielectric reflect-or-refract draw, random_unit_vector (Lambertian :70, Metal :123 — the
    // only draw of either), then the reflection (vec3d.h:144-155) shared by Metal and a
    // reflecting Dielectric. Every lane still makes its own material's draws in the reference's
    // order (no lane draws in two of these steps).
    double ux0 = 0, uy0 = 0, uz0 = 0;
    if (met || die) {
        const double il = recip_exact<FAST>(sqrt_exact<FAST>(P.d[0] * P.d[0] + P.d[1] * P.d[1] + P.d[2] * P.d[2]));
        ux0 = P.d[0] * il;
        uy0 = P.d[1] * il;
        uz0 = P.d[2] * il;
    }
    bool reflect = met;
    double cosv = 0, ratio = 0;
    if (die) {  // material.h:185-218, vec3d.h:168-200
        ratio = front ? M.color[0] : M.param;  // 1. / ri, ri / 1. (precomputed: upload)
        cosv = fmin((-ux0) * n[0] + (-uy0) * n[1] + (-uz0) * n[2], 1.);
        const double sinv = sqrt_exact<FAST>(1 - cosv * cosv);
        if (ratio * sinv > 1) {
            reflect = true;  // total internal reflection, no draw
        } else {
            const double r0 = front ? M.color[1] : M.color[2];  // reflectance's r0 (upload)
            const double pw = pow5(1 - cosv);
            const double u = rnd_01(P.rng);
            reflect = u < r0 + (1 - r0) * pw;
            // a branch a 1-ulp different pow could flip (crt_schlick.h): counted, never taken in
            // practice (probability ~2^-50 per decision)
            if (__builtin_expect(schlick_undecided(u, r0, pw), 0)) atomicAdd(S.guard, 1ull);
        }
    }
    double rx = 0, ry = 0, rz = 0;
    if (lam || met) random_unit_vector<FAST>(P.rng, rx, ry, rz);
    double nd[3];
    if (reflect) {  // Metal (material.h:116-139) or a reflecting Dielectric
        const double k2 = 2 * (ux0 * n[0] + uy0 * n[1] + uz0 * n[2]);
        nd[0] = ux0 - n[0] * k2;
        nd[1] = uy0 - n[1] * k2;
        nd[2] = uz0 - n[2] * k2;
        if (met) {
            nd[0] = nd[0] + rx * M.param;
            nd[1] = nd[1] + ry * M.param;
            nd[2] = nd[2] + rz * M.param;
            if (n[0] * nd[0] + n[1] * nd[1] + n[2] * nd[2] < 0) return true;  // absorbed; emits 0
        }
    } else if (die) {  // refraction
        const double px = (ux0 + n[0] * cosv) * ratio;
        const double py = (uy0 + n[1] * cosv) * ratio;
        const double pz = (uz0 + n[2] * cosv) * ratio;
        const double sq = -sqrt_exact<FAST>(fabs(1 - (px * px + py * py + pz * pz)));
        nd[0] = px + n[0] * sq;
        nd[1] = py + n[1] * sq;
        nd[2] = pz + n[2] * sq;
    } else {  // Lambertian (material.h:64-86)
        nd[0] = n[0] + rx; nd[1] = n[1] + ry; nd[2] = n[2] + rz;
        if (fabs(nd[0]) < 1e-8 && fabs(nd[1]) < 1e-8 && fabs(nd[2]) < 1e-8) {
            nd[0] = n[0]; nd[1] = n[1]; nd[2] = n[2];
        }
    }
    if (kind != CRT_DIELECTRIC) {  // attenuation = intrinsic colour (dielectric: 1)
        P.T[0] = P.T[0] * M.color[0];
        P.T[1] = P.T[1] * M.color[1];
        P.T[2] = P.T[2] * M.color[2];
    }
    P.o[0] = p[0]; P.o[1] = p[1]; P.o[2] = p[2];
    P.d[0] = nd[0]; P.d[1] = nd[1]; P.d[2] = nd[2];
    P.depth -= 1;
    return false;
}

// 16-byte cooperative copy global -> LDS (the scene staging of LSCENE kernels)
__device__ __forceinline__ void stage_lds(unsigned char* dst, const void* src, uint32_t bytes) {
    const uint4* s = static_cast<const uint4*>(src);
    uint4* d = reinterpret_cast<uint4*>(dst);
    for (uint32_t i = threadIdx.x; i < bytes / 16; i += kBlock) d[i] = s[i];
}

// The render kernel: a persistent grid (as many blocks as are resident) whose waves take work
// items from a queue in HBM, one atomic per item: item = (8x8 pixel tile, sample chunk), 64
// (chunk, pixel) units, in tile-major order. A wave's lanes draw units as they finish one,
// crossing from one item into the next without waiting, so a lane idles only once the queue is
// dry, and the grid drains within about one unit.
// Persistent per-lane state machine (WALK -> LEAF -> ... -> DONE -> shade -> WALK) in traversal
// rounds: every walking lane walks the DFS to its next entered leaf (or the end of its
// traversal), then the lanes holding a leaf test it together. Lanes whose ray is finished park
// until kShadeBatch of them are finished (or nobody traverses), then shade together, and a
// finished path starts the lane's next sample at once (path regeneration). So the shading code
// runs with many lanes active, and a wave is never held by its slowest ray or path.
// A unit's samples are summed in sample order into partial[chunk][pixel].
// LSCENE: nodes, primitive refs, spheres and parallelograms are staged in LDS first.
// 4 waves per SIMD (128 VGPRs): the f32 walk / packed sphere filter state does not fit 96
// VGPRs without ~66 spills (5 waves: 3932 vs 4158 Msamples/s on config 2)
#ifndef CRT_WAVES_PER_EU
#define CRT_WAVES_PER_EU 4
#endif
// LDS-scene kernels: 5 waves per SIMD (96 VGPRs) spill 65 VGPRs with the work-queue state and
// wrote 94 GB of scratch per config-2 frame: 5262 vs 5499 Msamples/s at 4 (config 3: 1958 vs
// 1939); with v10's block pools 5 had measured +0.7%. The HBM-scene kernels lose 14% at 5.
#ifndef CRT_WAVES_PER_EU_LDS
#define CRT_WAVES_PER_EU_LDS 4
#endif
#ifndef CRT_SHADE_BATCH
#define CRT_SHADE_BATCH 48
#endif
constexpr int kShadeBatch = CRT_SHADE_BATCH;

// HBM-scene kernels keep the top of the node array in LDS (CRT_NO_LDS_TOP=1 at run time: none)
constexpr bool kTopTreelet = true;
// The timed kernels walk speculatively (walk(): lanes that found their first leaf walk on to the
// next one). The instrumented pass (COUNT) walks like the reference by default, so its node counts
// are the reference's (the algorithmic-byte basis); with Work::count_spec (CRT_COUNT_SPEC=1 at run
// time) it walks speculatively too, for the timed kernel's phase timings and lane utilization (its
// node counts then include the speculative visits).
// Static wave priority per phase (s_setprio 0-3; the SQ issues a ready instruction of the highest
// priority wave first, then the oldest): the traversal phases are dependency chains (LDS read ->
// test -> next address), the shade and path-start phases have more independent work to fill in.
// Config 2 (ms/frame, one box): none 87.9; walk 1 86.6; walk+leaf 1 85.6; walk 2 / leaf 1 85.6;
// walk 1 / leaf 2 85.6; walk 2 / leaf 2 / start 1 85.4; walk 3 / leaf 2 / start 1 (kept) 85.3;
// walk 1 / leaf 1 / start 1 86.0.
constexpr int kPrioWalk = 3, kPrioLeaf = 2, kPrioShade = 0, kPrioInit = 1;
template <int P>
__device__ __forceinline__ void set_prio() {
    if constexpr ((kPrioWalk | kPrioLeaf | kPrioShade | kPrioInit) != 0) __builtin_amdgcn_s_setprio(P);
}

// PM (primitive mix): 0 sphere-only scenes (every parallelogram path compiled out), 1 any scene,
// 2 parallelogram-only scenes of axis-aligned parallelograms (LDS scenes: the flat-box filter
// only, no sphere paths)
// W5: 5 waves per SIMD (96 VGPRs, ~40-48 of them spilled), launched for sphere-only and
// flat-parallelogram LDS scenes whose LDS copy leaves room for five blocks per CU (dispatch_render)
template <typename SE, bool GSTACK, bool LSCENE, bool COUNT, int PM, bool W5>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(W5 ? kManyWaves : LSCENE ? CRT_WAVES_PER_EU_LDS : CRT_WAVES_PER_EU, 8))) void render_kernel(
    SceneView Sg, CamView C, Work W, double* __restrict__ partial, SE* __restrict__ gstack,
    Counters* __restrict__ counters) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // the instances with PM = 0 are launched for sphere-only scenes only, PM = 2 for scenes of
    // axis-aligned parallelograms only: the other primitive's paths are compiled out of them
    constexpr bool kSphOnly = PM == 0, kFlatOnly = PM == 2;
    // sqrt / reciprocal expansions without range fix-ups (sqrt_exact, recip_exact): measured
    // faster only in the five-wave sphere-only instance
    constexpr bool kFast = kSphOnly && W5;
    SceneView S = Sg;
    if (LSCENE) {  // f32 nodes at LDS offset 0 (fetch_nodef: a node's LDS address is its ref)
        if (static_cast<uint32_t>(reinterpret_cast<uintptr_t>((LdsByte*)smem)) != 0) __builtin_trap();
        stage_lds(smem, Sg.fnodes, W.bytes_nodes);
        stage_lds(smem + W.lds_quads, Sg.quads, W.bytes_quads);
        S.quads = reinterpret_cast<const DevQuad*>(smem + W.lds_quads);
        S.quads_lds = W.lds_quads;
        if (W.quads_f32) {  // the parallelogram filter's records (flat boxes when axis-aligned)
            stage_lds(smem + W.lds_quadf, W.quads_flat ? static_cast<const void*>(Sg.quadbox) : Sg.quadf, W.bytes_quadf);
            S.quadf_lds = W.lds_quadf;
        }
        S.refs_lds = W.lds_refs;
        S.spheres_lds = W.spheres_f32 ? (W.bytes_sph64 ? W.lds_sph64 : ~0u) : W.lds_spheres;
        if (W.spheres_f32) {
            // sphere-only: the filter's pair records in LDS; refs are unused (slot = sphere),
            // and the f64 spheres (candidates' exact tests, shading) stay in HBM / L1
            stage_lds(smem + W.lds_spheres, Sg.spair, W.bytes_spheres);
            if (W.bytes_sph64) stage_lds(smem + W.lds_sph64, Sg.spheres, W.bytes_sph64);
            S.spair_lds = W.lds_spheres;
        } else {
            stage_lds(smem + W.lds_refs, Sg.refs, W.bytes_refs);
            stage_lds(smem + W.lds_spheres, Sg.spheres, W.bytes_spheres);
            S.refs = reinterpret_cast<const uint32_t*>(smem + W.lds_refs);
            S.spheres = reinterpret_cast<const DevSphere*>(smem + W.lds_spheres);
        }
        __syncthreads();
    } else if (W.ntop) {  // HBM scene: keep the first ntop bytes of f32 nodes (top levels) in LDS
        if (static_cast<uint32_t>(reinterpret_cast<uintptr_t>((LdsByte*)smem)) != 0) __builtin_trap();
        stage_lds(smem, Sg.fnodes, W.ntop);
        S.ntop = W.ntop;
        __syncthreads();
    }
    // The camera constants are read from an LDS copy in start_path / shade: held in SGPRs for
    // the whole kernel they would spill (into VGPR lanes, reloaded with v_readlane per use).
    if (threadIdx.x == 0) *reinterpret_cast<CamView*>(smem + W.lds_cam) = C;
#if CRT_WATCHDOG
    if (threadIdx.x == 0) atomicCAS(&crt_wd_deadline, 0ull, wall_clock64() + 300000000ull);  // 3 s at 100 MHz
#endif
    __syncthreads();
    const CamView& CL = *reinterpret_cast<const CamView*>(smem + W.lds_cam);
    const float tmin32 = W.tmin32;  // a kernel argument (SGPR): no conversion in the walk loop
    const uint32_t lane = threadIdx.x & 63;
    LaneCounters ctr{};
    const unsigned long long t_start = COUNT ? wall_clock64() : 0;
    // stack levels 0..depth of this lane, above two guard levels holding the sentinel reference
    // and one more level walk() may read (three levels in HBM; in LDS that one is other data)
    Stack<SE> st;
    if (GSTACK) {
        st.stride = gridDim.x * kBlock;
        st.base = gstack + (static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x) + 3 * static_cast<size_t>(st.stride);
    } else {
        st.base = reinterpret_cast<SE*>(smem + W.lds_stack) + threadIdx.x;
        st.stride = kBlock;
    }
    st.base[-static_cast<ptrdiff_t>(st.stride)] = static_cast<SE>(W.sentinel);
    st.base[-2 * static_cast<ptrdiff_t>(st.stride)] = static_cast<SE>(W.sentinel);
    // The wave's current item (wave-uniform) and how many of its 64 units are drawn; lanes take
    // the next units in lane order. A unit's sum goes to partial[chunk][pixel] whichever lane
    // traced it, so frames do not depend on the schedule.
    uint32_t item_pos = 0, item_units = 0;
    uint32_t seg = blockIdx.x % W.segments, seg_tried = 0;  // the wave's queue (XCD-local first)
    uint32_t item_txy = 0, item_chunk = 0;
    // the lane's unit: tile (tx | ty << 16), chunk << 6 | tile pixel; and its current sample
    uint32_t u_txy = 0, u_cp = 0, s = 0;
    double acc[3] = {0, 0, 0};
    // the five-wave sphere-only instance: the pixel sum lives in LDS (three doubles a lane,
    // [k][lane]), not in six VGPRs live across every phase (spill stores 17 -> 9; config 2 73.1-73.4
    // -> 72.6 ms, config 3 0.4% slower with it in the flat instance); shade adds a path's
    // contribution to a zeroed local (0 + x = x) that then goes into the LDS sum: the same
    // additions as acc + x
    constexpr bool kAccLds = kFast;
    typedef __attribute__((address_space(3))) double LdsDouble;
    LdsDouble* const acc_l = (LdsDouble*)static_cast<uintptr_t>(W.lds_acc + threadIdx.x * 8);
    // the five-wave flat-parallelogram instance keeps each ray's f64 1 / d in LDS for the walk's f64
    // node tests (slab64_inv) instead of dividing at each one
    constexpr bool kInvLds = (kFlatOnly && LSCENE && W5) || (!LSCENE && !GSTACK);
    // the sibling-pair walk (walk_pairs) of the HBM-scene instances; the instrumented pass walks
    // that way only when it walks like the timed kernel (CRT_COUNT_SPEC=1)
    constexpr bool kPair = CRT_PAIR_WALK && !LSCENE;
    const bool pw = kPair && W.pair_walk && (!COUNT || W.count_spec);
    S.inv64_lds = W.lds_inv64;
    if (kAccLds) {
        acc_l[0] = 0;
        acc_l[kBlock] = 0;
        acc_l[2 * kBlock] = 0;
    }
    Path P;
    Trav R;
    R.state = kIdle;
    bool need = true, start = false, cont = false;
    uint32_t cw = 0, cl = 0, cs = 0;  // wall_clock64 ticks (100 MHz), differences mod 2^32
    uint32_t cd = 0, ci = 0;
    unsigned long long t_first_idle = 0;
    while (true) {
        CRT_WD(1, item_pos, item_units);
        // lanes without a unit draw until each holds a unit with samples to trace or the queue
        // is dry. A unit off the image has no pixel sum; one with max_depth == 0 sums
        // RGB::zero() (camera.h:211-213) and is written at once.
        if (COUNT) cd -= static_cast<uint32_t>(wall_clock64());
        set_prio<kPrioInit>();
        while (true) {
            CRT_WD(2, item_pos, item_units);
            const uint64_t m = __ballot(need);
            if (m == 0) break;
            if (item_pos >= item_units) {  // the item is used up: the next one from a queue
                const uint32_t leader = static_cast<uint32_t>(__ffsll(static_cast<long long>(m)) - 1);
                item_units = 0;
                item_pos = 0;
                // this wave's segment first, then the others in turn; seg == segments: all dry
                while (seg < W.segments) {
                    const uint32_t t0 = static_cast<uint32_t>(static_cast<uint64_t>(W.tiles) * seg / W.segments);
                    const uint32_t t1 = static_cast<uint32_t>(static_cast<uint64_t>(W.tiles) * (seg + 1) / W.segments);
                    const uint32_t nt = t1 - t0, bulk = nt * W.groups;
                    uint32_t v = 0;
                    if (lane == leader) v = atomicAdd(W.queue + seg, 1u);
                    const uint32_t j = __builtin_amdgcn_readlane(v, leader);
                    if (j < nt * (W.groups + W.tail_chunks)) {
                        uint32_t tile;
                        if (j < bulk) {
                            tile = j / W.groups;
                            item_chunk = (j - tile * W.groups) * W.item_chunks;
                            item_units = 64 * W.item_chunks;
                        } else {
                            const uint32_t jt = j - bulk;
                            tile = jt / W.tail_chunks;
                            item_chunk = W.bulk_chunks + (jt - tile * W.tail_chunks);
                            item_units = 64;
                        }
                        tile += t0;
                        item_txy = (tile % W.tiles_x) | ((tile / W.tiles_x) << 16);
                        break;
                    }
                    if (++seg_tried >= W.segments) seg = W.segments;  // every segment is dry
                    else seg = seg + 1 == W.segments ? 0 : seg + 1;
                }
            }
            if (item_units == 0) {  // the queues are dry
                need = false;
                break;
            }
            const uint32_t take = min(static_cast<uint32_t>(__popcll(m)), item_units - item_pos);
            const uint32_t r = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                         __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u));
            if (need && r < take) {
                const uint32_t uu = item_pos + r, pix = uu & 63, chunk = item_chunk + (uu >> 6);
                u_txy = item_txy;
                u_cp = (chunk << 6) | pix;
                // band-local column and owned row
                const uint32_t col = (item_txy & 0xffffu) * kTileW + pix % kTileW, k = (item_txy >> 16) * kTileH + pix / kTileW;
                if (chunk < W.chunks && col < W.bw && k < W.bh) {
                    s = chunk * W.chunk_len;
                    if (C.max_depth > 0) {
                        need = false;
                        start = true;
                    } else if (!COUNT) {
                        double* dst = partial + (static_cast<size_t>(chunk) * W.bh * W.bw +
                                                 static_cast<size_t>(k) * W.bw + col) * 3;
                        dst[0] = 0;
                        dst[1] = 0;
                        dst[2] = 0;
                    }
                }
            }
            item_pos += take;
        }
        if (COUNT) {
            const uint32_t now = static_cast<uint32_t>(wall_clock64());
            cd += now;
            ci -= now;
        }
        if (start) {
            const uint32_t pix = u_cp & 63;
            const uint32_t col = W.col0 + (u_txy & 0xffffu) * kTileW + pix % kTileW;
            const uint32_t row = owned_row(W, W.k0 + (u_txy >> 16) * kTileH + pix / kTileW);
            start_path(CL, row, col, sample_seed(C.base_seed, row * C.w + col, s), P);
        }
        // one traversal set-up for new samples and scattered rays alike (the wave runs it once);
        // the guard level below the stack gets the sentinel back (the f32 walk's store at the
        // sentinel overwrote it)
        if (start || cont) {
            trav_init(P.o, P.d, W.f32_ok != 0, R);
            // the pair walk's lanes hold tokens (walk_pairs): the root pair's left child, and the
            // sentinel's token in the guard level; rays that need the EXACT walk keep plain refs
            const bool tok = kPair && pw && !(R.neg & kZeroDir);
            st.base[-static_cast<ptrdiff_t>(st.stride)] = static_cast<SE>(W.sentinel | (tok ? kTokAlone : 0u));
            if (!kFlatOnly) st.base[-2 * static_cast<ptrdiff_t>(st.stride)] = static_cast<SE>(W.sentinel | (tok ? kTokAlone : 0u));
            if (tok) R.cur = kTokAlone;
            if (kInvLds) {  // the f64 node test's 1 / d, divided once per ray (slab64_inv)
                uint32_t t = threadIdx.x;
                asm volatile("" : "+v"(t));
                LdsDouble* const inv_l = (LdsDouble*)static_cast<uintptr_t>(W.lds_inv64 + t * 8);
                inv_l[0] = 1 / P.d[0];
                inv_l[kBlock] = 1 / P.d[1];
                inv_l[2 * kBlock] = 1 / P.d[2];
            }
            if (COUNT) ctr.rays++;
        }
        start = false;
        cont = false;
        if (COUNT) ci += static_cast<uint32_t>(wall_clock64());
        // traversal rounds (walk to the next entered leaf, test it) until enough lanes hold a
        // finished ray, or none is traversing
        while (true) {
            CRT_WD(3, R.state, R.cur);
            if (COUNT && W.round_counters) {
                const unsigned long long nw = __popcll(__ballot(R.state == kWalk));
                if (wave_leader()) {
                    atomicAdd(&counters->rounds, 1ull);
                    atomicAdd(&counters->round_walkers, nw);
                }
            }
            if (COUNT) cw -= static_cast<uint32_t>(wall_clock64());
            set_prio<kPrioWalk>();
            if (kPair && pw) {
                // W.pair_walk is off for scenes that need the EXACT walk (W.exact_slab); a ray
                // with a zero / tiny / huge direction component takes it, on plain refs
                if (__ballot(R.state == kWalk && (R.neg & kZeroDir)) != 0) {
                    if (R.state == kWalk && (R.neg & kZeroDir))
                        walk<SE, COUNT, true, kTopTreelet && !LSCENE, LSCENE, GSTACK, false>(S, st, P.o, P.d, C.t_min, tmin32, R, ctr);
                }
                if (R.state == kWalk && !(R.neg & kZeroDir))
                    walk_pairs<SE, COUNT, kTopTreelet && !LSCENE, kInvLds>(S, st, P.o, P.d, C.t_min, tmin32, R, ctr);
            } else if (!W.exact_slab && __ballot(R.state == kWalk && (R.neg & kZeroDir)) == 0) {
                if (R.state == kWalk) {
                    if (!COUNT || W.count_spec)
                        walk<SE, COUNT, false, kTopTreelet && !LSCENE, LSCENE, GSTACK, true, kInvLds, !kFlatOnly>(S, st, P.o, P.d, C.t_min, tmin32, R, ctr);
                    else
                        walk<SE, COUNT, false, kTopTreelet && !LSCENE, LSCENE, GSTACK, false, kInvLds>(S, st, P.o, P.d, C.t_min, tmin32, R, ctr);
                }
            } else {
                if (R.state == kWalk) walk<SE, COUNT, true, kTopTreelet && !LSCENE, LSCENE, GSTACK, false>(S, st, P.o, P.d, C.t_min, tmin32, R, ctr);
            }
            if (COUNT) cw += static_cast<uint32_t>(wall_clock64());
            set_prio<kPrioLeaf>();
            if (COUNT && W.round_counters) {
                const unsigned long long nl = __popcll(__ballot(R.state == kLeaf));
                if (wave_leader()) atomicAdd(&counters->round_leaves, nl);
            }
            if (COUNT) cl -= static_cast<uint32_t>(wall_clock64());
            if (R.state == kLeaf) leaf_step<SE, COUNT, kTopTreelet && !LSCENE, LSCENE, kFast, kFlatOnly>(S, st, P.o, P.d, C.t_min, tmin32, kSphOnly || (!kFlatOnly && W.sphere_only != 0), !kFlatOnly && W.spheres_f32 != 0, kFlatOnly || (!kSphOnly && W.quads_f32 != 0), kFlatOnly || (!kSphOnly && W.quads_flat != 0), R, ctr);
            if (COUNT) cl += static_cast<uint32_t>(wall_clock64());
            const uint64_t pending = __ballot(R.state == kWalk);
            const uint64_t finished = __ballot(R.state == kDone);
            const int nfin = __popcll(finished);
            if (COUNT && W.round_counters && wave_leader()) atomicAdd(&counters->round_done, static_cast<unsigned long long>(nfin));
            if (pending == 0 || nfin >= kShadeBatch) break;
        }
        const uint64_t m_done = __ballot(R.state == kDone);
        if (COUNT && t_first_idle == 0 && __ballot(R.state == kIdle) != 0) t_first_idle = wall_clock64();
        if (m_done == 0) break;  // every lane idle: the queue is dry
        if (COUNT) cs -= static_cast<uint32_t>(wall_clock64());
        set_prio<kPrioShade>();
        if (COUNT && W.round_counters && wave_leader()) atomicAdd(&counters->shade_rounds, 1ull);
        if (COUNT && ((ctr.rays | ctr.nodes | ctr.sphere_tests | ctr.quad_tests | ctr.it_walk | ctr.it_leaf |
                       ctr.it_shade | ctr.slow_nodes | ctr.it_slow | ctr.cand | ctr.it_cand) & 0x80000000u))
            flush_counts(ctr, counters);
        if (R.state == kDone) {
            if (COUNT && wave_leader()) ctr.it_shade++;
            double contrib[3] = {0, 0, 0};
            bool ended = shade<LSCENE, kSphOnly, kFlatOnly, kFast>(S, CL, P, R.found, R.ref, R.tmax, kAccLds ? contrib : acc);
            if (kAccLds && ended) {
                acc_l[0] = acc_l[0] + contrib[0];
                acc_l[kBlock] = acc_l[kBlock] + contrib[1];
                acc_l[2 * kBlock] = acc_l[2 * kBlock] + contrib[2];
            }
            // a scattered ray with no bounce left returns RGB::zero() (camera.h:211-213)
            if (!ended && P.depth == 0) ended = true;
            if (!ended) {
                cont = true;  // the scattered ray: traversal set-up with the new samples' (above)
            } else {
                const uint32_t chunk = u_cp >> 6;
                if (++s < min(C.spp, (chunk + 1) * W.chunk_len)) {
                    start = true;  // the unit's next sample (started after the draw, with the drawers)
                } else {  // the unit is done: its sum (samples in order) to partial[chunk][pixel]
                    if (!COUNT) {
                        const uint32_t pix = u_cp & 63;
                        const uint32_t col = (u_txy & 0xffffu) * kTileW + pix % kTileW, k = (u_txy >> 16) * kTileH + pix / kTileW;
                        double* dst = partial + (static_cast<size_t>(chunk) * W.bh * W.bw +
                                                 static_cast<size_t>(k) * W.bw + col) * 3;
                        dst[0] = kAccLds ? acc_l[0] : acc[0];
                        dst[1] = kAccLds ? acc_l[kBlock] : acc[1];
                        dst[2] = kAccLds ? acc_l[2 * kBlock] : acc[2];
                    }
                    if (kAccLds) {
                        acc_l[0] = 0;
                        acc_l[kBlock] = 0;
                        acc_l[2 * kBlock] = 0;
                    }
                    acc[0] = 0;
                    acc[1] = 0;
                    acc[2] = 0;
                    need = true;
                }
                R.state = kIdle;
            }
        }
        if (COUNT) cs += static_cast<uint32_t>(wall_clock64());
    }
    if (COUNT) {
        using ull = unsigned long long;
        flush_counts(ctr, counters);
        if (lane == 0) {  // per-wave phase times (the wave executes each phase as one)
            atomicAdd(&counters->cyc_walk, static_cast<ull>(cw));
            atomicAdd(&counters->cyc_leaf, static_cast<ull>(cl));
            atomicAdd(&counters->cyc_shade, static_cast<ull>(cs));
            atomicAdd(&counters->cyc_draw, static_cast<ull>(cd));
            atomicAdd(&counters->cyc_init, static_cast<ull>(ci));
            const unsigned long long t_end = wall_clock64();
            atomicAdd(&counters->cyc_total, t_end - t_start);
            atomicAdd(&counters->cyc_tail, t_first_idle ? t_end - t_first_idle : 0ull);
        }
    }
}

// pixel_color /= spp (camera.h:290, rgb.h:76): sum the chunks in order, multiply by 1/spp.
// One thread per pixel of the launch's band.
__global__ __launch_bounds__(256) void resolve_kernel(const double* __restrict__ partial,
                                                      double* __restrict__ out, Work W, uint32_t w,
                                                      uint32_t h, double inv_spp) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    const uint64_t band = static_cast<uint64_t>(W.bh) * W.bw;
    if (i >= band) return;
    const uint32_t k = W.k0 + static_cast<uint32_t>(i / W.bw), col = W.col0 + static_cast<uint32_t>(i % W.bw);
    const size_t pix = static_cast<size_t>(W.packed ? k : owned_row(W, k)) * w + col;
    const size_t plane = band * 3;
    double r = partial[i * 3 + 0], g = partial[i * 3 + 1], b = partial[i * 3 + 2];
    for (uint32_t c = 1; c < W.chunks; ++c) {
        r = r + partial[c * plane + i * 3 + 0];
        g = g + partial[c * plane + i * 3 + 1];
        b = b + partial[c * plane + i * 3 + 2];
    }
    out[pix * 3 + 0] = r * inv_spp;
    out[pix * 3 + 1] = g * inv_spp;
    out[pix * 3 + 2] = b * inv_spp;
}

// Image::send_as_ppm's integers (image.h:38-56; RGB::as_string rgb.h:99-115 with its defaults):
// Reinhard by luminance (rgb.h:27-29), gamma 2, static_cast<int>(255.999999 * .). The reference
// takes std::pow(x, 1/2) (rgb.h:10-13), a libm pow within ~1 ulp of the correctly rounded sqrt
// used here; where the truncated integer could differ for any value within 2 ulps of sqrt(x)
// (or v is NaN / out of int range), the kernel writes kPpmRedo and the host recomputes that
// pixel with std::pow (device_ppm_values), so every integer is the reference's.
constexpr double kPpmScale = 255 + 0.999999;
constexpr int32_t kPpmRedo = INT32_MIN + 1;

__device__ __forceinline__ int32_t ppm_channel(double c, double L) {
    const double x = c / (1 + L);
    const double s = sqrt(x);
    const double v = kPpmScale * s;
    if (!(v >= 0 && v < 2147483648.0)) return kPpmRedo;
    if (s < 0x1p-1000) return 0;  // pow(x, 0.5) is below 2^-999 too
    const uint64_t bits = static_cast<uint64_t>(__double_as_longlong(s));
    const double lo = __longlong_as_double(static_cast<long long>(bits - 2));
    const double hi = __longlong_as_double(static_cast<long long>(bits + 2));
    return static_cast<int32_t>(kPpmScale * lo) == static_cast<int32_t>(kPpmScale * hi) ? static_cast<int32_t>(v)
                                                                                          : kPpmRedo;
}

__global__ __launch_bounds__(256) void ppm_kernel(const double* __restrict__ rgb, uint64_t n,
                                                  int32_t* __restrict__ out) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i >= n) return;
    const double c[3] = {rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2]};
    const double L = 0.2126 * c[0] + 0.7152 * c[1] + 0.0722 * c[2];
#pragma unroll
    for (int k = 0; k < 3; ++k) out[3 * i + k] = ppm_channel(c[k], L);
}

// The same values as 8-bit bytes (the fused output of crt_render_ppm: 3 B a pixel cross xGMI and
// PCIe instead of 24). A pixel with a value the kernel cannot settle, or outside [0, 255] (a NaN
// pixel prints INT_MIN), is listed in redo = [count, pixel...] (at most cap) for the host.
__global__ __launch_bounds__(256) void ppm8_kernel(const double* __restrict__ rgb, uint64_t n,
                                                   uint8_t* __restrict__ out, uint32_t* __restrict__ redo,
                                                   uint32_t cap) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i >= n) return;
    const double c[3] = {rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2]};
    const double L = 0.2126 * c[0] + 0.7152 * c[1] + 0.0722 * c[2];
    int32_t q[3];
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        q[k] = ppm_channel(c[k], L);
        ok = ok && q[k] >= 0 && q[k] <= 255;
    }
    if (!ok) {
        const uint32_t j = atomicAdd(redo, 1u);
        if (j < cap) redo[1 + j] = static_cast<uint32_t>(i);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) out[3 * i + k] = ok ? static_cast<uint8_t>(q[k]) : 0;
}

// The f64 values of the pixels ppm8_kernel listed for the host (redo = [count, pixel...]),
// gathered into one compact buffer: the host then copies them in one transfer
__global__ __launch_bounds__(256) void redo_gather_kernel(const double* __restrict__ rgb,
                                                          const uint32_t* __restrict__ list, uint32_t n,
                                                          double* __restrict__ out) {
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    const size_t i = list[j];
#pragma unroll
    for (int k = 0; k < 3; ++k) out[3 * static_cast<size_t>(j) + k] = rgb[3 * i + k];
}

// Closest-hit queries (BVH::hit_by for an arbitrary ray batch).
__global__ __launch_bounds__(kBlock) void hits_kernel(SceneView S, const double* __restrict__ rays,
                                                      uint32_t n, double t_min, double t_max,
                                                      const uint32_t* __restrict__ ref_prim,
                                                      uint32_t num_spheres,
                                                      crt_hit* __restrict__ out,
                                                      uint32_t* __restrict__ gstack) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    Stack<uint32_t> st;
    st.base = gstack + i;
    st.stride = gridDim.x * kBlock;
    double o[3] = {rays[6 * i + 0], rays[6 * i + 1], rays[6 * i + 2]};
    double d[3] = {rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]};
    double tmax = t_max;
    uint32_t ref = 0;
    LaneCounters ctr{};
    crt_hit h{};
    h.prim = -1;
    if (trace<uint32_t, false>(S, st, o, d, t_min, tmax, ref, ctr)) {
        double p[3], nrm[3];
        bool front;
        h.material = hit_record<false>(S, ref, o, d, tmax, p, nrm, front);
        h.t = tmax;
        for (int k = 0; k < 3; ++k) { h.point[k] = p[k]; h.normal[k] = nrm[k]; }
        h.front_face = front ? 1 : 0;
        // ref_prim: spheres at [0, num_spheres), parallelograms after them
        const uint32_t k = (ref & kRefQuad) ? num_spheres + (ref & ~kRefQuad) : ref;
        h.prim = static_cast<int32_t>(ref_prim[k]);
    }
    out[i] = h;
}

}  // namespace dev

// =============================================================================================
// host launch plumbing

static dev::SceneView view_of(const DeviceCopy& c) {
    dev::SceneView v{c.nodes, c.fnodes, 0, c.refs, c.spheres, c.spair, 0, c.sphere_mat, c.quads, c.quad_mat,
                     c.mats, c.quadf, c.sphere_mrec, c.quad_mrec, 0, c.quadbox};
    v.guard = c.guard;
    return v;
}

int device_count(int* n) {
    hipError_t e = hipGetDeviceCount(n);
    if (e != hipSuccess) {
        *n = 0;
        return fail(CRT_E_NODEVICE, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    }
    return CRT_OK;
}

static int check_device(int device) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
        return fail(CRT_E_NODEVICE, "no HIP device visible (the render path has no CPU fallback)");
    if (device < 0 || device >= n || device >= kMaxDevices)
        return fail(CRT_E_NODEVICE, "device " + std::to_string(device) + " out of range");
    return CRT_OK;
}

struct DeviceGuard {
    int prev = 0;
    explicit DeviceGuard(int d) { (void)hipGetDevice(&prev); (void)hipSetDevice(d); }
    ~DeviceGuard() { (void)hipSetDevice(prev); }
};

static size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// The device image of a scene: every array of device_layout() at its offset in one host buffer,
// built once per scene (the first upload) and copied whole to each device. The derived arrays
// (f32 nodes, filter records, per-slot material records) are written straight into the image,
// per element in parallel (parallel_for); the image is not zero-filled first, only the guard words
// (and the padding, which nothing reads) are cleared.
static void stage_image(crt_scene* s) {
    const size_t n_nodes = s->num_dnodes, n_refs = s->num_prims;
    const size_t n_sp = s->num_spheres, n_q = s->num_quads, n_m = s->num_dmats;
    size_t off[kArrCount + 1];
    const size_t total = device_layout(s, off);
    BigVec<char>& img = s->image;
    img.resize(total);
    auto at = [&](int arr) { return img.data() + off[arr]; };
    // padding between the arrays (and the guard words): zero
    for (int a = 0; a < kArrCount; ++a) {
        static const size_t kElem[kArrCount] = {sizeof(DevNode), sizeof(DevNodeF), 4, sizeof(DevSphere), sizeof(DevSpherePair),
                                                4, sizeof(DevQuad), sizeof(DevQuadF), sizeof(DevQuadBox), 4,
                                                sizeof(DevMaterial), sizeof(DevMaterial), sizeof(DevMaterial), 1};
        const size_t cnt[kArrCount] = {n_nodes, n_nodes, n_refs, n_sp, n_sp, n_sp, n_q, n_q, n_q, n_q, n_m, n_sp, n_q, 64};
        const size_t used = a == kArrGuard ? 0 : cnt[a] * kElem[a];
        std::memset(img.data() + off[a] + used, 0, off[a + 1] - off[a] - used);
    }
    // plain copies, in parallel chunks
    auto put = [&](int arr, const void* src, size_t bytes) {
        char* dst = at(arr);
        const char* sp = static_cast<const char*>(src);
        parallel_for(bytes, size_t{1} << 22, [&](size_t a, size_t b) { std::memcpy(dst + a, sp + a, b - a); });
    };
    put(kArrNodes, s->dnodes.data(), n_nodes * sizeof(DevNode));
    put(kArrRefs, s->refs.data(), n_refs * 4);
    put(kArrSpheres, s->spheres.data(), n_sp * sizeof(DevSphere));
    put(kArrSphereMat, s->sphere_mat.data(), n_sp * 4);
    put(kArrQuads, s->quads.data(), n_q * sizeof(DevQuad));
    put(kArrQuadMat, s->quad_mat.data(), n_q * 4);
    put(kArrMats, s->dmats.data(), n_m * sizeof(DevMaterial));
    // f32 refs are byte offsets (index << 5) and interior w1 must stay below kLeafFlagF
    DevNodeF* fnodes = reinterpret_cast<DevNodeF*>(at(kArrFNodes));
    std::atomic<bool> f32_bad{false};
    parallel_for(n_nodes, 4096, [&](size_t a, size_t b) {
        bool bad = false;
        for (size_t i = a; i < b; ++i) bad = node_record(s->dnodes[i], static_cast<uint32_t>(i), fnodes[i]) || bad;
        if (bad) f32_bad = true;
    });
    // sphere pair records of the f32 candidate filter (slots i, i + 1): half i of record i from
    // sphere i, the other half from sphere i + 1 (the last record's second half zero)
    DevSpherePair* spair = reinterpret_cast<DevSpherePair*>(at(kArrSpherePairs));
    std::atomic<bool> sph_bad{false};
    parallel_for(n_sp, 4096, [&](size_t a, size_t b) {
        bool bad = false;
        for (size_t i = a; i < b; ++i) {
            DevSpherePair& r = spair[i];
            bad = sphere_pair_half(s->spheres[i], r.cx[0], r.cy[0], r.cz[0], r.r2e[0]) || bad;
            if (i + 1 < n_sp) (void)sphere_pair_half(s->spheres[i + 1], r.cx[1], r.cy[1], r.cz[1], r.r2e[1]);
            else r.cx[1] = r.cy[1] = r.cz[1] = r.r2e[1] = 0;
        }
        if (bad) sph_bad = true;
    });
    // parallelogram filter records (crt_quad_filter.h quad_record, quad_flat_box)
    DevQuadF* quadf = reinterpret_cast<DevQuadF*>(at(kArrQuadF));
    DevQuadBox* quadbox = reinterpret_cast<DevQuadBox*>(at(kArrQuadBox));
    std::atomic<bool> quads_bad{false}, flat_bad{false};
    parallel_for(n_q, 4096, [&](size_t a, size_t b) {
        bool qb = false, fb = false;
        for (size_t i = a; i < b; ++i) {
            const DevQuad& q = s->quads[i];
            if (!quad_record(q.v, q.s1, q.s2, q.sn, quadf[i])) qb = true;
            quadbox[i] = DevQuadBox{};  // a record quad_flat_box rejects stays zero
            if (!quad_flat_box(q.v, q.s1, q.s2, quadbox[i])) fb = true;
        }
        if (qb) quads_bad = true;
        if (fb) flat_bad = true;
    });
    // parallelogram-only scenes of axis-aligned parallelograms: each leaf's flat boxes grouped by
    // their flat axis (regroup_leaf)
    std::atomic<bool> regroup_bad{false};
    if (!flat_bad && n_sp == 0 && n_q > 0) {
        parallel_for(n_nodes, 1 << 12, [&](size_t a, size_t b) {
            bool bad = false;
            for (size_t k = a; k < b; ++k) bad = regroup_leaf(s->dnodes[k], k, quadbox) || bad;
            if (bad) regroup_bad = true;
        });
    }
    // shading constants per slot (shading_consts)
    DevMaterial* smrec = reinterpret_cast<DevMaterial*>(at(kArrSphereMrec));
    DevMaterial* qmrec = reinterpret_cast<DevMaterial*>(at(kArrQuadMrec));
    parallel_for(n_sp, 4096, [&](size_t a, size_t b) {
        for (size_t i = a; i < b; ++i) {
            smrec[i] = s->dmats[s->sphere_mat[i]];
            shading_consts(smrec[i], &s->spheres[i]);
        }
    });
    parallel_for(n_q, 4096, [&](size_t a, size_t b) {
        for (size_t i = a; i < b; ++i) {
            qmrec[i] = s->dmats[s->quad_mat[i]];
            shading_consts(qmrec[i], nullptr);
        }
    });
    s->image_f32_ok = !f32_bad;
    s->image_spheres_f32_ok = !sph_bad;
    s->image_quads_f32_ok = !quads_bad;
    s->image_quads_flat_ok = !flat_bad && !regroup_bad;
    s->staged = true;
}

// The pointers of a scene copy at `base` (device_layout's arrays at their offsets).
void device_bind_copy(crt_scene* s, int device, void* base, size_t total) {
    size_t off[kArrCount + 1];
    (void)device_layout(s, off);
    DeviceCopy& c = s->dev[device];
    char* b = static_cast<char*>(base);
    c.base = base;
    c.bytes = total;
    c.nodes = reinterpret_cast<DevNode*>(b + off[kArrNodes]);
    c.fnodes = reinterpret_cast<DevNodeF*>(b + off[kArrFNodes]);
    c.f32_ok = s->image_f32_ok && std::getenv("CRT_F64_NODES") == nullptr;
    c.refs = reinterpret_cast<uint32_t*>(b + off[kArrRefs]);
    c.spheres = reinterpret_cast<DevSphere*>(b + off[kArrSpheres]);
    c.spair = reinterpret_cast<DevSpherePair*>(b + off[kArrSpherePairs]);
    c.spheres_f32_ok = s->image_spheres_f32_ok && std::getenv("CRT_F64_SPHERES") == nullptr;
    c.sphere_mat = reinterpret_cast<uint32_t*>(b + off[kArrSphereMat]);
    c.quads = reinterpret_cast<DevQuad*>(b + off[kArrQuads]);
    c.quadf = reinterpret_cast<DevQuadF*>(b + off[kArrQuadF]);
    c.quads_f32_ok = s->image_quads_f32_ok && std::getenv("CRT_F64_QUADS") == nullptr;
    c.quadbox = reinterpret_cast<DevQuadBox*>(b + off[kArrQuadBox]);
    // CRT_GENERIC_QUADS=1: the generic parallelogram filter even for axis-aligned ones
    c.quads_flat_ok = s->image_quads_flat_ok && std::getenv("CRT_GENERIC_QUADS") == nullptr;
    c.quad_mat = reinterpret_cast<uint32_t*>(b + off[kArrQuadMat]);
    c.mats = reinterpret_cast<DevMaterial*>(b + off[kArrMats]);
    c.sphere_mrec = reinterpret_cast<DevMaterial*>(b + off[kArrSphereMrec]);
    c.quad_mrec = reinterpret_cast<DevMaterial*>(b + off[kArrQuadMrec]);
    c.guard = reinterpret_cast<unsigned long long*>(b + off[kArrGuard]);
    c.valid = true;
}

// Copy the scene into HBM of `device`: the staged image in one transfer. Uploads to different
// devices run concurrently (render_multi uploads from one thread per device); the image is
// staged once, under the scene's lock. A scene set up on a device (crt_stage_gpu.hip) is copied
// from that device's HBM instead (its copy there is already in place).
int device_upload(crt_scene* s, int device) {
    int rc = check_device(device);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(s->dev_mu[device]);
    DeviceCopy& c = s->dev[device];
    if (c.valid) return CRT_OK;
    if (s->num_dnodes >= (size_t{1} << (31 - kNodeFShift)))
        return fail(CRT_E_INVALID, "BVH too large for the device node layout");
    if (s->image_device < 0) {
        std::lock_guard<std::mutex> ls(s->mu);
        if (!s->staged) stage_image(s);
    }
    size_t off[kArrCount + 1];
    const size_t total = device_layout(s, off);
    DeviceGuard g(device);
    void* base = nullptr;
    HIP_TRY(hipMalloc(&base, total));
    hipError_t e = s->image_device >= 0
                       ? hipMemcpyPeer(base, device, s->dev[s->image_device].base, s->image_device, total)
                       : hipMemcpy(base, s->image.data(), total, hipMemcpyHostToDevice);
    // a peer copy also carries the source copy's guard words (its running Schlick count, counted
    // into by renders on that device): a new copy starts at zero, as a host-staged one does
    if (e == hipSuccess && s->image_device >= 0)
        e = hipMemset(static_cast<char*>(base) + off[kArrGuard], 0, total - off[kArrGuard]);
    if (e != hipSuccess) {
        (void)hipFree(base);
        return fail(CRT_E_HIP, std::string("scene upload: ") + hipGetErrorString(e));
    }
    device_bind_copy(s, device, base, total);
    return CRT_OK;
}

// the guard words of the scene's copy on `device` (after the renders that count into them have
// completed: synchronizes the device)
int device_guard(crt_scene* s, int device, uint64_t* schlick_undecided, bool reset) {
    int rc = check_device(device);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(s->dev_mu[device]);
    DeviceCopy& c = s->dev[device];
    if (!c.valid) return fail(CRT_E_NOT_UPLOADED, "crt_render_guard: scene not uploaded to this device");
    DeviceGuard g(device);
    HIP_TRY(hipDeviceSynchronize());
    unsigned long long v = 0;
    HIP_TRY(hipMemcpy(&v, c.guard, sizeof v, hipMemcpyDeviceToHost));
    if (reset) HIP_TRY(hipMemset(c.guard, 0, sizeof v));
    *schlick_undecided = v;
    return CRT_OK;
}

int device_image(crt_scene* s, int device, void* host, size_t bytes) {
    int rc = device_upload(s, device);
    if (rc) return rc;
    const DeviceCopy& c = s->dev[device];
    if (bytes != c.bytes)
        return fail(CRT_E_INVALID, "crt_scene_image: bytes must be " + std::to_string(c.bytes));
    DeviceGuard g(device);
    HIP_TRY(hipMemcpy(host, c.base, c.bytes, hipMemcpyDeviceToHost));
    return CRT_OK;
}

void device_release(crt_scene* s) {
    for (int d = 0; d < kMaxDevices; ++d) {
        DeviceCopy& c = s->dev[d];
        if (!c.valid) continue;
        DeviceGuard g(d);
        (void)hipFree(c.base);
        c = DeviceCopy{};
    }
}

static dev::CamView cam_view(const crt_camera* cam) {
    dev::CamView v{};
    for (int k = 0; k < 3; ++k) {
        v.o[k] = cam->origin[k];
        v.p00[k] = cam->pixel00[k];
        v.pdx[k] = cam->pixel_delta_x[k];
        v.pdy[k] = cam->pixel_delta_y[k];
        v.ddx[k] = cam->defocus_disk_x[k];
        v.ddy[k] = cam->defocus_disk_y[k];
        v.bg[k] = cam->background[k];
    }
    v.defocus_angle = cam->defocus_angle;
    v.t_min = cam->t_min;
    v.inv_spp = 1 / static_cast<double>(cam->samples_per_pixel);
    v.w = cam->image_w;
    v.h = cam->image_h;
    v.spp = cam->samples_per_pixel;
    v.max_depth = cam->max_depth;
    v.base_seed = cam->base_seed;
    return v;
}

static uint32_t count_owned(uint32_t h, uint32_t rb, uint32_t tc, uint32_t ti) {
    uint32_t n = 0;
    for (uint32_t r = 0; r < h; ++r)
        if ((r / rb) % tc == ti) ++n;
    return n;
}

static size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

constexpr size_t kAccBytes = 3 * dev::kBlock * sizeof(double);  // five-wave sphere-only pixel sums
constexpr size_t kInvBytes = 3 * dev::kBlock * sizeof(double);  // flat-parallelogram instances' 1 / d
constexpr size_t kLdsSceneBudget = 40 * 1024 * dev::kBlock / 256;  // scene + stack per block (4 blocks of 256 a CU)
// sphere-only LDS scenes also stage the f64 spheres (pass 2's exact tests, shading) when the block
// still fits 40 KB: rtow 40.6 KB, 84.7 vs 85.4 ms with them in HBM / L1 (v12; round 1's layout,
// with even-aligned filter records to make room, had measured the opposite)
constexpr size_t kLdsStackBudget = 32 * 1024 * dev::kBlock / 256;

// Partial-sum budget per launch (bytes): the owned frame is rendered in bands whose partial sums
// fit it (CRT_PARTIAL_MB overrides; tests force many small bands). 4 GiB holds a whole config-2
// frame (2.9 GB) in one band; config 5 on one GPU (37.6 GB of partial sums) takes 10.
static size_t partial_budget() {
    if (const char* e = std::getenv("CRT_PARTIAL_MB"))
        return static_cast<size_t>(std::max(1, std::atoi(e))) << 20;
    return size_t{4} << 30;
}

template <typename SE, bool GSTACK, bool LSCENE, int PM, bool W5 = false>
static int launch_render(const crt_scene* s, int device, const crt_camera* cam, const dev::Work& w0,
                         size_t lds, double* d_rgb, hipStream_t stream, crt_render_stats* count_stats) {
    const DeviceCopy& c = s->dev[device];
    dev::Work W = w0;
    W.lds_cam = static_cast<uint32_t>(align16(lds));  // the camera copy after the rest
    lds = W.lds_cam + align16(sizeof(dev::CamView));
    if (W5 && PM == 0) {  // then the pixel sums (render_kernel: kAccLds)
        W.lds_acc = static_cast<uint32_t>(align16(lds));
        lds = W.lds_acc + kAccBytes;
    }
    if ((LSCENE && PM == 2 && W5) || (!LSCENE && !GSTACK)) {  // or the rays' f64 1 / d (render_kernel: kInvLds)
        W.lds_inv64 = static_cast<uint32_t>(align16(lds));
        lds = W.lds_inv64 + kInvBytes;
    }
    constexpr int kThreads = dev::kBlock;
    const void* kfn = reinterpret_cast<const void*>(dev::render_kernel<SE, GSTACK, LSCENE, false, PM, W5>);
    const uint64_t pixels = static_cast<uint64_t>(W.owned_rows) * cam->image_w;
    // Sample chunks: a function of spp ONLY, so every pixel's sum is grouped identically whatever
    // the tiling / number of GPUs / lane schedule / band split (bit-identical frames for 1..N
    // devices): 4 samples, or spp / 192 above 768 spp. A unit is the grain the grid drains on:
    // per-rank share at 8 GPUs 12.2 ms with 4-sample chunks vs 13.0 with 8 (one GPU 87.4 vs 87.5;
    // the partial sums double to 2.9 GB per config-2 frame). The persistent grid's waves take
    // (tile, chunk) items from a queue in tile-major order (render_kernel).
    const uint32_t spp = cam->samples_per_pixel;
#ifndef CRT_CHUNK_MIN
#define CRT_CHUNK_MIN 4
#endif
    W.chunk_len = std::max<uint32_t>(CRT_CHUNK_MIN, (spp + 191) / 192);
    W.chunks = (spp + W.chunk_len - 1) / W.chunk_len;
    W.rb_shift = 32;
    for (uint32_t sh = 0; sh < 31; ++sh)
        if ((1u << sh) == W.row_block) W.rb_shift = sh;
    // Bands: rectangles of bx x by tiles over the owned rows x width, each one launch (render +
    // resolve). bx, by <= 65535 (a unit packs its tile as tx | ty << 16), and a band's partial
    // sums (64 pixels x 3 x chunks doubles per tile) fit the budget. A pixel's chunks are summed
    // in the same order in any band, so the split does not change frames.
    constexpr uint64_t kMaxTiles = 65535;
    const uint64_t tiles_x_all = (static_cast<uint64_t>(cam->image_w) + dev::kTileW - 1) / dev::kTileW;
    const uint64_t tiles_y_all = (static_cast<uint64_t>(W.owned_rows) + dev::kTileH - 1) / dev::kTileH;
    const uint64_t tile_bytes = 64ull * 3 * sizeof(double) * W.chunks;
    const uint64_t cap = std::max<uint64_t>(1, partial_budget() / tile_bytes);
    const uint32_t bx = static_cast<uint32_t>(std::min({tiles_x_all, kMaxTiles, cap}));
    const uint32_t by = static_cast<uint32_t>(std::min({tiles_y_all, kMaxTiles, std::max<uint64_t>(1, cap / bx)}));
    // the grid: every resident block (more would only wait), fewer when a band's items are fewer
    int cus = 0, per_cu = 0;
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, kThreads, lds));
    constexpr uint32_t kWavesPerBlock = kThreads / 64;
    uint64_t resident = static_cast<uint64_t>(std::max(1, cus)) * std::max(1, per_cu);
    if (const char* e = std::getenv("CRT_GRID_BLOCKS"))  // schedule tests: a smaller grid, same frame
        resident = std::max<uint64_t>(1, std::min<uint64_t>(resident, static_cast<uint64_t>(std::max(1, std::atoi(e)))));
    auto knob = [](const char* name, uint32_t dflt) {
        const char* e = std::getenv(name);
        return e ? static_cast<uint32_t>(std::max(0, std::min(4096, std::atoi(e)))) : dflt;
    };

    double* partial = nullptr;
    SE* gstack = nullptr;
    dev::Counters* ctr = nullptr;
    const bool count = count_stats != nullptr;
    const uint64_t band_px = std::min<uint64_t>(static_cast<uint64_t>(bx) * dev::kTileW, cam->image_w) *
                             std::min<uint64_t>(static_cast<uint64_t>(by) * dev::kTileH, W.owned_rows);
    if (!count)
        HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&partial), band_px * 3 * W.chunks * sizeof(double), stream));
    if (GSTACK) {
        size_t bytes = static_cast<size_t>(s->depth + 4) * resident * dev::kBlock * sizeof(SE);  // + 3 levels below
        HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&gstack), bytes, stream));
    }
    if (count) {
        HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&ctr), sizeof(dev::Counters), stream));
        HIP_TRY(hipMemsetAsync(ctr, 0, sizeof(dev::Counters), stream));
    }
    uint32_t* queue = nullptr;
    HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&queue), 256, stream));
    W.queue = queue;
    dev::SceneView S = view_of(c);
    dev::CamView C = cam_view(cam);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (count) {
        HIP_TRY(hipEventCreate(&e0));
        HIP_TRY(hipEventCreate(&e1));
        HIP_TRY(hipEventRecord(e0, stream));
    }
    for (uint64_t ty0 = 0; ty0 < tiles_y_all; ty0 += by) {
        for (uint64_t tx0 = 0; tx0 < tiles_x_all; tx0 += bx) {
            W.col0 = static_cast<uint32_t>(tx0 * dev::kTileW);
            W.k0 = static_cast<uint32_t>(ty0 * dev::kTileH);
            W.bw = static_cast<uint32_t>(std::min<uint64_t>(static_cast<uint64_t>(bx) * dev::kTileW, cam->image_w - W.col0));
            W.bh = static_cast<uint32_t>(std::min<uint64_t>(static_cast<uint64_t>(by) * dev::kTileH, W.owned_rows - W.k0));
            W.tiles_x = (W.bw + dev::kTileW - 1) / dev::kTileW;
            W.tiles_y = (W.bh + dev::kTileH - 1) / dev::kTileH;
            W.tiles = W.tiles_x * W.tiles_y;
            const uint64_t blocks = std::max<uint64_t>(
                1, std::min<uint64_t>(resident, (static_cast<uint64_t>(W.tiles) * W.chunks + kWavesPerBlock - 1) / kWavesPerBlock));
            // Items: bulk items of K chunks for the first part of each tile's chunks, then the
            // rest in one-chunk items at the end of the queue (CRT_TAIL_CHUNKS), so the grid
            // drains on small items; a wave's lanes cross from item to item without waiting
            // either way. Large items keep a wave's lanes on one tile (coherent rays: config 2 on
            // one GPU takes 72.5 ms with K = 7, 77.1 with K = 1), small ones balance the drain
            // against a ~10x spread of tile costs. With p = (tile, chunk) pairs per wave: K =
            // min(7, p / 15) for p >= 60, else 3, and the tail takes max(1/9, 30 / p) of the
            // chunks (all of them for p <= 30). Config 2, the slowest rank's share
            // (tools/item_sweep.py, tools/grid_sweep.py, profiles/r03_schedule): N = 2 (p = 183)
            // 36.9 -> 36.7 ms, N = 4 (p = 92) 19.7 -> 19.0, N = 8 (p = 46, K = 3 with an 81-chunk
            // tail) 10.34-10.49 -> 10.17-10.31 against the earlier K = p / 30 with a 1/9 tail;
            // N = 1 (7, 13 of 125 chunks) unchanged. (CRT_ITEM_CHUNKS, CRT_TAIL_CHUNKS override.)
            const uint64_t per_lane = static_cast<uint64_t>(W.tiles) * W.chunks / (blocks * kWavesPerBlock);
            const uint32_t k_auto = per_lane >= 60 ? static_cast<uint32_t>(std::min<uint64_t>(7, per_lane / 15)) : 3u;
            W.item_chunks = std::max<uint32_t>(1, knob("CRT_ITEM_CHUNKS", k_auto));
            const uint32_t tail_auto = static_cast<uint32_t>(std::max<uint64_t>(
                W.chunks / 9, std::min<uint64_t>(W.chunks, static_cast<uint64_t>(W.chunks) * 30 / std::max<uint64_t>(1, per_lane))));
            const uint32_t tail_want = std::min(W.chunks, knob("CRT_TAIL_CHUNKS", W.item_chunks > 1 ? tail_auto : 0));
            W.groups = (W.chunks - tail_want) / W.item_chunks;
            W.bulk_chunks = W.groups * W.item_chunks;
            W.tail_chunks = W.chunks - W.bulk_chunks;
            const uint64_t bulk_items = static_cast<uint64_t>(W.tiles) * W.groups;
            const uint64_t items = bulk_items + static_cast<uint64_t>(W.tiles) * W.tail_chunks;
            if (items >= 0xffffffffull) return fail(CRT_E_INVALID, "band too large for one launch");
            W.n_items = static_cast<uint32_t>(items);
            W.bulk_items = static_cast<uint32_t>(bulk_items);
            // HBM-resident scenes: one queue per XCD (blocks b and b + 8 share one), so an XCD's L2
            // serves the rays of one region of the band (config 4: 163.5 vs 166.2 ms); LDS scenes
            // keep one queue (config 2: 88.5 vs 89.0 ms with eight). CRT_XCD_QUEUES=0/1 forces.
            W.segments = knob("CRT_XCD_QUEUES", LSCENE ? 0 : 1) ? 8u : 1u;
            HIP_TRY(hipMemsetAsync(queue, 0, 8 * sizeof(uint32_t), stream));
#if CRT_WATCHDOG
            {
                void* wd = nullptr;
                HIP_TRY(hipGetSymbolAddress(&wd, HIP_SYMBOL(dev::crt_wd_deadline)));
                HIP_TRY(hipMemsetAsync(wd, 0, sizeof(unsigned long long), stream));
            }
#endif
            if (count) {
                hipLaunchKernelGGL((dev::render_kernel<SE, GSTACK, LSCENE, true, PM, W5>), dim3(static_cast<uint32_t>(blocks)),
                                   dim3(dev::kBlock), lds, stream, S, C, W, partial, gstack, ctr);
                HIP_TRY(hipGetLastError());
            } else {
                hipLaunchKernelGGL((dev::render_kernel<SE, GSTACK, LSCENE, false, PM, W5>), dim3(static_cast<uint32_t>(blocks)),
                                   dim3(dev::kBlock), lds, stream, S, C, W, partial, gstack, ctr);
                HIP_TRY(hipGetLastError());
                const uint64_t rb = (static_cast<uint64_t>(W.bw) * W.bh + 255) / 256;
                hipLaunchKernelGGL(dev::resolve_kernel, dim3(static_cast<uint32_t>(rb)), dim3(256), 0, stream, partial,
                                   d_rgb, W, cam->image_w, cam->image_h, C.inv_spp);
                HIP_TRY(hipGetLastError());
            }
        }
    }
    if (count) HIP_TRY(hipEventRecord(e1, stream));
    if (partial) HIP_TRY(hipFreeAsync(partial, stream));
    HIP_TRY(hipFreeAsync(queue, stream));
    if (gstack) HIP_TRY(hipFreeAsync(gstack, stream));
    if (count) {
        dev::Counters h{};
        HIP_TRY(hipMemcpyAsync(&h, ctr, sizeof h, hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        HIP_TRY(hipFreeAsync(ctr, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        count_stats->samples = pixels * cam->samples_per_pixel;
        count_stats->rays = h.rays;
        count_stats->nodes_visited = h.nodes;
        count_stats->sphere_tests = h.sphere_tests;
        count_stats->parallelogram_tests = h.quad_tests;
        count_stats->kernel_ms = ms;
        count_stats->ticks_walk = h.cyc_walk;
        count_stats->ticks_leaf = h.cyc_leaf;
        count_stats->ticks_shade = h.cyc_shade;
        count_stats->ticks_total = h.cyc_total;
        count_stats->wave_iters_walk = h.it_walk;
        count_stats->wave_iters_leaf = h.it_leaf;
        count_stats->wave_iters_shade = h.it_shade;
        count_stats->ticks_tail = h.cyc_tail;
        count_stats->slow_node_tests = h.slow_nodes;
        count_stats->wave_iters_slow = h.it_slow;
        count_stats->candidate_tests = h.cand;
        count_stats->wave_iters_candidates = h.it_cand;
        if (std::getenv("CRT_DEBUG_COUNTERS"))
            std::fprintf(stderr, "crt counters: rays %llu nodes %llu sphere_tests %llu quad_tests %llu it_walk %llu "
                         "it_leaf %llu it_shade %llu rounds %llu walkers/round %.2f leaves/round %.2f done/round %.2f "
"shade_rounds %llu; wave time: walk %.3f leaf %.3f shade %.3f draw %.3f init %.3f\n", h.rays, h.nodes, h.sphere_tests, h.quad_tests, h.it_walk,
                         h.it_leaf, h.it_shade, h.rounds, double(h.round_walkers) / double(h.rounds ? h.rounds : 1),
                         double(h.round_leaves) / double(h.rounds ? h.rounds : 1),
                         double(h.round_done) / double(h.rounds ? h.rounds : 1), h.shade_rounds,
                         double(h.cyc_walk) / double(h.cyc_total), double(h.cyc_leaf) / double(h.cyc_total),
                         double(h.cyc_shade) / double(h.cyc_total), double(h.cyc_draw) / double(h.cyc_total),
                         double(h.cyc_init) / double(h.cyc_total));
    }
    return CRT_OK;
}

// Kernel variant per scene: u16 stack entries below 65536 nodes; the scene itself in LDS when it
// and the stack fit the LDS budget, else the stack alone in LDS, else everything in HBM.
template <typename SE>
static int dispatch_render(const crt_scene* s, int device, const crt_camera* cam, dev::Work W,
                           double* d_rgb, hipStream_t st, crt_render_stats* count_stats) {
    // depth + 1 levels: walk_step stores the far child at level sp unconditionally
    const size_t stack_bytes = align16(static_cast<size_t>(s->depth + 1) * dev::kBlock * sizeof(SE));
    W.bytes_nodes = static_cast<uint32_t>(align16(s->num_dnodes * sizeof(DevNodeF)));
    // sphere-only scenes in f32 range stage the filter's pair records instead of refs + spheres
    W.bytes_refs = W.spheres_f32 ? 0u : static_cast<uint32_t>(align16(s->num_prims * 4));
    W.bytes_spheres = static_cast<uint32_t>(align16(s->num_spheres * (W.spheres_f32 ? sizeof(DevSpherePair)
                                                                                         : sizeof(DevSphere))));
    W.bytes_quads = static_cast<uint32_t>(align16(s->num_quads * sizeof(DevQuad)));
    W.bytes_quadf = W.quads_f32 ? static_cast<uint32_t>(s->num_quads * (W.quads_flat ? sizeof(DevQuadBox) : sizeof(DevQuadF)))
                                : 0u;
    const size_t scene_bytes = static_cast<size_t>(W.bytes_nodes) + W.bytes_refs + W.bytes_spheres + W.bytes_quads +
                               W.bytes_quadf;
    const uint32_t level = static_cast<uint32_t>(dev::kBlock * sizeof(SE));  // one stack level
    // the sentinel is the last node; refs are byte offsets into the f32 node array
    W.sentinel = static_cast<uint32_t>(s->num_dnodes - 1) << kNodeFShift;
    W.f32_ok = s->dev[device].f32_ok ? 1u : 0u;
    W.tmin32 = static_cast<float>(cam->t_min);
    const bool force_global = std::getenv("CRT_NO_LDS_SCENE") != nullptr;
    // LDS stacks: [data][second guard: sentinel][guard level: sentinel][levels 0..depth]. A lane
    // that reaches the sentinel with no leaf recorded pops the second guard (round 6: it holds the
    // sentinel too, so the walks need no sentinel compare), and the speculative read reaches one
    // level below it: the guard starts at least three levels into the allocation and the second
    // guard lies past the data, so every level the pointer reaches has a non-negative LDS address. (With one
    // level, a 640-thread block on a small scene put that pointer at a negative address; the
    // level count derived from it then wrapped, and the flat-parallelogram instance walked a
    // garbage stack forever: the round-4 hang, found with -DCRT_WATCHDOG=1. Power-of-two blocks
    // had wrapped back onto the right level by the modular arithmetic alone.)
    auto stack_at = [&](size_t data_bytes) { return static_cast<uint32_t>(std::max<size_t>(data_bytes, 2 * level) + 2 * level); };
    if (!force_global && stack_at(scene_bytes) + stack_bytes <= kLdsSceneBudget) {
        W.lds_nodes = 0;
        W.lds_refs = W.lds_nodes + W.bytes_nodes;
        W.lds_spheres = W.lds_refs + W.bytes_refs;
        W.lds_quads = W.lds_spheres + W.bytes_spheres;
        W.lds_quadf = W.lds_quads + W.bytes_quads;
        W.lds_sph64 = W.lds_quadf + W.bytes_quadf;
        const size_t cam_bytes = align16(sizeof(dev::CamView));
        // Sphere-only scenes and scenes of axis-aligned parallelograms run five waves per SIMD when
        // five blocks fit a CU's LDS (32 KB each), staging the f64 spheres only if they fit that
        // too (config 2: 73.7 ms at five waves without them vs 75.8 at four with them; config 3:
        // 89.8 vs 92.6); the others four, with up to 40 KB (the general instance at five: config
        // 3 116.5 vs 100.6 ms).
        const size_t budget5 = 160 * 1024 * dev::kBlock / (64 * dev::kManyWaves * 4);  // LDS a block at five waves a SIMD
        const bool w5 = (64 * dev::kManyWaves * 4) % dev::kBlock == 0 && (W.sphere_only || W.quads_flat) && std::getenv("CRT_FOUR_WAVES") == nullptr &&
                        stack_at(scene_bytes) + stack_bytes + cam_bytes + (W.sphere_only ? kAccBytes : 0) +
                            (W.quads_flat ? kInvBytes : 0) <= budget5;
        const size_t budget = w5 ? budget5 : kLdsSceneBudget;
        const uint32_t sph64 = static_cast<uint32_t>(s->num_spheres * sizeof(DevSphere));
        if (W.spheres_f32 && stack_at(scene_bytes + sph64) + stack_bytes + cam_bytes + (w5 ? kAccBytes : 0) <= budget)
            W.bytes_sph64 = sph64;
        W.lds_stack = stack_at(scene_bytes + W.bytes_sph64);
        const size_t lds = W.lds_stack + stack_bytes;
        if (W.sphere_only)
            return w5 ? launch_render<SE, false, true, 0, true>(s, device, cam, W, lds, d_rgb, st, count_stats)
                      : launch_render<SE, false, true, 0, false>(s, device, cam, W, lds, d_rgb, st, count_stats);
        if (W.quads_flat)
            return w5 ? launch_render<SE, false, true, 2, true>(s, device, cam, W, lds, d_rgb, st, count_stats)
                      : launch_render<SE, false, true, 2, false>(s, device, cam, W, lds, d_rgb, st, count_stats);
        return launch_render<SE, false, true, 1>(s, device, cam, W, W.lds_stack + stack_bytes, d_rgb, st, count_stats);
    }
    // HBM scene: the top of the (breadth-first) node array goes to LDS as far as it fits beside
    // the stack without costing resident blocks (CRT_WAVES_PER_EU blocks of 4 waves, the VGPR
    // limit); W.ntop counts bytes of f32 nodes
    const size_t per_block = 160 * 1024 * dev::kBlock / (256 * CRT_WAVES_PER_EU);  // LDS per block at the VGPR occupancy
    const bool no_top = std::getenv("CRT_NO_LDS_TOP") != nullptr;
    const size_t all_nodes = s->num_dnodes * sizeof(DevNodeF);
    auto top_bytes = [&](size_t room) {
        // whole 64-byte sibling pairs (walk_pairs reads a pair from LDS or from HBM, not both)
        return no_top ? 0u : static_cast<uint32_t>(std::min(all_nodes, room / (2 * sizeof(DevNodeF)) * (2 * sizeof(DevNodeF))));
    };
    if (stack_bytes <= kLdsStackBudget && std::getenv("CRT_FORCE_GSTACK") == nullptr) {
        const size_t taken = stack_bytes + 3 * level + kInvBytes;
        const size_t room = per_block > taken ? per_block - taken : 0;
        W.ntop = top_bytes(room);
        W.lds_nodes = 0;
        W.lds_stack = stack_at(align16(W.ntop));
        if (W.sphere_only)
            return launch_render<SE, false, false, 0>(s, device, cam, W, W.lds_stack + stack_bytes, d_rgb, st, count_stats);
        return launch_render<SE, false, false, 1>(s, device, cam, W, W.lds_stack + stack_bytes, d_rgb, st, count_stats);
    }
    W.ntop = top_bytes(per_block);
    W.lds_nodes = 0;
    if (W.sphere_only) return launch_render<SE, true, false, 0>(s, device, cam, W, W.ntop, d_rgb, st, count_stats);
    return launch_render<SE, true, false, 1>(s, device, cam, W, W.ntop, d_rgb, st, count_stats);
}

int device_render(const crt_scene* s, int device, const crt_camera* cam, const crt_tiling* t,
                  double* d_rgb, void* stream, crt_render_stats* count_stats) {
    int rc = check_device(device);
    if (rc) return rc;
    if (!s->dev[device].valid)
        return fail(CRT_E_NOT_UPLOADED, "scene not uploaded to device " + std::to_string(device));
    if (cam->image_w == 0 || cam->image_h == 0) return fail(CRT_E_INVALID, "empty image");
    if (static_cast<uint64_t>(cam->image_w) * cam->image_h >= 0xffffffffull)
        return fail(CRT_E_INVALID, "image has more than 2^32-1 pixels");
    crt_tiling tl{1, 1, 0, 0};
    if (t) tl = *t;
    if (tl.flags & ~CRT_TILING_PACKED) return fail(CRT_E_INVALID, "unknown tiling flags");
    if (tl.row_block == 0 || tl.tile_count == 0 || tl.tile_index >= tl.tile_count)
        return fail(CRT_E_INVALID, "bad tiling");
    DeviceGuard g(device);
    dev::Work W{};
    W.row_block = tl.row_block;
    W.tile_count = tl.tile_count;
    W.tile_index = tl.tile_index;
    W.owned_rows = count_owned(cam->image_h, tl.row_block, tl.tile_count, tl.tile_index);
    W.packed = (tl.flags & CRT_TILING_PACKED) ? 1u : 0u;
    if (W.owned_rows == 0 || cam->samples_per_pixel == 0) {
        if (count_stats) *count_stats = crt_render_stats{};
        if (cam->samples_per_pixel == 0 && d_rgb && W.owned_rows) {
            // 0 spp: the reference multiplies a zero sum by 1/0 -> NaN (0 * inf)
            std::vector<double> nanrow(static_cast<size_t>(cam->image_w) * 3,
                                       std::numeric_limits<double>::quiet_NaN());
            for (uint32_t k = 0; k < W.owned_rows; ++k) {
                uint32_t blk = k / W.row_block, in = k % W.row_block;
                uint32_t row = (tl.flags & CRT_TILING_PACKED) ? k : (blk * W.tile_count + W.tile_index) * W.row_block + in;
                HIP_TRY(hipMemcpyAsync(d_rgb + static_cast<size_t>(row) * cam->image_w * 3, nanrow.data(),
                                       nanrow.size() * 8, hipMemcpyHostToDevice,
                                       static_cast<hipStream_t>(stream)));
            }
            HIP_TRY(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
        }
        return CRT_OK;
    }
    W.sphere_only = (s->num_quads == 0 && s->num_spheres != 0) ? 1u : 0u;
    W.spheres_f32 = (W.sphere_only && s->dev[device].spheres_f32_ok) ? 1u : 0u;
    W.quads_f32 = (s->num_spheres == 0 && s->num_quads != 0 && s->dev[device].quads_f32_ok) ? 1u : 0u;
    // the flat-box filter is the walk's f32 node test: it needs the walk's f32 range (f32_ok)
    W.quads_flat = (W.quads_f32 && s->dev[device].quads_flat_ok && s->dev[device].f32_ok) ? 1u : 0u;
    W.exact_slab = (s->exact_slab || std::getenv("CRT_EXACT_SLAB") != nullptr) ? 1u : 0u;
    W.pair_walk = (CRT_PAIR_WALK && !W.exact_slab && std::getenv("CRT_NO_PAIR_WALK") == nullptr) ? 1u : 0u;
    W.count_spec = std::getenv("CRT_COUNT_SPEC") != nullptr ? 1u : 0u;
    W.round_counters = std::getenv("CRT_ROUND_COUNTERS") != nullptr ? 1u : 0u;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (count_stats) HIP_TRY(hipStreamCreate(&st));
    int r;
    if ((s->num_dnodes << kNodeFShift) <= 65536)  // every ref fits a u16 stack entry
        r = dispatch_render<uint16_t>(s, device, cam, W, d_rgb, st, count_stats);
    else
        r = dispatch_render<uint32_t>(s, device, cam, W, d_rgb, st, count_stats);
    if (count_stats) (void)hipStreamDestroy(st);
    return r;
}

int device_closest_hits(crt_scene* s, int device, const double* rays, size_t n, double t_min,
                        double t_max, crt_hit* out) {
    int rc = device_upload(s, device);
    if (rc) return rc;
    if (n == 0) return CRT_OK;
    if (n > 0x7fffffffu) return fail(CRT_E_INVALID, "too many rays");
    DeviceGuard g(device);
    const DeviceCopy& c = s->dev[device];
    const uint32_t blocks = static_cast<uint32_t>((n + dev::kBlock - 1) / dev::kBlock);
    // ref -> primitive index: spheres at [0, nsp), parallelograms at [nsp, nsp + nq)
    const size_t nsp = s->num_spheres, nq = s->num_quads;
    std::vector<uint32_t> ref_prim(std::max<size_t>(1, nsp + nq));
    std::vector<uint32_t> dev_refs;  // a scene set up on the device has no host refs
    const uint32_t* refs = s->refs.data();
    if (s->refs.size() != s->num_prims) {
        dev_refs.resize(s->num_prims);
        HIP_TRY(hipMemcpy(dev_refs.data(), c.refs, s->num_prims * 4, hipMemcpyDeviceToHost));
        refs = dev_refs.data();
    }
    for (size_t slot = 0; slot < s->num_prims; ++slot) {
        uint32_t r = refs[slot];
        ref_prim[(r & kRefQuad) ? nsp + (r & ~kRefQuad) : r] = s->order[slot];
    }
    double* d_rays = nullptr;
    crt_hit* d_out = nullptr;
    uint32_t *d_sp = nullptr, *d_stack = nullptr;
    HIP_TRY(hipMalloc(&d_rays, n * 6 * sizeof(double)));
    HIP_TRY(hipMalloc(&d_out, n * sizeof(crt_hit)));
    HIP_TRY(hipMalloc(&d_sp, ref_prim.size() * 4));
    HIP_TRY(hipMalloc(&d_stack, static_cast<size_t>(s->depth + 1) * blocks * dev::kBlock * 4));
    HIP_TRY(hipMemcpy(d_rays, rays, n * 6 * sizeof(double), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(d_sp, ref_prim.data(), ref_prim.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(dev::hits_kernel, dim3(blocks), dim3(dev::kBlock), 0, 0, view_of(c), d_rays,
                       static_cast<uint32_t>(n), t_min, t_max, d_sp, static_cast<uint32_t>(nsp), d_out, d_stack);
    hipError_t le = hipGetLastError();
    hipError_t se = hipDeviceSynchronize();
    if (le == hipSuccess && se == hipSuccess)
        se = hipMemcpy(out, d_out, n * sizeof(crt_hit), hipMemcpyDeviceToHost);
    (void)hipFree(d_rays);
    (void)hipFree(d_out);
    (void)hipFree(d_sp);
    (void)hipFree(d_stack);
    if (le != hipSuccess) return fail(CRT_E_HIP, std::string("hits_kernel launch: ") + hipGetErrorString(le));
    if (se != hipSuccess) return fail(CRT_E_HIP, std::string("hits_kernel: ") + hipGetErrorString(se));
    return CRT_OK;
}

int device_ppm_values(int device, const double* d_rgb, size_t n, int32_t* h_values, void* stream) {
    int rc = check_device(device);
    if (rc) return rc;
    if (n == 0) return CRT_OK;
    if (n > (1ull << 40)) return fail(CRT_E_INVALID, "crt_ppm_values: frame too large");
    DeviceGuard g(device);
    hipStream_t st = static_cast<hipStream_t>(stream);
    int32_t* d_out = nullptr;
    HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&d_out), n * 3 * sizeof(int32_t), st));
    hipLaunchKernelGGL(dev::ppm_kernel, dim3(static_cast<uint32_t>((n + 255) / 256)), dim3(256), 0, st,
                       d_rgb, static_cast<uint64_t>(n), d_out);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(h_values, d_out, n * 3 * sizeof(int32_t), hipMemcpyDeviceToHost, st);
    (void)hipFreeAsync(d_out, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return fail(CRT_E_HIP, std::string("ppm_kernel: ") + hipGetErrorString(e));
    // pixels the kernel could not settle: recompute on the host with std::pow
    std::vector<size_t> redo;
    for (size_t p = 0; p < n; ++p)
        if (h_values[3 * p] == dev::kPpmRedo || h_values[3 * p + 1] == dev::kPpmRedo ||
            h_values[3 * p + 2] == dev::kPpmRedo)
            redo.push_back(p);
    if (redo.empty()) return CRT_OK;
    // their f64 values: the whole frame when many, else gathered on the device (one upload of the
    // list, one copy back)
    const bool whole = redo.size() > 4096;
    std::vector<double> px(whole ? n * 3 : redo.size() * 3);
    if (whole) {
        HIP_TRY(hipMemcpy(px.data(), d_rgb, n * 3 * sizeof(double), hipMemcpyDeviceToHost));
    } else {
        std::vector<uint32_t> list(redo.begin(), redo.end());
        uint32_t* d_list = nullptr;
        double* d_px = nullptr;
        HIP_TRY(hipMalloc(&d_list, list.size() * sizeof(uint32_t)));
        hipError_t ge = hipMalloc(&d_px, px.size() * sizeof(double));
        if (ge == hipSuccess) ge = hipMemcpy(d_list, list.data(), list.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
        if (ge == hipSuccess) {
            hipLaunchKernelGGL(dev::redo_gather_kernel, dim3(static_cast<uint32_t>((list.size() + 255) / 256)), dim3(256), 0,
                               st, d_rgb, d_list, static_cast<uint32_t>(list.size()), d_px);
            ge = hipGetLastError();
        }
        if (ge == hipSuccess) ge = hipStreamSynchronize(st);
        if (ge == hipSuccess) ge = hipMemcpy(px.data(), d_px, px.size() * sizeof(double), hipMemcpyDeviceToHost);
        (void)hipFree(d_list);
        if (d_px) (void)hipFree(d_px);
        if (ge != hipSuccess) return fail(CRT_E_HIP, std::string("ppm redo gather: ") + hipGetErrorString(ge));
    }
    for (size_t j = 0; j < redo.size(); ++j)
        ppm_pixel_host(px.data() + 3 * (whole ? redo[j] : j), h_values + 3 * redo[j]);
    return CRT_OK;
}

// Peer access from device `to` to device `from`'s memory, enabled once per pair per process
// (hipDeviceEnablePeerAccess fails with AlreadyEnabled on a repeat call; HIP keeps such an error as
// the thread's last error, so it is read off here, not left for a later hipGetLastError).
static void enable_peer_once(int to, int from) {
    static std::mutex mu;
    static bool done[kMaxDevices][kMaxDevices] = {};
    std::lock_guard<std::mutex> lk(mu);
    if (done[to][from]) return;
    done[to][from] = true;
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, to, from) != hipSuccess || !can) {
        (void)hipGetLastError();
        return;  // the copies still work, staged by the runtime
    }
    DeviceGuard g(to);
    if (hipDeviceEnablePeerAccess(from, 0) != hipSuccess) (void)hipGetLastError();
}

// Device d's owned rows (crt_tiling{rb, n, d}) are packed in its buffer; copy them to their frame
// rows in `dst` (on device 0): full rb-row blocks with one strided copy (rb rows apart in the
// source, n x rb rows apart in the frame), a short last block on its own. bytes_per_row: one row.
static hipError_t gather_packed(char* dst, const char* src, size_t H, size_t rb, int n, int d,
                                size_t bytes_per_row, hipStream_t st) {
    const size_t first = static_cast<size_t>(d) * rb, step = static_cast<size_t>(n) * rb;
    if (first >= H) return hipSuccess;
    const size_t blocks = (H - first + step - 1) / step;     // blocks of device d
    const size_t last = first + (blocks - 1) * step;         // frame row of its last block
    const size_t full = last + rb <= H ? blocks : blocks - 1; // blocks with all rb rows
    hipError_t e = hipSuccess;
    if (full)
        e = hipMemcpy2DAsync(dst + first * bytes_per_row, step * bytes_per_row, src, rb * bytes_per_row,
                             rb * bytes_per_row, full, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess && full < blocks)
        e = hipMemcpyAsync(dst + last * bytes_per_row, src + full * rb * bytes_per_row, (H - last) * bytes_per_row,
                           hipMemcpyDeviceToDevice, st);
    return e;
}

// crt_render / crt_render_ppm: the whole frame over devices [0, n). Rows are dealt in 4-row
// blocks (row r on device (r / 4) % n, crt_tiling{4, n, d}); the scene is uploaded to every device
// concurrently (one host thread per device, one copy of the staged image each); each device renders
// its own rows only, packed (CRT_TILING_PACKED: a device holds its share of the frame, 1/n of it)
// on its own stream; device 0's stream then waits for each device and pulls that device's row
// blocks into the frame with ONE strided peer copy (hipMemcpy2DAsync over xGMI), and the assembled
// frame crosses PCIe once. Frames are bit-identical for any n (per-sample RNG, spp-only sample
// chunks).
//   h_rgb (f64 frame, crt_render): 24 B a pixel cross xGMI and PCIe; device 0 renders straight
//     into the frame.
//   h_ppm (int32 PPM values, crt_render_ppm; image.h:38-56, rgb.h:90-115): every device converts
//     its rows to 8-bit PPM values before the gather (ppm8_kernel), so 3 B a pixel cross xGMI and
//     PCIe; the few pixels the kernel leaves to the host (NaN, out of range, or within 2 ulps of
//     an integer step) are recomputed from their f64 values with std::pow (ppm_pixel_host).
// CRT_EMULATE_DEVICES=k (tests): k logical devices all on device 0, through the same tiling and
// gather code.
static int render_multi_impl(crt_scene* s, const crt_camera* cam, int num_devices, double* h_rgb,
                             int32_t* h_ppm, crt_render_stats* stats) {
    int avail = 0;
    if (hipGetDeviceCount(&avail) != hipSuccess || avail == 0)
        return fail(CRT_E_NODEVICE, "no HIP device visible (the render path has no CPU fallback)");
    if (num_devices <= 0) num_devices = avail;
    num_devices = std::min(num_devices, std::min(avail, kMaxDevices));
    bool emulate = false;
    if (const char* e = std::getenv("CRT_EMULATE_DEVICES")) {
        num_devices = std::max(1, std::min(std::atoi(e), 64));
        emulate = true;
    }
    const int n = num_devices;
    const bool ppm = h_ppm != nullptr;
    auto phys = [&](int d) { return emulate ? 0 : d; };
    const size_t W = cam->image_w, H = cam->image_h;
    const uint32_t rb = 4;  // 4-row blocks: 800 rows split exactly over 1, 2, 4, 8 devices
    // 1. concurrent uploads, one thread per physical device; a worker's error message is taken
    // from its own thread (crt_last_error is per thread) and raised again on this one
    const int n_phys = emulate ? 1 : n;
    std::vector<int> urc(n_phys, CRT_OK);
    std::vector<std::string> umsg(n_phys);
    {
        std::vector<std::thread> th;
        for (int d = 0; d < n_phys; ++d)
            th.emplace_back([&, d] {
                urc[d] = device_upload(s, d);
                if (urc[d]) umsg[d] = crt_last_error();
            });
        for (auto& t : th) t.join();
    }
    for (int d = 0; d < n_phys; ++d)
        if (urc[d]) return fail(urc[d], "device " + std::to_string(d) + ": " + umsg[d]);
    // 2. render: each logical device its own rows on its own stream (f64 mode: device 0 into the
    // whole frame, the others packed; ppm mode: every device packed, then to 8-bit values)
    std::vector<double*> bufs(n, nullptr);
    std::vector<uint8_t*> b8(n, nullptr);
    std::vector<uint32_t*> redo(n, nullptr);  // [count, indices...] per device (ppm mode)
    std::vector<size_t> rows(n, 0);
    std::vector<hipStream_t> streams(n, nullptr);
    std::vector<hipEvent_t> ev0(n, nullptr), ev1(n, nullptr);
    constexpr uint32_t kRedoCap = 1u << 16;
    int rc = CRT_OK;
    for (int d = 0; d < n && rc == CRT_OK; ++d) {
        DeviceGuard g(phys(d));
        rows[d] = count_owned(cam->image_h, rb, static_cast<uint32_t>(n), static_cast<uint32_t>(d));
        const bool packed = ppm || d > 0;
        const size_t px = (packed ? rows[d] : H) * W;
        if (hipStreamCreateWithFlags(&streams[d], hipStreamNonBlocking) != hipSuccess ||
            hipMalloc(&bufs[d], std::max<size_t>(1, px) * 3 * sizeof(double)) != hipSuccess ||
            (ppm && hipMalloc(&b8[d], std::max<size_t>(1, px) * 3) != hipSuccess) ||
            (ppm && hipMalloc(&redo[d], (1 + kRedoCap) * sizeof(uint32_t)) != hipSuccess) ||
            hipEventCreate(&ev0[d]) != hipSuccess || hipEventCreate(&ev1[d]) != hipSuccess) {
            (void)hipGetLastError();
            rc = fail(CRT_E_HIP, "render: per-device setup failed on device " + std::to_string(phys(d)));
            break;
        }
        crt_tiling t{rb, static_cast<uint32_t>(n), static_cast<uint32_t>(d), packed ? CRT_TILING_PACKED : 0u};
        (void)hipEventRecord(ev0[d], streams[d]);
        rc = device_render(s, phys(d), cam, &t, bufs[d], streams[d], nullptr);
        if (rc == CRT_OK && ppm && px) {
            if (hipMemsetAsync(redo[d], 0, sizeof(uint32_t), streams[d]) != hipSuccess) {
                rc = fail(CRT_E_HIP, "render: redo counter");
                break;
            }
            hipLaunchKernelGGL(dev::ppm8_kernel, dim3(static_cast<uint32_t>((px + 255) / 256)), dim3(256), 0, streams[d],
                               bufs[d], static_cast<uint64_t>(px), b8[d], redo[d], kRedoCap);
            if (hipGetLastError() != hipSuccess) rc = fail(CRT_E_HIP, "render: ppm8_kernel launch");
        }
        (void)hipEventRecord(ev1[d], streams[d]);
    }
    // 3. gather into device 0: one strided copy per device, then one device-to-host copy
    uint8_t* frame8 = nullptr;
    std::vector<uint8_t> h8;
    if (rc == CRT_OK) {
        DeviceGuard g(0);
        if (ppm && hipMalloc(&frame8, std::max<size_t>(1, H * W * 3)) != hipSuccess) {
            (void)hipGetLastError();
            rc = fail(CRT_E_HIP, "render: frame buffer");
        }
        const size_t row_bytes = W * 3 * (ppm ? 1 : sizeof(double));
        for (int d = ppm ? 0 : 1; d < n && rc == CRT_OK; ++d) {
            if (!emulate && d > 0) enable_peer_once(0, d);
            if (hipStreamWaitEvent(streams[0], ev1[d], 0) != hipSuccess) {
                rc = fail(CRT_E_HIP, "render: gather wait failed");
                break;
            }
            const hipError_t e = ppm ? gather_packed(reinterpret_cast<char*>(frame8), reinterpret_cast<const char*>(b8[d]),
                                                     H, rb, n, d, row_bytes, streams[0])
                                     : gather_packed(reinterpret_cast<char*>(bufs[0]), reinterpret_cast<const char*>(bufs[d]),
                                                     H, rb, n, d, row_bytes, streams[0]);
            if (e != hipSuccess) rc = fail(CRT_E_HIP, std::string("render: gather from device ") +
                                                         std::to_string(d) + ": " + hipGetErrorString(e));
        }
        if (rc == CRT_OK) {
            hipError_t e;
            if (ppm) {
                h8.resize(H * W * 3);
                e = hipMemcpyAsync(h8.data(), frame8, h8.size(), hipMemcpyDeviceToHost, streams[0]);
            } else {
                e = hipMemcpyAsync(h_rgb, bufs[0], H * W * 3 * sizeof(double), hipMemcpyDeviceToHost, streams[0]);
            }
            if (e == hipSuccess) e = hipStreamSynchronize(streams[0]);
            if (e != hipSuccess) rc = fail(CRT_E_HIP, std::string("render: ") + hipGetErrorString(e));
        }
    }
    float max_ms = 0;
    for (int d = 0; d < n; ++d) {
        if (!streams[d]) continue;
        DeviceGuard g(phys(d));
        hipError_t e = hipStreamSynchronize(streams[d]);
        if (e != hipSuccess && rc == CRT_OK)
            rc = fail(CRT_E_HIP, std::string("render on device ") + std::to_string(phys(d)) + ": " + hipGetErrorString(e));
        float ms = 0;
        if (rc == CRT_OK && hipEventElapsedTime(&ms, ev0[d], ev1[d]) == hipSuccess) max_ms = std::max(max_ms, ms);
    }
    // 4. ppm mode: 8-bit values to int32, and the pixels each device left to the host
    if (rc == CRT_OK && ppm) {
        for (size_t i = 0; i < H * W * 3; ++i) h_ppm[i] = h8[i];
        for (int d = 0; d < n && rc == CRT_OK; ++d) {
            if (!rows[d]) continue;
            DeviceGuard g(phys(d));
            uint32_t cnt = 0;
            if (hipMemcpy(&cnt, redo[d], sizeof cnt, hipMemcpyDeviceToHost) != hipSuccess) {
                rc = fail(CRT_E_HIP, "render: redo count");
                break;
            }
            if (!cnt) continue;
            const size_t px = rows[d] * W;
            std::vector<uint32_t> idx;
            if (cnt <= kRedoCap) {  // the listed pixels
                idx.resize(cnt);
                if (hipMemcpy(idx.data(), redo[d] + 1, cnt * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess) {
                    rc = fail(CRT_E_HIP, "render: redo list");
                    break;
                }
            }
            std::vector<double> rgb(cnt <= kRedoCap ? 3 * idx.size() : 3 * px);
            const bool whole = cnt > kRedoCap;  // more than the list holds: every pixel of the device
            if (whole) {
                if (hipMemcpy(rgb.data(), bufs[d], 3 * px * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) rc = CRT_E_HIP;
            } else {
                // the listed pixels gathered on the device, then one copy (not one per pixel)
                double* packed = nullptr;
                if (hipMalloc(&packed, 3 * idx.size() * sizeof(double)) != hipSuccess) {
                    rc = CRT_E_HIP;
                } else {
                    hipLaunchKernelGGL(dev::redo_gather_kernel, dim3(static_cast<uint32_t>((idx.size() + 255) / 256)), dim3(256),
                                       0, nullptr, bufs[d], redo[d] + 1, static_cast<uint32_t>(idx.size()), packed);
                    if (hipGetLastError() != hipSuccess ||
                        hipMemcpy(rgb.data(), packed, 3 * idx.size() * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
                        rc = CRT_E_HIP;
                    (void)hipFree(packed);
                }
            }
            if (rc != CRT_OK) {
                rc = fail(CRT_E_HIP, "render: redo pixels");
                break;
            }
            const size_t m = whole ? px : idx.size();
            for (size_t j = 0; j < m; ++j) {
                const size_t k = whole ? j : idx[j];  // packed pixel index on device d
                const size_t kr = k / W, col = k % W;
                const size_t row = (kr / rb * static_cast<size_t>(n) + static_cast<size_t>(d)) * rb + kr % rb;
                ppm_pixel_host(rgb.data() + 3 * j, h_ppm + 3 * (row * W + col));
            }
        }
    }
    for (int d = 0; d < n; ++d) {
        DeviceGuard g(phys(d));
        if (bufs[d]) (void)hipFree(bufs[d]);
        if (b8[d]) (void)hipFree(b8[d]);
        if (redo[d]) (void)hipFree(redo[d]);
        if (streams[d]) (void)hipStreamDestroy(streams[d]);
        if (ev0[d]) (void)hipEventDestroy(ev0[d]);
        if (ev1[d]) (void)hipEventDestroy(ev1[d]);
    }
    if (frame8) {
        DeviceGuard g(0);
        (void)hipFree(frame8);
    }
    if (stats && rc == CRT_OK) {
        *stats = crt_render_stats{};
        stats->samples = static_cast<uint64_t>(cam->image_w) * cam->image_h * cam->samples_per_pixel;
        stats->kernel_ms = max_ms;
    }
    return rc;
}

int render_multi(crt_scene* s, const crt_camera* cam, int num_devices, double* h_rgb,
                 crt_render_stats* stats) {
    return render_multi_impl(s, cam, num_devices, h_rgb, nullptr, stats);
}

int render_multi_ppm(crt_scene* s, const crt_camera* cam, int num_devices, int32_t* h_values,
                     crt_render_stats* stats) {
    return render_multi_impl(s, cam, num_devices, nullptr, h_values, stats);
}

// The compile-time switches this library was built with (bench.py hashes them with the kernel
// sources, so a PMC summary is only used for the exact build it was collected on).
#ifndef CRT_ARCH
#define CRT_ARCH "unknown"
#endif
#define CRT_STR2(x) #x
#define CRT_STR(x) CRT_STR2(x)
const char* device_build_info() {
    // every compile-time parameter of the kernels (the numeric tuning knobs; the library has no
    // other build switches), and the offload target the Makefile compiled for
    return "arch=" CRT_ARCH " CRT_BLOCK=" CRT_STR(CRT_BLOCK) " CRT_TILE_W=" CRT_STR(CRT_TILE_W)
           " CRT_WAVES_PER_EU=" CRT_STR(CRT_WAVES_PER_EU) " CRT_WAVES_PER_EU_LDS=" CRT_STR(CRT_WAVES_PER_EU_LDS)
           " CRT_SHADE_BATCH=" CRT_STR(CRT_SHADE_BATCH) " CRT_CHUNK_MIN=" CRT_STR(CRT_CHUNK_MIN)
           " CRT_WATCHDOG=" CRT_STR(CRT_WATCHDOG) " CRT_PAIR_WALK=" CRT_STR(CRT_PAIR_WALK);
}

}  // namespace crt
