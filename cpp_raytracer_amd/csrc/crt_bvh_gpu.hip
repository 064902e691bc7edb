// GPU build of the reference's binned-SAH BVH (bvh.h:183-550), node for node and bit for bit
// the tree crt_host.cpp's Builder (and the reference) produces: same node bounds, split axes,
// leaf ranges, primitive order and preorder numbering.
//
// Level-synchronous: every task (a node's primitive range [lo, hi) of `order`) of one tree level
// is one workgroup of kThreads. Per task:
//   1. node bounds as the ordered fold of the primitives' boxes over [lo, hi) (Interval::merge
//      with fmin/fmax, a tie keeps the newer operand: each thread folds a contiguous chunk and the
//      chunks are combined in order, which is the same fold), and the centroid bounds;
//   2. per axis with a non-empty centroid extent, the 32 buckets' counts and boxes (LDS atomics
//      on order-preserving integer keys; only the values of these boxes are used);
//   3. thread 0 evaluates the SAH costs exactly as the reference (same loops, same operation
//      order, the "after" sweep starting at bucket nb-2 and merging bucket k itself) and decides
//      leaf / split;
//   4. a split partitions [lo, hi) as libstdc++'s std::partition does (the bidirectional
//      algorithm: the i-th "false" from the left is swapped with the i-th "true" from the right),
//      computed with block scans instead of the two converging scans;
//   5. the two children become tasks of the next level.
// The host then numbers the nodes in preorder (the reference's flattening, bvh.h:468-550).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "crt_internal.h"

namespace crt {
namespace bvhgpu {

constexpr int kThreads = 256;
constexpr uint32_t kMaxBuckets = 64;

struct Task {
    uint32_t lo, hi, node, pad;
};

struct TNode {
    double b[6];
    uint32_t lo, count;    // leaf: primitive range in `order`
    uint32_t left, right;  // inner: children (build ids)
    uint32_t axis, leaf;
};

struct Params {
    uint32_t nb, max_leaf;
};

// Interval::merge with std::fmin / std::fmax (glibc: a tie returns the second operand)
__device__ __forceinline__ double fmin_g(double acc, double x) { return acc < x ? acc : x; }
__device__ __forceinline__ double fmax_g(double acc, double x) { return acc > x ? acc : x; }

// order-preserving integer keys for the bucket-box atomics
__device__ __forceinline__ unsigned long long okey(double d) {
    const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(d));
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double unkey(unsigned long long k) {
    const unsigned long long b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    return __longlong_as_double(static_cast<long long>(b));
}

struct Box {
    double mn[3], mx[3];
    __device__ void empty() {
        for (int k = 0; k < 3; ++k) {
            mn[k] = __builtin_inf();
            mx[k] = -__builtin_inf();
        }
    }
    __device__ void merge(const Box& o) {
        for (int k = 0; k < 3; ++k) {
            mn[k] = fmin_g(mn[k], o.mn[k]);
            mx[k] = fmax_g(mx[k], o.mx[k]);
        }
    }
    __device__ double area() const {  // aabb.h:29-31
        const double x = mx[0] - mn[0], y = mx[1] - mn[1], z = mx[2] - mn[2];
        return 2 * (x * x + y * y + z * z);
    }
};

// bvh.h:275-292 (the partition predicate of :418-433 uses the same bucket)
__device__ __forceinline__ uint32_t bucket_of(double c, double cmin, double csize, uint32_t nb) {
    const double offset = (c - cmin) / csize;
    uint32_t b = static_cast<uint32_t>(static_cast<double>(nb) * offset);
    if (b == nb) --b;
    return b;
}

// SAH costs (bvh.h:340-397) from the bucket counts bn[axis * kMaxBuckets + k] and boxes
// bb[(axis * kMaxBuckets + k) * 6 + q] (order-preserving keys), the reference's loops and
// operation order; returns 1 to split at (best_axis, best_bucket), 0 for a leaf.
__device__ int sah_decide(const unsigned int* bn, const unsigned long long* bb, uint32_t nb,
                          const bool live[3], uint32_t count, uint32_t max_leaf,
                          uint32_t& best_axis, uint32_t& best_bucket) {
    double min_cost = __builtin_inf();
    best_axis = 0;
    best_bucket = 0;
    double costs[kMaxBuckets];
    for (int ax = 0; ax < 3; ++ax) {
        if (!live[ax]) continue;
        Box before, after, bk;
        before.empty();
        uint32_t nbef = 0;
        for (uint32_t k = 0; k + 1 < nb; ++k) {
            const unsigned long long* kb = bb + (ax * kMaxBuckets + k) * 6;
            for (int q = 0; q < 3; ++q) {
                bk.mn[q] = unkey(kb[q]);
                bk.mx[q] = unkey(kb[3 + q]);
            }
            before.merge(bk);
            nbef += bn[ax * kMaxBuckets + k];
            costs[k] = before.area() * static_cast<double>(nbef);
        }
        after.empty();
        uint32_t naft = 0;
        for (int k = static_cast<int>(nb) - 2; k >= 0; --k) {  // merges bucket k itself (:360-369)
            const unsigned long long* kb = bb + (ax * kMaxBuckets + k) * 6;
            for (int q = 0; q < 3; ++q) {
                bk.mn[q] = unkey(kb[q]);
                bk.mx[q] = unkey(kb[3 + q]);
            }
            after.merge(bk);
            naft += bn[ax * kMaxBuckets + k];
            costs[k] = costs[k] + after.area() * static_cast<double>(naft);
        }
        for (uint32_t k = 0; k + 1 < nb; ++k) {
            if (costs[k] < min_cost) {
                min_cost = costs[k];
                best_axis = ax;
                best_bucket = k;
            }
        }
    }
    if (__builtin_isinf(min_cost)) return 0;  // bvh.h:395-397
    return (count > max_leaf || min_cost < static_cast<double>(count)) ? 1 : 0;
}

// exclusive prefix of `flag` over the block (thread order) and the block total
template <int NT>
__device__ __forceinline__ uint32_t block_scan(bool flag, uint32_t* wsum, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t m = __ballot(flag);
    const uint32_t in_wave = __popcll(m & ((1ull << lane) - 1));
    if (lane == 0) wsum[wv] = __popcll(m);
    __syncthreads();
    uint32_t before = 0;
    total = 0;
    for (int w = 0; w < NT / 64; ++w) {
        if (w < static_cast<int>(wv)) before += wsum[w];
        total += wsum[w];
    }
    __syncthreads();
    return before + in_wave;
}

// the ordered fold of one contiguous range [a, e) over the block: bounds (fold order) and
// centroid bounds; result in red[0] / cred[0]
template <int NT>
__device__ void block_fold(uint32_t a0, uint32_t e0, const uint32_t* __restrict__ order,
                           const double* __restrict__ pb, const double* __restrict__ pc,
                           double (*red)[6], double (*cred)[6]) {
    const uint32_t t = threadIdx.x, count = e0 - a0;
    Box acc, cacc;
    acc.empty();
    cacc.empty();
    const uint32_t chunk = (count + NT - 1) / NT;
    const uint32_t a = a0 + min(count, t * chunk), e = a0 + min(count, (t + 1) * chunk);
    for (uint32_t j = a; j < e; ++j) {
        const uint32_t p = order[j];
        const double* b = pb + static_cast<size_t>(p) * 6;
        const double* c = pc + static_cast<size_t>(p) * 3;
        for (int k = 0; k < 3; ++k) {
            acc.mn[k] = fmin_g(acc.mn[k], b[2 * k]);
            acc.mx[k] = fmax_g(acc.mx[k], b[2 * k + 1]);
            cacc.mn[k] = fmin_g(cacc.mn[k], c[k]);
            cacc.mx[k] = fmax_g(cacc.mx[k], c[k]);
        }
    }
    for (int k = 0; k < 3; ++k) {
        red[t][k] = acc.mn[k];
        red[t][3 + k] = acc.mx[k];
        cred[t][k] = cacc.mn[k];
        cred[t][3 + k] = cacc.mx[k];
    }
    __syncthreads();
    for (int s = 1; s < NT; s *= 2) {
        if ((t % (2 * s)) == 0 && t + s < NT) {
            for (int k = 0; k < 3; ++k) {
                red[t][k] = fmin_g(red[t][k], red[t + s][k]);
                red[t][3 + k] = fmax_g(red[t][3 + k], red[t + s][3 + k]);
                cred[t][k] = fmin_g(cred[t][k], cred[t + s][k]);
                cred[t][3 + k] = fmax_g(cred[t][3 + k], cred[t + s][3 + k]);
            }
        }
        __syncthreads();
    }
}

// SAH costs of all (axis, bucket) split candidates in parallel: candidate i = (ax, k) computes
// the prefix union / count of buckets 0..k and the suffix union / count of k..nb-2 itself. The
// unions' values do not depend on the merge order (min / max; a signed-zero difference never
// changes a size), so each cost is bit-identical to the reference's sweep; the argmin keeps the
// first candidate in (axis, bucket) order with the strictly smallest cost, as the sweep does.
template <int NT>
__device__ int sah_parallel(const unsigned int* bn, const unsigned long long* bb, uint32_t nb,
                            const bool live[3], uint32_t count, uint32_t max_leaf, double* costs,
                            uint32_t& best_axis, uint32_t& best_bucket) {
    const uint32_t nc = nb - 1;
    for (uint32_t i = threadIdx.x; i < 3 * nc; i += NT) {
        const uint32_t ax = i / nc, k = i % nc;
        double c = __builtin_nan("");
        if (live[ax]) {
            Box before, after, bk;
            before.empty();
            after.empty();
            uint32_t nbef = 0, naft = 0;
            for (uint32_t j = 0; j < nc; ++j) {
                const unsigned long long* kb = bb + (ax * kMaxBuckets + j) * 6;
                for (int q = 0; q < 3; ++q) {
                    bk.mn[q] = unkey(kb[q]);
                    bk.mx[q] = unkey(kb[3 + q]);
                }
                if (j <= k) {
                    before.merge(bk);
                    nbef += bn[ax * kMaxBuckets + j];
                }
                if (j >= k) {
                    after.merge(bk);
                    naft += bn[ax * kMaxBuckets + j];
                }
            }
            c = before.area() * static_cast<double>(nbef);
            c = c + after.area() * static_cast<double>(naft);
        }
        costs[i] = c;
    }
    __syncthreads();
    double min_cost = __builtin_inf();
    best_axis = 0;
    best_bucket = 0;
    for (uint32_t i = 0; i < 3 * nc; ++i) {
        if (costs[i] < min_cost) {
            min_cost = costs[i];
            best_axis = i / nc;
            best_bucket = i % nc;
        }
    }
    if (__builtin_isinf(min_cost)) return 0;
    return (count > max_leaf || min_cost < static_cast<double>(count)) ? 1 : 0;
}

template <int NT>
__global__ __launch_bounds__(NT) void build_level(
    const Task* __restrict__ tasks, const double* __restrict__ pb, const double* __restrict__ pc,
    uint32_t* __restrict__ order, uint8_t* __restrict__ pred, uint32_t* __restrict__ scr_f,
    uint32_t* __restrict__ scr_t, TNode* __restrict__ nodes, uint32_t* __restrict__ node_ctr,
    Task* __restrict__ next, uint32_t* __restrict__ next_ctr, Params P, const uint32_t* __restrict__ task_count) {
    __shared__ double red[NT][6];
    __shared__ double cred[NT][6];
    __shared__ unsigned int bn[3][kMaxBuckets];
    __shared__ unsigned long long bb[3][kMaxBuckets][6];
    __shared__ double costs[3 * kMaxBuckets];
    __shared__ uint32_t wsum[NT / 64];
    __shared__ uint32_t s_ntrue;

    // one task per block, or (task_count given: levels launched without a host round trip) the
    // level's tasks strided over a grid of resident blocks
    const uint32_t ntasks = task_count ? *task_count : gridDim.x;
    for (uint32_t ti = blockIdx.x; ti < ntasks; ti += gridDim.x) {
    __syncthreads();  // the previous task's reads of the shared arrays are done
    const Task tk = tasks[ti];
    const uint32_t lo = tk.lo, hi = tk.hi, count = hi - lo, t = threadIdx.x;

    // 1. bounds (ordered fold over contiguous chunks) and centroid bounds
    block_fold<NT>(lo, hi, order, pb, pc, red, cred);
    TNode* me = nodes + tk.node;
    if (count == 1) {  // bvh.h: a single primitive is a leaf
        if (t < 6) me->b[t] = (t & 1) ? red[0][3 + t / 2] : red[0][t / 2];
        if (t == 0) {
            me->lo = lo;
            me->count = 1;
            me->leaf = 1;
            me->axis = 0;
        }
        continue;
    }

    // 2. bucket counts and boxes per axis
    const uint32_t nb = P.nb;
    double cmin[3], csize[3];
    bool live[3];
    for (int k = 0; k < 3; ++k) {
        cmin[k] = cred[0][k];
        csize[k] = cred[0][3 + k] - cred[0][k];
        live[k] = !(csize[k] <= 0);  // is_empty_exclusive skips the axis (bvh.h:244)
    }
    for (uint32_t i = t; i < 3 * nb; i += NT) {
        const uint32_t ax = i / nb, b = i % nb;
        bn[ax][b] = 0;
        for (int k = 0; k < 3; ++k) {
            bb[ax][b][k] = okey(__builtin_inf());
            bb[ax][b][3 + k] = okey(-__builtin_inf());
        }
    }
    __syncthreads();
    for (uint32_t j = lo + t; j < hi; j += NT) {
        const uint32_t p = order[j];
        const double* b = pb + static_cast<size_t>(p) * 6;
        const double* c = pc + static_cast<size_t>(p) * 3;
        for (int ax = 0; ax < 3; ++ax) {
            if (!live[ax]) continue;
            const uint32_t k = bucket_of(c[ax], cmin[ax], csize[ax], nb);
            atomicAdd(&bn[ax][k], 1u);
            for (int q = 0; q < 3; ++q) {
                atomicMin(&bb[ax][k][q], okey(b[2 * q]));
                atomicMax(&bb[ax][k][3 + q], okey(b[2 * q + 1]));
            }
        }
    }
    __syncthreads();

    // 3. SAH costs (bvh.h:340-397), all candidates in parallel
    uint32_t axis, bucket;
    const int split = sah_parallel<NT>(&bn[0][0], &bb[0][0][0], nb, live, count, P.max_leaf, costs, axis, bucket);
    if (t == 0) {
        for (int q = 0; q < 6; ++q) me->b[q] = (q & 1) ? red[0][3 + q / 2] : red[0][q / 2];
        if (!split) {
            me->lo = lo;
            me->count = count;
            me->leaf = 1;
            me->axis = 0;
        }
    }
    if (!split) continue;

    // 4. std::partition (libstdc++ bidirectional): predicate, then pair the falses of the left
    //    part with the trues of the right part from the outside in
    const double pmin = cmin[axis], psize = csize[axis];
    if (t == 0) s_ntrue = 0;
    __syncthreads();
    uint32_t my_true = 0;
    for (uint32_t j = lo + t; j < hi; j += NT) {
        const uint32_t p = order[j];
        const bool pr = bucket_of(pc[static_cast<size_t>(p) * 3 + axis], pmin, psize, nb) <= bucket;
        pred[j] = pr ? 1 : 0;
        my_true += pr ? 1 : 0;
    }
    atomicAdd(&s_ntrue, my_true);
    __syncthreads();
    const uint32_t mid = lo + s_ntrue;
    // m = falses in [lo, mid) = trues in [mid, hi); ranks by block scans over [lo, hi) in order
    uint32_t carry_f = 0, carry_t = 0, m = 0;
    {
        uint32_t mt = 0;
        for (uint32_t j = mid + t; j < hi; j += NT) mt += pred[j];
        __syncthreads();
        if (t == 0) s_ntrue = 0;
        __syncthreads();
        atomicAdd(&s_ntrue, mt);
        __syncthreads();
        m = s_ntrue;
        __syncthreads();
    }
    for (uint32_t base = lo; base < hi; base += NT) {
        const uint32_t j = base + t;
        const bool in = j < hi;
        const bool pr = in && pred[j];
        const bool is_f = in && j < mid && !pr;
        const bool is_t = in && j >= mid && pr;
        uint32_t tot_f, tot_t;
        const uint32_t rf = block_scan<NT>(is_f, wsum, tot_f);
        const uint32_t rt = block_scan<NT>(is_t, wsum, tot_t);
        if (is_f) scr_f[lo + carry_f + rf] = j;               // r-th false from the left
        if (is_t) scr_t[lo + (m - 1 - (carry_t + rt))] = j;   // r-th true from the right
        carry_f += tot_f;
        carry_t += tot_t;
    }
    __syncthreads();
    for (uint32_t r = t; r < m; r += NT) {
        const uint32_t a = scr_f[lo + r], b = scr_t[lo + r];
        const uint32_t va = order[a], vb = order[b];
        order[a] = vb;
        order[b] = va;
    }

    // 5. children
    if (t == 0) {
        const uint32_t c = atomicAdd(node_ctr, 2u);
        me->left = c;
        me->right = c + 1;
        me->axis = axis;
        me->leaf = 0;
        const uint32_t q = atomicAdd(next_ctr, 2u);
        next[q] = Task{lo, mid, c, 0};
        next[q + 1] = Task{mid, hi, c + 1, 0};
    }
    }
}

// the node count after a level (its build ids end there)
__global__ void mark_level(const uint32_t* __restrict__ node_ctr, uint32_t* __restrict__ out) { *out = *node_ctr; }


// ---- tasks above kBigTask primitives: each level spreads them over chunks of kChunk -----------
// The same five steps as build_level, with the per-task work split into per-chunk kernels and
// per-task kernels (the ordered bounds fold is per chunk, then over the chunks in order).
constexpr uint32_t kChunk = 4096;
constexpr uint32_t kBigTask = 4096;
constexpr int kSmallThreads = 64;  // tasks of at most kBigTask primitives: one wave each

struct BigTask {
    uint32_t lo, hi, node, chunk0, nchunks, pad[3];
};
struct BigInfo {
    double cmin[3], csize[3];
    uint32_t live[3];
    uint32_t split, axis, bucket, mid, m;
};
struct ChunkInfo {
    uint32_t task, lo, hi, ntrue, pf, pt, pad[2];
};

__global__ __launch_bounds__(kThreads) void big_fold(const ChunkInfo* __restrict__ chunks,
                                                     const uint32_t* __restrict__ order,
                                                     const double* __restrict__ pb,
                                                     const double* __restrict__ pc,
                                                     double* __restrict__ chunk_red) {
    __shared__ double red[kThreads][6];
    __shared__ double cred[kThreads][6];
    const ChunkInfo ck = chunks[blockIdx.x];
    block_fold<kThreads>(ck.lo, ck.hi, order, pb, pc, red, cred);
    if (threadIdx.x < 6) chunk_red[blockIdx.x * 12 + threadIdx.x] = red[0][threadIdx.x];
    else if (threadIdx.x < 12) chunk_red[blockIdx.x * 12 + threadIdx.x] = cred[0][threadIdx.x - 6];
}

__global__ __launch_bounds__(kThreads) void big_combine(const BigTask* __restrict__ big,
                                                        BigInfo* __restrict__ info,
                                                        const double* __restrict__ chunk_red,
                                                        TNode* __restrict__ nodes,
                                                        unsigned int* __restrict__ bn_g,
                                                        unsigned long long* __restrict__ bb_g, uint32_t nb) {
    const BigTask bt = big[blockIdx.x];
    if (threadIdx.x == 0) {
        Box acc, cacc;
        acc.empty();
        cacc.empty();
        for (uint32_t c = bt.chunk0; c < bt.chunk0 + bt.nchunks; ++c) {  // chunks in order
            const double* r = chunk_red + c * 12;
            for (int k = 0; k < 3; ++k) {
                acc.mn[k] = fmin_g(acc.mn[k], r[k]);
                acc.mx[k] = fmax_g(acc.mx[k], r[3 + k]);
                cacc.mn[k] = fmin_g(cacc.mn[k], r[6 + k]);
                cacc.mx[k] = fmax_g(cacc.mx[k], r[9 + k]);
            }
        }
        TNode* me = nodes + bt.node;
        BigInfo& in = info[blockIdx.x];
        for (int k = 0; k < 3; ++k) {
            me->b[2 * k] = acc.mn[k];
            me->b[2 * k + 1] = acc.mx[k];
            in.cmin[k] = cacc.mn[k];
            in.csize[k] = cacc.mx[k] - cacc.mn[k];
            in.live[k] = !(in.csize[k] <= 0) ? 1u : 0u;
        }
    }
    unsigned int* bn = bn_g + blockIdx.x * 3 * kMaxBuckets;
    unsigned long long* bb = bb_g + blockIdx.x * 3 * kMaxBuckets * 6;
    for (uint32_t i = threadIdx.x; i < 3 * kMaxBuckets; i += kThreads) {
        bn[i] = 0;
        for (int q = 0; q < 3; ++q) {
            bb[i * 6 + q] = okey(__builtin_inf());
            bb[i * 6 + 3 + q] = okey(-__builtin_inf());
        }
    }
    (void)nb;
}

__global__ __launch_bounds__(kThreads) void big_buckets(const ChunkInfo* __restrict__ chunks,
                                                        const BigInfo* __restrict__ info,
                                                        const uint32_t* __restrict__ order,
                                                        const double* __restrict__ pb,
                                                        const double* __restrict__ pc,
                                                        unsigned int* __restrict__ bn_g,
                                                        unsigned long long* __restrict__ bb_g, uint32_t nb) {
    __shared__ unsigned int bn[3][kMaxBuckets];
    __shared__ unsigned long long bb[3][kMaxBuckets][6];
    const ChunkInfo ck = chunks[blockIdx.x];
    const BigInfo& in = info[ck.task];
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < 3 * nb; i += kThreads) {
        const uint32_t ax = i / nb, b = i % nb;
        bn[ax][b] = 0;
        for (int k = 0; k < 3; ++k) {
            bb[ax][b][k] = okey(__builtin_inf());
            bb[ax][b][3 + k] = okey(-__builtin_inf());
        }
    }
    __syncthreads();
    for (uint32_t j = ck.lo + t; j < ck.hi; j += kThreads) {
        const uint32_t p = order[j];
        const double* b = pb + static_cast<size_t>(p) * 6;
        const double* c = pc + static_cast<size_t>(p) * 3;
        for (int ax = 0; ax < 3; ++ax) {
            if (!in.live[ax]) continue;
            const uint32_t k = bucket_of(c[ax], in.cmin[ax], in.csize[ax], nb);
            atomicAdd(&bn[ax][k], 1u);
            for (int q = 0; q < 3; ++q) {
                atomicMin(&bb[ax][k][q], okey(b[2 * q]));
                atomicMax(&bb[ax][k][3 + q], okey(b[2 * q + 1]));
            }
        }
    }
    __syncthreads();
    unsigned int* gbn = bn_g + ck.task * 3 * kMaxBuckets;
    unsigned long long* gbb = bb_g + ck.task * 3 * kMaxBuckets * 6;
    for (uint32_t i = t; i < 3 * nb; i += kThreads) {
        const uint32_t ax = i / nb, b = i % nb;
        if (!bn[ax][b]) continue;
        atomicAdd(&gbn[ax * kMaxBuckets + b], bn[ax][b]);
        for (int q = 0; q < 3; ++q) {
            atomicMin(&gbb[(ax * kMaxBuckets + b) * 6 + q], bb[ax][b][q]);
            atomicMax(&gbb[(ax * kMaxBuckets + b) * 6 + 3 + q], bb[ax][b][3 + q]);
        }
    }
}

__global__ void big_sah(const BigTask* __restrict__ big, BigInfo* __restrict__ info,
                        const unsigned int* __restrict__ bn_g, const unsigned long long* __restrict__ bb_g,
                        TNode* __restrict__ nodes, Params P) {
    if (threadIdx.x != 0) return;
    const BigTask bt = big[blockIdx.x];
    BigInfo& in = info[blockIdx.x];
    const bool live[3] = {in.live[0] != 0, in.live[1] != 0, in.live[2] != 0};
    uint32_t axis, bucket;
    const int split = sah_decide(bn_g + blockIdx.x * 3 * kMaxBuckets, bb_g + blockIdx.x * 3 * kMaxBuckets * 6,
                                 P.nb, live, bt.hi - bt.lo, P.max_leaf, axis, bucket);
    in.split = split;
    in.axis = axis;
    in.bucket = bucket;
    if (!split) {
        TNode* me = nodes + bt.node;
        me->lo = bt.lo;
        me->count = bt.hi - bt.lo;
        me->leaf = 1;
        me->axis = 0;
    }
}

__global__ __launch_bounds__(kThreads) void big_pred(ChunkInfo* __restrict__ chunks,
                                                     const BigInfo* __restrict__ info,
                                                     const uint32_t* __restrict__ order,
                                                     const double* __restrict__ pc,
                                                     uint8_t* __restrict__ pred, uint32_t nb) {
    __shared__ uint32_t s_true;
    ChunkInfo& ck = chunks[blockIdx.x];
    const BigInfo& in = info[ck.task];
    if (!in.split) return;
    if (threadIdx.x == 0) s_true = 0;
    __syncthreads();
    const uint32_t ax = in.axis;
    uint32_t mine = 0;
    for (uint32_t j = ck.lo + threadIdx.x; j < ck.hi; j += kThreads) {
        const uint32_t p = order[j];
        const bool pr = bucket_of(pc[static_cast<size_t>(p) * 3 + ax], in.cmin[ax], in.csize[ax], nb) <= in.bucket;
        pred[j] = pr ? 1 : 0;
        mine += pr ? 1 : 0;
    }
    atomicAdd(&s_true, mine);
    __syncthreads();
    if (threadIdx.x == 0) ck.ntrue = s_true;
}

__global__ __launch_bounds__(kThreads) void big_mid(const BigTask* __restrict__ big, BigInfo* __restrict__ info,
                                                    ChunkInfo* __restrict__ chunks,
                                                    const uint8_t* __restrict__ pred, TNode* __restrict__ nodes,
                                                    uint32_t* __restrict__ node_ctr, BigTask* __restrict__ next_big,
                                                    uint32_t* __restrict__ next_big_ctr, Task* __restrict__ next_small,
                                                    uint32_t* __restrict__ next_small_ctr) {
    __shared__ uint32_t s_mid, s_tl;
    const BigTask bt = big[blockIdx.x];
    BigInfo& in = info[blockIdx.x];
    if (!in.split) return;
    if (threadIdx.x == 0) {
        uint32_t T = 0;
        for (uint32_t c = bt.chunk0; c < bt.chunk0 + bt.nchunks; ++c) T += chunks[c].ntrue;
        s_mid = bt.lo + T;
        s_tl = 0;
    }
    __syncthreads();
    const uint32_t mid = s_mid;
    // trues left of mid inside the chunk that straddles mid
    uint32_t straddle = 0xffffffffu;
    for (uint32_t c = bt.chunk0; c < bt.chunk0 + bt.nchunks; ++c)
        if (chunks[c].lo < mid && chunks[c].hi > mid) straddle = c;
    if (straddle != 0xffffffffu) {
        uint32_t mine = 0;
        for (uint32_t j = chunks[straddle].lo + threadIdx.x; j < mid; j += kThreads) mine += pred[j];
        atomicAdd(&s_tl, mine);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t pf = 0, pt = 0;
        for (uint32_t c = bt.chunk0; c < bt.chunk0 + bt.nchunks; ++c) {
            ChunkInfo& ck = chunks[c];
            uint32_t f, tr;
            if (ck.hi <= mid) {
                f = (ck.hi - ck.lo) - ck.ntrue;
                tr = 0;
            } else if (ck.lo >= mid) {
                f = 0;
                tr = ck.ntrue;
            } else {
                f = (mid - ck.lo) - s_tl;
                tr = ck.ntrue - s_tl;
            }
            ck.pf = pf;
            ck.pt = pt;
            pf += f;
            pt += tr;
        }
        in.mid = mid;
        in.m = pf;
        const uint32_t c = atomicAdd(node_ctr, 2u);
        TNode* me = nodes + bt.node;
        me->left = c;
        me->right = c + 1;
        me->axis = in.axis;
        me->leaf = 0;
        const uint32_t r[2][2] = {{bt.lo, mid}, {mid, bt.hi}};
        for (int k = 0; k < 2; ++k) {
            if (r[k][1] - r[k][0] > kBigTask) {
                const uint32_t q = atomicAdd(next_big_ctr, 1u);
                next_big[q] = BigTask{r[k][0], r[k][1], c + k, 0, 0, {0, 0, 0}};
            } else {
                const uint32_t q = atomicAdd(next_small_ctr, 1u);
                next_small[q] = Task{r[k][0], r[k][1], c + k, 0};
            }
        }
    }
}

__global__ __launch_bounds__(kThreads) void big_ranks(const ChunkInfo* __restrict__ chunks,
                                                      const BigInfo* __restrict__ info,
                                                      const BigTask* __restrict__ big,
                                                      const uint8_t* __restrict__ pred,
                                                      uint32_t* __restrict__ scr_f, uint32_t* __restrict__ scr_t) {
    __shared__ uint32_t wsum[kThreads / 64];
    const ChunkInfo ck = chunks[blockIdx.x];
    const BigInfo& in = info[ck.task];
    if (!in.split) return;
    const uint32_t lo = big[ck.task].lo, mid = in.mid, m = in.m;
    uint32_t carry_f = ck.pf, carry_t = ck.pt;
    for (uint32_t base = ck.lo; base < ck.hi; base += kThreads) {
        const uint32_t j = base + threadIdx.x;
        const bool inr = j < ck.hi;
        const bool pr = inr && pred[j];
        const bool is_f = inr && j < mid && !pr;
        const bool is_t = inr && j >= mid && pr;
        uint32_t tot_f, tot_t;
        const uint32_t rf = block_scan<kThreads>(is_f, wsum, tot_f);
        const uint32_t rt = block_scan<kThreads>(is_t, wsum, tot_t);
        if (is_f) scr_f[lo + carry_f + rf] = j;
        if (is_t) scr_t[lo + (m - 1 - (carry_t + rt))] = j;
        carry_f += tot_f;
        carry_t += tot_t;
    }
}

__global__ __launch_bounds__(kThreads) void big_swap(const ChunkInfo* __restrict__ chunks,
                                                     const BigInfo* __restrict__ info,
                                                     const BigTask* __restrict__ big,
                                                     const uint32_t* __restrict__ scr_f,
                                                     const uint32_t* __restrict__ scr_t,
                                                     uint32_t* __restrict__ order) {
    const ChunkInfo ck = chunks[blockIdx.x];
    const BigInfo& in = info[ck.task];
    if (!in.split) return;
    const BigTask bt = big[ck.task];
    const uint32_t r0 = (blockIdx.x - bt.chunk0) * kChunk, r1 = min(in.m, r0 + kChunk);
    for (uint32_t r = r0 + threadIdx.x; r < r1; r += kThreads) {
        const uint32_t a = scr_f[bt.lo + r], b = scr_t[bt.lo + r];
        const uint32_t va = order[a], vb = order[b];
        order[a] = vb;
        order[b] = va;
    }
}

}  // namespace bvhgpu

#define BV_TRY(expr)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) {                                                             \
            rc = fail(CRT_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));       \
            goto done;                                                                      \
        }                                                                                   \
    } while (0)

// ---- device-side preparation and numbering ----------------------------------------------------
using bvhgpu::kThreads;
using bvhgpu::TNode;
__global__ __launch_bounds__(kThreads) void iota_order(uint32_t* __restrict__ order, uint32_t n) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i < n) order[i] = i;
}
// std::midpoint(double, double) as libstdc++ implements it (interval.h:31 Interval::mid, the
// centroid of aabb.h:27): (a + b) / 2 when neither operand can overflow, else halving first.
__device__ __forceinline__ double midpoint_ls(double a, double b) {
    constexpr double lo = 2.2250738585072014e-308 * 2, hi = 1.7976931348623157e308 / 2;
    const double aa = a < 0 ? -a : a, ab = b < 0 ? -b : b;
    if (aa <= hi && ab <= hi) return (a + b) / 2;
    if (aa < lo) return a + b / 2;
    if (ab < lo) return a / 2 + b;
    return a / 2 + b / 2;
}
// the primitives' centroids from their boxes (what crt_host.cpp's Builder computes)
__global__ __launch_bounds__(kThreads) void centroids(const double* __restrict__ pb, double* __restrict__ pc, size_t n) {
    const size_t i = static_cast<size_t>(blockIdx.x) * kThreads + threadIdx.x;
    if (i >= n) return;
    for (int k = 0; k < 3; ++k) pc[3 * i + k] = midpoint_ls(pb[6 * i + 2 * k], pb[6 * i + 2 * k + 1]);
}
// Preorder numbering (bvh.h:468-550) level by level: a level's build ids are contiguous [a, b)
// (children are allocated while their parents' level is processed). Subtree sizes bottom-up,
// then preorder positions top-down, then every node written at its position.
__global__ __launch_bounds__(kThreads) void subtree_sizes(const TNode* __restrict__ t, uint32_t* __restrict__ size,
                                                          uint32_t a, uint32_t b) {
    const uint32_t i = a + blockIdx.x * kThreads + threadIdx.x;
    if (i >= b) return;
    size[i] = t[i].leaf ? 1u : 1u + size[t[i].left] + size[t[i].right];
}
__global__ __launch_bounds__(kThreads) void preorder_level(const TNode* __restrict__ t, const uint32_t* __restrict__ size,
                                                           uint32_t* __restrict__ pre, uint32_t a, uint32_t b) {
    const uint32_t i = a + blockIdx.x * kThreads + threadIdx.x;
    if (i >= b || t[i].leaf) return;
    pre[t[i].left] = pre[i] + 1;
    pre[t[i].right] = pre[i] + 1 + size[t[i].left];
}
__global__ __launch_bounds__(kThreads) void emit_preorder(const TNode* __restrict__ t, const uint32_t* __restrict__ pre,
                                                          uint32_t n, crt_bvh_node* __restrict__ out,
                                                          uint32_t* __restrict__ max_leaf) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const TNode& x = t[i];
    crt_bvh_node o;
    for (int q = 0; q < 6; ++q) o.bounds[q] = x.b[q];
    o.flags = 0;
    if (x.leaf) {
        o.index = x.lo;
        o.count = x.count;
        o.axis = 0;
        atomicMax(max_leaf, x.count);
    } else {
        o.index = pre[x.right];
        o.count = 0;
        o.axis = x.axis;
    }
    out[pre[i]] = o;
}

void device_tree_free(DeviceTree& t) {
    (void)hipFree(t.nodes);
    (void)hipFree(t.order);
    t.nodes = nullptr;
    t.order = nullptr;
}

// The tree of n (> 0) primitives from their boxes in HBM of the current device (d_pb: 6 doubles
// each, in primitive order): centroids, the levels and the preorder numbering on the device. The
// preorder node array and the slot order stay in HBM (out.nodes / out.order, freed by
// device_tree_free).
int device_build_tree(size_t n, const double* d_pb, uint32_t num_buckets, uint32_t max_leaf, DeviceTree& out) {
    using namespace bvhgpu;
    if (num_buckets < 2 || num_buckets > kMaxBuckets)
        return fail(CRT_E_INVALID, "GPU BVH build supports 2..64 buckets");
    int rc = CRT_OK;
    double* d_pc = nullptr;
    uint32_t *d_order = nullptr, *d_f = nullptr, *d_t = nullptr, *d_ctr = nullptr;
    uint8_t* d_pred = nullptr;
    Task *d_ta = nullptr, *d_tb = nullptr;
    TNode* d_nodes = nullptr;
    BigTask *d_big = nullptr, *d_big_next = nullptr;
    BigInfo* d_info = nullptr;
    ChunkInfo* d_chunks = nullptr;
    double* d_chunk_red = nullptr;
    unsigned int* d_bn = nullptr;
    unsigned long long* d_bb = nullptr;
    uint32_t nnodes = 0;
    std::vector<uint32_t> level_end;  // build ids [level_end[L - 1], level_end[L]) are level L
    uint32_t *d_size = nullptr, *d_pre = nullptr, *d_maxleaf = nullptr, *d_batch = nullptr;
    constexpr uint32_t kBatch = 8;
    int dev_id = 0;
    (void)hipGetDevice(&dev_id);
    crt_bvh_node* d_out = nullptr;
    const bool dbg = std::getenv("CRT_DEBUG_BUILD") != nullptr;
    auto tp = std::chrono::steady_clock::now();
    auto phase = [&](const char* what) {  // CRT_DEBUG_BUILD: where the build's time goes
        if (!dbg) return;
        (void)hipDeviceSynchronize();
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "bvh phase %-10s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(now - tp).count());
        tp = now;
    };
    {
        BV_TRY(hipMalloc(&d_pc, n * 3 * sizeof(double)));
        BV_TRY(hipMalloc(&d_order, n * 4));
        BV_TRY(hipMalloc(&d_f, n * 4));
        BV_TRY(hipMalloc(&d_t, n * 4));
        BV_TRY(hipMalloc(&d_pred, n));
        BV_TRY(hipMalloc(&d_ta, n * sizeof(Task)));
        BV_TRY(hipMalloc(&d_tb, n * sizeof(Task)));
        BV_TRY(hipMalloc(&d_nodes, 2 * n * sizeof(TNode)));
        BV_TRY(hipMalloc(&d_ctr, 3 * 4));
        const size_t max_big = n / kBigTask + 2, max_chunks = n / kChunk + 2 * max_big;
        BV_TRY(hipMalloc(&d_big, max_big * sizeof(BigTask)));
        BV_TRY(hipMalloc(&d_big_next, max_big * sizeof(BigTask)));
        BV_TRY(hipMalloc(&d_info, max_big * sizeof(BigInfo)));
        BV_TRY(hipMalloc(&d_chunks, max_chunks * sizeof(ChunkInfo)));
        BV_TRY(hipMalloc(&d_chunk_red, max_chunks * 12 * sizeof(double)));
        BV_TRY(hipMalloc(&d_bn, max_big * 3 * kMaxBuckets * sizeof(unsigned int)));
        BV_TRY(hipMalloc(&d_bb, max_big * 3 * kMaxBuckets * 6 * sizeof(unsigned long long)));
        phase("alloc");
        hipLaunchKernelGGL(centroids, dim3(static_cast<uint32_t>((n + kThreads - 1) / kThreads)), dim3(kThreads), 0, 0,
                           d_pb, d_pc, n);
        hipLaunchKernelGGL(iota_order, dim3(static_cast<uint32_t>((n + kThreads - 1) / kThreads)), dim3(kThreads), 0, 0,
                           d_order, static_cast<uint32_t>(n));
        BV_TRY(hipGetLastError());
        // counters: [0] nodes allocated, [1] next small tasks, [2] next big tasks
        uint32_t ctr[3] = {1, 0, 0};
        uint32_t nsmall = 0, nbig = 0;
        std::vector<BigTask> bigs;
        if (n > kBigTask) {
            bigs.push_back(BigTask{0, static_cast<uint32_t>(n), 0, 0, 0, {0, 0, 0}});
            nbig = 1;
        } else {
            const Task root{0, static_cast<uint32_t>(n), 0, 0};
            BV_TRY(hipMemcpy(d_ta, &root, sizeof root, hipMemcpyHostToDevice));
            nsmall = 1;
        }
        BV_TRY(hipMemcpy(d_ctr, ctr, sizeof ctr, hipMemcpyHostToDevice));
        const Params P{num_buckets, max_leaf};
        phase("upload");
        level_end.push_back(1);  // level 1: the root
        auto tl = std::chrono::steady_clock::now();
        int level = 0;
        std::vector<ChunkInfo> chunks;
        while (nsmall || nbig) {
            if (!nbig) break;  // only small tasks left: the batched loop below
            if (nbig) {
                chunks.clear();
                for (uint32_t i = 0; i < nbig; ++i) {
                    BigTask& bt = bigs[i];
                    bt.chunk0 = static_cast<uint32_t>(chunks.size());
                    for (uint32_t lo = bt.lo; lo < bt.hi; lo += kChunk)
                        chunks.push_back(ChunkInfo{i, lo, std::min(bt.hi, lo + kChunk), 0, 0, 0, {0, 0}});
                    bt.nchunks = static_cast<uint32_t>(chunks.size()) - bt.chunk0;
                }
                const uint32_t nch = static_cast<uint32_t>(chunks.size());
                BV_TRY(hipMemcpy(d_big, bigs.data(), nbig * sizeof(BigTask), hipMemcpyHostToDevice));
                BV_TRY(hipMemcpy(d_chunks, chunks.data(), nch * sizeof(ChunkInfo), hipMemcpyHostToDevice));
                hipLaunchKernelGGL(big_fold, dim3(nch), dim3(kThreads), 0, 0, d_chunks, d_order, d_pb, d_pc, d_chunk_red);
                hipLaunchKernelGGL(big_combine, dim3(nbig), dim3(kThreads), 0, 0, d_big, d_info, d_chunk_red, d_nodes,
                                   d_bn, d_bb, num_buckets);
                hipLaunchKernelGGL(big_buckets, dim3(nch), dim3(kThreads), 0, 0, d_chunks, d_info, d_order, d_pb, d_pc,
                                   d_bn, d_bb, num_buckets);
                hipLaunchKernelGGL(big_sah, dim3(nbig), dim3(64), 0, 0, d_big, d_info, d_bn, d_bb, d_nodes, P);
                hipLaunchKernelGGL(big_pred, dim3(nch), dim3(kThreads), 0, 0, d_chunks, d_info, d_order, d_pc, d_pred,
                                   num_buckets);
                hipLaunchKernelGGL(big_mid, dim3(nbig), dim3(kThreads), 0, 0, d_big, d_info, d_chunks, d_pred, d_nodes,
                                   d_ctr, d_big_next, d_ctr + 2, d_tb, d_ctr + 1);
                hipLaunchKernelGGL(big_ranks, dim3(nch), dim3(kThreads), 0, 0, d_chunks, d_info, d_big, d_pred, d_f, d_t);
                hipLaunchKernelGGL(big_swap, dim3(nch), dim3(kThreads), 0, 0, d_chunks, d_info, d_big, d_f, d_t, d_order);
                BV_TRY(hipGetLastError());
            }
            if (nsmall) {
                hipLaunchKernelGGL(build_level<kSmallThreads>, dim3(nsmall), dim3(kSmallThreads), 0, 0, d_ta, d_pb, d_pc, d_order,
                                   d_pred, d_f, d_t, d_nodes, d_ctr, d_tb, d_ctr + 1, P, nullptr);
                BV_TRY(hipGetLastError());
            }
            BV_TRY(hipMemcpy(ctr, d_ctr, sizeof ctr, hipMemcpyDeviceToHost));
            if (dbg) {
                const auto now = std::chrono::steady_clock::now();
                std::fprintf(stderr, "bvh level %d: %u big + %u small tasks %.3f ms\n", level, nbig, nsmall,
                             std::chrono::duration<double, std::milli>(now - tl).count());
                tl = now;
            }
            ++level;
            if (ctr[0] > level_end.back()) level_end.push_back(ctr[0]);
            nsmall = ctr[1];
            nbig = ctr[2];
            if (nbig) {
                bigs.resize(nbig);
                BV_TRY(hipMemcpy(bigs.data(), d_big_next, nbig * sizeof(BigTask), hipMemcpyDeviceToHost));
            }
            ctr[1] = ctr[2] = 0;
            BV_TRY(hipMemcpy(d_ctr + 1, &ctr[1], 8, hipMemcpyHostToDevice));
            std::swap(d_ta, d_tb);
        }
        // Only tasks of at most kBigTask primitives left: kBatch levels at a time with no host round
        // trip between them. Level j of a batch reads its task count from cnt[j] and appends the
        // next level's tasks to cnt[j + 1] (zeroed with the batch), striding them over a grid of
        // resident blocks; its node count goes to lend[j]; the host reads the batch's counters once.
        if (nsmall) {
            int cus = 0;
            BV_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev_id));
            const uint32_t resident = static_cast<uint32_t>(std::max(1, cus)) * 8;  // ~17.5 KB of LDS a block
            BV_TRY(hipMalloc(&d_batch, (2 * kBatch + 1) * 4));
            std::vector<uint32_t> hb(2 * kBatch + 1);
            uint32_t count = nsmall;
            while (count) {
                std::fill(hb.begin(), hb.end(), 0u);
                hb[0] = count;
                BV_TRY(hipMemcpy(d_batch, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
                for (uint32_t j = 0; j < kBatch; ++j) {
                    const uint32_t g = j == 0 ? std::min(count, resident) : resident;
                    hipLaunchKernelGGL(build_level<kSmallThreads>, dim3(g), dim3(kSmallThreads), 0, 0, d_ta, d_pb, d_pc,
                                       d_order, d_pred, d_f, d_t, d_nodes, d_ctr, d_tb, d_batch + j + 1, P, d_batch + j);
                    hipLaunchKernelGGL(mark_level, dim3(1), dim3(1), 0, 0, d_ctr, d_batch + kBatch + 1 + j);
                    std::swap(d_ta, d_tb);
                }
                BV_TRY(hipGetLastError());
                BV_TRY(hipMemcpy(hb.data(), d_batch, hb.size() * 4, hipMemcpyDeviceToHost));
                for (uint32_t j = 0; j < kBatch; ++j) {
                    if (dbg)
                        std::fprintf(stderr, "bvh level %d: %u small tasks (batched)\n", level, hb[j]);
                    ++level;
                    if (hb[kBatch + 1 + j] > level_end.back()) level_end.push_back(hb[kBatch + 1 + j]);
                }
                count = hb[kBatch];
            }
            ctr[0] = level_end.back();
        }
        phase("levels");
        nnodes = ctr[0];
        // preorder numbering on the device: sizes bottom-up, positions top-down, then the nodes
        BV_TRY(hipMalloc(&d_size, nnodes * 4));
        BV_TRY(hipMalloc(&d_pre, nnodes * 4));
        BV_TRY(hipMalloc(&d_maxleaf, 4));
        BV_TRY(hipMalloc(&d_out, nnodes * sizeof(crt_bvh_node)));
        BV_TRY(hipMemset(d_pre, 0, 4));
        BV_TRY(hipMemset(d_maxleaf, 0, 4));
        const size_t nl = level_end.size();
        auto grid = [](uint32_t a, uint32_t b) { return dim3((b - a + kThreads - 1) / kThreads); };
        for (size_t L = nl; L-- > 0;) {
            const uint32_t a = L ? level_end[L - 1] : 0, b = level_end[L];
            hipLaunchKernelGGL(subtree_sizes, grid(a, b), dim3(kThreads), 0, 0, d_nodes, d_size, a, b);
        }
        for (size_t L = 0; L + 1 < nl; ++L) {
            const uint32_t a = L ? level_end[L - 1] : 0, b = level_end[L];
            hipLaunchKernelGGL(preorder_level, grid(a, b), dim3(kThreads), 0, 0, d_nodes, d_size, d_pre, a, b);
        }
        hipLaunchKernelGGL(emit_preorder, grid(0, nnodes), dim3(kThreads), 0, 0, d_nodes, d_pre, nnodes, d_out, d_maxleaf);
        BV_TRY(hipGetLastError());
        BV_TRY(hipMemcpy(&out.max_leaf, d_maxleaf, 4, hipMemcpyDeviceToHost));
        out.nnodes = nnodes;
        out.depth = static_cast<uint32_t>(nl);
        out.nodes = d_out;
        out.order = d_order;
        d_out = nullptr;
        d_order = nullptr;
    }
    phase("preorder");
done:
    (void)hipFree(d_pc);
    (void)hipFree(d_order);
    (void)hipFree(d_f);
    (void)hipFree(d_t);
    (void)hipFree(d_pred);
    (void)hipFree(d_ta);
    (void)hipFree(d_tb);
    (void)hipFree(d_nodes);
    (void)hipFree(d_ctr);
    (void)hipFree(d_big);
    (void)hipFree(d_big_next);
    (void)hipFree(d_info);
    (void)hipFree(d_chunks);
    (void)hipFree(d_chunk_red);
    (void)hipFree(d_bn);
    (void)hipFree(d_bb);
    (void)hipFree(d_size);
    (void)hipFree(d_pre);
    (void)hipFree(d_maxleaf);
    (void)hipFree(d_out);
    (void)hipFree(d_batch);
    return rc;
}

// Builds s->nodes / s->order on `device` for the (non-empty, non-linear) primitive list, from the
// primitives' boxes (6 doubles each, in primitive order, on the host).
int device_build_bvh(crt_scene* s, uint32_t num_buckets, uint32_t max_leaf, int device,
                     const BigVec<double>& boxes) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return fail(CRT_E_NODEVICE, "GPU BVH build: device " + std::to_string(device) + " not visible");
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    const size_t n = s->prims.size();
    int rc = CRT_OK;
    double* d_pb = nullptr;
    DeviceTree t;
    {
        BV_TRY(hipMalloc(&d_pb, n * 6 * sizeof(double)));
        BV_TRY(hipMemcpy(d_pb, boxes.data(), n * 6 * sizeof(double), hipMemcpyHostToDevice));
        rc = device_build_tree(n, d_pb, num_buckets, max_leaf, t);
        if (rc) goto done;
        s->nodes.resize(t.nnodes);
        s->order.resize(n);
        BV_TRY(hipMemcpy(s->nodes.data(), t.nodes, t.nnodes * sizeof(crt_bvh_node), hipMemcpyDeviceToHost));
        BV_TRY(hipMemcpy(s->order.data(), t.order, n * 4, hipMemcpyDeviceToHost));
        s->max_leaf = t.max_leaf;
        s->depth = t.depth;
    }
done:
    (void)hipFree(d_pb);
    device_tree_free(t);
    (void)hipSetDevice(prev);
    return rc;
}

}  // namespace crt
