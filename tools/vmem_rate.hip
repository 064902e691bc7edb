// Microbenchmark of the vector-memory path (TA / TD / L1) for the render kernel's node gathers:
// how the cost of one wave64 global_load depends on the number of active lanes, the load width,
// the number of distinct cache lines the lanes touch and the level that serves them. Every lane
// runs 4 independent dependent-load chains (addresses from the loaded data, as a BVH walk does)
// over a table of 16-B records; a step is one load per chain.
//   hipcc --offload-arch=gfx950 -O3 tools/vmem_rate.hip -o tools/build/vmem_rate
//   tools/build/vmem_rate  -> one JSON line per case: ns per wave-instruction per CU
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int kSteps = 2048;

// WIDTH: dwords per load (1, 2, 4); PAIR: a second 16-B load from the same 32-B record per step
template <int WIDTH, bool PAIR>
__global__ __launch_bounds__(256) void gather_kernel(const uint32_t* __restrict__ table, uint32_t mask,
                                                     uint32_t active, uint32_t group, uint32_t* __restrict__ sink) {
    const uint32_t lane = threadIdx.x & 63;
    if (lane >= active) return;
    // lanes of one group (group lanes) follow the same address sequence: a coherent wave has
    // few distinct lines per instruction, an incoherent one 64
    const uint32_t g = (blockIdx.x * 256 + threadIdx.x) / group;
    uint32_t i0 = g * 2654435761u, i1 = g * 40503u + 7, i2 = g * 2246822519u + 3, i3 = g * 3266489917u + 11;
    uint32_t acc = 0;
    for (int s = 0; s < kSteps; ++s) {
        uint32_t v[4];
        const uint32_t idx[4] = {i0 & mask, i1 & mask, i2 & mask, i3 & mask};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t* p = table + static_cast<size_t>(idx[c]) * 8;  // 32-B records
            if (WIDTH == 4) {
                const uint4 q = *reinterpret_cast<const uint4*>(p);
                v[c] = q.x ^ q.y ^ q.z ^ q.w;
                if (PAIR) {
                    const uint4 r = *reinterpret_cast<const uint4*>(p + 4);
                    v[c] ^= r.x ^ r.w;
                }
            } else if (WIDTH == 2) {
                const uint2 q = *reinterpret_cast<const uint2*>(p);
                v[c] = q.x ^ q.y;
            } else {
                v[c] = *p;
            }
        }
        i0 = i0 * 1664525u + v[0];
        i1 = i1 * 1664525u + v[1];
        i2 = i2 * 1664525u + v[2];
        i3 = i3 * 1664525u + v[3];
        acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int WIDTH, bool PAIR>
static double run(const uint32_t* table, uint32_t records, uint32_t active, uint32_t group, uint32_t* sink,
                  int cus) {
    const int blocks = cus * 8;  // 32 waves per CU
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    gather_kernel<WIDTH, PAIR><<<blocks, 256>>>(table, records - 1, active, group, sink);  // warm
    hipEventRecord(a);
    gather_kernel<WIDTH, PAIR><<<blocks, 256>>>(table, records - 1, active, group, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    const double wave_insts_per_cu = 32.0 * kSteps * 4 * (PAIR ? 2 : 1);
    return ms * 1e6 / wave_insts_per_cu;  // ns per wave-instruction per CU
}

int main() {
    int dev = 0;
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, dev);
    const int cus = prop.multiProcessorCount;
    const size_t max_records = size_t(1) << 22;  // 4M x 32 B = 128 MB
    std::vector<uint32_t> h(max_records * 8);
    for (size_t i = 0; i < h.size(); ++i) h[i] = static_cast<uint32_t>(i * 2654435761u >> 7);
    uint32_t *table, *sink;
    hipMalloc(&table, h.size() * 4);
    hipMalloc(&sink, 4);
    hipMemcpy(table, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    const uint32_t sizes[] = {1u << 9, 1u << 16, 1u << 22};  // 16 KB (L1), 2 MB (L2), 128 MB (MALL)
    const uint32_t actives[] = {64, 32, 16, 8};
    const uint32_t groups[] = {1, 8, 64};
    for (uint32_t rec : sizes)
        for (uint32_t grp : groups)
            for (uint32_t act : actives) {
                const double x4 = run<4, false>(table, rec, act, grp, sink, cus);
                const double x4p = run<4, true>(table, rec, act, grp, sink, cus);
                const double x2 = run<2, false>(table, rec, act, grp, sink, cus);
                const double x1 = run<1, false>(table, rec, act, grp, sink, cus);
                printf("{\"table_bytes\": %zu, \"lanes_per_address\": %u, \"active_lanes\": %u, "
                       "\"ns_per_wave_load\": {\"dwordx4\": %.3f, \"dwordx4_pair\": %.3f, \"dwordx2\": %.3f, \"dword\": %.3f}}\n",
                       static_cast<size_t>(rec) * 32, grp, act, x4, x4p, x2, x1);
                fflush(stdout);
            }
    hipFree(table);
    hipFree(sink);
    return 0;
}
