// Microbenchmark pinning the VALU issue model of tools/pmc_summary.py on the MI355X: the SIMD
// cycles one wave64 VALU instruction occupies, for the instruction kinds the render kernel issues
// (f32 fma, f64 add / mul / fma, f64 reciprocal), measured with s_memtime (shader clock) inside
// each wave. Every wave runs 8 independent accumulator chains (latency hidden by ILP) of
// kIters x 16 instructions; with w waves on one SIMD the SIMD's issue cost per instruction is
// elapsed_cycles / (w x instructions per wave).
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o tools/build/valu_rate
//   tools/build/valu_rate  -> one JSON line
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int kIters = 4096;
constexpr int kUnroll = 16;

#define CHAIN8(OP)                                                                               \
    asm volatile(OP " %0, %0, %8\n\t" OP " %1, %1, %8\n\t" OP " %2, %2, %8\n\t" OP " %3, %3, %8\n\t" \
                 OP " %4, %4, %8\n\t" OP " %5, %5, %8\n\t" OP " %6, %6, %8\n\t" OP " %7, %7, %8"      \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)  \
                 : "v"(b))
#define CHAIN8_FMA(OP)                                                                                   \
    asm volatile(OP " %0, %0, %8, %8\n\t" OP " %1, %1, %8, %8\n\t" OP " %2, %2, %8, %8\n\t"              \
                 OP " %3, %3, %8, %8\n\t" OP " %4, %4, %8, %8\n\t" OP " %5, %5, %8, %8\n\t"              \
                 OP " %6, %6, %8, %8\n\t" OP " %7, %7, %8, %8"                                           \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)      \
                 : "v"(b))
#define CHAIN8_UN(OP)                                                                            \
    asm volatile(OP " %0, %0\n\t" OP " %1, %1\n\t" OP " %2, %2\n\t" OP " %3, %3\n\t"             \
                 OP " %4, %4\n\t" OP " %5, %5\n\t" OP " %6, %6\n\t" OP " %7, %7"                 \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7))

template <int KIND, typename T>
__global__ void rate_kernel(unsigned long long* cycles, T* sink, T seed) {
    T a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3, a4 = seed + 4, a5 = seed + 5, a6 = seed + 6,
      a7 = seed + 7, b = seed * T(0.5);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int u = 0; u < kUnroll / 8; ++u) {
            if constexpr (KIND == 0) CHAIN8_FMA("v_fma_f32");
            if constexpr (KIND == 1) CHAIN8("v_add_f64");
            if constexpr (KIND == 2) CHAIN8("v_mul_f64");
            if constexpr (KIND == 3) CHAIN8_FMA("v_fma_f64");
            if constexpr (KIND == 4) CHAIN8_UN("v_rcp_f64");
            if constexpr (KIND == 5) CHAIN8("v_add_f32");
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    // every lane writes (vector stores): the chains stay live
    sink[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if ((threadIdx.x & 63) == 0) cycles[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;
}

template <int KIND, typename T>
static double measure(int blocks, int threads) {
    const int waves = blocks * threads / 64;
    unsigned long long* d_cyc = nullptr;
    T* d_sink = nullptr;
    if (hipMalloc(&d_cyc, waves * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (hipMalloc(&d_sink, static_cast<size_t>(blocks) * threads * sizeof(T)) != hipSuccess) return -1;
    for (int rep = 0; rep < 2; ++rep)  // the first launch warms up clocks and code
        hipLaunchKernelGGL((rate_kernel<KIND, T>), dim3(blocks), dim3(threads), 0, 0, d_cyc, d_sink, T(1.0001));
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    std::vector<unsigned long long> cyc(waves);
    if (hipMemcpy(cyc.data(), d_cyc, waves * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    (void)hipFree(d_cyc);
    (void)hipFree(d_sink);
    double mean = 0;
    for (auto c : cyc) mean += static_cast<double>(c);
    mean /= waves;
    // waves per SIMD: a block of `threads` lands on one CU, its waves dealt over the 4 SIMDs
    const double per_simd = (threads / 64) / 4.0;
    return mean / (per_simd * kIters * kUnroll);
}

int main() {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
    const char* names[] = {"v_fma_f32", "v_add_f64", "v_mul_f64", "v_fma_f64", "v_rcp_f64", "v_add_f32"};
    std::printf("{\"cus\": %d, \"cycles_per_wave64_instruction\": {", cus);
    for (int k = 0; k < 6; ++k) {
        double c1 = 0, c2 = 0;
        switch (k) {
            case 0: c1 = measure<0, float>(cus, 256); c2 = measure<0, float>(cus, 512); break;
            case 1: c1 = measure<1, double>(cus, 256); c2 = measure<1, double>(cus, 512); break;
            case 2: c1 = measure<2, double>(cus, 256); c2 = measure<2, double>(cus, 512); break;
            case 3: c1 = measure<3, double>(cus, 256); c2 = measure<3, double>(cus, 512); break;
            case 4: c1 = measure<4, double>(cus, 256); c2 = measure<4, double>(cus, 512); break;
            case 5: c1 = measure<5, float>(cus, 256); c2 = measure<5, float>(cus, 512); break;
        }
        std::printf("%s\"%s\": {\"1_wave_per_simd\": %.3f, \"2_waves_per_simd\": %.3f}", k ? ", " : "", names[k], c1, c2);
    }
    std::printf("}}\n");
    return 0;
}
