// Microbenchmark pinning the VALU issue model of tools/pmc_summary.py on the MI355X: the SIMD
// cycles one wave64 VALU instruction occupies, for the instruction kinds the render kernel issues
// (f32 fma, f64 add / mul / fma, f64 reciprocal), measured with s_memtime (shader clock) inside
// each wave. Every wave runs 8 independent accumulator chains (latency hidden by ILP) of
// kIters x 16 instructions; with w waves on one SIMD the SIMD's issue cost per instruction is
// elapsed_cycles / (w x instructions per wave).
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o tools/build/valu_rate
//   tools/build/valu_rate  -> one JSON line
#include <hip/hip_runtime.h>

#include <algorithm>
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
__global__ __launch_bounds__(1024) void rate_kernel(unsigned long long* cycles, unsigned long long* real, T* sink, T seed) {
    T a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3, a4 = seed + 4, a5 = seed + 5, a6 = seed + 6,
      a7 = seed + 7, b = seed * T(0.5);
    __syncthreads();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
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
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    // every lane writes (vector stores): the chains stay live
    sink[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if ((threadIdx.x & 63) == 0) {
        cycles[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;
        real[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = r1 - r0;  // 100 MHz
    }
}

// waves per SIMD: `blocks_per_cu` blocks of `threads` on every CU, their waves dealt over the 4
// SIMDs. Returns memtime ticks per instruction per SIMD, and (via ghz) the memtime tick rate
// against s_memrealtime (a constant 100 MHz) over the waves' own spans: the shader clock the
// ticks run at.
template <int KIND, typename T>
static double measure(int cus, int threads, int blocks_per_cu, double* ghz) {
    const int blocks = cus * blocks_per_cu;
    const int waves = blocks * threads / 64;
    unsigned long long *d_cyc = nullptr, *d_real = nullptr;
    T* d_sink = nullptr;
    if (hipMalloc(&d_cyc, waves * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (hipMalloc(&d_real, waves * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (hipMalloc(&d_sink, static_cast<size_t>(blocks) * threads * sizeof(T)) != hipSuccess) return -1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((rate_kernel<KIND, T>), dim3(blocks), dim3(threads), 0, 0, d_cyc, d_real, d_sink, T(1.0001));  // warm-up
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((rate_kernel<KIND, T>), dim3(blocks), dim3(threads), 0, 0, d_cyc, d_real, d_sink, T(1.0001));
    (void)hipEventRecord(e1, 0);
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> cyc(waves), rt(waves);
    if (hipMemcpy(cyc.data(), d_cyc, waves * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    if (hipMemcpy(rt.data(), d_real, waves * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    (void)hipFree(d_cyc);
    (void)hipFree(d_real);
    (void)hipFree(d_sink);
    double mean = 0, sum_rt = 0;
    for (int i = 0; i < waves; ++i) {
        mean += static_cast<double>(cyc[i]);
        sum_rt += static_cast<double>(rt[i]);
    }
    // memtime ticks per ns of the constant 100 MHz clock, over the waves' own spans
    if (ghz) *ghz = mean / (sum_rt * 10.0);
    mean /= waves;
    const double per_simd = (threads / 64) * blocks_per_cu / 4.0;
    return mean / (per_simd * kIters * kUnroll);
}

int main() {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
    const char* names[] = {"v_fma_f32", "v_add_f64", "v_mul_f64", "v_fma_f64", "v_rcp_f64", "v_add_f32"};
    const int cfg[4][2] = {{256, 1}, {512, 1}, {1024, 1}, {1024, 2}};  // 1, 2, 4, 8 waves per SIMD
    double ghz = 0;
    std::printf("{\"cus\": %d, \"memtime_ticks_per_wave64_instruction_per_simd\": {", cus);
    for (int k = 0; k < 6; ++k) {
        std::printf("%s\"%s\": {", k ? ", " : "", names[k]);
        for (int c = 0; c < 4; ++c) {
            double r = 0;
            const int th = cfg[c][0], bp = cfg[c][1];
            switch (k) {
                case 0: r = measure<0, float>(cus, th, bp, &ghz); break;
                case 1: r = measure<1, double>(cus, th, bp, &ghz); break;
                case 2: r = measure<2, double>(cus, th, bp, &ghz); break;
                case 3: r = measure<3, double>(cus, th, bp, &ghz); break;
                case 4: r = measure<4, double>(cus, th, bp, &ghz); break;
                case 5: r = measure<5, float>(cus, th, bp, &ghz); break;
            }
            std::printf("%s\"%d_waves\": %.3f", c ? ", " : "", th / 64 * bp / 4, r);
        }
        std::printf("}");
    }
    std::printf("}, \"memtime_ghz_vs_memrealtime\": %.3f}\n", ghz);
    return 0;
}
