// Microbenchmark pinning the VALU issue model of tools/pmc_summary.py on the MI355X: the SIMD
// cycles one wave64 VALU instruction occupies, for the instruction kinds the render kernel issues
// (f32 add / mul / fma / rcp, int32, f64 add / mul / fma / rcp), from the wall time of grids with
// 1, 2, 4 and 8 waves per SIMD at the shader clock (s_memtime against s_memrealtime). Every wave
// runs 8 independent accumulator chains (latency hidden by ILP) of kIters x 16 instructions.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o tools/build/valu_rate
//   tools/build/valu_rate  -> one JSON line
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float F2 __attribute__((ext_vector_type(2)));
constexpr int kIters = 4096;
constexpr int kUnroll = 16;

#define CHAIN8(OP)                                                                               \
    asm volatile(OP " %0, %0, %8\n\t" OP " %1, %1, %8\n\t" OP " %2, %2, %8\n\t" OP " %3, %3, %8\n\t" \
                 OP " %4, %4, %8\n\t" OP " %5, %5, %8\n\t" OP " %6, %6, %8\n\t" OP " %7, %7, %8"      \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)  \
                 : "v"(b))
#define CHAIN8_FMA(OP)                                                                                   \
    asm volatile(OP " %0, %0, %8, %9\n\t" OP " %1, %1, %8, %9\n\t" OP " %2, %2, %8, %9\n\t"              \
                 OP " %3, %3, %8, %9\n\t" OP " %4, %4, %8, %9\n\t" OP " %5, %5, %8, %9\n\t"              \
                 OP " %6, %6, %8, %9\n\t" OP " %7, %7, %8, %9"                                           \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)      \
                 : "v"(b), "v"(c))
#define CHAIN8_MASK(OP)                                                                                  \
    asm volatile(OP " %0, %0, %8, %9\n\t" OP " %1, %1, %8, %9\n\t" OP " %2, %2, %8, %9\n\t"              \
                 OP " %3, %3, %8, %9\n\t" OP " %4, %4, %8, %9\n\t" OP " %5, %5, %8, %9\n\t"              \
                 OP " %6, %6, %8, %9\n\t" OP " %7, %7, %8, %9"                                           \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)      \
                 : "v"(b), "s"(mask))
#define CHAIN8_CMP(OP)                                                                                   \
    asm volatile(OP " %0, %1, %9\n\t" OP " %0, %2, %9\n\t" OP " %0, %3, %9\n\t" OP " %0, %4, %9\n\t"     \
                 OP " %0, %5, %9\n\t" OP " %0, %6, %9\n\t" OP " %0, %7, %9\n\t" OP " %0, %8, %9"         \
                 : "=s"(mask) : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7), "v"(b))
#define CHAIN8_CVT(OP)                                                                           \
    asm volatile(OP " %0, %8\n\t" OP " %1, %8\n\t" OP " %2, %8\n\t" OP " %3, %8\n\t"             \
                 OP " %4, %8\n\t" OP " %5, %8\n\t" OP " %6, %8\n\t" OP " %7, %8"                 \
                 : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7)  \
                 : "v"(ub))
#define CHAIN8_UN(OP)                                                                            \
    asm volatile(OP " %0, %0\n\t" OP " %1, %1\n\t" OP " %2, %2\n\t" OP " %3, %3\n\t"             \
                 OP " %4, %4\n\t" OP " %5, %5\n\t" OP " %6, %6\n\t" OP " %7, %7"                 \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7))

template <int KIND, typename T>
__global__ __launch_bounds__(1024) void rate_kernel(unsigned long long* cycles, unsigned long long* real, T* sink, T seed) {
    unsigned long long mask = 0x5555555555555555ull;
    unsigned ub = threadIdx.x * 7919u + 13u;
    T a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3, a4 = seed + 4, a5 = seed + 5, a6 = seed + 6,
      a7 = seed + 7, b = seed * T(0.5), c = seed * T(0.25);
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
            if constexpr (KIND == 6) CHAIN8("v_mul_f32");
            if constexpr (KIND == 7) CHAIN8("v_xor_b32");
            if constexpr (KIND == 8) CHAIN8_UN("v_rcp_f32");
            if constexpr (KIND == 9) CHAIN8_FMA("v_pk_fma_f32");
            if constexpr (KIND == 10) CHAIN8("v_pk_add_f32");
            if constexpr (KIND == 11) CHAIN8("v_min_f32");
            if constexpr (KIND == 12) CHAIN8_FMA("v_max3_f32");
            if constexpr (KIND == 13) CHAIN8_MASK("v_cndmask_b32_e64");
            if constexpr (KIND == 14) CHAIN8("v_min_i32");
            if constexpr (KIND == 15) CHAIN8("v_max_u32");
            if constexpr (KIND == 16) CHAIN8_FMA("v_med3_f32");
            if constexpr (KIND == 17) CHAIN8_FMA("v_min3_i32");
            if constexpr (KIND == 18) CHAIN8("v_min_f64");
            if constexpr (KIND == 19) CHAIN8_CMP("v_cmp_lt_f32_e64");
            if constexpr (KIND == 20) CHAIN8_FMA("v_bfe_u32");
            if constexpr (KIND == 21) CHAIN8_FMA("v_lshl_or_b32");
            if constexpr (KIND == 22) CHAIN8("v_mul_lo_u32");
            if constexpr (KIND == 23) CHAIN8("v_mul_hi_u32");
            if constexpr (KIND == 24) CHAIN8_FMA("v_mad_u32_u24");
            if constexpr (KIND == 25) CHAIN8_CVT("v_cvt_f32_u32");
            if constexpr (KIND == 26) CHAIN8_CVT("v_cvt_f64_u32");
            if constexpr (KIND == 27) CHAIN8_UN("v_rsq_f64");
            if constexpr (KIND == 28) CHAIN8_UN("v_sqrt_f64");
            if constexpr (KIND == 29) CHAIN8_CMP("v_cmp_lt_f64_e64");
            if constexpr (KIND == 30) CHAIN8_UN("v_mov_b32");
            if constexpr (KIND == 31) CHAIN8("v_add_u32");
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    // every lane writes (vector stores): the chains stay live
    sink[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + T(static_cast<float>(mask & 1));
    if ((threadIdx.x & 63) == 0) {
        cycles[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;
        real[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = r1 - r0;  // 100 MHz
    }
}

// A grid of `blocks_per_cu` blocks of `threads` per CU. Returns the SIMD cycles per wave64
// instruction: the launch's wall time (HIP events) x the shader clock over the instructions each
// of the 1024 SIMDs executes; the clock is s_memtime against s_memrealtime (a constant 100 MHz)
// over the waves' spans. Launch overhead is included (< 1% at these sizes).
static double g_last_ms = 0;  // wall time of the last timed launch
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
    g_last_ms = ms;
    std::vector<unsigned long long> cyc(waves), rt(waves);
    if (hipMemcpy(cyc.data(), d_cyc, waves * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    if (hipMemcpy(rt.data(), d_real, waves * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    (void)hipFree(d_cyc);
    (void)hipFree(d_real);
    (void)hipFree(d_sink);
    double sum_t = 0, sum_rt = 0;
    for (int i = 0; i < waves; ++i) {
        sum_t += static_cast<double>(cyc[i]);
        sum_rt += static_cast<double>(rt[i]);
    }
    // the shader clock: memtime ticks per ns of the constant 100 MHz clock, over the waves' spans
    const double clk = sum_t / (sum_rt * 10.0);
    if (ghz) *ghz = clk;
    // cycles per wave64 instruction per SIMD from the launch's wall time (the waves' own spans
    // would assume every wave of the grid resident at once, which the dispatch does not guarantee)
    const double insts_per_simd = static_cast<double>(waves) * kIters * kUnroll / (cus * 4.0);
    return ms * 1e-3 * clk * 1e9 / insts_per_simd;
}

int main() {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
    const char* names[] = {"v_fma_f32", "v_add_f64", "v_mul_f64", "v_fma_f64", "v_rcp_f64", "v_add_f32",
                           "v_mul_f32", "v_xor_b32", "v_rcp_f32", "v_pk_fma_f32", "v_pk_add_f32", "v_min_f32",
                           "v_max3_f32", "v_cndmask_b32", "v_min_i32", "v_max_u32", "v_med3_f32", "v_min3_i32",
                           "v_min_f64", "v_cmp_lt_f32", "v_bfe_u32", "v_lshl_or_b32", "v_mul_lo_u32",
                           "v_mul_hi_u32", "v_mad_u32_u24", "v_cvt_f32_u32", "v_cvt_f64_u32", "v_rsq_f64",
                           "v_sqrt_f64", "v_cmp_lt_f64", "v_mov_b32", "v_add_u32"};
    constexpr int kKinds = sizeof(names) / sizeof(names[0]);
    const int cfg[4][2] = {{256, 1}, {512, 1}, {1024, 1}, {1024, 2}};  // 1, 2, 4, 8 waves per SIMD
    double ghz = 0, fma64_tflops = 0;
    std::printf("{\"cus\": %d, \"cycles_per_wave64_instruction_per_simd\": {", cus);
    for (int k = 0; k < kKinds; ++k) {
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
                case 6: r = measure<6, float>(cus, th, bp, &ghz); break;
                case 7: r = measure<7, float>(cus, th, bp, &ghz); break;
                case 8: r = measure<8, float>(cus, th, bp, &ghz); break;
                case 9: r = measure<9, F2>(cus, th, bp, &ghz); break;
                case 10: r = measure<10, F2>(cus, th, bp, &ghz); break;
                case 11: r = measure<11, float>(cus, th, bp, &ghz); break;
                case 12: r = measure<12, float>(cus, th, bp, &ghz); break;
                case 13: r = measure<13, float>(cus, th, bp, &ghz); break;
                case 14: r = measure<14, float>(cus, th, bp, &ghz); break;
                case 15: r = measure<15, float>(cus, th, bp, &ghz); break;
                case 16: r = measure<16, float>(cus, th, bp, &ghz); break;
                case 17: r = measure<17, float>(cus, th, bp, &ghz); break;
                case 18: r = measure<18, double>(cus, th, bp, &ghz); break;
                case 19: r = measure<19, float>(cus, th, bp, &ghz); break;
                case 20: r = measure<20, float>(cus, th, bp, &ghz); break;
                case 21: r = measure<21, float>(cus, th, bp, &ghz); break;
                case 22: r = measure<22, float>(cus, th, bp, &ghz); break;
                case 23: r = measure<23, float>(cus, th, bp, &ghz); break;
                case 24: r = measure<24, float>(cus, th, bp, &ghz); break;
                case 25: r = measure<25, float>(cus, th, bp, &ghz); break;
                case 26: r = measure<26, double>(cus, th, bp, &ghz); break;
                case 27: r = measure<27, double>(cus, th, bp, &ghz); break;
                case 28: r = measure<28, double>(cus, th, bp, &ghz); break;
                case 29: r = measure<29, double>(cus, th, bp, &ghz); break;
                case 30: r = measure<30, float>(cus, th, bp, &ghz); break;
                case 31: r = measure<31, float>(cus, th, bp, &ghz); break;
            }
            if (k == 3 && c == 3) {  // v_fma_f64 at 8 waves: the wall-clock rate
                const double insts = static_cast<double>(cus) * bp * (th / 64) * kIters * kUnroll;
                std::fprintf(stderr, "v_fma_f64 8 waves: %.3f ms, %.1f TFLOP/s f64\n", g_last_ms, insts * 64 * 2 / (g_last_ms * 1e-3) / 1e12);
                fma64_tflops = insts * 64 * 2 / (g_last_ms * 1e-3) / 1e12;
            }
            std::printf("%s\"%d_waves\": %.3f", c ? ", " : "", th / 64 * bp / 4, r);
        }
        std::printf("}");
    }
    std::printf("}, \"shader_clock_ghz\": %.3f, \"v_fma_f64_8_waves_wall_tflops\": %.1f}\n", ghz, fma64_tflops);
    return 0;
}
