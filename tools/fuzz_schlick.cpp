// Host fuzzer of crt_schlick.h (the render kernel's Schlick term): compares the kernel's
// correctly rounded pow5(x) with this host's glibc pow(x, 5.0) — the function the reference's
// Dielectric::reflectance calls (material.h:180) — over n pseudo-random x in (0, 1] (uniform,
// plus a log-uniform share reaching tiny x) and reports the mismatch count and the largest
// distance in ulps. The kernel's per-decision guard (schlick_undecided) is exact only if that
// distance is <= 1; tests/test_schlick.py runs this under both of glibc's x86-64 pow variants
// (FMA and SSE2, selected with GLIBC_TUNABLES).
//   g++ -std=c++20 -O2 -ffp-contract=off -fopenmp tools/fuzz_schlick.cpp -o fuzz_schlick
//   ./fuzz_schlick <n>   -> JSON line
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../cpp_raytracer_amd/csrc/crt_schlick.h"

static int64_t ulp_key(double x) {  // monotone integer key of a double
    int64_t b;
    __builtin_memcpy(&b, &x, 8);
    return b < 0 ? INT64_MIN - b : b;
}

int main(int argc, char** argv) {
    const long long n = argc > 1 ? std::atoll(argv[1]) : 100000000LL;
    long long mismatches = 0, max_ulps = 0, undecided = 0;
    double worst_x = 0;
#pragma omp parallel for schedule(static) reduction(+ : mismatches, undecided) reduction(max : max_ulps)
    for (long long i = 0; i < n; ++i) {
        uint64_t z = static_cast<uint64_t>(i) * 0x9E3779B97F4A7C15ull + 0x1234567ull;  // splitmix64
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        double x = static_cast<double>(z >> 11) * 0x1p-53;
        if (i % 8 == 7) x = std::ldexp(1.0 + x, -static_cast<int>(z % 200));  // log-uniform share
        if (x == 0) x = 1;
        const double mine = crt::pow5(x), ref = std::pow(x, 5.0);
        if (mine != ref) {
            ++mismatches;
            const long long d = std::llabs(ulp_key(mine) - ulp_key(ref));
            if (d > max_ulps) max_ulps = d;
        }
        // the guard with the Schlick r0 of the reference scenes' glass (ri 1.5 / 1/1.5 -> 0.04)
        const double r = (1 - 1.5) / (1 + 1.5), r0 = r * r;
        const double u = static_cast<double>(static_cast<uint32_t>(z)) * (1 / static_cast<double>(4294967295u - 1));
        if (crt::schlick_undecided(u, r0, mine)) ++undecided;
    }
    (void)worst_x;
    std::printf("{\"n\": %lld, \"mismatches\": %lld, \"max_ulps\": %lld, \"undecided\": %lld}\n", n, mismatches,
                max_ulps, undecided);
    return 0;
}
