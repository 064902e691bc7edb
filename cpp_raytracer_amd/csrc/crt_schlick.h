// Schlick's reflectance term of Dielectric::reflectance (material.h:175-181),
//   r0 + (1 - r0) * pow(1 - cosine, 5),
// shared by the render kernel (shade) and its host fuzzer (tools/fuzz_schlick.cpp).
//
// The reference calls glibc's pow, which is not correctly rounded: its error bound is ~0.52 ulp,
// and measured over random x in (0, 1] its pow(x, 5) differs from the correctly rounded x^5 in
// ~8e-4 of inputs, always by one ulp. glibc's two x86-64 variants (FMA and SSE2, picked by the
// host CPU) also disagree with EACH OTHER on ~7e-4 of inputs, so "glibc's result" depends on the
// machine the reference runs on. The kernel therefore computes x^5 correctly rounded (pow5: a
// double-double product rounded once) and proves, per decision, that the reference's
// `rand_double() < reflectance` takes the same branch for ANY pow result within one ulp of it:
// the reflectance is monotone in the pow value (1 - r0 >= 0, rounding is monotone), so the
// branch is the same for every value in [pred(p), succ(p)] unless the draw u satisfies
// R(pred(p)) <= u < R(succ(p)). schlick_undecided() flags exactly those draws; the kernel counts
// them in the scene's guard word (crt_render_guard), and a render whose count is 0 took every
// Dielectric branch as the reference does on either glibc variant. tools/fuzz_schlick.cpp checks
// the premise: |glibc pow(x, 5) - pow5(x)| <= 1 ulp for both variants over 1e9 draws.
#pragma once

#include <cstdint>
#include <cstring>

#ifndef CRT_HD
#define CRT_HD inline
#define CRT_FMA(a, b, c) std::fma(a, b, c)
#include <cmath>
#else
#define CRT_FMA(a, b, c) __builtin_fma(a, b, c)
#endif

namespace crt {

// x^5 rounded once from a double-double product (x >= 0)
CRT_HD double pow5(double x) {
    const double x2h = x * x;
    const double x2l = CRT_FMA(x, x, -x2h);
    const double x4h = x2h * x2h;
    const double x4l = CRT_FMA(x2h, x2h, -x4h) + 2 * x2h * x2l;
    const double x5h = x4h * x;
    const double x5l = CRT_FMA(x4h, x, -x5h) + x4l * x;
    return x5h + x5l;
}

// the neighbours of p >= 0 in the doubles (p finite)
CRT_HD double schlick_pred(double p) {
    uint64_t b;
    __builtin_memcpy(&b, &p, 8);
    b = p > 0 ? b - 1 : 0x8000000000000001ull;  // pred(+0) = -denorm_min
    double r;
    __builtin_memcpy(&r, &b, 8);
    return r;
}
CRT_HD double schlick_succ(double p) {
    uint64_t b;
    __builtin_memcpy(&b, &p, 8);
    b += 1;
    double r;
    __builtin_memcpy(&r, &b, 8);
    return r;
}

// true when `u < r0 + (1 - r0) * q` is not the same for every q in [pred(p), succ(p)]
CRT_HD bool schlick_undecided(double u, double r0, double p) {
    const double lo = r0 + (1 - r0) * schlick_pred(p);
    const double hi = r0 + (1 - r0) * schlick_succ(p);
    return lo <= u && u < hi;
}

}  // namespace crt
