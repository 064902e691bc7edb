// The parallelogram candidate filter of the render kernel's two-pass leaves (crt_device.hip
// leaf_step), shared with its host fuzzer (tools/fuzz_quad_filter.cpp), which runs this exact
// f32 sequence against the exact test.
//
// The exact test is Parallelogram::hit_by (parallelogram.h:177-240) in f64:
//   den = n.d; |den| < 1e-9 -> miss; t = n.(v - o) / den; !(tmin < t < tmax) -> miss;
//   w = (o + d t) - v; alpha = sn.(w x s2), beta = sn.(s1 x w); hit iff alpha, beta in [0, 1]
// (n = unit normal, sn = n / |n|^2 of the ctor, parallelogram.h:269-296). The filter returns false
// only where that test provably misses, for this t_max and any smaller one: t <= t_min, t >= t_max,
// alpha or beta outside [0, 1]. It computes the same quantities in f32 from f32-rounded inputs,
// alpha and beta through the triple-product identities alpha = w.(s2 x sn), beta = w.(sn x s1)
// with g1 = s2 x sn and g2 = sn x s1 precomputed per parallelogram (quad_record):
//   num' = sn'.(v' - o'), den' = sn'.d', t' = num' * rcp(den')       (sn is parallel to n, so
//   num'/den' estimates t; the |n| scale cancels)
//   w' = d' t' - (v' - o'), alpha' = g1'.w', beta' = g2'.w'
// Error bounds, with u = 2^-24, V = max|v|, O = max|o|, D = max|d|, SN1 = |sn|_1, S1 = |s1|_1,
// S2 = |s2|_1 (each input rounding, product and sum rounds once, fma once):
//   |num' - num| <= a' = 6u SN1 (V + O),   |den' - den| <= b' = 5u SN1 D
//   for |den'| > 2 b':   |num'/den' - t| <= 2 (a' + b' |num'/den'|) / |den'|
//   rcp (1 ulp) and the product add 3.2u |t'|                      =>  Et
//   |w'_k - w_k| <= D Et + 3u Mw,  Mw = O + D |t'| + V  (bounds |o|, |d t|, |v|, |w|)
//   g1' = RN32(RN64(s2 x sn)): |g1' - g1|_1 <= u |g1|_1 + 2^-51 S2 SN1, and |g1|_1 <= SN1 S2
//   (likewise g2 with S1); the three roundings of the dot product add <= 3u(1 + u) |g1'|_1 Mw:
//   |alpha' - alpha| <= SN1 S2 (D Et + 7.01u Mw),  |beta' - beta| <= SN1 S1 (D Et + 7.01u Mw)
// The filter uses a = 7u SN1 (V + O), b = 6u SN1 D, Et = 2.5 (a + b|t'|)|rcp| + 4u|t'| and
// Ea = Ka (1.25 D Et + 14u Mw) with Ka = SN1 S2, Kb = SN1 S1 rounded up on the host (slack >= 15%
// over every bound, 2x on the alpha / beta rounding terms: it also covers the rounding of these
// bound computations and the f64 test's own rounding errors, which are ~2^-29 of the f32 ones),
// plus absolute floors (2^-80 in a and b, 2^-50 in Ea, Eb) for underflow. A rejection needs a TRUE
// strict comparison against a bound rounded in f32 (x > RN(1 + Ea) implies x > 1 + Ea), so NaN /
// inf anywhere (0/0, overflowed bounds) keeps the quad a candidate. Valid for |v_k|, |s1_k|,
// |s2_k|, |o_k| <= 2^30, SN1 in [2^-64, 2^40] per quad (the host sets the scene flag), and D in
// [2^-30, 2^30] per ray (quad_ray32_ok).
#pragma once

#include <cmath>
#include <cstdint>

#ifndef CRT_HD
#define CRT_HD inline
#endif

namespace crt {

// one f32 parallelogram record (64 bytes, four 16-byte loads)
struct alignas(16) DevQuadF {
    float v[3], g1[3], g2[3], sn[3];  // g1 = s2 x sn, g2 = sn x s1 (alpha = g1.w, beta = g2.w)
    float sn1;      // |sn|_1, rounded up
    float ka, kb;   // |sn|_1 |s2|_1, |sn|_1 |s1|_1, rounded up
    float vmax;     // max_k |v'_k| (exact)
};
static_assert(sizeof(DevQuadF) == 64, "f32 quad record");
constexpr double kF32QuadMax = 0x1p30;

// the ray in f32 for the filter (per entered leaf)
struct QuadRay32 {
    float o[3], d[3];
    float O, D;      // max |o'_k|, max |d'_k|
    float b6;        // 6u D (b = SN1 * b6)
    float tlo, thi;  // f32 bounds with tlo <= t_min, thi >= t_max
};

constexpr float kU = 0x1p-24f;

// RN32 of x rounded down / up to a float bound (x finite or inf)
CRT_HD float f32_down(double x) {
    float f = static_cast<float>(x);
    if (static_cast<double>(f) > x) f = std::nextafter(f, -INFINITY);
    return f;
}
CRT_HD float f32_up(double x) {
    float f = static_cast<float>(x);
    if (static_cast<double>(f) < x) f = std::nextafter(f, INFINITY);
    return f;
}

CRT_HD bool quad_ray32_ok(const double o[3], const double d[3]) {
    bool ok = true;
    double dm = 0;
    for (int k = 0; k < 3; ++k) {
        ok = ok && std::fabs(o[k]) <= kF32QuadMax && std::fabs(d[k]) <= 0x1p30;
        dm = std::fmax(dm, std::fabs(d[k]));
    }
    return ok && dm >= 0x1p-30;
}

CRT_HD void quad_ray32(const double o[3], const double d[3], double tmin, double tmax, QuadRay32& L) {
    float O = 0, D = 0;
    for (int k = 0; k < 3; ++k) {
        L.o[k] = static_cast<float>(o[k]);
        L.d[k] = static_cast<float>(d[k]);
        O = std::fmax(O, std::fabs(L.o[k]));
        D = std::fmax(D, std::fabs(L.d[k]));
    }
    L.O = O;
    L.D = D;
    L.b6 = D * (6 * kU);
    L.tlo = f32_down(tmin);
    L.thi = f32_up(tmax);
}

// the filter record of a parallelogram (the ctor's v, s1, s2, sn in f64); false when it is outside
// the filter's range (the scene then decides its parallelograms in f64)
CRT_HD bool quad_record(const double v[3], const double s1[3], const double s2[3], const double sn[3],
                        DevQuadF& f) {
    double sn1 = 0, S1 = 0, S2 = 0;
    bool ok = true;
    const double g1[3] = {s2[1] * sn[2] - s2[2] * sn[1], s2[2] * sn[0] - s2[0] * sn[2], s2[0] * sn[1] - s2[1] * sn[0]};
    const double g2[3] = {sn[1] * s1[2] - sn[2] * s1[1], sn[2] * s1[0] - sn[0] * s1[2], sn[0] * s1[1] - sn[1] * s1[0]};
    float vmax = 0;
    for (int k = 0; k < 3; ++k) {
        f.v[k] = static_cast<float>(v[k]);
        f.g1[k] = static_cast<float>(g1[k]);
        f.g2[k] = static_cast<float>(g2[k]);
        f.sn[k] = static_cast<float>(sn[k]);
        vmax = std::fmax(vmax, std::fabs(f.v[k]));
        sn1 += std::fabs(sn[k]);
        S1 += std::fabs(s1[k]);
        S2 += std::fabs(s2[k]);
        ok = ok && std::fabs(v[k]) <= kF32QuadMax && std::fabs(s1[k]) <= kF32QuadMax && std::fabs(s2[k]) <= kF32QuadMax;
    }
    f.sn1 = f32_up(sn1 * (1 + 0x1p-20));
    f.ka = f32_up(sn1 * S2 * (1 + 0x1p-20));
    f.kb = f32_up(sn1 * S1 * (1 + 0x1p-20));
    f.vmax = vmax;
    return ok && sn1 >= 0x1p-64 && sn1 <= 0x1p40;
}

// false only where Parallelogram::hit_by provably misses for t_max (and any smaller t_max);
// rcp(x) is the hardware reciprocal (within 1 ulp of 1/x)
template <typename Rcp>
CRT_HD bool quad_candidate(const DevQuadF& q, const QuadRay32& L, Rcp rcp) {
    const float vx = q.v[0] - L.o[0], vy = q.v[1] - L.o[1], vz = q.v[2] - L.o[2];
    const float num = std::fma(q.sn[2], vz, std::fma(q.sn[1], vy, q.sn[0] * vx));
    const float den = std::fma(q.sn[2], L.d[2], std::fma(q.sn[1], L.d[1], q.sn[0] * L.d[0]));
    const float V = q.vmax;
    const float a = std::fma(q.sn1 * (7 * kU), V + L.O, 0x1p-80f);
    const float b = std::fma(q.sn1, L.b6, 0x1p-80f);
    const float r = rcp(den);
    const float t = num * r;
    const float at = std::fabs(t);
    const float Et = std::fma(std::fma(b, at, a), std::fabs(r) * 2.5f, at * (4 * kU));
    const bool den_ok = std::fabs(den) > 2 * b;
    const bool t_out = (t + Et < L.tlo) | (t - Et > L.thi);
    const float wx = std::fma(L.d[0], t, -vx), wy = std::fma(L.d[1], t, -vy), wz = std::fma(L.d[2], t, -vz);
    // alpha = sn . (w x s2) = w . g1, beta = sn . (s1 x w) = w . g2
    const float alpha = std::fma(q.g1[2], wz, std::fma(q.g1[1], wy, q.g1[0] * wx));
    const float beta = std::fma(q.g2[2], wz, std::fma(q.g2[1], wy, q.g2[0] * wx));
    const float Mw = std::fma(L.D, at, L.O + V);
    const float base = std::fma(L.D, Et * 1.25f, Mw * (14 * kU));
    const float Ea = std::fma(q.ka, base, 0x1p-50f), Eb = std::fma(q.kb, base, 0x1p-50f);
    const bool a_out = (alpha < -Ea) | (alpha > 1 + Ea);
    const bool b_out = (beta < -Eb) | (beta > 1 + Eb);
    return !(den_ok & (t_out | a_out | b_out));
}

// ---- axis-aligned parallelograms: the walk's node test on a flat box ---------------------------
// A parallelogram whose sides lie along two different axes i, j (every face of a Box, box.h:53-84,
// and the Cornell walls) is the rectangle p_k = v_k, p_i in [a_i, b_i], p_j in [a_j, b_j]: the
// flat box with a_k = b_k = v_k. Its unit normal and sn are exactly zero off axis k (each cross-
// product component has a zero factor in both products), so the reference computes
//   t = n_k (v_k - o_k) / (n_k d_k),   alpha = (p_i - v_i) / s1_i,   beta = (p_j - v_j) / s2_j
// up to a few f64 roundings: within ~10 u64 (|t| + |o_i / d_i| + |v_i / d_i|) of the exact values
// in t units (u64 = 2^-53; an alpha error e is a t error e |s1_i / d_i|). "alpha in [0, 1]" is
// "t within the i-slab of the box", so the reference's hit is the slab test of the flat box
// (t in (t_min, t_max), every slab containing t) up to those errors.
// The filter runs the render kernel's f32 node test (crt_device.hip walk(): t'_jk = fma(b32_jk,
// inv32_k, -oinv32_k), lo' = max of the mins and tmin', hi' = min of the maxes and tmax',
// gap' = hi' - lo', th = 2^-19 max(|lo'|, |hi'|) + marg) on the box rounded to f32 and rejects
// when gap' < -th. The walk's analysis bounds |gap' - gap64| by 2^-20.1 M + 2^-19.8 A + 2^-84
// (M = max(|lo'|, |hi'|), A = max_k |o_k / d_k|, gap64 the f64 slab gap), so a rejection means
// gap64 < -2^-20.3 (M + A): the ray misses the closed rectangle (or the (t_min, t_max) range) by
// at least that much in exact arithmetic, ~2^30 times the reference's rounding errors above (|t|,
// the bounding slab values and |v_i / d_i| <= |slab value| + A are all <= M + A where they
// decide), so the reference misses it too, for this t_max and any smaller one. Rays outside the
// walk's range carry marg = inf (every quad a candidate), and NaN never rejects.
// flat_box_candidate below is that sequence; the kernel (leaf_step) and tools/fuzz_quad_filter.cpp
// (against the exact test) both call it.
struct alignas(16) DevQuadBox {
    float b[6];      // x.min x.max y.min y.max z.min z.max (RN32 of the f64 bounds)
    uint32_t pad[2];
};
static_assert(sizeof(DevQuadBox) == 32, "flat quad box record");

// the flat box of an axis-aligned parallelogram; false for any other one (or bounds beyond the
// walk's 2^40 range)
CRT_HD bool quad_flat_box(const double v[3], const double s1[3], const double s2[3], DevQuadBox& f) {
    int a1 = -1, a2 = -1;
    for (int k = 0; k < 3; ++k) {
        if (s1[k] != 0) {
            if (a1 >= 0) return false;
            a1 = k;
        }
        if (s2[k] != 0) {
            if (a2 >= 0) return false;
            a2 = k;
        }
    }
    if (a1 < 0 || a2 < 0 || a1 == a2) return false;
    for (int k = 0; k < 3; ++k) {
        double lo = v[k], hi = v[k];
        const double e = k == a1 ? v[k] + s1[k] : k == a2 ? v[k] + s2[k] : v[k];
        lo = std::fmin(lo, e);
        hi = std::fmax(hi, e);
        if (!(std::fabs(lo) <= 0x1p40 && std::fabs(hi) <= 0x1p40)) return false;
        f.b[2 * k] = static_cast<float>(lo);
        f.b[2 * k + 1] = static_cast<float>(hi);
    }
    f.pad[0] = f.pad[1] = 0;
    return true;
}

// The flat-box filter: false only where the exact test provably misses (see above). b = the box
// (DevQuadBox::b), inv32 / oinv32 / marg = the ray's f32 walk constants (crt_device.hip
// trav_init), tmin32 = RN32(t_min), tmax32 = RN32(min(t_max, 2^100)). MM supplies min / max /
// min3 / max3 / max_s (second operand wave-uniform) / max_abs of non-NaN floats: the kernel's
// v_min_f32 family, or std::fmin / std::fmax on the host (the same values for non-NaN operands).
template <typename MM>
CRT_HD bool flat_box_candidate(const float b[6], const float inv32[3], const float oinv32[3], float tmin32,
                               float tmax32, float marg) {
    const float x0 = std::fma(b[0], inv32[0], -oinv32[0]);
    const float x1 = std::fma(b[1], inv32[0], -oinv32[0]);
    const float y0 = std::fma(b[2], inv32[1], -oinv32[1]);
    const float y1 = std::fma(b[3], inv32[1], -oinv32[1]);
    const float z0 = std::fma(b[4], inv32[2], -oinv32[2]);
    const float z1 = std::fma(b[5], inv32[2], -oinv32[2]);
    const float lo = MM::max3(MM::min(x0, x1), MM::min(y0, y1), MM::max_s(MM::min(z0, z1), tmin32));
    const float hi = MM::min3(MM::max(x0, x1), MM::max(y0, y1), MM::min(MM::max(z0, z1), tmax32));
    const float th = std::fma(MM::max_abs(lo, hi), 0x1p-19f, marg);
    return !(hi - lo < -th);
}

// flat_box_candidate for a box flat on axis K (b[2K] == b[2K + 1], so the axis' two slab values
// are one, t): lo' = max(t, the other axes' mins, tmin') and hi' = min(t, the other axes' maxes,
// tmax') take the min / max of the same values as flat_box_candidate's lo' / hi' (min(t, t) =
// max(t, t) = t), in another order; min / max of non-NaN values are exact, so they are the same
// floats and the decision is the same bit, with one FMA and two min / max fewer. (A NaN arises
// only for rays outside the walk's range, where marg = inf makes both return true.) The kernel
// runs it over the leaf's records grouped by flat axis (crt_device.hip stage_image, leaf_step);
// tools/fuzz_quad_filter.cpp checks it against flat_box_candidate on every flat case.
template <int K, typename MM>
CRT_HD bool flat_axis_candidate(const float b[6], const float inv32[3], const float oinv32[3], float tmin32,
                                float tmax32, float marg) {
    constexpr int I = K == 0 ? 1 : 0, J = K == 2 ? 1 : 2;
    const float t = std::fma(b[2 * K], inv32[K], -oinv32[K]);
    const float i0 = std::fma(b[2 * I], inv32[I], -oinv32[I]);
    const float i1 = std::fma(b[2 * I + 1], inv32[I], -oinv32[I]);
    const float j0 = std::fma(b[2 * J], inv32[J], -oinv32[J]);
    const float j1 = std::fma(b[2 * J + 1], inv32[J], -oinv32[J]);
    const float lo = MM::max3(MM::min(i0, i1), MM::min(j0, j1), MM::max_s(t, tmin32));
    const float hi = MM::min3(MM::max(i0, i1), MM::max(j0, j1), MM::min(t, tmax32));
    const float th = std::fma(MM::max_abs(lo, hi), 0x1p-19f, marg);
    return !(hi - lo < -th);
}

// host min / max for flat_box_candidate
struct HostMinMax {
    static float min(float a, float b) { return std::fmin(a, b); }
    static float max(float a, float b) { return std::fmax(a, b); }
    static float min3(float a, float b, float c) { return std::fmin(std::fmin(a, b), c); }
    static float max3(float a, float b, float c) { return std::fmax(std::fmax(a, b), c); }
    static float max_s(float a, float b) { return std::fmax(a, b); }
    static float max_abs(float a, float b) { return std::fmax(std::fabs(a), std::fabs(b)); }
};

}  // namespace crt
