// Fuzz check of the render kernel's parallelogram candidate filter (csrc/crt_quad_filter.h
// quad_candidate, the code the kernel runs): the filter may keep a parallelogram the exact test
// rejects, but must never reject one the exact test (Parallelogram::hit_by, parallelogram.h:177-240,
// as in crt_device.hip hit_quad / oracle/crt_oracle.c) accepts for the same t_max.
// Build: g++ -std=c++20 -O2 -ffp-contract=off -o /tmp/fuzzq tools/fuzz_quad_filter.cpp
// Run:   /tmp/fuzzq [millions of cases per family]
// The hardware reciprocal (v_rcp_f32, within 1 ulp) is modelled adversarially: RN(1/x) moved one
// ulp up or down at random. Families: random rays around random parallelograms at scales 2^-10 to
// 2^20 (and Cornell-box-like ones), rays aimed at edges and corners (alpha or beta within a few ulps
// of 0 or 1), grazing rays (direction almost in the plane), rays leaving the surface (t ~ t_min),
// and t_max within a few ulps of the hit. Prints violations (must be 0) and the rejection rate.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../cpp_raytracer_amd/csrc/crt_quad_filter.h"

using crt::DevQuadF;
using crt::QuadRay32;

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint64_t next_u64() {
    rs ^= rs >> 12; rs ^= rs << 25; rs ^= rs >> 27;
    return rs * 2685821657736338717ull;
}
static double u01() { return static_cast<double>(next_u64() >> 11) * 0x1p-53; }
static double urange(double lo, double hi) { return lo + (hi - lo) * u01(); }
static double ulps(double x, int k) {  // x moved by k ulps
    for (; k > 0; --k) x = std::nextafter(x, INFINITY);
    for (; k < 0; ++k) x = std::nextafter(x, -INFINITY);
    return x;
}

struct Quad {
    double v[3], s1[3], s2[3], n[3], sn[3];
};

// the ctor's derived data (parallelogram.h:269-296; crt_host.cpp make_quad): n = unit(cross),
// sn = cross * (1 / |cross|^2), vec3d.h:34 divides by multiplying with the reciprocal
static Quad make_quad(const double v[3], const double s1[3], const double s2[3]) {
    Quad q;
    for (int k = 0; k < 3; ++k) { q.v[k] = v[k]; q.s1[k] = s1[k]; q.s2[k] = s2[k]; }
    const double c[3] = {s1[1] * s2[2] - s1[2] * s2[1], s1[2] * s2[0] - s1[0] * s2[2], s1[0] * s2[1] - s1[1] * s2[0]};
    const double m2 = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
    const double il = 1 / std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    const double i2 = 1 / m2;
    for (int k = 0; k < 3; ++k) { q.n[k] = c[k] * il; q.sn[k] = c[k] * i2; }
    return q;
}

// crt_device.hip hit_quad, operation for operation
static bool exact(const Quad& q, const double o[3], const double d[3], double tmin, double tmax, double* tout) {
    double den = q.n[0] * d[0] + q.n[1] * d[1] + q.n[2] * d[2];
    if (std::fabs(den) < 1e-9) return false;
    double vx = q.v[0] - o[0], vy = q.v[1] - o[1], vz = q.v[2] - o[2];
    double ht = (q.n[0] * vx + q.n[1] * vy + q.n[2] * vz) / den;
    if (tout) *tout = ht;
    if (!(tmin < ht && ht < tmax)) return false;
    double px = o[0] + d[0] * ht, py = o[1] + d[1] * ht, pz = o[2] + d[2] * ht;
    double wx = px - q.v[0], wy = py - q.v[1], wz = pz - q.v[2];
    double c1x = wy * q.s2[2] - wz * q.s2[1];
    double c1y = wz * q.s2[0] - wx * q.s2[2];
    double c1z = wx * q.s2[1] - wy * q.s2[0];
    double alpha = q.sn[0] * c1x + q.sn[1] * c1y + q.sn[2] * c1z;
    double c2x = q.s1[1] * wz - q.s1[2] * wy;
    double c2y = q.s1[2] * wx - q.s1[0] * wz;
    double c2z = q.s1[0] * wy - q.s1[1] * wx;
    double beta = q.sn[0] * c2x + q.sn[1] * c2y + q.sn[2] * c2z;
    return 0 <= alpha && alpha <= 1 && 0 <= beta && beta <= 1;
}

// the host side of the record (crt_quad_filter.h quad_record, as crt_device.hip device_upload)
static bool record(const Quad& q, DevQuadF& f) { return crt::quad_record(q.v, q.s1, q.s2, q.sn, f); }

static float rcp_adversarial(float x) {
    float r = 1.0f / x;
    const uint64_t k = next_u64() % 3;
    if (k == 1) r = std::nextafter(r, INFINITY);
    if (k == 2) r = std::nextafter(r, -INFINITY);
    return r;
}

static void rand_dir(double s, double d[3]) {
    double m;
    do {
        for (int k = 0; k < 3; ++k) d[k] = urange(-1, 1);
        m = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
    } while (m > 1 || m < 1e-6);
    for (int k = 0; k < 3; ++k) d[k] *= s;
}

static long viol = 0, miss_total = 0, miss_rejected = 0, hits = 0, skipped = 0;
static long fviol = 0, fmiss_total = 0, fmiss_rejected = 0, fhits = 0;
static long axis_checked = 0, axis_diff = 0;  // flat_axis_candidate vs flat_box_candidate

// the render kernel's flat-box filter for axis-aligned parallelograms (crt_device.hip leaf_step
// calls the same crt::flat_box_candidate), with the ray constants of trav_init (inv32 =
// v_rcp_f32(RN32(d)), oinv32 = RN32(RN32(o) inv32), marg) and tmin' = RN32(t_min),
// tmax' = RN32(min(t_max, 2^100)). The walk's range (|d'_k| in [2^-39, 2^39], |o'_k| <= 2^40) is
// the filter's own; outside it marg = inf keeps every parallelogram.
static bool flat_candidate(const crt::DevQuadBox& b, const double o[3], const double d[3], double tmin,
                           double tmax) {
    float inv[3], oinv[3], A = 0;
    bool f32 = true;
    for (int k = 0; k < 3; ++k) {
        const float d32 = static_cast<float>(d[k]), o32 = static_cast<float>(o[k]);
        inv[k] = rcp_adversarial(d32);
        oinv[k] = o32 * inv[k];
        A = std::fmax(A, std::fabs(oinv[k]));
        f32 = f32 && std::fabs(d32) <= 0x1p39f && std::fabs(d32) >= 0x1p-39f && std::fabs(o32) <= 0x1p40f;
    }
    const float marg = f32 ? std::fmax(A * 0x1p-19f, 0x1p-60f) : INFINITY;
    const float tmin32 = static_cast<float>(tmin), tmax32 = static_cast<float>(std::fmin(tmax, 0x1p100));
    const bool c = crt::flat_box_candidate<crt::HostMinMax>(b.b, inv, oinv, tmin32, tmax32, marg);
    // the kernel's per-axis form (grouped leaves) must give the same bit
    int flat = -1;
    for (int k = 0; k < 3 && flat < 0; ++k)
        if (b.b[2 * k] == b.b[2 * k + 1]) flat = k;
    const bool ca = flat == 0   ? crt::flat_axis_candidate<0, crt::HostMinMax>(b.b, inv, oinv, tmin32, tmax32, marg)
                    : flat == 1 ? crt::flat_axis_candidate<1, crt::HostMinMax>(b.b, inv, oinv, tmin32, tmax32, marg)
                                : crt::flat_axis_candidate<2, crt::HostMinMax>(b.b, inv, oinv, tmin32, tmax32, marg);
    ++axis_checked;
    axis_diff += flat < 0 || ca != c;
    return c;
}

static long fwide = 0;  // flat cases outside the generic filter's range (quad_ray32_ok false)

static void check(const Quad& q, const double o[3], const double d[3], double tmin, double tmax) {
    const bool hit = exact(q, o, d, tmin, tmax, nullptr);
    // the flat-box filter first: its range is the walk's, not the generic filter's
    crt::DevQuadBox box;
    if (crt::quad_flat_box(q.v, q.s1, q.s2, box)) {
        const bool fc = flat_candidate(box, o, d, tmin, tmax);
        if (hit) {
            ++fhits;
            if (!fc && ++fviol <= 10)
                std::printf("FLAT VIOLATION o=(%a %a %a) d=(%a %a %a) v=(%a %a %a) s1=(%a %a %a) s2=(%a %a %a) tmin=%a tmax=%a\n",
                            o[0], o[1], o[2], d[0], d[1], d[2], q.v[0], q.v[1], q.v[2], q.s1[0], q.s1[1], q.s1[2],
                            q.s2[0], q.s2[1], q.s2[2], tmin, tmax);
        } else {
            ++fmiss_total;
            fmiss_rejected += !fc;
        }
        if (!crt::quad_ray32_ok(o, d)) ++fwide;
    }
    DevQuadF f;
    if (!record(q, f) || !crt::quad_ray32_ok(o, d)) { ++skipped; return; }
    QuadRay32 L;
    crt::quad_ray32(o, d, tmin, tmax, L);
    const bool cand = crt::quad_candidate(f, L, rcp_adversarial);
    if (hit) {
        ++hits;
        if (!cand) {
            if (++viol <= 10)
                std::printf("VIOLATION o=(%a %a %a) d=(%a %a %a) v=(%a %a %a) s1=(%a %a %a) s2=(%a %a %a) tmin=%a tmax=%a\n",
                            o[0], o[1], o[2], d[0], d[1], d[2], q.v[0], q.v[1], q.v[2], q.s1[0], q.s1[1], q.s1[2],
                            q.s2[0], q.s2[1], q.s2[2], tmin, tmax);
        }
    } else {
        ++miss_total;
        miss_rejected += !cand;
    }
}

static Quad rand_quad(double S) {
    double v[3], s1[3], s2[3];
    for (int k = 0; k < 3; ++k) v[k] = urange(-S, S);
    rand_dir(S * urange(0.05, 1), s1);
    rand_dir(S * urange(0.05, 1), s2);
    if (u01() < 0.5) {  // axis-aligned (Cornell walls and boxes)
        const int a = static_cast<int>(next_u64() % 3), b = (a + 1 + static_cast<int>(next_u64() % 2)) % 3;
        for (int k = 0; k < 3; ++k) { s1[k] = 0; s2[k] = 0; }
        s1[a] = S * urange(0.05, 1) * (u01() < 0.5 ? -1 : 1);
        s2[b] = S * urange(0.05, 1) * (u01() < 0.5 ? -1 : 1);
        if (u01() < 0.5) for (int k = 0; k < 3; ++k) v[k] = std::round(v[k]);
    }
    return make_quad(v, s1, s2);
}

static void point_on(const Quad& q, double al, double be, double p[3]) {
    for (int k = 0; k < 3; ++k) p[k] = q.v[k] + q.s1[k] * al + q.s2[k] * be;
}

int main(int argc, char** argv) {
    const long M = (argc > 1 ? std::atol(argv[1]) : 2) * 1000000;
    const double scales[] = {0x1p-10, 0.01, 1, 555, 1e4, 0x1p20};
    const double tmin = 1e-5;
    for (long i = 0; i < M; ++i) {  // random rays around random quads
        const double S = scales[next_u64() % 6];
        Quad q = rand_quad(S);
        double o[3], d[3];
        for (int k = 0; k < 3; ++k) o[k] = urange(-2 * S, 2 * S);
        rand_dir(std::exp2(urange(-12, 12)), d);
        const double tmax = u01() < 0.5 ? INFINITY : std::exp2(urange(-10, 30));
        check(q, o, d, tmin, tmax);
    }
    for (long i = 0; i < M; ++i) {  // aimed at edges and corners
        const double S = scales[next_u64() % 6];
        Quad q = rand_quad(S);
        const double e[] = {0, 1};
        double al = u01() < 0.5 ? e[next_u64() % 2] : u01(), be = u01() < 0.5 ? e[next_u64() % 2] : u01();
        al = ulps(al, static_cast<int>(next_u64() % 9) - 4);
        be = ulps(be, static_cast<int>(next_u64() % 9) - 4);
        double p[3], d[3], o[3];
        point_on(q, al, be, p);
        rand_dir(std::exp2(urange(-8, 8)), d);
        const double t0 = S * std::exp2(urange(-6, 4)) / std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
        for (int k = 0; k < 3; ++k) o[k] = p[k] - d[k] * t0;
        double th = 0;
        exact(q, o, d, tmin, INFINITY, &th);
        const double tmax = u01() < 0.5 ? INFINITY : ulps(th, static_cast<int>(next_u64() % 9) - 2);
        check(q, o, d, tmin, tmax);
    }
    for (long i = 0; i < M; ++i) {  // grazing rays: direction almost in the plane
        const double S = scales[next_u64() % 6];
        Quad q = rand_quad(S);
        double p[3], d[3], o[3];
        point_on(q, urange(-0.1, 1.1), urange(-0.1, 1.1), p);
        const double eps = std::exp2(urange(-45, -5));
        for (int k = 0; k < 3; ++k) d[k] = q.s1[k] * urange(-1, 1) + q.s2[k] * urange(-1, 1) + q.n[k] * S * eps;
        const double t0 = urange(0.01, 3);
        for (int k = 0; k < 3; ++k) o[k] = p[k] - d[k] * t0;
        check(q, o, d, tmin, INFINITY);
    }
    for (long i = 0; i < M; ++i) {  // leaving the surface (scattered rays): t ~ 0 vs t_min
        const double S = scales[next_u64() % 6];
        Quad q = rand_quad(S);
        double p[3], d[3];
        point_on(q, u01(), u01(), p);
        rand_dir(std::exp2(urange(-4, 4)), d);
        if (u01() < 0.5)  // just above or below the plane
            for (int k = 0; k < 3; ++k) p[k] += q.n[k] * S * std::exp2(urange(-40, -10)) * (u01() < 0.5 ? -1 : 1);
        check(q, p, d, tmin, INFINITY);
    }
    for (long i = 0; i < M; ++i) {  // Cornell box: 555-unit walls, rays from the walls
        Quad q = rand_quad(555);
        double o[3], d[3];
        for (int k = 0; k < 3; ++k) o[k] = urange(0, 555);
        if (u01() < 0.5) o[next_u64() % 3] = u01() < 0.5 ? 0 : 555;
        rand_dir(urange(0.2, 2), d);
        check(q, o, d, tmin, u01() < 0.5 ? INFINITY : urange(1, 2000));
    }
    for (long i = 0; i < M; ++i) {  // the walk's range edges: |o| up to 2^40, |d_k| from 2^-39 to 2^39
        const double S = std::exp2(urange(20, 38));
        Quad q = rand_quad(S);
        double o[3], d[3];
        for (int k = 0; k < 3; ++k) o[k] = urange(-1, 1) * std::exp2(urange(30, 40));
        for (int k = 0; k < 3; ++k) d[k] = (u01() < 0.5 ? -1 : 1) * std::exp2(urange(-39, 39));
        if (u01() < 0.5) {  // aimed at the rectangle (or just past an edge)
            double p[3];
            point_on(q, urange(-0.01, 1.01), urange(-0.01, 1.01), p);
            const double t0 = std::exp2(urange(-20, 20));
            for (int k = 0; k < 3; ++k) o[k] = std::fmax(-0x1p40, std::fmin(0x1p40, p[k] - d[k] * t0));
        }
        const double tmax = u01() < 0.5 ? INFINITY : std::exp2(urange(-30, 60));
        check(q, o, d, tmin, tmax);
    }
    std::printf("cases %ld (skipped %ld): exact hits %ld, violations %ld; exact misses %ld, rejected by the "
                "filter %.4f\n", 6 * M, skipped, hits, viol, miss_total,
                miss_total ? static_cast<double>(miss_rejected) / miss_total : 0.0);
    std::printf("flat-box filter (axis-aligned parallelograms): exact hits %ld, violations %ld; exact misses %ld, "
                "rejected %.4f; %ld of them outside the generic filter's range\n", fhits, fviol, fmiss_total,
                fmiss_total ? static_cast<double>(fmiss_rejected) / fmiss_total : 0.0, fwide);
    std::printf("per-axis flat filter: %ld cases, %ld differ from the flat-box filter\n", axis_checked, axis_diff);
    return viol != 0 || fviol != 0 || axis_diff != 0 || axis_checked == 0;
}
