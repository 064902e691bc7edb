/* Fuzz check of the render kernel's sphere candidate filter (crt_device.hip sphere_candidate):
 * the filter may keep a sphere the exact test rejects, but must never reject a sphere the exact
 * test (Sphere::hit_by, sphere.h:45-96, as in oracle/crt_oracle.c) accepts for the same t_max.
 * Build: gcc -O2 -ffp-contract=off -o /tmp/fuzz tools/fuzz_sphere_filter.c -lm
 * Run:   /tmp/fuzz [millions of cases per family]
 * Families: random rays near random spheres at several scales, rays leaving a sphere's surface
 * (the self-intersection case), near-tangent rays, rtow-like scenes (ground sphere r = 1000),
 * and wide exponent spreads. Prints violations (must be 0) and the filter's rejection rate. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static double u01(void) { /* xorshift64* -> [0,1) */
    rs ^= rs >> 12; rs ^= rs << 25; rs ^= rs >> 27;
    return (double)((rs * 2685821657736338717ull) >> 11) * 0x1p-53;
}
static double urange(double lo, double hi) { return lo + (hi - lo) * u01(); }

/* the exact test (oracle/crt_oracle.c hit_sphere) */
static int exact(const double c[3], double r, const double o[3], const double d[3], double tmin, double tmax) {
    double oc[3] = {o[0] - c[0], o[1] - c[1], o[2] - c[2]};
    double a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
    double b = d[0] * oc[0] + d[1] * oc[1] + d[2] * oc[2];
    double cc = (oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2]) - r * r;
    double disc = b * b - a * cc;
    if (disc < 0) return 0;
    double sq = sqrt(disc);
    double root = (-b - sq) / a;
    if (!(tmin < root && root < tmax)) {
        root = (-b + sq) / a;
        if (!(tmin < root && root < tmax)) return 0;
    }
    return 1;
}

/* the kernel's filter, operation for operation */
static int candidate(const double c[3], double r, const double o[3], const double d[3], double a,
                     double lo, double hi) {
    const double ocx = o[0] - c[0], ocy = o[1] - c[1], ocz = o[2] - c[2];
    const double b = fma(d[2], ocz, fma(d[1], ocy, d[0] * ocx));
    const double q = fma(ocz, ocz, fma(ocy, ocy, ocx * ocx));
    const double r2 = r * r;
    const double cc = q - r2;
    const double disc = fma(b, b, -(a * cc));
    const double S = a * (q + r2);
    const double D = fma(S, 0x1p-30, disc) + 0x1p-500;
    const double y = -b - hi, w = b + lo;
    const int rej = (D < 0) | (y * fabs(y) > D) | (w * fabs(w) > D);
    return !rej;
}

/* the previous filter (v7): exact disc, hardware rsq, 2^-12 margins (rsq modelled by 1/sqrt) */
static int candidate_v7(const double c[3], double r, const double o[3], const double d[3], double a,
                        double lo, double hi) {
    double ocx = o[0] - c[0], ocy = o[1] - c[1], ocz = o[2] - c[2];
    double b = d[0] * ocx + d[1] * ocy + d[2] * ocz;
    double cc = (ocx * ocx + ocy * ocy + ocz * ocz) - r * r;
    double disc = b * b - a * cc;
    if (disc < 0) return 0;
    const double sqa = disc * (1 / sqrt(disc));
    const double m = (fabs(b) + sqa) * 0x1p-12;
    return !((-b - sqa) - m > hi || (-b + sqa) + m < lo);
}

/* The f32 filter (crt_device.hip sphere_candidate_f32 + sphere_f32 / leaf_f32 setup), operation
 * for operation: per sphere c32 = RN32(c), r2e = RN32(r^2 (1 + 2^-14) + 2^22 |c - c32|^2); per ray
 * o32, d32, a32 = RN32(a), kap = RN32(2^22 |o - o32|^2 + 2^-50), hi32 = RN32(tmax a (1 + 2^-20)),
 * lo32 = RN32(tmin a (1 - 2^-20)). Returns -1 when the ray or sphere is outside the f32 range
 * (the kernel then runs the exact test on every sphere). */
static int f32_ray_ok(const double o[3], const double d[3], double a) {
    for (int k = 0; k < 3; ++k)
        if (!(fabs(o[k]) <= 0x1p30 && fabs(d[k]) <= 0x1p30)) return 0;
    return a >= 0x1p-60 && a <= 0x1p60;
}
static int f32_sphere_ok(const double c[3], double r) {
    for (int k = 0; k < 3; ++k)
        if (!(fabs(c[k]) <= 0x1p30)) return 0;
    return r >= 0 && r <= 0x1p30;
}
static int candidate_f32(const double c[3], double r, const double o[3], const double d[3], double a,
                         double tmin, double tmax) {
    float c32[3], o32[3], d32[3];
    double dc2 = 0, do2 = 0;
    for (int k = 0; k < 3; ++k) {
        c32[k] = (float)c[k];
        o32[k] = (float)o[k];
        d32[k] = (float)d[k];
        dc2 += (c[k] - (double)c32[k]) * (c[k] - (double)c32[k]);
        do2 += (o[k] - (double)o32[k]) * (o[k] - (double)o32[k]);
    }
    const float r2e = (float)(r * r * (1 + 0x1p-14) + dc2 * 0x1p22);
    const float kap = (float)(do2 * 0x1p22 + 0x1p-50);
    const float a32 = (float)a;
    const float hi32 = (float)(tmax * a * (1 + 0x1p-20));
    const float lo32 = (float)(tmin * a * (1 - 0x1p-20));
    /* per sphere */
    const float xx = o32[0] - c32[0], xy = o32[1] - c32[1], xz = o32[2] - c32[2];
    const float b = fmaf(d32[2], xz, fmaf(d32[1], xy, d32[0] * xx));
    const float q = fmaf(xz, xz, fmaf(xy, xy, xx * xx));
    const float g = fmaf(q, 1 - 0x1p-15f, -(r2e + kap));
    const float D = fmaf(b, b, -(a32 * g));
    const float y = -b - hi32, w = b + lo32;
    const float z = fmaxf(y, w);
    const float zz = z * fabsf(z);
    return !(fmaxf(zz, 0.f) > D);
}

static long viol32 = 0, rej32 = 0, tot32 = 0;
static int cur_fam = 0;
static long fam_tot[6], fam_rej64[6], fam_rej32[6];

static double lim_tmax(double tmax, double a) { return tmax * a * (1 + 0x1p-30); }
static double lim_tmin(double tmin, double a) { return tmin * a * (1 - 0x1p-30); }

static long viol = 0, acc = 0, rej = 0, total = 0, rej7 = 0, weaker = 0;

static void check(const double c[3], double r, const double o[3], const double d[3], double tmin, double tmax) {
    const double a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
    if (!(a >= 0x1p-500 && a <= 0x1p500)) return; /* the kernel takes the sequential exact path */
    const int e = exact(c, r, o, d, tmin, tmax);
    const int f = candidate(c, r, o, d, a, lim_tmin(tmin, a), lim_tmax(tmax, a));
    const int f7 = candidate_v7(c, r, o, d, a, lim_tmin(tmin, a), lim_tmax(tmax, a));
    if (f32_ray_ok(o, d, a) && f32_sphere_ok(c, r)) {
        const int g = candidate_f32(c, r, o, d, a, tmin, tmax);
        ++tot32;
        rej32 += !g;
        fam_tot[cur_fam]++;
        fam_rej32[cur_fam] += !g;
        fam_rej64[cur_fam] += !f;
        if (e && !g) {
            if (viol32 < 10)
                printf("F32 VIOLATION c=(%a %a %a) r=%a o=(%a %a %a) d=(%a %a %a) tmin=%a tmax=%a\n", c[0], c[1], c[2],
                       r, o[0], o[1], o[2], d[0], d[1], d[2], tmin, tmax);
            ++viol32;
        }
    }
    rej7 += !f7;
    weaker += (!f7 && f);
    ++total;
    acc += e;
    rej += !f;
    if (e && !f) {
        if (viol < 10)
            printf("VIOLATION c=(%a %a %a) r=%a o=(%a %a %a) d=(%a %a %a) tmin=%a tmax=%a\n", c[0], c[1], c[2], r,
                   o[0], o[1], o[2], d[0], d[1], d[2], tmin, tmax);
        ++viol;
    }
}

static void rand_unit(double v[3]) {
    double m;
    do {
        v[0] = urange(-1, 1); v[1] = urange(-1, 1); v[2] = urange(-1, 1);
        m = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    } while (!(m < 1 && m > 1e-6));
    m = 1 / sqrt(m);
    v[0] *= m; v[1] *= m; v[2] *= m;
}

int main(int argc, char** argv) {
    const long n = (argc > 1 ? atol(argv[1]) : 5) * 1000000L;
    const double tmin = 0.00001;
    for (long i = 0; i < n; ++i) {
        const int fam = (int)(i % 6);
        cur_fam = fam;
        double c[3], o[3], d[3], r, tmax;
        const double scale = pow(10.0, urange(-3, 3));
        rand_unit(d);
        const double dl = pow(10.0, urange(-2, 2)); /* unnormalized directions */
        for (int k = 0; k < 3; ++k) d[k] *= dl;
        r = scale * pow(10.0, urange(-2, 0.5));
        for (int k = 0; k < 3; ++k) c[k] = urange(-20, 20) * scale;
        tmax = u01() < 0.3 ? INFINITY : urange(0, 50) * scale / dl;
        if (fam == 0) { /* random rays passing near the sphere */
            double p[3];
            rand_unit(p);
            const double miss = r * urange(0.5, 1.5);
            const double back = urange(-5, 30) * scale;
            for (int k = 0; k < 3; ++k) o[k] = c[k] + p[k] * miss - d[k] / dl * back;
        } else if (fam == 1) { /* leaving the sphere's surface (self intersection) */
            double n3[3];
            rand_unit(n3);
            for (int k = 0; k < 3; ++k) o[k] = c[k] + n3[k] * r;
            /* outgoing or grazing directions */
            const double dn = d[0] * n3[0] + d[1] * n3[1] + d[2] * n3[2];
            if (dn < 0 && u01() < 0.8)
                for (int k = 0; k < 3; ++k) d[k] -= 2 * dn * n3[k] * (u01() < 0.5 ? 1.0 : 0.999999);
        } else if (fam == 2) { /* near-tangent rays */
            double n3[3], t3[3];
            rand_unit(n3);
            /* tangent direction: d minus its component along n3 */
            const double dn = d[0] * n3[0] + d[1] * n3[1] + d[2] * n3[2];
            for (int k = 0; k < 3; ++k) t3[k] = d[k] - dn * n3[k];
            const double off = r * (1 + urange(-1e-9, 1e-9));
            const double back = urange(0, 20) * scale;
            for (int k = 0; k < 3; ++k) o[k] = c[k] + n3[k] * off - t3[k] * back / dl;
            for (int k = 0; k < 3; ++k) d[k] = t3[k];
        } else if (fam == 3) { /* rtow-like: ground sphere and small spheres, camera-ish origins */
            if (u01() < 0.5) { c[0] = 0; c[1] = -1000; c[2] = 0; r = 1000; }
            else { c[0] = urange(-11, 11); c[1] = 0.2; c[2] = urange(-11, 11); r = 0.2; }
            if (u01() < 0.5) { o[0] = 13; o[1] = 2; o[2] = 3; }
            else { o[0] = urange(-12, 12); o[1] = urange(0, 1e-9); o[2] = urange(-12, 12); }
            double t3[3] = {urange(-1, 1), urange(-0.3, 0.5), urange(-1, 1)};
            for (int k = 0; k < 3; ++k) d[k] = t3[k] * dl;
            tmax = u01() < 0.5 ? INFINITY : urange(0, 30) / dl;
        } else if (fam == 4) { /* wide exponent spreads */
            const double e1 = pow(2.0, urange(-200, 200)), e2 = pow(2.0, urange(-200, 200));
            for (int k = 0; k < 3; ++k) { c[k] = urange(-1, 1) * e1; o[k] = c[k] + urange(-1, 1) * e2; }
            r = fabs(urange(0, 2)) * e2;
            tmax = u01() < 0.5 ? INFINITY : urange(0, 4) * e2 / dl;
        } else { /* origin inside the sphere, near the surface */
            double n3[3];
            rand_unit(n3);
            const double f = 1 - pow(10.0, urange(-16, -1));
            for (int k = 0; k < 3; ++k) o[k] = c[k] + n3[k] * r * f;
        }
        check(c, r, o, d, tmin, tmax);
        /* the same ray with t_max just above / below the exact root */
        if (fam < 3) {
            const double a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
            double oc[3] = {o[0] - c[0], o[1] - c[1], o[2] - c[2]};
            double b = d[0] * oc[0] + d[1] * oc[1] + d[2] * oc[2];
            double cc = (oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2]) - r * r;
            double disc = b * b - a * cc;
            if (disc >= 0) {
                const double root = (-b - sqrt(disc)) / a;
                check(c, r, o, d, tmin, nextafter(root, INFINITY));
                check(c, r, o, d, tmin, nextafter(nextafter(root, INFINITY), INFINITY));
                const double root2 = (-b + sqrt(disc)) / a;
                check(c, r, o, d, tmin, nextafter(root2, INFINITY));
                check(c, r, o, d, nextafter(root2, -INFINITY), INFINITY);
                check(c, r, o, d, nextafter(root, -INFINITY), nextafter(root2, INFINITY));
            }
        }
    }
    printf("cases %ld  exact accepts %ld  filter rejects %ld (%.1f%%)  violations %ld\n", total, acc, rej,
           100.0 * rej / total, viol);
    printf("v7 filter rejects %ld; kept by this filter but rejected by v7: %ld\n", rej7, weaker);
    printf("f32 filter: cases %ld  rejects %ld (%.1f%%)  violations %ld\n", tot32, rej32, 100.0 * rej32 / (tot32 ? tot32 : 1),
           viol32);
    for (int k = 0; k < 6; ++k)
        printf("  family %d: %ld cases, f64 filter rejects %.1f%%, f32 filter %.1f%%\n", k, fam_tot[k],
               100.0 * fam_rej64[k] / (fam_tot[k] ? fam_tot[k] : 1), 100.0 * fam_rej32[k] / (fam_tot[k] ? fam_tot[k] : 1));
    return viol != 0 || viol32 != 0;
}
