// Primitive construction, shared by the host flattening (crt_host.cpp flatten) and the device
// scene set-up (crt_stage_gpu.hip): Scene::get_primitive_components (scene.h:85-106) with the
// ctors' derived data and get_aabb(). One definition for both sides, compiled with
// -ffp-contract=off on each, so a primitive staged on the device is bit-identical to the host's.
#pragma once

#include <cmath>
#include <cstdint>

#include "../../include/crt_render.h"

#ifndef CRT_HD
#define CRT_HD inline
#endif

namespace crt {
namespace prim {

// std::fmin / std::fmax as the reference's g++ build evaluates them: calls into glibc, whose
// x86-64 versions return the SECOND operand on a tie (so fmin(+0, -0) = -0) and the other operand
// when one is NaN. clang inlines them with the operands commuted, which differs on signed zeros,
// so the glibc semantics are spelled out.
CRT_HD double gfmin(double x, double y) {
    if (std::isnan(x)) return y;
    if (std::isnan(y)) return x;
    return x < y ? x : y;
}
CRT_HD double gfmax(double x, double y) {
    if (std::isnan(x)) return y;
    if (std::isnan(y)) return x;
    return x > y ? x : y;
}

// AABB::empty() then merge of each point (aabb.h, interval.h:45-54)
CRT_HD void box_empty(double b[6]) {
    for (int k = 0; k < 3; ++k) {
        b[2 * k] = INFINITY;
        b[2 * k + 1] = -INFINITY;
    }
}
CRT_HD void box_merge(double b[6], const double p[3]) {
    for (int k = 0; k < 3; ++k) {
        b[2 * k] = gfmin(b[2 * k], p[k]);
        b[2 * k + 1] = gfmax(b[2 * k + 1], p[k]);
    }
}

// Sphere (sphere.h:16-18, :112-122): centre, radius; AABB::from_points({c - rv, c + rv})
CRT_HD void sphere_prim(const double c[3], double r, double v[4], double box[6]) {
    const double lo[3] = {c[0] - r, c[1] - r, c[2] - r}, hi[3] = {c[0] + r, c[1] + r, c[2] + r};
    for (int k = 0; k < 3; ++k) v[k] = c[k];
    v[3] = r;
    box_empty(box);
    box_merge(box, lo);
    box_merge(box, hi);
}

// Parallelogram (parallelogram.h:269-296): v, s1, s2, the unit normal n / |n| and the scaled normal
// n / |n|^2 of n = s1 x s2 (vec3d.h:34 divides by multiplying with the reciprocal), the box of the
// four corners padded to ensure_min_axis_length(1e-4) (aabb.h:197-202).
CRT_HD void quad_prim(const double v[3], const double s1[3], const double s2[3], double out[15], double box[6]) {
    const double n[3] = {s1[1] * s2[2] - s1[2] * s2[1], s1[2] * s2[0] - s1[0] * s2[2], s1[0] * s2[1] - s1[1] * s2[0]};
    const double m2 = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];
    const double inv_mag = 1 / std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    const double inv_m2 = 1 / m2;
    for (int k = 0; k < 3; ++k) {
        out[k] = v[k];
        out[3 + k] = s1[k];
        out[6 + k] = s2[k];
        out[9 + k] = n[k] * inv_mag;
        out[12 + k] = n[k] * inv_m2;
    }
    const double a[3] = {v[0] + s1[0], v[1] + s1[1], v[2] + s1[2]};
    const double b[3] = {v[0] + s2[0], v[1] + s2[1], v[2] + s2[2]};
    const double ab[3] = {a[0] + s2[0], a[1] + s2[1], a[2] + s2[2]};
    box_empty(box);
    box_merge(box, v);
    box_merge(box, a);
    box_merge(box, b);
    box_merge(box, ab);
    const double m = 1e-4;
    for (int k = 0; k < 3; ++k) {
        const double size = box[2 * k + 1] - box[2 * k];
        if (size < m) {
            const double pad = (m - size) / 2;
            box[2 * k] -= pad;
            box[2 * k + 1] += pad;
        }
    }
}

// primitives an object flattens to: a Box is six parallelograms (box.h:53-84)
CRT_HD uint32_t object_prims(const crt_object& o) { return o.kind == CRT_BOX ? 6u : 1u; }

// Primitive j of object o: its kind (CRT_SPHERE / CRT_PARALLELOGRAM), its 15 doubles (sphere:
// c, r; parallelogram: v, s1, s2, unit n, scaled n; unused doubles zero) and its box.
// A Box's faces in box.h:64-84 order: min / max corners from fmin / fmax, sides along x, y, z.
CRT_HD uint32_t object_prim(const crt_object& o, uint32_t j, double out[15], double box[6]) {
    for (int k = 0; k < 15; ++k) out[k] = 0;
    if (o.kind == CRT_SPHERE) {
        sphere_prim(o.v, o.v[3], out, box);
        return CRT_SPHERE;
    }
    if (o.kind == CRT_PARALLELOGRAM) {
        quad_prim(o.v, o.v + 3, o.v + 6, out, box);
        return CRT_PARALLELOGRAM;
    }
    double mn[3], mx[3];
    for (int k = 0; k < 3; ++k) {
        mn[k] = gfmin(o.v[k], o.v[3 + k]);
        mx[k] = gfmax(o.v[k], o.v[3 + k]);
    }
    const double sx[3] = {mx[0] - mn[0], 0, 0}, sy[3] = {0, mx[1] - mn[1], 0}, sz[3] = {0, 0, mx[2] - mn[2]};
    const double nx[3] = {-sx[0], -sx[1], -sx[2]}, ny[3] = {-sy[0], -sy[1], -sy[2]}, nz[3] = {-sz[0], -sz[1], -sz[2]};
    switch (j) {
        case 0: quad_prim(mn, sx, sy, out, box); break;
        case 1: quad_prim(mn, sx, sz, out, box); break;
        case 2: quad_prim(mn, sy, sz, out, box); break;
        case 3: quad_prim(mx, nx, ny, out, box); break;
        case 4: quad_prim(mx, nx, nz, out, box); break;
        default: quad_prim(mx, ny, nz, out, box); break;
    }
    return CRT_PARALLELOGRAM;
}

}  // namespace prim
}  // namespace crt
