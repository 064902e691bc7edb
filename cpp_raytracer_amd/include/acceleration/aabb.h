// Drop-in for the reference's acceleration/aabb.h (used by the host-side BVH build and the
// Hittable::get_aabb interface; the GPU kernel has its own copy of the slab test).
#ifndef AABB_H
#define AABB_H

#include <array>
#include <initializer_list>
#include <iostream>
#include <utility>

#include "math/interval.h"
#include "math/ray3d.h"

class AABB {
    Interval x, y, z;
    AABB(const Interval& x_, const Interval& y_, const Interval& z_) : x{x_}, y{y_}, z{z_} {}

public:
    Interval& operator[](size_t axis) { return axis == 0 ? x : (axis == 1 ? y : z); }
    const Interval& operator[](size_t axis) const { return axis == 0 ? x : (axis == 1 ? y : z); }

    Point3D centroid() const { return Point3D{x.midpoint(), y.midpoint(), z.midpoint()}; }
    double surface_area() const { return 2 * (x.size() * x.size() + y.size() * y.size() + z.size() * z.size()); }
    double volume() const { return x.size() * y.size() * z.size(); }

    bool is_hit_by(const Ray3D& ray, Interval t) const {
        for (size_t a = 0; a < 3; ++a) {
            const Interval& s = (*this)[a];
            double inv = 1 / ray.dir[a];
            double t0 = (s.min - ray.origin[a]) * inv, t1 = (s.max - ray.origin[a]) * inv;
            if (inv < 0) std::swap(t0, t1);
            if (t0 > t.min) t.min = t0;
            if (t1 < t.max) t.max = t1;
            if (t.max <= t.min) return false;
        }
        return true;
    }

    bool is_hit_by_optimized(const Ray3D& ray, const Interval& t, const Vec3D& inv,
                             const std::array<bool, 3>& neg) const {
        double xtmin = (x[neg[0]] - ray.origin.x) * inv.x, xtmax = (x[!neg[0]] - ray.origin.x) * inv.x;
        double ytmin = (y[neg[1]] - ray.origin.y) * inv.y, ytmax = (y[!neg[1]] - ray.origin.y) * inv.y;
        if (xtmin > ytmax || ytmin > xtmax) return false;
        if (ytmin > xtmin) xtmin = ytmin;
        if (ytmax < xtmax) xtmax = ytmax;
        double ztmin = (z[neg[2]] - ray.origin.z) * inv.z, ztmax = (z[!neg[2]] - ray.origin.z) * inv.z;
        if (xtmin > ztmax || ztmin > xtmax) return false;
        if (ztmin > xtmin) xtmin = ztmin;
        if (ztmax < xtmax) xtmax = ztmax;
        return (xtmin < t.max) && (xtmax > t.min);
    }

    AABB& merge_with(const AABB& o) { x.merge_with(o.x); y.merge_with(o.y); z.merge_with(o.z); return *this; }
    AABB& merge_with(const Point3D& p) { x.merge_with(p.x); y.merge_with(p.y); z.merge_with(p.z); return *this; }
    AABB& ensure_min_axis_length(double m) {
        if (x.size() < m) x.pad_with((m - x.size()) / 2);
        if (y.size() < m) y.pad_with((m - y.size()) / 2);
        if (z.size() < m) z.pad_with((m - z.size()) / 2);
        return *this;
    }

    AABB() : AABB(Interval::empty(), Interval::empty(), Interval::empty()) {}
    static AABB empty() { return AABB(); }
    static AABB from_axis_intervals(const Interval& a, const Interval& b, const Interval& c) { return AABB(a, b, c); }
    static AABB from_points(std::initializer_list<Point3D> pts) {
        AABB r;
        for (const auto& p : pts) r.merge_with(p);
        return r;
    }
    static AABB merge(const AABB& a, const AABB& b) {
        return AABB(Interval::merge(a.x, b.x), Interval::merge(a.y, b.y), Interval::merge(a.z, b.z));
    }
    friend std::ostream& operator<<(std::ostream& os, const AABB& b) {
        return os << "AABB {x: " << b.x << ", y: " << b.y << ", z: " << b.z << "} ";
    }
};

#endif
