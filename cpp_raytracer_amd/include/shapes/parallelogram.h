// Drop-in for the reference's shapes/parallelogram.h.
#ifndef PARALLELOGRAM_H
#define PARALLELOGRAM_H

#include <memory>

#include "base/hittable.h"
#include "base/material.h"
#include "math/vec3d.h"

class Parallelogram : public Hittable {
    Point3D vertex;
    Vec3D side1, side2;
    std::shared_ptr<Material> material;
    Vec3D unit_plane_normal, scaled_plane_normal;
    AABB aabb;

public:
    std::optional<hit_info> hit_by(const Ray3D& ray, const Interval& t) const override {
        auto den = dot(unit_plane_normal, ray.dir);
        if (std::fabs(den) < 1e-9) return {};
        auto ht = dot(unit_plane_normal, vertex - ray.origin) / den;
        if (!t.contains_exclusive(ht)) return {};
        auto p = ray(ht);
        auto w = p - vertex;
        auto alpha = dot(scaled_plane_normal, cross(w, side2));
        auto beta = dot(scaled_plane_normal, cross(side1, w));
        if (auto i = Interval(0, 1); i.contains_inclusive(alpha) && i.contains_inclusive(beta))
            return hit_info(ht, p, unit_plane_normal, ray, material);
        return {};
    }
    AABB get_aabb() const override { return aabb; }
    void print_to(std::ostream& os) const override {
        os << "Parallelogram {vertex: " << vertex << ", side 1 vector: " << side1
           << ", side 2 vector: " << side2 << " } " << std::flush;
    }
    bool crt_describe(crt_object& o, const Material*& m) const override {
        o = crt_object{};
        o.kind = CRT_PARALLELOGRAM;
        const Vec3D* v[3] = {&vertex, &side1, &side2};
        for (int i = 0; i < 3; ++i) {
            o.v[3 * i + 0] = v[i]->x;
            o.v[3 * i + 1] = v[i]->y;
            o.v[3 * i + 2] = v[i]->z;
        }
        m = material.get();
        return true;
    }
    Parallelogram(const Point3D& v, const Vec3D& s1, const Vec3D& s2, std::shared_ptr<Material> mat)
        : vertex{v}, side1{s1}, side2{s2}, material{std::move(mat)} {
        auto n = cross(side1, side2);
        unit_plane_normal = n.unit_vector();
        scaled_plane_normal = n / n.mag_squared();
        aabb = AABB::from_points({vertex, vertex + side1, vertex + side2, vertex + side1 + side2})
                   .ensure_min_axis_length(1e-4);
    }
};

#endif
