// Drop-in for the reference's shapes/sphere.h.
#ifndef SPHERE_H
#define SPHERE_H

#include <iostream>
#include <memory>

#include "base/hittable.h"
#include "base/material.h"
#include "math/ray3d.h"
#include "math/vec3d.h"

struct Sphere : public Hittable {
    Point3D center;
    double radius;
    std::shared_ptr<Material> material;
    AABB aabb;

    std::optional<hit_info> hit_by(const Ray3D& ray, const Interval& t) const override {
        auto oc = ray.origin - center;
        auto a = dot(ray.dir, ray.dir);
        auto b = dot(ray.dir, oc);
        auto c = dot(oc, oc) - radius * radius;
        auto disc = b * b - a * c;
        if (disc < 0) return {};
        auto sq = std::sqrt(disc);
        auto root = (-b - sq) / a;
        if (!t.contains_exclusive(root)) {
            root = (-b + sq) / a;
            if (!t.contains_exclusive(root)) return {};
        }
        auto p = ray(root);
        return hit_info(root, p, (p - center) / radius, ray, material);
    }
    AABB get_aabb() const override { return aabb; }
    void print_to(std::ostream& os) const override {
        os << "Sphere {center: " << center << ", radius: " << radius << ", material: " << *material << "} "
           << std::flush;
    }
    bool crt_describe(crt_object& o, const Material*& m) const override {
        o = crt_object{};
        o.kind = CRT_SPHERE;
        o.v[0] = center.x; o.v[1] = center.y; o.v[2] = center.z; o.v[3] = radius;
        m = material.get();
        return true;
    }
    Sphere(const Point3D& c, double r, std::shared_ptr<Material> mat)
        : center{c}, radius{r}, material{std::move(mat)} {
        auto rv = Vec3D{r, r, r};
        aabb = AABB::from_points({center - rv, center + rv});
    }
};

#endif
