// Drop-in for the reference's base/hittable.h. Every built-in Hittable also describes itself in
// the C ABI's terms (crt_describe) so Camera::render can flatten a world for the GPU; a
// user-defined Hittable without a description is rejected loudly by the flattener.
#ifndef HITTABLE_AND_HIT_INFO_H
#define HITTABLE_AND_HIT_INFO_H

#include <cmath>
#include <iostream>
#include <limits>
#include <memory>
#include <optional>
#include <vector>

#include "../../../include/crt_render.h"
#include "acceleration/aabb.h"
#include "math/interval.h"
#include "math/ray3d.h"

class Material;

struct hit_info {
    double hit_time;
    Point3D hit_point;
    Vec3D unit_surface_normal;
    bool hit_from_outside = false;
    const Material* material;

    hit_info(double t, const Point3D& p, const Vec3D& outward_unit_normal, const Ray3D& ray,
             const std::shared_ptr<Material>& mat)
        : hit_time{t}, hit_point{p}, material{mat.get()} {
        set_face(outward_unit_normal, ray);
    }
    hit_info(double t, const Point3D& p, const Vec3D& outward_unit_normal, const Ray3D& ray,
             const Material* mat)
        : hit_time{t}, hit_point{p}, material{mat} {
        set_face(outward_unit_normal, ray);
    }

private:
    void set_face(const Vec3D& n, const Ray3D& ray) {
        if (dot(ray.dir, n) > 0) {
            unit_surface_normal = -n;
            hit_from_outside = false;
        } else {
            unit_surface_normal = n;
            hit_from_outside = true;
        }
    }
};

inline std::ostream& operator<<(std::ostream& os, const hit_info& h) {
    return os << "hit_info {\n\thit_time: " << h.hit_time << "\n\thit_point: " << h.hit_point
              << "\n\tsurface_normal: " << h.unit_surface_normal
              << "\n\thit_from_outside: " << h.hit_from_outside << "\n}\n";
}

struct Hittable {
    virtual std::optional<hit_info> hit_by(const Ray3D& ray, const Interval& ray_times) const = 0;
    virtual AABB get_aabb() const = 0;
    virtual std::vector<std::shared_ptr<Hittable>> get_primitive_components() const { return {}; }
    virtual void print_to(std::ostream& os) const = 0;
    // GPU description of an indivisible primitive: fills kind / v[] and the material pointer.
    virtual bool crt_describe(crt_object& /*obj*/, const Material*& /*mat*/) const { return false; }
    virtual ~Hittable() = default;
};

inline std::ostream& operator<<(std::ostream& os, const Hittable& h) {
    h.print_to(os);
    return os;
}

#endif
