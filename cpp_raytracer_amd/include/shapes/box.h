// Drop-in for the reference's shapes/box.h: six Parallelogram faces (the BVH sees the faces).
#ifndef BOX_SURFACE_H
#define BOX_SURFACE_H

#include <array>
#include <cmath>

#include "base/hittable.h"
#include "base/scene.h"
#include "shapes/parallelogram.h"

class Box : public Hittable {
    Scene faces;
    std::shared_ptr<Material> material;

public:
    std::optional<hit_info> hit_by(const Ray3D& ray, const Interval& t) const override { return faces.hit_by(ray, t); }
    std::vector<std::shared_ptr<Hittable>> get_primitive_components() const override {
        return faces.get_primitive_components();
    }
    void print_to(std::ostream& os) const override { os << "Box {faces: " << faces << "} " << std::flush; }
    AABB get_aabb() const override { return faces.get_aabb(); }

    Box(const Point3D& a, const Point3D& b, std::shared_ptr<Material> mat) : material{std::move(mat)} {
        Point3D lo, hi;
        for (int i = 0; i < 3; ++i) {
            lo[i] = std::fmin(a[i], b[i]);
            hi[i] = std::fmax(a[i], b[i]);
        }
        auto sx = Vec3D{hi.x - lo.x, 0, 0}, sy = Vec3D{0, hi.y - lo.y, 0}, sz = Vec3D{0, 0, hi.z - lo.z};
        faces.add(std::make_shared<Parallelogram>(lo, sx, sy, material));
        faces.add(std::make_shared<Parallelogram>(lo, sx, sz, material));
        faces.add(std::make_shared<Parallelogram>(lo, sy, sz, material));
        faces.add(std::make_shared<Parallelogram>(hi, -sx, -sy, material));
        faces.add(std::make_shared<Parallelogram>(hi, -sx, -sz, material));
        faces.add(std::make_shared<Parallelogram>(hi, -sy, -sz, material));
    }
};

#endif
