// Drop-in for the reference's math/ray3d.h.
#ifndef RAY3D_H
#define RAY3D_H

#include <iostream>

#include "math/vec3d.h"

struct Ray3D {
    Point3D origin{0, 0, 0};
    Vec3D dir{0, 0, 0};
    Point3D operator()(double t) const { return origin + t * dir; }
};

inline std::ostream& operator<<(std::ostream& os, const Ray3D& r) {
    return os << "Ray3D {origin: " << r.origin << ", dir: " << r.dir << "}";
}

#endif
