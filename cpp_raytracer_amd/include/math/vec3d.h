// Drop-in for the reference's math/vec3d.h (same operator semantics: a / d is a * (1 / d)).
#ifndef VEC3D_H
#define VEC3D_H

#include <cmath>
#include <iostream>
#include <optional>

#include "util/rand_util.h"

struct Vec3D {
    double x = 0, y = 0, z = 0;

    const double& operator[](size_t axis) const { return axis == 0 ? x : (axis == 1 ? y : z); }
    double& operator[](size_t axis) { return axis == 0 ? x : (axis == 1 ? y : z); }

    Vec3D operator-() const { return Vec3D{-x, -y, -z}; }
    Vec3D& operator+=(const Vec3D& r) { x += r.x; y += r.y; z += r.z; return *this; }
    Vec3D& operator-=(const Vec3D& r) { x -= r.x; y -= r.y; z -= r.z; return *this; }
    Vec3D& operator*=(double d) { x *= d; y *= d; z *= d; return *this; }
    Vec3D& operator/=(double d) { return *this *= (1 / d); }

    double mag() const { return std::sqrt(x * x + y * y + z * z); }
    double mag_squared() const { return x * x + y * y + z * z; }
    Vec3D unit_vector() const;
    bool near_zero(double eps = 1e-8) {
        return std::fabs(x) < eps && std::fabs(y) < eps && std::fabs(z) < eps;
    }

    static Vec3D zero() { return Vec3D{0, 0, 0}; }
    static Vec3D random(double min = 0, double max = 1) {
        return Vec3D{rand_double(min, max), rand_double(min, max), rand_double(min, max)};
    }
    static Vec3D random_unit_vector();
    static Vec3D random_vector_in_unit_disk() {
        Vec3D r;
        do {
            r = Vec3D{rand_double(-1, 1), rand_double(-1, 1), 0};
        } while (!(r.mag_squared() < 1));
        return r;
    }
    static Vec3D random_unit_vector_on_hemisphere(const Vec3D& surface_normal);
};

inline Vec3D operator+(const Vec3D& a, const Vec3D& b) { auto r = a; r += b; return r; }
inline Vec3D operator-(const Vec3D& a, const Vec3D& b) { auto r = a; r -= b; return r; }
inline Vec3D operator*(const Vec3D& a, double d) { auto r = a; r *= d; return r; }
inline Vec3D operator*(double d, const Vec3D& a) { return a * d; }
inline Vec3D operator/(const Vec3D& a, double d) { auto r = a; r /= d; return r; }
inline double dot(const Vec3D& a, const Vec3D& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline Vec3D cross(const Vec3D& a, const Vec3D& b) {
    return Vec3D{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline std::ostream& operator<<(std::ostream& os, const Vec3D& v) {
    return os << "(" << v.x << ", " << v.y << ", " << v.z << ")";
}

inline Vec3D Vec3D::unit_vector() const { return *this / this->mag(); }

inline Vec3D Vec3D::random_unit_vector() {
    Vec3D r;
    do {
        r = Vec3D::random(-1, 1);
    } while (!(r.mag_squared() < 1));
    return r.unit_vector();
}

inline Vec3D Vec3D::random_unit_vector_on_hemisphere(const Vec3D& n) {
    auto r = Vec3D::random_unit_vector();
    return dot(n, r) > 0 ? r : -r;
}

inline Vec3D reflected(const Vec3D& dir, const Vec3D& unit_normal) {
    return dir - 2 * dot(dir, unit_normal) * unit_normal;
}

inline std::optional<Vec3D> refracted(const Vec3D& unit_dir, const Vec3D& unit_normal,
                                      double ratio) {
    auto cos_theta = std::fmin(dot(-unit_dir, unit_normal), 1.);
    auto sin_theta = std::sqrt(1 - cos_theta * cos_theta);
    if (ratio * sin_theta > 1) return {};
    auto perp = ratio * (unit_dir + cos_theta * unit_normal);
    auto para = -std::sqrt(std::fabs(1 - perp.mag_squared())) * unit_normal;
    return perp + para;
}

using Point3D = Vec3D;

#endif
