// Drop-in for the reference's base/material.h. scatter/emit keep the reference's semantics for
// callers of the API; the GPU kernel implements the same four materials itself (crt_describe
// hands it their parameters). A user-defined Material has no GPU description and is rejected.
#ifndef MATERIAL_H
#define MATERIAL_H

#include <cmath>
#include <iostream>
#include <optional>

#include "base/hittable.h"
#include "math/ray3d.h"
#include "util/rand_util.h"
#include "util/rgb.h"

struct scatter_info {
    Ray3D ray;
    RGB attenuation;
    scatter_info(const Ray3D& r, const RGB& a) : ray{r}, attenuation{a} {}
};

struct Material {
    virtual std::optional<scatter_info> scatter(const Ray3D& ray, const hit_info& info) const = 0;
    virtual RGB emit() const { return RGB::zero(); }
    virtual void print_to(std::ostream& os) const = 0;
    virtual bool crt_describe(crt_material& /*m*/) const { return false; }
    virtual ~Material() = default;
};

inline std::ostream& operator<<(std::ostream& os, const Material& m) {
    m.print_to(os);
    return os;
}

inline crt_material crt_make_material(uint32_t kind, const RGB& c, double param) {
    crt_material m{};
    m.kind = kind;
    m.color[0] = c.r;
    m.color[1] = c.g;
    m.color[2] = c.b;
    m.param = param;
    return m;
}

class Lambertian : public Material {
    RGB intrinsic_color;

public:
    std::optional<scatter_info> scatter(const Ray3D&, const hit_info& info) const override {
        auto dir = info.unit_surface_normal + Vec3D::random_unit_vector();
        if (dir.near_zero()) dir = info.unit_surface_normal;
        return scatter_info(Ray3D{info.hit_point, dir}, intrinsic_color);
    }
    void print_to(std::ostream& os) const override {
        os << "Lambertian {color: " << intrinsic_color.as_string(", ", "()") << "} " << std::flush;
    }
    bool crt_describe(crt_material& m) const override {
        m = crt_make_material(CRT_LAMBERTIAN, intrinsic_color, 0);
        return true;
    }
    Lambertian(const RGB& c) : intrinsic_color{c} {}
};

class Metal : public Material {
    RGB intrinsic_color;
    double fuzz_factor;

public:
    std::optional<scatter_info> scatter(const Ray3D& ray, const hit_info& info) const override {
        auto r = reflected(ray.dir.unit_vector(), info.unit_surface_normal);
        auto dir = r + fuzz_factor * Vec3D::random_unit_vector();
        if (dot(info.unit_surface_normal, dir) < 0) return {};
        return scatter_info(Ray3D{info.hit_point, dir}, intrinsic_color);
    }
    void print_to(std::ostream& os) const override {
        os << "Metal {color: " << intrinsic_color.as_string(", ", "()") << ", fuzz factor: " << fuzz_factor
           << "} " << std::flush;
    }
    bool crt_describe(crt_material& m) const override {
        m = crt_make_material(CRT_METAL, intrinsic_color, fuzz_factor);
        return true;
    }
    Metal(const RGB& c, double fuzz = 0) : intrinsic_color{c}, fuzz_factor{std::fmin(fuzz, 1.)} {}
};

class Dielectric : public Material {
    double refr_index;

    static double reflectance(double cos_theta, double ratio) {
        auto r0 = (1 - ratio) / (1 + ratio);
        r0 *= r0;
        return r0 + (1 - r0) * std::pow(1 - cos_theta, 5);
    }

public:
    std::optional<scatter_info> scatter(const Ray3D& ray, const hit_info& info) const override {
        auto ratio = info.hit_from_outside ? 1. / refr_index : refr_index / 1.;
        auto u = ray.dir.unit_vector();
        auto dir = refracted(u, info.unit_surface_normal, ratio);
        if (!dir) {
            dir = reflected(u, info.unit_surface_normal);
        } else {
            auto cos_theta = std::fmin(dot(-u, info.unit_surface_normal), 1.);
            if (rand_double() < reflectance(cos_theta, ratio)) dir = reflected(u, info.unit_surface_normal);
        }
        return scatter_info(Ray3D{info.hit_point, *dir}, RGB::from_mag(1, 1, 1));
    }
    void print_to(std::ostream& os) const override {
        os << "Dielectric {refractive index: " << refr_index << "} " << std::flush;
    }
    bool crt_describe(crt_material& m) const override {
        m = crt_make_material(CRT_DIELECTRIC, RGB::zero(), refr_index);
        return true;
    }
    Dielectric(double ri) : refr_index{ri} {}
};

class DiffuseLight : public Material {
    RGB intrinsic_color;
    double intensity;

public:
    std::optional<scatter_info> scatter(const Ray3D&, const hit_info&) const override { return {}; }
    RGB emit() const override { return intensity * intrinsic_color; }
    void print_to(std::ostream& os) const override {
        os << "DiffuseLight {color: " << intrinsic_color.as_string(", ", "()") << ", intensity: " << intensity
           << "} " << std::flush;
    }
    bool crt_describe(crt_material& m) const override {
        m = crt_make_material(CRT_DIFFUSE_LIGHT, intrinsic_color, intensity);
        return true;
    }
    DiffuseLight(const RGB& c, double k) : intrinsic_color{c}, intensity{k} {}
};

#endif
