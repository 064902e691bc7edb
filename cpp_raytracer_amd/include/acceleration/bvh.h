// Drop-in for the reference's acceleration/bvh.h. BVH(world, num_buckets, max_primitives_in_node)
// flattens the world (Scene::get_primitive_components) and builds the reference's binned-SAH BVH
// in libcrt_hip (crt_scene_create: identical node arrays, tests/test_host_abi.py); the node arrays
// then live in HBM for Camera::render. BVH::hit_by runs the same traversal on the GPU
// (crt_closest_hits). There is no CPU traversal.
#ifndef BVH_H
#define BVH_H

#include <chrono>
#include <cstdlib>
#include <iostream>
#include <memory>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "base/material.h"
#include "base/scene.h"
#include "util/time_util.h"

namespace crt_api {

[[noreturn]] inline void die(const std::string& what) {
    std::cout << "Error: " << what << ": " << crt_last_error() << std::endl;
    std::exit(-1);
}

// A world flattened for the C ABI, plus the material pointer of every material index.
struct Flat {
    std::vector<crt_material> materials;
    std::vector<crt_object> objects;
    std::vector<const Material*> material_ptrs;
    std::unordered_map<const Material*, uint32_t> index;

    void add_primitive(const Hittable& h) {
        crt_object o{};
        const Material* m = nullptr;
        if (!h.crt_describe(o, m)) {
            auto parts = h.get_primitive_components();
            if (parts.empty()) {
                std::cout << "Error: a Hittable type without a GPU description (only Sphere, "
                             "Parallelogram, Box and Scene render on the MI355X path)"
                          << std::endl;
                std::exit(-1);
            }
            for (const auto& p : parts) add_primitive(*p);
            return;
        }
        auto it = index.find(m);
        uint32_t mi;
        if (it == index.end()) {
            crt_material cm{};
            if (!m || !m->crt_describe(cm)) {
                std::cout << "Error: a Material type without a GPU description (only Lambertian, Metal, "
                             "Dielectric and DiffuseLight render on the MI355X path)"
                          << std::endl;
                std::exit(-1);
            }
            mi = static_cast<uint32_t>(materials.size());
            materials.push_back(cm);
            material_ptrs.push_back(m);
            index.emplace(m, mi);
        } else {
            mi = it->second;
        }
        o.material = mi;
        objects.push_back(o);
    }

    // the BVH is built over get_primitive_components() (bvh.h:757 of the reference)
    explicit Flat(const Hittable& world) {
        auto parts = world.get_primitive_components();
        if (parts.empty()) add_primitive(world);
        for (const auto& p : parts) add_primitive(*p);
    }
};

// Owns one crt_scene (host arrays + per-device HBM copies).
class GpuScene {
    crt_scene* s = nullptr;

public:
    std::vector<const Material*> materials;
    std::vector<crt_material> material_records;  // the flattened world, as handed to the C ABI
    std::vector<crt_object> object_records;
    GpuScene(const Hittable& world, uint32_t num_buckets, uint32_t max_prims, bool linear) {
        Flat f(world);
        // the tree is the reference's either way; with a GPU visible it is built on device 0
        // (crt_bvh_params.build_device), above 100k primitives where that pays
        int ndev = 0;
        const uint32_t on_gpu = (!linear && f.objects.size() > 100000 && crt_device_count(&ndev) == 0 && ndev > 0) ? 1u : 0u;
        crt_bvh_params p{num_buckets, max_prims, linear ? 1u : 0u, on_gpu};
        if (crt_scene_create(f.materials.data(), f.materials.size(), f.objects.data(), f.objects.size(), &p, &s))
            die("crt_scene_create");
        materials = std::move(f.material_ptrs);
        material_records = std::move(f.materials);
        object_records = std::move(f.objects);
    }
    ~GpuScene() { crt_scene_destroy(s); }
    GpuScene(const GpuScene&) = delete;
    GpuScene& operator=(const GpuScene&) = delete;
    crt_scene* get() const { return s; }
    crt_scene_info info() const {
        crt_scene_info i{};
        crt_scene_info_get(s, &i);
        return i;
    }
};

}  // namespace crt_api

class BVH : public Hittable {
    std::shared_ptr<crt_api::GpuScene> scene;
    AABB bounds;
    size_t num_objects;

public:
    template <typename T>
    requires std::is_base_of_v<Hittable, T>
    BVH(const T& world, size_t num_buckets = 32, size_t max_primitives_in_node = 12) {
        if constexpr (requires { world.size(); }) num_objects = world.size();
        else num_objects = 1;
        auto start = std::chrono::steady_clock::now();
        scene = std::make_shared<crt_api::GpuScene>(world, static_cast<uint32_t>(num_buckets),
                                                     static_cast<uint32_t>(max_primitives_in_node), false);
        auto info = scene->info();
        std::cout << "Building BVH over " << num_objects << " objects (" << info.num_primitives
                  << " primitives)..." << std::endl;
        std::cout << "Constructed BVH in " << ms_diff(start, std::chrono::steady_clock::now())
                  << "ms (created " << info.num_nodes << " BVHNodes total)\n" << std::endl;
        bounds = world.get_aabb();
    }

    const crt_api::GpuScene& gpu_scene() const { return *scene; }

    // BVH::hit_by (bvh.h:585-715) for one ray, on the GPU
    std::optional<hit_info> hit_by(const Ray3D& ray, const Interval& t) const override {
        double r[6] = {ray.origin.x, ray.origin.y, ray.origin.z, ray.dir.x, ray.dir.y, ray.dir.z};
        crt_hit h{};
        if (crt_closest_hits(scene->get(), 0, r, 1, t.min, t.max, &h)) crt_api::die("crt_closest_hits");
        if (h.prim < 0) return {};
        hit_info info(h.t, Point3D{h.point[0], h.point[1], h.point[2]},
                      Vec3D{h.normal[0], h.normal[1], h.normal[2]}, ray, scene->materials[h.material]);
        // crt_hit.normal already faces the ray: restore the side flag the kernel reported
        info.hit_from_outside = h.front_face != 0;
        info.unit_surface_normal = Vec3D{h.normal[0], h.normal[1], h.normal[2]};
        return info;
    }

    AABB get_aabb() const override { return bounds; }

    void print_to(std::ostream& os) const override {
        auto i = scene->info();
        os << "BVH {" << i.num_primitives << " primitives, " << i.num_nodes << " nodes, depth " << i.depth
           << "}" << std::flush;
    }
};

#endif
