// Drop-in for the reference's base/scene.h.
#ifndef SCENE_H
#define SCENE_H

#include <iterator>
#include <memory>
#include <span>
#include <vector>

#include "base/hittable.h"

class Scene : public Hittable {
    std::vector<std::shared_ptr<Hittable>> objects;
    AABB aabb;

public:
    operator std::vector<std::shared_ptr<Hittable>>&() { return objects; }
    operator const std::vector<std::shared_ptr<Hittable>>&() const { return objects; }

    size_t size() const { return objects.size(); }
    void clear() { objects.clear(); }
    std::shared_ptr<Hittable>& operator[](size_t i) { return objects[i]; }
    const std::shared_ptr<Hittable>& operator[](size_t i) const { return objects[i]; }
    auto begin() { return objects.begin(); }
    auto begin() const { return objects.cbegin(); }
    auto end() { return objects.end(); }
    auto end() const { return objects.cend(); }

    void add(std::shared_ptr<Hittable> object) {
        aabb.merge_with(object->get_aabb());
        objects.push_back(std::move(object));
    }
    void add(const Scene& scene) {
        for (const auto& o : scene) add(o);
    }

    // linear closest hit (scene.h:59-75 of the reference); rendering a Scene never uses this: it
    // goes through the BVH on the GPU
    std::optional<hit_info> hit_by(const Ray3D& ray, const Interval& ray_times) const override {
        std::optional<hit_info> result;
        auto tmax = ray_times.max;
        for (const auto& o : objects) {
            if (auto cur = o->hit_by(ray, Interval(ray_times.min, tmax)); cur) {
                result = cur;
                tmax = cur->hit_time;
            }
        }
        return result;
    }

    AABB get_aabb() const override { return aabb; }

    std::vector<std::shared_ptr<Hittable>> get_primitive_components() const override {
        std::vector<std::shared_ptr<Hittable>> ret;
        for (const auto& o : objects) {
            if (auto parts = o->get_primitive_components(); !parts.empty())
                ret.insert(ret.end(), std::make_move_iterator(parts.begin()), std::make_move_iterator(parts.end()));
            else
                ret.push_back(o);
        }
        return ret;
    }

    void print_to(std::ostream& os) const override {
        os << "Scene with " << size() << " objects:\n";
        for (const auto& o : objects) {
            o->print_to(os);
            os << '\n';
        }
        os << std::flush;
    }

    Scene() = default;
    Scene(std::span<const std::shared_ptr<Hittable>> objs) {
        for (const auto& o : objs) add(o);
    }
};

#endif
