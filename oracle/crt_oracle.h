/* TEST INFRASTRUCTURE — the CPU oracle. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline may load it; the product (cpp_raytracer_amd/lib/libcrt_hip.so) never does.
 *
 * A plain-C restatement of the reference's render path (DeltaPavonis/cpp_raytracer):
 * Camera::init / random_ray_through_pixel / ray_color (camera.h), BVH build + BVH::hit_by
 * (bvh.h), Sphere / Parallelogram / Box (shapes/), the four materials (material.h), Vec3D
 * helpers (vec3d.h) and the LCG of rand_util.h — with the per-(pixel, sample) RNG seeding of
 * include/crt_render.h. Pinned against the reference itself: tests/test_oracle.py checks it
 * bit-for-bit against the golden vectors oracle/_ref produced from /root/reference.
 *
 * Data formats are those of include/crt_render.h.
 */
#ifndef CRT_ORACLE_H
#define CRT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/crt_render.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_stats {
    uint64_t samples, rays, nodes_visited, sphere_tests, parallelogram_tests;
} oracle_stats;

/* Camera::init (camera.h:87-157) */
int oracle_camera(const crt_camera_settings* s, crt_camera* out);

/* Scene::get_primitive_components + BVH(world, num_buckets, max_prims) (bvh.h:183-550).
 * nodes: capacity max_nodes; returns the node count in *num_nodes, prim order in order[]. */
int oracle_bvh(const crt_material* mats, size_t nm, const crt_object* objs, size_t no,
               uint32_t num_buckets, uint32_t max_prims, crt_bvh_node* nodes, size_t max_nodes,
               size_t* num_nodes, uint32_t* order, size_t max_prims_out, size_t* num_prims);

/* Per-sample-seeded render of rows [r0,r1) x cols [c0,c1) with `threads` OpenMP threads.
 * rgb: (r1-r0)*(c1-c0)*3; samples (nullable): per-sample radiance, (r1-r0)*(c1-c0)*spp*3. */
int oracle_render(const crt_material* mats, size_t nm, const crt_object* objs, size_t no,
                  const crt_camera_settings* s, uint32_t base_seed, int threads, uint32_t r0,
                  uint32_t r1, uint32_t c0, uint32_t c1, double* rgb, double* samples,
                  oracle_stats* stats);

/* BVH::hit_by for n rays {ox,oy,oz,dx,dy,dz}, interval (t_min, t_max). */
int oracle_hits(const crt_material* mats, size_t nm, const crt_object* objs, size_t no,
                const double* rays, size_t n, double t_min, double t_max, crt_hit* out);

uint32_t oracle_sample_seed(uint32_t base, uint32_t pixel, uint32_t sample);

/* The integers Image::send_as_ppm prints (image.h:38-56) for n RGB pixels: RGB::as_string
 * (rgb.h:99-115) with its defaults — Reinhard by luminance (rgb.h:27-29), gamma 2 via
 * std::pow(x, 1/2) (rgb.h:10-13), static_cast<int>(255.999999 * .) — as the x86-64 g++ build
 * computes them (cvttsd2si: NaN / out of range -> INT_MIN). out: 3n values. */
void oracle_ppm_values(const double* rgb, size_t n, int32_t* out);

#ifdef __cplusplus
}
#endif
#endif
