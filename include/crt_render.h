/*
 * crt_render.h — C ABI of the MI355X (gfx950) render path.
 *
 * This is the drop-in boundary for the reference's hot path
 *   Camera::render(const Scene&)            include/base/camera.h:301-303
 *   template<T> Camera::render(const T&)    include/base/camera.h:264-297
 *   BVH(world, 32, 12) build + BVH::hit_by  include/acceleration/bvh.h:183-550, 585-715
 * (paths relative to the reference repository DeltaPavonis/cpp_raytracer).
 *
 * Plain C types only: pointers, sizes, POD structs. No HIP or torch types in any signature;
 * streams are passed as `void*` (a hipStream_t, or NULL for the default stream).
 * Every function returns 0 on success and a negative CRT_E* code on failure; the message of the
 * last failure on the calling thread is available from crt_last_error().
 *
 * The C++ reference-compatible API (cpp_raytracer_amd/include/base/camera.h etc.) is built on
 * top of these entry points; INTEGRATION.md shows the bindings.
 */
#ifndef CRT_RENDER_H
#define CRT_RENDER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI versions:
 *   1  rounds 1-4.
 *   2  round 5: crt_scene_image added; crt_bvh_params.build_device = d + 1 now also sets the scene
 *      up on GPU d (its copy there lives as long as the scene; other devices peer-copy it, guard
 *      words zeroed) and leaves the host-side staging image empty. */
#define CRT_ABI_VERSION 2

/* ---- status codes ---------------------------------------------------------------------- */
#define CRT_OK 0
#define CRT_E_INVALID (-1)     /* bad argument / unsupported object                         */
#define CRT_E_HIP (-2)         /* a HIP runtime call failed (message names it)              */
#define CRT_E_NODEVICE (-3)    /* no gfx950 device visible, or device index out of range    */
#define CRT_E_NOT_UPLOADED (-4)/* scene not resident on the requested device               */
#define CRT_E_ALLOC (-5)       /* host or device allocation failed                          */

/* ---- scene description ----------------------------------------------------------------- */
/* Material kinds: base/material.h:58 (Lambertian), :105 (Metal), :164 (Dielectric),
 * :231 (DiffuseLight). */
enum {
    CRT_LAMBERTIAN = 1,    /* color = intrinsic colour                                       */
    CRT_METAL = 2,         /* color, param = fuzz AFTER the ctor's fmin(fuzz, 1) clamp (:150) */
    CRT_DIELECTRIC = 3,    /* param = refractive index                                       */
    CRT_DIFFUSE_LIGHT = 4  /* color, param = intensity                                       */
};

/* Object kinds: shapes/sphere.h:12, shapes/parallelogram.h:133, shapes/box.h:432. */
enum {
    CRT_SPHERE = 1,        /* v[0..2] centre, v[3] radius                                    */
    CRT_PARALLELOGRAM = 2, /* v[0..2] vertex, v[3..5] side1, v[6..8] side2                  */
    CRT_BOX = 3            /* v[0..2] vertex, v[3..5] opposite vertex (6 faces, box.h:53-84) */
};

typedef struct crt_material {
    uint32_t kind;
    uint32_t reserved;
    double color[3];
    double param;
} crt_material; /* 40 bytes */

typedef struct crt_object {
    uint32_t kind;
    uint32_t material; /* index into the material array */
    double v[9];
} crt_object; /* 80 bytes */

/* BVH build knobs, BVH(world, num_buckets = 32, max_primitives_in_node = 12) bvh.h:754-756.
 * linear != 0 builds a single always-entered leaf in object order: the semantics of rendering a
 * non-BVH Hittable (Scene::hit_by scene.h:59-75 / Box::hit_by box.h:24-28). */
typedef struct crt_bvh_params {
    uint32_t num_buckets;
    uint32_t max_prims_in_node;
    uint32_t linear;
    uint32_t build_device;  /* 0: build on the host; d + 1: build on GPU d (the same tree), and
                             * set the scene up on GPU d: its copy there is in place after
                             * crt_scene_create (the same bytes the host staging uploads) */
} crt_bvh_params;

/* ---- camera ---------------------------------------------------------------------------- */
/* The Camera's user-set state (camera.h:16-82 members, set by the setters at :308-406).
 * Angles are RADIANS, exactly as the Camera stores them after its degree conversions. */
typedef struct crt_camera_settings {
    uint32_t image_w, image_h;
    uint32_t samples_per_pixel, max_depth;
    double center[3];
    double direction[3];
    double lookat[3];
    double up[3];
    double focus_dist;
    double fov;            /* vertical if fov_is_vertical, else horizontal; radians          */
    double defocus_angle;  /* radians                                                        */
    double background[3];
    uint32_t has_lookat;
    uint32_t has_focus_dist;
    uint32_t fov_is_vertical;
    uint32_t reserved;
} crt_camera_settings;

/* The camera after Camera::init() (camera.h:87-157): what the per-sample loop reads. */
typedef struct crt_camera {
    uint32_t image_w, image_h;
    uint32_t samples_per_pixel, max_depth;
    double origin[3];
    double pixel00[3];
    double pixel_delta_x[3];
    double pixel_delta_y[3];
    double defocus_disk_x[3];
    double defocus_disk_y[3];
    double defocus_angle;
    double background[3];
    double t_min;          /* Interval::with_min(0.00001), camera.h:217                      */
    uint32_t base_seed;    /* per-render seed of the per-sample RNG stream (crt_sample_seed)  */
    uint32_t reserved;
} crt_camera;

/* Rows owned by one device/rank: row r is rendered iff (r / row_block) % tile_count == tile_index.
 * {1,1,0,0} (or NULL) = the whole frame. flags: CRT_TILING_PACKED = the output buffer holds only
 * the owned rows, packed in order (owned row k at offset k * image_w * 3): a rank or device then
 * allocates its share of the frame, not the whole frame.
 * ABI change (round 4): this word was `reserved` before CRT_TILING_PACKED existed; any other bit
 * set is rejected with CRT_E_INVALID, so a caller that left it uninitialised must now zero it. */
#define CRT_TILING_PACKED 1u
typedef struct crt_tiling {
    uint32_t row_block;
    uint32_t tile_count;
    uint32_t tile_index;
    uint32_t flags;
} crt_tiling;

typedef struct crt_scene crt_scene; /* opaque: flattened primitives + BVH + device copies */

typedef struct crt_scene_info {
    uint64_t num_objects, num_materials, num_primitives, num_spheres, num_parallelograms;
    uint64_t num_nodes;
    uint32_t depth;          /* levels in the BVH (root = 1)                                 */
    uint32_t max_leaf_size;
    uint64_t device_bytes;   /* bytes of one device copy                                     */
    double build_ms;         /* host BVH build time                                          */
} crt_scene_info;

/* A LinearBVHNode (bvh.h:117-161) as exported for parity checks. */
typedef struct crt_bvh_node {
    double bounds[6];        /* x.min x.max y.min y.max z.min z.max                          */
    uint32_t index;          /* first primitive (leaf) / second child (interior)             */
    uint32_t count;          /* primitives in leaf, 0 for interior                           */
    uint32_t axis;           /* split axis of an interior node                               */
    uint32_t flags;          /* bit0: always entered (linear leaf)                           */
} crt_bvh_node;

/* Closest hit of one ray (the hit_info of hittable.h:20-72 that BVH::hit_by returns). */
typedef struct crt_hit {
    double t;
    double point[3];
    double normal[3];        /* faces the ray (front-face flip applied)                      */
    int32_t prim;            /* flattened primitive index (Scene::get_primitive_components), -1 = miss */
    int32_t front_face;      /* hit_from_outside                                             */
    uint32_t material;
    uint32_t reserved;
} crt_hit;

/* Work counters of one render (instrumented pass): the algorithmic-byte basis of bench.py. */
typedef struct crt_render_stats {
    uint64_t samples;
    uint64_t rays;           /* ray segments traced (primary + scattered)                    */
    uint64_t nodes_visited;  /* BVH nodes whose AABB was tested                              */
    uint64_t sphere_tests;
    uint64_t parallelogram_tests;
    double kernel_ms;
    /* wave-time breakdown of the instrumented pass (sum over waves, 100 MHz ticks): interior
     * BVH walk, leaf primitive tests, shading + path regeneration, whole wave lifetime */
    uint64_t ticks_walk, ticks_leaf, ticks_shade, ticks_total;
    /* wave iterations of each phase: lane utilization = lane work / (iterations * 64) with lane
     * work = nodes_visited, sphere+parallelogram tests, rays respectively */
    uint64_t wave_iters_walk, wave_iters_leaf, wave_iters_shade;
    uint64_t ticks_tail;  /* summed per wave: ticks from its first idle lane to its end */
    /* node tests the f32 walk could not decide (decided in f64), and the wave iterations that
     * ran such a test */
    uint64_t slow_node_tests, wave_iters_slow;
    /* two-pass sphere leaves: exact tests of the filter's candidates, and the wave iterations
     * of that pass (sphere_tests counts the filter's tests) */
    uint64_t candidate_tests, wave_iters_candidates;
} crt_render_stats;

/* ---- entry points ---------------------------------------------------------------------- */
int crt_abi_version(void);
const char* crt_last_error(void);
/* The library's compile-time configuration ("arch=gfx950 CRT_BLOCK=256 ..."): the kernel build
 * switches documented in INTEGRATION.md. */
const char* crt_build_info(void);
int crt_device_count(int* count);
void crt_free(void* p);

/* Per-sample RNG seed: state X0 of the reference's LCG (rand_util.h:85-117) for one (pixel,
 * sample); the kernel then draws X1, X2, ... exactly as rand_double does. */
uint32_t crt_sample_seed(uint32_t base_seed, uint32_t pixel, uint32_t sample);

/* One reference-LCG draw: advances *state and returns min + (max-min)*X*(1/(2^32-2)). */
double crt_rand_double(uint32_t* state, double min, double max);

/* Scenes of the reference's src/main.cpp, built with the reference's RNG semantics
 * (SeedSeqGenerator + LCG, evaluation order of a g++ build). has_seed = 0 keeps the scene
 * function's own seeding (rtow_final_image never seeds; such a call is rejected).
 * Arrays are malloc'd; release with crt_free. cam receives the scene's camera settings. */
int crt_scene_build_named(const char* name, uint32_t seed, int has_seed,
                          crt_material** materials, size_t* num_materials,
                          crt_object** objects, size_t* num_objects,
                          crt_camera_settings* cam);

/* Flatten (Scene::get_primitive_components, scene.h:85-106) and build the BVH (bvh.h:183-550)
 * on the host, or with params->build_device on that GPU, where the whole scene is then set up.
 * params may be NULL (= {32, 12, 0, 0}). */
int crt_scene_create(const crt_material* materials, size_t num_materials,
                     const crt_object* objects, size_t num_objects,
                     const crt_bvh_params* params, crt_scene** out);
int crt_scene_info_get(const crt_scene* scene, crt_scene_info* info);
/* nodes: num_nodes entries; prim_order: num_primitives entries (slot -> primitive index). */
int crt_scene_export_bvh(const crt_scene* scene, crt_bvh_node* nodes, uint32_t* prim_order);
/* Copy the scene into HBM of `device` (synchronous). Idempotent. */
int crt_scene_upload(crt_scene* scene, int device);
/* The scene's copy in HBM of `device` (uploaded first if needed) copied to host memory: bytes =
 * crt_scene_info.device_bytes. The layout is internal (tests and tooling compare copies). */
int crt_scene_image(crt_scene* scene, int device, void* host, size_t bytes);
void crt_scene_destroy(crt_scene* scene);

/* Camera::init() (camera.h:87-157). */
int crt_camera_resolve(const crt_camera_settings* settings, crt_camera* out);

/* Render the owned rows of the frame into d_rgb (DEVICE pointer on the scene's device,
 * image_h*image_w*3 doubles, row-major, the layout of Image::operator[] image.h:32-33; with
 * CRT_TILING_PACKED only owned_rows*image_w*3 doubles, the owned rows in order).
 * Enqueued on `stream`; returns without waiting. Rows not owned are left untouched.
 * Output is the per-pixel mean over samples_per_pixel samples (camera.h:285-292). */
int crt_render_async(const crt_scene* scene, int device, const crt_camera* cam,
                     const crt_tiling* tiling, double* d_rgb, void* stream);

/* Instrumented pass: counts the work of the same render (never timed). */
int crt_render_count(const crt_scene* scene, int device, const crt_camera* cam,
                     const crt_tiling* tiling, crt_render_stats* stats);

/* Blocking whole-frame render over devices [0, num_devices): rows are dealt to devices in
 * blocks of 4 (crt_tiling{4, num_devices, d}), rendered concurrently, and gathered into HOST
 * memory h_rgb. */
int crt_render(crt_scene* scene, const crt_camera* cam, int num_devices, double* h_rgb,
               crt_render_stats* stats);

/* crt_render fused with Image::send_as_ppm's integers (image.h:38-56; RGB::as_string
 * rgb.h:99-115, the values crt_ppm_values gives): every device tone-maps its own rows to 8-bit
 * values before the gather, so 3 bytes a pixel cross xGMI and PCIe instead of 24. h_values: host,
 * image_w*image_h*3 int32, identical to crt_ppm_values of crt_render's frame. */
int crt_render_ppm(crt_scene* scene, const crt_camera* cam, int num_devices, int32_t* h_values,
                   crt_render_stats* stats);

/* Closest hits of n rays (host arrays; rays[i] = {ox,oy,oz,dx,dy,dz}) against the scene on
 * `device`, time interval (t_min, t_max) exclusive, as BVH::hit_by (bvh.h:585-715). */
int crt_closest_hits(crt_scene* scene, int device, const double* rays, size_t n,
                     double t_min, double t_max, crt_hit* out);

/* The integers Image::send_as_ppm prints (image.h:38-56; RGB::as_string rgb.h:99-115 with its
 * defaults: Reinhard tone map by luminance, gamma 2, static_cast<int>(255.999999 * v)) for the
 * n-pixel frame d_rgb (device memory on `device`, row-major RGB f64, e.g. crt_render_async's
 * output), computed on the GPU; h_values (host, 3n int32) receives them, identical to the
 * x86-64 reference build's (NaN / out of range -> INT_MIN). Synchronous on `stream`. */
int crt_ppm_values(int device, const double* d_rgb, size_t n, int32_t* h_values, void* stream);

/* Writes w x h pixel values (3 per pixel) as Image::send_as_ppm does: "P3\nw h\n255\n", then
 * one "r g b\n" line per pixel, rows top to bottom. */
int crt_ppm_write(const char* path, uint32_t w, uint32_t h, const int32_t* values);

/* Parity guard of the renders of `scene` on `device` since its upload (or the last reset):
 * *schlick_undecided = Dielectric reflect-or-refract decisions (material.h:199-210) whose branch
 * would differ for a pow(1 - cos, 5) one ulp away from the kernel's correctly rounded value
 * (cpp_raytracer_amd/csrc/crt_schlick.h). glibc's pow, which the reference calls, is within one
 * ulp but not correctly rounded, so a render during which this stays 0 took every such branch as
 * the reference does. Synchronizes the device; reset != 0 zeroes the count. */
int crt_render_guard(crt_scene* scene, int device, uint64_t* schlick_undecided, int reset);

#ifdef __cplusplus
}
#endif

#endif /* CRT_RENDER_H */
