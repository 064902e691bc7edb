// End-to-end run of the C++ drop-in API on the GPU, written as a src/main.cpp scene function
// would be: BASELINE config 1 built through Scene / Sphere / Lambertian, rendered by
// Camera::render(const Scene&) (camera.h:301-303: BVH + the per-sample loop, here crt_render on
// every visible GPU) and written by Image::send_as_ppm (image.h:38-56).
//   config1_e2e <seed> <out.ppm>
// The render's base seed is the first SeedSeqGenerator::next_seed() after set_seed(seed)
// (2483477 * seed + 2987434823 mod 2^32, rand_util.h:51-79), so tests/test_gpu_cpp_e2e.py can
// compare the PPM bytes with the reference's (tests/golden/ppm_cases.npz, oracle/_ref).
#include <cstdlib>
#include <memory>

#include "base/camera.h"
#include "base/scene.h"
#include "shapes/shapes.h"
#include "util/rand_util.h"

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    SeedSeqGenerator::get_instance().set_seed(static_cast<uint32_t>(std::strtoul(argv[1], nullptr, 10)));
    Scene world;
    world.add(std::make_shared<Sphere>(Point3D(0, -1000, 0), 1000, std::make_shared<Lambertian>(RGB::from_mag(0.5))));
    world.add(std::make_shared<Sphere>(Point3D(0, 1, 0), 1, std::make_shared<Lambertian>(RGB::from_mag(0.4, 0.2, 0.1))));
    Camera()
        .set_image_by_width_and_aspect_ratio(400, 16. / 9.)
        .set_vertical_fov(20)
        .set_camera_center(Point3D(13, 2, 3))
        .set_camera_lookat(Point3D(0, 0, 0))
        .set_samples_per_pixel(1)
        .set_max_depth(50)
        .set_background(RGB::from_mag(0.7, 0.8, 1))
        .render(world)
        .send_as_ppm(argv[2]);
    return 0;
}
