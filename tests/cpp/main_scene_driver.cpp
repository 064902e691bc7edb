// Test driver: calls one scene function of the reference's src/main.cpp (compiled unchanged
// against cpp_raytracer_amd/include, with -Dmain=crt_reference_main) after an optional
// set_seed, with CRT_DUMP_SCENE set so Camera::render writes the flattened scene and exits.
#include <cstdlib>
#include <cstring>
#include <iostream>

#include "util/rand_util.h"

void rtow_final_image();
void rtow_final_lights_with_tone_mapping();
void millions_of_spheres();
void millions_of_spheres_with_lights();
void parallelogram_test();
void cornell_box_test(bool);
void raining_on_the_dance_floor();
void christmas_tree_made_of_spheres();

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    if (argc >= 3) SeedSeqGenerator::get_instance().set_seed(static_cast<uint32_t>(std::strtoul(argv[2], nullptr, 10)));
    const std::string n = argv[1];
    if (n == "rtow_final") rtow_final_image();
    else if (n == "rtow_final_lights") rtow_final_lights_with_tone_mapping();
    else if (n == "millions") millions_of_spheres();
    else if (n == "millions_lights") millions_of_spheres_with_lights();
    else if (n == "parallelograms") parallelogram_test();
    else if (n == "cornell") cornell_box_test(false);
    else if (n == "cornell_empty") cornell_box_test(true);
    else if (n == "dance_floor") raining_on_the_dance_floor();
    else if (n == "christmas_tree") christmas_tree_made_of_spheres();
    else return 2;
    return 3;  // render should have exited
}
