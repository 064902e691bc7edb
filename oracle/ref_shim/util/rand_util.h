/* TEST INFRASTRUCTURE — oracle/_ref build only, never part of the product.
 *
 * Instrumentation shim placed AHEAD of /root/reference/include on the include path of the
 * oracle/_ref build, so the reference's quoted `#include "util/rand_util.h"` (math/vec3d.h:7,
 * util/rgb.h:6, base/material.h:7) resolves here. It keeps the reference RNG's semantics
 * (util/rand_util.h:40-127: SeedSeqGenerator's LCG x <- 2483477x + 2987434823, the per-thread
 * LCG x <- 1664525x + 1013904223 mapped to min + (max-min)*x*(1/(2^32-2)), rand_int through a
 * thread_local mt19937 seeded from the same sequence) and adds ONE hook:
 *   crt_oracle_set_state(x0)  — set this thread's LCG state, so the next draw is X1 of the
 *                               per-(pixel, sample) stream the GPU kernel uses.
 * Without the hook the behaviour equals the reference's; oracle/Makefile builds the driver once
 * with this shim and once with the reference's own rand_util.h and checks both agree.
 */
#ifndef RAND_UTIL_H
#define RAND_UTIL_H

#include <cstdint>
#include <iostream>
#include <limits>
#include <mutex>
#include <optional>
#include <random>

#define CRT_ORACLE_SHIM 1

class SeedSeqGenerator {
    std::optional<uint32_t> seed_;
    std::mutex mu_;
    SeedSeqGenerator() = default;

public:
    static SeedSeqGenerator& get_instance() {
        static SeedSeqGenerator g;
        return g;
    }
    SeedSeqGenerator(const SeedSeqGenerator&) = delete;
    SeedSeqGenerator& operator=(const SeedSeqGenerator&) = delete;

    uint32_t next_seed() {
        std::lock_guard<std::mutex> lk(mu_);
        if (!seed_) {
            seed_ = std::random_device{}();
            std::cout << "SeedSeqGenerator(shim): no seed set, using " << *seed_ << std::endl;
        }
        seed_ = static_cast<uint32_t>(2483477u * (*seed_) + 2987434823u);
        return *seed_;
    }

    void set_seed(uint32_t s) {
        std::cout << "SeedSeqGenerator(shim): seed " << s << std::endl;
        seed_ = s;
    }
};

namespace crt_shim {
inline thread_local bool have_state = false;
inline thread_local uint32_t state = 0;
}  // namespace crt_shim

inline void crt_oracle_set_state(uint32_t x0) {
    crt_shim::state = x0;
    crt_shim::have_state = true;
}

inline double rand_double(double min = 0, double max = 1) {
    if (!crt_shim::have_state) {
        crt_shim::state = SeedSeqGenerator::get_instance().next_seed();
        crt_shim::have_state = true;
    }
    crt_shim::state = 1664525u * crt_shim::state + 1013904223u;
    constexpr double scale = 1 / static_cast<double>(std::numeric_limits<uint32_t>::max() - 1);
    return min + (max - min) * static_cast<double>(crt_shim::state) * scale;
}

inline int rand_int(int min = 0, int max = 1) {
    thread_local std::mt19937 gen{SeedSeqGenerator::get_instance().next_seed()};
    thread_local std::uniform_int_distribution<> dist;
    dist.param(std::uniform_int_distribution<>::param_type{min, max});
    return dist(gen);
}

#endif
