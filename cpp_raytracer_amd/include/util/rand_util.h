// Drop-in for the reference's util/rand_util.h: the same seed sequence and per-thread LCG
// (SeedSeqGenerator x <- 2483477x + 2987434823; rand_double x <- 1664525x + 1013904223 mapped to
// [min, max] by x / (2^32 - 2); rand_int via a thread_local mt19937), so scene code that draws
// random numbers builds the same scenes as with the reference.
#ifndef RAND_UTIL_H
#define RAND_UTIL_H

#include <cstdint>
#include <iostream>
#include <limits>
#include <mutex>
#include <optional>
#include <random>

class SeedSeqGenerator {
    std::optional<uint32_t> custom_seed;
    std::mutex mtx;
    SeedSeqGenerator() = default;

public:
    static SeedSeqGenerator& get_instance() {
        static SeedSeqGenerator instance;
        return instance;
    }
    SeedSeqGenerator(const SeedSeqGenerator&) = delete;
    SeedSeqGenerator& operator=(const SeedSeqGenerator&) = delete;
    SeedSeqGenerator(SeedSeqGenerator&&) = delete;
    SeedSeqGenerator& operator=(SeedSeqGenerator&&) = delete;

    uint32_t next_seed() {
        std::lock_guard<std::mutex> lock(mtx);
        if (!custom_seed) {
            custom_seed = std::random_device{}();
            std::cout << "SeedSeqGenerator: No random seed provided, using " << *custom_seed
                      << " (Use SeedSeqGenerator::get_instance().set_seed([custom seed]) "
                         "to set a custom seed)"
                      << std::endl;
        }
        custom_seed = static_cast<uint32_t>(2'483'477u * (*custom_seed) + 2'987'434'823u);
        return *custom_seed;
    }

    void set_seed(uint32_t seed) {
        std::cout << "SeedSeqGenerator: Using user-provided random seed " << seed << '\n'
                  << std::endl;
        custom_seed = seed;
    }
};

inline double rand_double(double min = 0, double max = 1) {
    thread_local uint32_t state = SeedSeqGenerator::get_instance().next_seed();
    state = 1'664'525u * state + 1'013'904'223u;
    constexpr double scale = 1 / static_cast<double>(std::numeric_limits<uint32_t>::max() - 1);
    return min + (max - min) * static_cast<double>(state) * scale;
}

inline int rand_int(int min = 0, int max = 1) {
    thread_local std::mt19937 generator{SeedSeqGenerator::get_instance().next_seed()};
    thread_local std::uniform_int_distribution<> dist;
    dist.param(std::uniform_int_distribution<>::param_type{min, max});
    return dist(generator);
}

#endif
