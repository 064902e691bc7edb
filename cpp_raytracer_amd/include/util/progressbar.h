// Drop-in for the reference's util/progressbar.h (same interface; prints a percentage line).
#ifndef PROGRESS_BAR_H
#define PROGRESS_BAR_H

#include <chrono>
#include <iostream>
#include <mutex>
#include <string>

#include "util/time_util.h"

template <bool DISABLE_PRINTING = false>
class ProgressBar {
    using Clock = std::chrono::steady_clock;
    size_t total, done = 0;
    unsigned last_percent = 0;
    std::string description;
    Clock::time_point start = Clock::now();
    std::mutex mtx;

public:
    explicit ProgressBar(size_t total_iterations, const std::string& task = "Progress",
                         unsigned /*downscale_factor*/ = 2)
        : total{total_iterations}, description{task} {
        if constexpr (!DISABLE_PRINTING) std::cout << description << std::endl;
    }

    void complete_iteration() {
        if constexpr (DISABLE_PRINTING) return;
        std::lock_guard<std::mutex> lock(mtx);
        ++done;
        unsigned pct = total ? static_cast<unsigned>(100 * done / total) : 100;
        if (pct >= last_percent + 10 || done == total) {
            last_percent = pct;
            std::cout << "  " << pct << "% (" << seconds_to_dhms(seconds_diff(start, Clock::now()))
                      << ")" << std::endl;
        }
        if (done == total)
            std::cout << description << ": Finished in "
                      << seconds_to_dhms(seconds_diff(start, Clock::now())) << '\n' << std::endl;
    }
};

#endif
