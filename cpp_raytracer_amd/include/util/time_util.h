// Drop-in for the reference's util/time_util.h.
#ifndef TIME_UTIL_H
#define TIME_UTIL_H

#include <array>
#include <chrono>
#include <string>
#include <utility>

template <typename T>
auto seconds_diff(const std::chrono::time_point<T>& start, const std::chrono::time_point<T>& end) {
    return std::chrono::duration_cast<std::chrono::seconds>(end - start).count();
}

template <typename T>
auto ms_diff(const std::chrono::time_point<T>& start, const std::chrono::time_point<T>& end) {
    return std::chrono::duration_cast<std::chrono::milliseconds>(end - start).count();
}

inline std::string seconds_to_dhms(unsigned long long seconds) {
    static const std::array<std::pair<unsigned, const char*>, 4> units{
        {{86400, "d"}, {3600, "hr"}, {60, "min"}, {1, "s"}}};
    std::string out;
    for (const auto& [factor, name] : units) {
        if (seconds >= factor) {
            out += std::to_string(seconds / factor) + name + " ";
            seconds %= factor;
        }
    }
    if (out.empty()) return "0s";
    out.pop_back();
    return out;
}

#endif
