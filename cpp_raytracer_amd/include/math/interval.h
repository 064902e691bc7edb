// Drop-in for the reference's math/interval.h.
#ifndef INTERVAL_H
#define INTERVAL_H

#include <cmath>
#include <iostream>
#include <limits>
#include <numeric>

struct Interval {
    constexpr static double DOUBLE_INF = std::numeric_limits<double>::infinity();
    double min, max;

    const double& operator[](size_t index) const { return index ? max : min; }
    double midpoint() const { return std::midpoint(min, max); }
    double size() const { return max - min; }
    bool is_empty_inclusive() const { return size() < 0; }
    bool is_empty_exclusive() const { return size() <= 0; }
    bool contains_inclusive(double d) const { return min <= d && d <= max; }
    bool contains_exclusive(double d) const { return min < d && d < max; }
    double clamp(double d) const { return d <= min ? min : (d >= max ? max : d); }
    void merge_with(const Interval& o) { min = std::fmin(min, o.min); max = std::fmax(max, o.max); }
    void merge_with(double d) { min = std::fmin(min, d); max = std::fmax(max, d); }
    Interval& pad_with(double padding) {
        min -= padding;
        max += padding;
        return *this;
    }

    Interval(double min_, double max_) : min{min_}, max{max_} {}

    static Interval empty() { return Interval(DOUBLE_INF, -DOUBLE_INF); }
    static Interval nonnegative() { return Interval(0, DOUBLE_INF); }
    static Interval with_min(double m) { return Interval(m, DOUBLE_INF); }
    static Interval with_max(double m) { return Interval(-DOUBLE_INF, m); }
    static Interval universe() { return Interval(-DOUBLE_INF, DOUBLE_INF); }
    static Interval merge(const Interval& a, const Interval& b) {
        return Interval(std::fmin(a.min, b.min), std::fmax(a.max, b.max));
    }
};

inline std::ostream& operator<<(std::ostream& os, const Interval& i) {
    return os << "Interval {min: " << i.min << ", max: " << i.max << "} ";
}

#endif
