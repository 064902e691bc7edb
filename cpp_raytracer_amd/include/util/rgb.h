// Drop-in for the reference's util/rgb.h.
#ifndef RGB_H
#define RGB_H

#include <cmath>
#include <cstdlib>
#include <iostream>
#include <string>

#include "math/interval.h"
#include "util/rand_util.h"

inline double linear_to_gamma(double d, double gamma = 2) { return std::pow(d, 1 / gamma); }

class RGB {
    RGB(double r_, double g_, double b_) : r{r_}, g{g_}, b{b_} {}

public:
    double r, g, b;

    double luminance() const { return 0.2126 * r + 0.7152 * g + 0.0722 * b; }

    static RGB from_mag(double red, double green, double blue) { return RGB(red, green, blue); }
    static RGB from_mag(double v) { return from_mag(v, v, v); }
    static RGB from_rgb(double red, double green, double blue, double max_magnitude = 255) {
        return RGB(red / max_magnitude, green / max_magnitude, blue / max_magnitude);
    }
    static RGB from_rgb(double v, double max_magnitude = 255) { return from_rgb(v, v, v, max_magnitude); }
    static RGB zero() { return from_mag(0); }
    // The reference writes from_mag(rand, rand, rand); a g++ build evaluates those arguments right
    // to left, so the blue channel is drawn first. That order is made explicit here so scenes
    // match the reference whatever compiler builds them.
    static RGB random(double min = 0, double max = 1) {
        const double bb = rand_double(min, max);
        const double gg = rand_double(min, max);
        const double rr = rand_double(min, max);
        return from_mag(rr, gg, bb);
    }

    RGB& operator+=(const RGB& o) { r += o.r; g += o.g; b += o.b; return *this; }
    RGB& operator*=(double d) { r *= d; g *= d; b *= d; return *this; }
    RGB& operator/=(double d) { return *this *= (1 / d); }

    // Reinhard tone map (/(1 + L)), gamma, scale by max + 0.999999, truncate (rgb.h:90-113)
    std::string as_string(std::string delimiter = " ", std::string surrounding = "",
                          double max_magnitude = 255, double gamma = 2,
                          bool use_tone_mapping = true) const {
        double r2 = r, g2 = g, b2 = b;
        if (use_tone_mapping) {
            const double L = luminance();
            r2 /= 1 + L;
            g2 /= 1 + L;
            b2 /= 1 + L;
        }
        const double scale = max_magnitude + 0.999999;
        return (surrounding.empty() ? "" : std::string{surrounding[0]}) +
               std::to_string(static_cast<int>(scale * linear_to_gamma(r2, gamma))) + delimiter +
               std::to_string(static_cast<int>(scale * linear_to_gamma(g2, gamma))) + delimiter +
               std::to_string(static_cast<int>(scale * linear_to_gamma(b2, gamma))) +
               (surrounding.empty() ? "" : std::string{surrounding[1]});
    }
};

inline RGB operator+(const RGB& a, const RGB& b) { return RGB::from_mag(a.r + b.r, a.g + b.g, a.b + b.b); }
inline RGB operator*(const RGB& a, double d) { auto r = a; r *= d; return r; }
inline RGB operator*(double d, const RGB& a) { return a * d; }
inline RGB operator*(const RGB& a, const RGB& b) { return RGB::from_mag(a.r * b.r, a.g * b.g, a.b * b.b); }

inline RGB lerp(const RGB& a, const RGB& b, double d) {
    if (!Interval(0, 1).contains_inclusive(d)) {
        std::cout << "Error: In `lerp(" << a.as_string(", ", "()", 255, 1) << ", "
                  << b.as_string(", ", "()", 255, 1) << ", " << d << "), lerp proportion " << d
                  << " is not in the range [0, 1]." << std::endl;
        std::exit(-1);
    }
    return RGB::from_mag((1 - d) * a.r + d * b.r, (1 - d) * a.g + d * b.g, (1 - d) * a.b + d * b.b);
}

#endif
