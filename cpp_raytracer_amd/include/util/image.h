// Drop-in for the reference's util/image.h: Image (row-major RGB pixels, P3 PPM writer/reader)
// and ImagePPMStream. Errors print and std::exit(-1), as the reference does.
#ifndef IMAGE_H
#define IMAGE_H

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "util/progressbar.h"
#include "util/rgb.h"

class Image {
    size_t w, h;
    std::vector<std::vector<RGB>> pixels;

    Image(size_t w_, size_t h_) : w{w_}, h{h_}, pixels(h_, std::vector<RGB>(w_, RGB::zero())) {}
    explicit Image(const std::vector<std::vector<RGB>>& p) : w{p[0].size()}, h{p.size()}, pixels{p} {}

public:
    size_t width() const { return w; }
    size_t height() const { return h; }
    std::vector<RGB>& operator[](size_t row) { return pixels[row]; }
    const std::vector<RGB>& operator[](size_t row) const { return pixels[row]; }
    double aspect_ratio() const { return static_cast<double>(w) / static_cast<double>(h); }

    void send_as_ppm(const std::string& destination) const {
        std::ofstream fout(destination);
        if (!fout.is_open()) {
            std::cout << "Error: In Image::print_as_ppm(), could not open the file \"" << destination
                      << "\"" << std::endl;
            std::exit(-1);
        }
        fout << "P3\n" << w << " " << h << "\n255\n";
        for (size_t row = 0; row < h; ++row)
            for (size_t col = 0; col < w; ++col) fout << pixels[row][col].as_string() << '\n';
        std::cout << "Image successfully saved to \"" << destination << "\"" << std::endl;
    }

    Image& outline_border() {
        for (size_t row = 0; row < h; ++row) pixels[row][0] = pixels[row][w - 1] = RGB::from_mag(1);
        for (size_t col = 1; col + 1 < w; ++col) pixels[0][col] = pixels[h - 1][col] = RGB::from_mag(1);
        return *this;
    }

    static Image with_dimensions(size_t width, size_t height) { return Image(width, height); }
    static Image with_width_and_aspect_ratio(size_t width, double aspect_ratio) {
        auto height = static_cast<size_t>(std::round(static_cast<double>(width) / aspect_ratio));
        return with_dimensions(width, std::max(size_t{1}, height));
    }
    static Image with_height_and_aspect_ratio(size_t height, double aspect_ratio) {
        auto width = static_cast<size_t>(std::round(static_cast<double>(height) * aspect_ratio));
        return with_dimensions(std::max(size_t{1}, width), height);
    }
    static Image from_data(const std::vector<std::vector<RGB>>& img) { return Image(img); }

    static Image from_ppm_file(const std::string& file_name) {
        auto die = [&](const std::string& msg) {
            std::cout << "Error: In Image::from_ppm_file(\"" << file_name << "\"), " << msg << std::endl;
            std::exit(-1);
        };
        std::ifstream fin(file_name);
        if (!fin.is_open()) {
            std::cout << "Error: In Image::from_ppm_file(), could not find/open the file \""
                      << file_name << "\"" << std::endl;
            std::exit(-1);
        }
        std::string first;
        std::getline(fin, first);
        if (first != "P3") die("first line of file was not \"P3\", but instead was " + first);
        size_t iw, ih;
        if (!(fin >> iw >> ih)) die("could not parse image width and height (two integers) on second line");
        int maxv;
        if (!(fin >> maxv)) die("could not parse RGB max magnitude (one integer)");
        std::vector<std::vector<RGB>> data(ih, std::vector<RGB>(iw, RGB::zero()));
        for (size_t row = 0; row < ih; ++row) {
            for (size_t col = 0; col < iw; ++col) {
                int r, g, b;
                if (!(fin >> r >> g >> b))
                    die("failed to parse color #" + std::to_string(row * iw + col + 1) +
                        " (three integers (r, g, b))");
                if (r < 0 || g < 0 || b < 0)
                    die("found negative RGB channel value; color #" + std::to_string(row * iw + col + 1));
                data[row][col] = RGB::from_rgb(r, g, b, maxv);
            }
        }
        return from_data(data);
    }
};

class ImagePPMStream {
    std::string file;
    std::ofstream fout;
    size_t w, h, curr_index;

    ImagePPMStream(const std::string& file_, size_t w_, size_t h_)
        : file{file_}, fout{file_}, w{w_}, h{h_}, curr_index{0} {
        fout << "P3\n" << w << " " << h << "\n255\n";
    }

public:
    size_t width() const { return w; }
    size_t height() const { return h; }
    size_t size() const { return w * h; }
    double aspect_ratio() const { return static_cast<double>(w) / static_cast<double>(h); }

    void set_file(const std::string& file_name) {
        fout.open(file_name);
        if (!fout.is_open()) {
            std::cout << "Error: In ImagePPMStream::set_file(), could not open the file \"" << file_name
                      << "\"" << std::endl;
            std::exit(-1);
        }
        if (curr_index > 0)
            std::cout << "Warning: In ImagePPMStream::set_file(\"" << file_name << "\"), original file \""
                      << file << "\" is left incomplete; " << curr_index << " out of " << w * h
                      << " pixels printed" << std::endl;
        file = file_name;
        curr_index = 0;
    }

    void add(const RGB& rgb) {
        if (curr_index == size()) {
            std::cout << "Error: Called ImagePPMStream::add() " << size() + 1 << " times for image"
                      << "of size " << size() << std::endl;
            std::exit(-1);
        }
        fout << rgb.as_string() << '\n';
        ++curr_index;
    }

    static ImagePPMStream with_dimensions(size_t width, size_t height, const std::string& file_name) {
        return ImagePPMStream(file_name, width, height);
    }
    static ImagePPMStream with_width_and_aspect_ratio(size_t width, double aspect, const std::string& f) {
        auto height = static_cast<size_t>(std::round(static_cast<double>(width) / aspect));
        return with_dimensions(width, std::max(size_t{1}, height), f);
    }
    static ImagePPMStream with_height_and_aspect_ratio(size_t height, double aspect, const std::string& f) {
        auto width = static_cast<size_t>(std::round(static_cast<double>(height) * aspect));
        return with_dimensions(std::max(size_t{1}, width), height, f);
    }

    ~ImagePPMStream() {
        if (curr_index == w * h)
            std::cout << "Image successfully saved to \"" << file << "\"" << std::endl;
        else
            std::cout << "Warning: ImagePPMStream to \"" << file << "\" incomplete; " << curr_index
                      << " out of (" << w << " * " << h << ") = " << w * h
                      << " RGB strings printed at time of destruction" << std::endl;
    }
};

#endif
