/*
 * crt_ppm.cpp — ASCII P3 writer, same bytes as crt::write_ppm
 * (src/core/crt_image_ppm.cpp:9-23): header "P3\nW H\nmax\n", then per pixel
 * "r g b\t" with clamp(static_cast<int>(c * max), 0, max) and '\n' per row.
 */
#include <cstdio>
#include <string>
#include <vector>

#include "crt_host.h"

namespace {

/* static_cast<int>(float) as x86-64 cvttss2si executes it (NaN / out of range → INT_MIN) */
inline int to_int_x86(float f) {
    if (f >= -2147483648.0f && f < 2147483648.0f) return (int)f;
    return (int)0x80000000;
}

inline void put_int(std::string &o, int v) {
    char buf[16];
    const int n = std::snprintf(buf, sizeof buf, "%d", v);
    o.append(buf, (size_t)n);
}

}  // namespace

extern "C" int crt_write_ppm(const char *path, const float *rgb, int32_t width, int32_t height,
                             int32_t max_color_component) {
    using crt_amd::set_error;
    if (!path || (!rgb && width * height > 0) || width < 0 || height < 0)
        return set_error(CRT_E_INVALID, "bad argument");
    std::FILE *f = std::fopen(path, "wb");
    if (!f) return set_error(CRT_E_IO, std::string("Could not open output file: ") + path);
    std::string row;
    row.reserve((size_t)width * 13 + 1);
    row = "P3\n";
    put_int(row, width);
    row += ' ';
    put_int(row, height);
    row += '\n';
    put_int(row, max_color_component);
    row += '\n';
    std::fwrite(row.data(), 1, row.size(), f);
    const float m = (float)max_color_component;
    for (int32_t y = 0; y < height; ++y) {
        row.clear();
        for (int32_t x = 0; x < width; ++x) {
            const float *p = rgb + 3 * ((size_t)y * width + x);
            for (int k = 0; k < 3; ++k) {
                int v = to_int_x86(p[k] * m);
                v = v < 0 ? 0 : (v > max_color_component ? max_color_component : v);
                put_int(row, v);
                row += k < 2 ? ' ' : '\t';
            }
        }
        row += '\n';
        std::fwrite(row.data(), 1, row.size(), f);
    }
    const bool ok = std::fclose(f) == 0;
    return ok ? CRT_OK : set_error(CRT_E_IO, std::string("write failed: ") + path);
}
