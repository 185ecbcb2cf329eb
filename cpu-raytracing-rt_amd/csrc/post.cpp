// post.cpp — host output surface: ACES tonemap + gamma (postprocessing.rs:5-37)
// and the binary P6 PPM writer (ppm.rs:4-19), applied to the mean radiance
// that rt_render returns, exactly where main.rs:104 / :74 apply them.
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/rt_api.h"
#include "api_internal.h"

namespace {

double aces(double x) {  // saturate((x*(a*x+b)) / (x*(c*x+d)+e)), postprocessing.rs:9-28
    const double a = 2.51, b = 0.03, c = 2.43, d = 0.59, e = 0.14;
    double v = ((a * x + b) * x) / ((c * x + d) * x + e);
    if (v < 0.0) return 0.0;  // num_traits::clamp (NaN passes through)
    if (v > 1.0) return 1.0;
    return v;
}
unsigned char to_byte(double v) {  // float_to_byte (ppm.rs:13-15)
    if (v < 0.0) v = 0.0;
    if (v > 1.0) v = 1.0;
    double r = std::round(v * 255.0);  // round half away from zero
    if (r != r) return 0;              // `as u8` maps NaN to 0
    return (unsigned char)r;
}

}  // namespace

extern "C" void rt_tonemap_gamma(const double* in, uint64_t n, double* out) {
    if (!in || !out) return;
    for (uint64_t i = 0; i < 3 * n; ++i) out[i] = std::pow(aces(in[i]), 1.0 / 2.2);  // correct_gamma
}

extern "C" int rt_save_ppm(const char* path, uint32_t w, uint32_t h, const double* rgb) {
    if (!path || !rgb) return rt::set_error(RT_ERR_INVALID, "path/rgb is NULL");
    FILE* f = std::fopen(path, "wb");
    if (!f) return rt::set_error(RT_ERR_IO, std::string("cannot create ") + path);
    std::fprintf(f, "P6\n%u %u\n255\n", w, h);
    std::vector<unsigned char> bytes((size_t)w * h * 3);
    for (size_t i = 0; i < bytes.size(); ++i) bytes[i] = to_byte(rgb[i]);
    size_t wrote = std::fwrite(bytes.data(), 1, bytes.size(), f);
    int rc = std::fclose(f);
    if (wrote != bytes.size() || rc != 0) return rt::set_error(RT_ERR_IO, std::string("short write to ") + path);
    return RT_OK;
}
