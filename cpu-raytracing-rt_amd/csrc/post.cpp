// post.cpp — host output surface: ACES tonemap + gamma (postprocessing.rs:5-37)
// and the binary P6 PPM writer (ppm.rs:4-19), applied to the mean radiance
// that rt_render returns, exactly where main.rs:104 / :74 apply them.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
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

// The PPM byte of a tonemapped value a (main.rs:104 correct_gamma, then ppm.rs:13-15)
unsigned char gamma_byte(double a) { return to_byte(std::pow(a, 1.0 / 2.2)); }

double from_bits(uint64_t b) {
    double d;
    std::memcpy(&d, &b, 8);
    return d;
}
uint64_t to_bits(double d) {
    uint64_t b;
    std::memcpy(&b, &d, 8);
    return b;
}

}  // namespace

namespace rt {

// thr[k - 1] = the least double a >= 0 with gamma_byte(a) >= k, k = 1..255, so
// for every tonemapped value a (aces() is in [0, 1], -0 or NaN) the byte is the
// number of thresholds <= a — what the device epilogue computes by a binary
// search (post_dev.hip), with the host's own `pow` behind every threshold.
//
// Found by bisection over the bit patterns of [0, 1] (non-negative doubles
// order like their bits), then proven: the byte is a monotone function of v =
// pow(a, 1/2.2) (a product by 255 and round, both monotone), and glibc's pow is
// within 1 ulp of the monotone exact power, so the predicate "byte >= k" can
// disagree with "a >= thr" only where the exact power is within ~1 ulp of the
// byte boundary — a run of a few ulps of a around the bisection point.  Every
// double within kWin ulps on either side is checked, so the table is exact for
// all inputs or the function reports failure (the device then keeps its own
// pow: post_dev.hip).
bool byte_thresholds(double thr[255]) {
    constexpr uint64_t kWin = 512;
    const uint64_t one = to_bits(1.0);
    for (int k = 1; k <= 255; ++k) {
        uint64_t lo = 0, hi = one;  // gamma_byte(0) = 0 < k <= 255 = gamma_byte(1)
        while (hi - lo > 1) {
            const uint64_t mid = lo + (hi - lo) / 2;
            if (gamma_byte(from_bits(mid)) >= k) hi = mid;
            else lo = mid;
        }
        for (uint64_t i = 1; i <= kWin; ++i) {
            if (i <= hi && gamma_byte(from_bits(hi - i)) >= k) return false;
            if (hi + i - 1 <= one && gamma_byte(from_bits(hi + i - 1)) < k) return false;
        }
        thr[k - 1] = from_bits(hi);
        if (k > 1 && !(thr[k - 2] < thr[k - 1])) return false;
    }
    return true;
}

}  // namespace rt

extern "C" int rt_byte_thresholds(double* out) {
    if (!out) return rt::set_error(RT_ERR_INVALID, "out is NULL");
    if (!rt::byte_thresholds(out)) return rt::set_error(RT_ERR_UNSUPPORTED, "host pow: byte thresholds not provable");
    return RT_OK;
}

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
