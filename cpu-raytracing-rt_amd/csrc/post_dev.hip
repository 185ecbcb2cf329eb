// post_dev.hip — device output surface: ACES tonemap + gamma (postprocessing.rs:5-37)
// and the PPM byte quantisation (ppm.rs:13-19), fused so the 8-byte-per-channel
// mean radiance never leaves the device.
//
// Bytes are the host path's bit for bit.  aces_tonemap is computed with the
// same IEEE operations in the same order as post.cpp (no contraction), so the
// tonemapped value a is the host's.  The rest — correct_gamma's pow(a, 1/2.2),
// the product by 255 and the rounding — is a monotone step function of a whose
// 255 steps the host derives from ITS pow and proves (post.cpp byte_thresholds):
// the device byte is a binary search of a over those thresholds, so no device
// libm rounding can move a byte.  (If the host proof ever failed, the kernels
// would fall back to the device pow — thr == nullptr.)
#include <hip/hip_runtime.h>

#include <mutex>

#include "api_internal.h"
#include "render.h"

namespace rt {

__device__ double g_byte_thr[256];  // thresholds of bytes 1..255 (entry 255 unused)

namespace {

__device__ __forceinline__ double aces_d(double x) {  // saturate((x*(a*x+b)) / (x*(c*x+d)+e))
    const double a = 2.51, b = 0.03, c = 2.43, d = 0.59, e = 0.14;
    double v = ((a * x + b) * x) / ((c * x + d) * x + e);
    if (v < 0.0) return 0.0;  // num_traits::clamp (NaN passes through)
    if (v > 1.0) return 1.0;
    return v;
}
__device__ __forceinline__ uint8_t to_byte_d(double v) {  // float_to_byte (fallback form)
    if (v < 0.0) v = 0.0;
    if (v > 1.0) v = 1.0;
    const double r = round(v * 255.0);  // half away from zero
    if (r != r) return 0;               // `as u8`: NaN -> 0
    return (uint8_t)r;
}
// main.rs:104 then ppm.rs:13-15: the number of thresholds <= a (NaN compares
// false everywhere: byte 0, as `NaN as u8`)
__device__ __forceinline__ uint8_t pixel_byte(double mean, const double* __restrict__ thr) {
    const double a = aces_d(mean);
    if (!thr) return to_byte_d(pow(a, 1.0 / 2.2));
    uint32_t k = 0;
#pragma unroll
    for (uint32_t step = 128; step; step >>= 1)
        if (k + step <= 255u && a >= thr[k + step - 1]) k += step;
    return (uint8_t)k;
}

__global__ void tonemap_bytes_kernel(const double* __restrict__ rgb, uint64_t n, uint8_t* __restrict__ out,
                                     const double* __restrict__ thr) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = pixel_byte(rgb[i], thr);
}

// unpack_kernel (render.hip) fused with the tonemap + byte packing: one pass
// from the gathered tiles to the PPM payload [H][W][3] u8.
__global__ void unpack_bytes_kernel(const double* __restrict__ g, uint8_t* __restrict__ bytes, uint32_t W,
                                    uint32_t H, uint32_t tiles_x, uint32_t world, uint32_t per_rank,
                                    const double* __restrict__ thr) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)W * H) return;
    const uint32_t x = (uint32_t)(i % W), y = (uint32_t)(i / W);
    const uint64_t tile = (uint64_t)(y / RT_TILE) * tiles_x + x / RT_TILE;
    const uint64_t rank = tile % world, slot = tile / world;
    const double* src = g + (((rank * per_rank + slot) * 256u) + (y % RT_TILE) * RT_TILE + (x % RT_TILE)) * 3;
    bytes[3 * i] = pixel_byte(src[0], thr);
    bytes[3 * i + 1] = pixel_byte(src[1], thr);
    bytes[3 * i + 2] = pixel_byte(src[2], thr);
}

// The threshold table on the current device: derived on the host once per
// process, uploaded once per device.  nullptr when the host proof failed.
hipError_t device_thresholds(const double** out) {
    static std::mutex mu;
    static int state = 0;  // 0 not derived, 1 exact, -1 proof failed
    static double thr[256];
    static bool uploaded[64];
    std::lock_guard<std::mutex> lock(mu);
    *out = nullptr;
    if (state == 0) state = byte_thresholds(thr) ? 1 : -1;
    if (state < 0) return hipSuccess;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    void* p = nullptr;
    e = hipGetSymbolAddress(&p, HIP_SYMBOL(g_byte_thr));
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64 || !uploaded[dev]) {
        e = hipMemcpy(p, thr, sizeof(thr), hipMemcpyHostToDevice);
        if (e != hipSuccess) return e;
        if (dev >= 0 && dev < 64) uploaded[dev] = true;
    }
    *out = (const double*)p;
    return hipSuccess;
}

}  // namespace

hipError_t launch_tonemap_bytes(const double* rgb, uint64_t n_values, uint8_t* out, hipStream_t st) {
    if (n_values == 0) return hipSuccess;
    const double* thr = nullptr;
    hipError_t e = device_thresholds(&thr);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(tonemap_bytes_kernel, dim3((unsigned)((n_values + 255) / 256)), dim3(256), 0, st, rgb,
                       n_values, out, thr);
    return hipGetLastError();
}
hipError_t launch_unpack_bytes(const double* g, uint8_t* bytes, uint32_t W, uint32_t H, uint32_t tiles_x,
                               uint32_t world, uint32_t per_rank, hipStream_t st) {
    const uint64_t n = (uint64_t)W * H;
    const double* thr = nullptr;
    hipError_t e = device_thresholds(&thr);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(unpack_bytes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, g, bytes, W, H,
                       tiles_x, world, per_rank, thr);
    return hipGetLastError();
}

}  // namespace rt
