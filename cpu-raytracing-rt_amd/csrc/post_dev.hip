// post_dev.hip — device output surface: ACES tonemap + gamma (postprocessing.rs:5-37)
// and the PPM byte quantisation (ppm.rs:13-19), fused so the 8-byte-per-channel
// mean radiance never leaves the device.  The same IEEE
// operations in the same order as post.cpp; `pow` is the device libm's, whose
// rounding may differ from glibc's in the last ulp — which can move a byte only
// when 255*v lands on a .5 boundary (tests/test_gpu_post.py counts them).
#include <hip/hip_runtime.h>

#include "render.h"

namespace rt {
namespace {

__device__ __forceinline__ double aces_d(double x) {  // saturate((x*(a*x+b)) / (x*(c*x+d)+e))
    const double a = 2.51, b = 0.03, c = 2.43, d = 0.59, e = 0.14;
    double v = ((a * x + b) * x) / ((c * x + d) * x + e);
    if (v < 0.0) return 0.0;  // num_traits::clamp (NaN passes through)
    if (v > 1.0) return 1.0;
    return v;
}
__device__ __forceinline__ uint8_t to_byte_d(double v) {  // float_to_byte
    if (v < 0.0) v = 0.0;
    if (v > 1.0) v = 1.0;
    const double r = round(v * 255.0);  // half away from zero
    if (r != r) return 0;               // `as u8`: NaN -> 0
    return (uint8_t)r;
}
__device__ __forceinline__ uint8_t pixel_byte(double mean) {  // main.rs:104 then ppm.rs:13-15
    return to_byte_d(pow(aces_d(mean), 1.0 / 2.2));
}

__global__ void tonemap_bytes_kernel(const double* __restrict__ rgb, uint64_t n, uint8_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = pixel_byte(rgb[i]);
}

// unpack_kernel (render.hip) fused with the tonemap + byte packing: one pass
// from the gathered tiles to the PPM payload [H][W][3] u8.
__global__ void unpack_bytes_kernel(const double* __restrict__ g, uint8_t* __restrict__ bytes, uint32_t W,
                                    uint32_t H, uint32_t tiles_x, uint32_t world, uint32_t per_rank) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)W * H) return;
    const uint32_t x = (uint32_t)(i % W), y = (uint32_t)(i / W);
    const uint64_t tile = (uint64_t)(y / RT_TILE) * tiles_x + x / RT_TILE;
    const uint64_t rank = tile % world, slot = tile / world;
    const double* src = g + (((rank * per_rank + slot) * 256u) + (y % RT_TILE) * RT_TILE + (x % RT_TILE)) * 3;
    bytes[3 * i] = pixel_byte(src[0]);
    bytes[3 * i + 1] = pixel_byte(src[1]);
    bytes[3 * i + 2] = pixel_byte(src[2]);
}

}  // namespace

hipError_t launch_tonemap_bytes(const double* rgb, uint64_t n_values, uint8_t* out, hipStream_t st) {
    if (n_values == 0) return hipSuccess;
    hipLaunchKernelGGL(tonemap_bytes_kernel, dim3((unsigned)((n_values + 255) / 256)), dim3(256), 0, st, rgb,
                       n_values, out);
    return hipGetLastError();
}
hipError_t launch_unpack_bytes(const double* g, uint8_t* bytes, uint32_t W, uint32_t H, uint32_t tiles_x,
                               uint32_t world, uint32_t per_rank, hipStream_t st) {
    const uint64_t n = (uint64_t)W * H;
    hipLaunchKernelGGL(unpack_bytes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, g, bytes, W, H,
                       tiles_x, world, per_rank);
    return hipGetLastError();
}

}  // namespace rt
