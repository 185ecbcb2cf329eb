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
// would fall back to the device pow — ByteTable::exact == 0.)
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>

#include "api_internal.h"
#include "render.h"

namespace rt {

namespace {

// The 255 byte thresholds, passed BY VALUE as a kernel argument (2 KB of the
// kernarg segment): no per-device table, no synchronous upload, nothing that
// breaks stream capture.  Each workgroup stages them in LDS for its searches.
struct ByteTable {
    double thr[256];  // thresholds of bytes 1..255 (entry 255 unused)
    uint32_t exact;   // 0: the host proof failed, the device pow is used instead
};

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
__device__ __forceinline__ uint8_t pixel_byte(double mean, const double* thr, bool exact) {
    const double a = aces_d(mean);
    if (!exact) return to_byte_d(pow(a, 1.0 / 2.2));
    uint32_t k = 0;
#pragma unroll
    for (uint32_t step = 128; step; step >>= 1)
        if (k + step <= 255u && a >= thr[k + step - 1]) k += step;
    return (uint8_t)k;
}
// the table into LDS (blockDim.x == 256)
__device__ __forceinline__ void stage_table(double* s_thr, const ByteTable& T) {
    s_thr[threadIdx.x] = T.thr[threadIdx.x];
    __syncthreads();
}

__global__ __launch_bounds__(256) void tonemap_bytes_kernel(const double* __restrict__ rgb, uint64_t n,
                                                            uint8_t* __restrict__ out, ByteTable T) {
    __shared__ double s_thr[256];
    stage_table(s_thr, T);
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = pixel_byte(rgb[i], s_thr, T.exact != 0);
}

// unpack_kernel (render.hip) fused with the tonemap + byte packing: one pass
// from the gathered tiles to the PPM payload [H][W][3] u8.
__global__ __launch_bounds__(256) void unpack_bytes_kernel(const double* __restrict__ g, uint8_t* __restrict__ bytes,
                                                           uint32_t W, uint32_t H, uint32_t tiles_x, uint32_t world,
                                                           uint32_t per_rank, ByteTable T) {
    __shared__ double s_thr[256];
    stage_table(s_thr, T);
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)W * H) return;
    const uint32_t x = (uint32_t)(i % W), y = (uint32_t)(i / W);
    const uint64_t tile = (uint64_t)(y / RT_TILE) * tiles_x + x / RT_TILE;
    const uint64_t rank = tile % world, slot = tile / world;
    const double* src = g + (((rank * per_rank + slot) * 256u) + (y % RT_TILE) * RT_TILE + (x % RT_TILE)) * 3;
    const bool exact = T.exact != 0;
    bytes[3 * i] = pixel_byte(src[0], s_thr, exact);
    bytes[3 * i + 1] = pixel_byte(src[1], s_thr, exact);
    bytes[3 * i + 2] = pixel_byte(src[2], s_thr, exact);
}

// The threshold table, derived (and proven) on the host once per process.
const ByteTable& byte_table() {
    static std::once_flag once;
    static ByteTable T;
    std::call_once(once, [] {
        std::memset(&T, 0, sizeof(T));
        T.exact = byte_thresholds(T.thr) ? 1u : 0u;
    });
    return T;
}

}  // namespace

hipError_t launch_tonemap_bytes(const double* rgb, uint64_t n_values, uint8_t* out, hipStream_t st) {
    if (n_values == 0) return hipSuccess;
    hipLaunchKernelGGL(tonemap_bytes_kernel, dim3((unsigned)((n_values + 255) / 256)), dim3(256), 0, st, rgb,
                       n_values, out, byte_table());
    return hipGetLastError();
}
hipError_t launch_unpack_bytes(const double* g, uint8_t* bytes, uint32_t W, uint32_t H, uint32_t tiles_x,
                               uint32_t world, uint32_t per_rank, hipStream_t st) {
    const uint64_t n = (uint64_t)W * H;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(unpack_bytes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, g, bytes, W, H,
                       tiles_x, world, per_rank, byte_table());
    return hipGetLastError();
}

}  // namespace rt
