// exec_mask_rate.hip — does a gfx950 SIMD issue a wave64 f64 instruction faster
// when some of its 16-lane quarters are masked off?  If it did, lanes regrouped
// inside a wave by shading branch (contiguous quarters) would run divergent
// branches in fewer cycles.  Measures cycles per v_fma_f64 / v_add_f32 wave
// instruction with every SIMD loaded (8 waves per SIMD) under several exec masks.
//
//   hipcc -O3 --offload-arch=gfx950 tools/exec_mask_rate.hip -o tools/exec_mask_rate && tools/exec_mask_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int kIters = 8192;

template <bool F64>
__global__ __launch_bounds__(256) void masked(double* out, unsigned long long* cyc, unsigned long long lanes_mask,
                                              double seed) {
    const unsigned lane = threadIdx.x & 63u;
    double a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7;
    float f0 = (float)a0, f1 = f0 + 1, f2 = f0 + 2, f3 = f0 + 3, f4 = f0 + 4, f5 = f0 + 5, f6 = f0 + 6, f7 = f0 + 7;
    const double m = 1.0000001, c = 1e-9;
    __syncthreads();
    unsigned long long t = 0;
    if ((lanes_mask >> lane) & 1ull) {
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        for (int it = 0; it < kIters; ++it) {
            if (F64) {
#define D(X) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(X) : "v"(m), "v"(c));
                D(a0) D(a1) D(a2) D(a3) D(a4) D(a5) D(a6) D(a7)
            } else {
#define F(X) asm volatile("v_add_f32 %0, %0, %1" : "+v"(X) : "v"((float)m));
                F(f0) F(f1) F(f2) F(f3) F(f4) F(f5) F(f6) F(f7)
            }
        }
        t = __builtin_amdgcn_s_memtime() - t0;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + f0 + f1 + f2 + f3 + f4 + f5 +
                                                 f6 + f7;
    if ((threadIdx.x & 63u) == (unsigned)__builtin_ctzll(lanes_mask)) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t;
}

int main() {
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int waves_per_simd = 8, blocks = cus * waves_per_simd;  // 4 waves per block: one per SIMD
    double* out;
    unsigned long long* cyc;
    CK(hipMalloc(&out, (size_t)blocks * 256 * sizeof(double)));
    CK(hipMalloc(&cyc, (size_t)blocks * 4 * sizeof(unsigned long long)));
    unsigned long long* h = (unsigned long long*)malloc((size_t)blocks * 4 * sizeof(unsigned long long));
    const struct { const char* name; unsigned long long m; } masks[] = {
        {"all 64 lanes", ~0ull},
        {"lanes 0-31 (two quarters)", 0x00000000FFFFFFFFull},
        {"lanes 0-15 (one quarter)", 0x000000000000FFFFull},
        {"16 lanes spread (every 4th)", 0x1111111111111111ull},
        {"lanes 0-7", 0xFFull},
        {"one lane", 1ull},
    };
    for (int f64 = 1; f64 >= 0; --f64) {
        for (const auto& mk : masks) {
            for (int rep = 0; rep < 2; ++rep) {
                if (f64) hipLaunchKernelGGL(masked<true>, dim3(blocks), dim3(256), 0, 0, out, cyc, mk.m, 1.0);
                else hipLaunchKernelGGL(masked<false>, dim3(blocks), dim3(256), 0, 0, out, cyc, mk.m, 1.0);
                CK(hipGetLastError());
                CK(hipDeviceSynchronize());
            }
            CK(hipMemcpy(h, cyc, (size_t)blocks * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
            double s = 0;
            for (int i = 0; i < blocks * 4; ++i) s += (double)h[i];
            const double per_wave = s / (blocks * 4);
            // each SIMD runs waves_per_simd waves side by side: SIMD cycles per instruction
            const double cpi = per_wave / (kIters * 8.0) / waves_per_simd;
            printf("%-8s %-30s cycles per wave-instruction per SIMD %6.2f\n", f64 ? "v_fma_f64" : "v_add_f32", mk.name,
                   cpi);
        }
    }
    return 0;
}
