// gather_rate.hip — what a scattered per-lane record read costs in the vector-memory
// path, by record shape (DESIGN.md §4 "what bounds the traversal").  The compact
// inner-node visit is three 16-B loads plus one 8-B load per lane, every lane its
// own line; this asks whether the path's rate is set by load instructions, by bytes,
// or by cache lines, which decides whether a smaller node format could pay.
//
// Every lane reads ITERS records at independent random 64-B-aligned slots of a table
// (no dependent chain: 8 waves per SIMD keep the path saturated), XOR-folds the words
// into one output word.  Shapes (16-B words unless noted):
//   n56  3 x 16 B + 1 x 8 B  (the compact node: boxes + child words)
//   w64  4 x 16 B            w48  3 x 16 B      w32  2 x 16 B     w16  1 x 16 B
//   d16  2 x 8 B             s16  4 x 4 B       q64  4 x 16 B, the four lanes of a quad
//                                                    reading ONE record (16 lines per load)
// Tables of 2 MiB (L2), 128 MiB (Infinity Cache) and 2 GiB (HBM).  Prints, per shape
// and table: G records/s, GB/s of record bytes, and CU cycles per wave-load.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/gather_rate tools/gather_rate.hip && tools/gather_rate
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

constexpr int kIters = 256;

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

template <int SHAPE>
__global__ __launch_bounds__(256) void gather(const uint4* __restrict__ tab, uint64_t n_slots, uint32_t* out) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    uint64_t key = mix(tid + 1);
    for (int it = 0; it < kIters; ++it) {
        key = key * 6364136223846793005ull + 1442695040888963407ull;
        uint64_t slot = (key >> 20) & (n_slots - 1);  // tables are powers of two
        if (SHAPE == 7) slot = __shfl(slot, threadIdx.x & ~3u);  // the quad's first lane's record
        const uint4* r = tab + slot * 4;                          // 64-B slot = 4 x uint4
        if (SHAPE == 0) {          // n56
            const uint4 a = r[0], b = r[1], c = r[2];
            const uint2 d = ((const uint2*)r)[6];
            acc ^= a.x ^ a.w ^ b.y ^ b.z ^ c.x ^ c.w ^ d.x ^ d.y;
        } else if (SHAPE == 1) {   // w64
            const uint4 a = r[0], b = r[1], c = r[2], d = r[3];
            acc ^= a.x ^ a.w ^ b.y ^ b.z ^ c.x ^ c.w ^ d.x ^ d.y;
        } else if (SHAPE == 2) {   // w48
            const uint4 a = r[0], b = r[1], c = r[2];
            acc ^= a.x ^ a.w ^ b.y ^ b.z ^ c.x ^ c.w;
        } else if (SHAPE == 3) {   // w32
            const uint4 a = r[0], b = r[1];
            acc ^= a.x ^ a.w ^ b.y ^ b.z;
        } else if (SHAPE == 4) {   // w16
            const uint4 a = r[0];
            acc ^= a.x ^ a.w ^ a.y;
        } else if (SHAPE == 5) {   // d16
            const uint2* q = (const uint2*)r;
            const uint2 a = q[0], b = q[1];
            asm volatile("" ::"v"(a.x), "v"(a.y));
            acc ^= a.x ^ b.y;
        } else if (SHAPE == 6) {   // s16
            const uint32_t* q = (const uint32_t*)r;
            const uint32_t a = q[0], b = q[1], c = q[2], d = q[3];
            asm volatile("" ::"v"(a), "v"(b), "v"(c));
            acc ^= a ^ b ^ c ^ d;
        } else {                   // q64: lane l of the quad reads word l of the quad's record
            const uint4 a = r[threadIdx.x & 3u];
            acc ^= a.x ^ a.w ^ a.y;
        }
    }
    if (acc == 0x12345678u) out[tid] = acc;  // keeps the loads
}

int main() {
    int dev = 0, cus = 0, clk_khz = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev));
    const uint64_t max_bytes = 2ull << 30;
    uint4* tab;
    uint32_t* out;
    CK(hipMalloc(&tab, max_bytes));
    CK(hipMemset(tab, 0x5a, max_bytes));
    const int blocks = cus * 8;  // 8 x 256 threads per CU = 8 waves per SIMD
    CK(hipMalloc(&out, (size_t)blocks * 256 * sizeof(uint32_t)));
    const char* names[] = {"n56", "w64", "w48", "w32", "w16", "d16", "s16", "q64"};
    const int bytes[] = {56, 64, 48, 32, 16, 16, 16, 16};
    const int loads[] = {4, 4, 3, 2, 1, 2, 4, 1};
    const uint64_t tables[] = {2ull << 20, 128ull << 20, 2ull << 30};
    const char* tnames[] = {"2MiB", "128MiB", "2GiB"};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("clock %.0f MHz (attribute), %d CUs, %d waves per SIMD, %d records per lane\n", clk_khz / 1e3, cus, 8,
           kIters);
    for (int t = 0; t < 3; ++t) {
        const uint64_t slots = tables[t] / 64;
        for (int s = 0; s < 8; ++s) {
            float best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                CK(hipEventRecord(e0, 0));
                switch (s) {
                    case 0: hipLaunchKernelGGL(gather<0>, dim3(blocks), dim3(256), 0, 0, tab, slots, out); break;
                    case 1: hipLaunchKernelGGL(gather<1>, dim3(blocks), dim3(256), 0, 0, tab, slots, out); break;
                    case 2: hipLaunchKernelGGL(gather<2>, dim3(blocks), dim3(256), 0, 0, tab, slots, out); break;
                    case 3: hipLaunchKernelGGL(gather<3>, dim3(blocks), dim3(256), 0, 0, tab, slots, out); break;
                    case 4: hipLaunchKernelGGL(gather<4>, dim3(blocks), dim3(256), 0, 0, tab, slots, out); break;
                    case 5: hipLaunchKernelGGL(gather<5>, dim3(blocks), dim3(256), 0, 0, tab, slots, out); break;
                    case 6: hipLaunchKernelGGL(gather<6>, dim3(blocks), dim3(256), 0, 0, tab, slots, out); break;
                    default: hipLaunchKernelGGL(gather<7>, dim3(blocks), dim3(256), 0, 0, tab, slots, out); break;
                }
                CK(hipGetLastError());
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            const double lanes = (double)blocks * 256, recs = lanes * kIters;
            const double wave_loads = recs / 64 * loads[s];
            const double cyc = best * 1e-3 * clk_khz * 1e3 * cus;  // CU cycles
            // q64: a record per quad, i.e. 16 records per wave-load
            const double recs_eff = s == 7 ? recs / 4 : recs;
            printf("%-7s %-4s %7.3f ms  %6.2f G records/s  %7.1f GB/s  %6.2f CU cycles per wave-load\n", tnames[t],
                   names[s], best, recs_eff / (best * 1e-3) / 1e9,
                   recs_eff * (s == 7 ? 64 : bytes[s]) / (best * 1e-3) / 1e9, cyc / wave_loads);
        }
    }
    return 0;
}
