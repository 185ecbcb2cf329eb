// fetch_calib.hip — calibrates rocprofv3's FETCH_SIZE / TCC_EA0_RDREQ* counters for
// the path kernel's memory access pattern (VERDICT r02 "calibrate the HBM claim").
//
// Each lane does ITERS dependent random record reads (the next index depends on
// the data just loaded, like a BVH descent), with the record shapes the
// traversal reads:
//   128 B  fat f64 node (rt_layout.h DevNode): 8 x 16-B loads, 128-B aligned
//    80 B  f64 triangle record (DevTri): 5 x 16-B loads, 80-B stride
//    64 B  compact node (DevNodeC): 4 x 16-B loads, 64-B aligned
//    36 B  compact triangle (kTriC f32): 3 x 12-B loads, 36-B stride
// over a table that fits the 256-MiB Infinity Cache (128 MiB) and one that does
// not (4 GiB).  The algorithmic byte count of every dispatch is exact
// (lanes x ITERS x record bytes); comparing it with the counters of the same
// dispatch gives the factor to apply to the path kernel's counters.
//   hipcc -O3 --offload-arch=gfx950 -o tools/fetch_calib tools/fetch_calib.hip
//   rocprofv3 --pmc FETCH_SIZE -- tools/fetch_calib   (one counter group per run)
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

struct W3 { uint32_t x, y, z; };

template <int RB>
__global__ __launch_bounds__(256) void gather(const uint8_t* __restrict__ buf, uint64_t n_rec, uint32_t iters,
                                              uint32_t* __restrict__ out) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t x = tid * 0x9E3779B97F4A7C15ull + 12345u;
    uint32_t acc = 0;
    for (uint32_t it = 0; it < iters; ++it) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        const uint64_t idx = ((x >> 20) ^ acc) % n_rec;  // depends on the last record: a dependent chain
        const uint8_t* p = buf + idx * RB;
        if constexpr (RB == 36) {
            const W3* q = (const W3*)p;
            const W3 a = q[0], b = q[1], c = q[2];
            acc ^= a.x ^ a.y ^ a.z ^ b.x ^ b.y ^ b.z ^ c.x ^ c.y ^ c.z;
        } else {
            const uint4* q = (const uint4*)p;
#pragma unroll
            for (int k = 0; k < RB / 16; ++k) {
                const uint4 w = q[k];
                acc ^= w.x ^ w.y ^ w.z ^ w.w;
            }
        }
        acc &= 0xFFu;  // keep the dependence, not the magnitude
    }
    out[tid] = acc;
}

template <int RB>
void run(const uint8_t* buf, uint64_t bytes, uint32_t* out, uint32_t blocks, uint32_t iters, const char* tag) {
    const uint64_t n_rec = bytes / RB;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int rep = 0; rep < 2; ++rep) {  // rep 0 warms the table's cache residency; rep 1 is the one to read
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(gather<RB>, dim3(blocks), dim3(256), 0, 0, buf, n_rec, iters, out);
        CK(hipGetLastError());
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, a, b));
        const double algo = (double)blocks * 256.0 * iters * RB;
        std::printf("{\"kernel\": \"gather<%d>\", \"table\": \"%s\", \"table_bytes\": %llu, \"rep\": %d, "
                    "\"record_bytes\": %d, \"reads\": %.0f, \"algo_bytes\": %.0f, \"ms\": %.4f, \"GBps\": %.1f}\n",
                    RB, tag, (unsigned long long)bytes, rep, RB, (double)blocks * 256.0 * iters, algo, ms,
                    algo / (ms * 1e-3) / 1e9);
        std::fflush(stdout);
    }
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

int main() {
    const uint64_t small = 128ull << 20, big = 4ull << 30;
    const uint32_t blocks = 4096, iters = 64;  // 1M lanes (16 waves per CU), 64 dependent reads each
    uint8_t *bs = nullptr, *bb = nullptr;
    uint32_t* out = nullptr;
    CK(hipMalloc(&bs, small));
    CK(hipMalloc(&bb, big));
    CK(hipMalloc(&out, (size_t)blocks * 256 * sizeof(uint32_t)));
    CK(hipMemset(bs, 0x5A, small));
    CK(hipMemset(bb, 0x5A, big));
    CK(hipDeviceSynchronize());
    const struct { const uint8_t* p; uint64_t n; const char* tag; } tables[2] = {{bs, small, "128MiB"},
                                                                                 {bb, big, "4GiB"}};
    for (const auto& t : tables) {
        run<128>(t.p, t.n, out, blocks, iters, t.tag);
        run<80>(t.p, t.n, out, blocks, iters, t.tag);
        run<64>(t.p, t.n, out, blocks, iters, t.tag);
        run<36>(t.p, t.n, out, blocks, iters, t.tag);
    }
    CK(hipFree(bs));
    CK(hipFree(bb));
    CK(hipFree(out));
    return 0;
}
