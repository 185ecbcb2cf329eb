// valu_rates.hip — issue cost of the VALU instruction classes the path kernel
// is made of, per wave64 instruction on one gfx950 SIMD, measured with every
// SIMD of the chip loaded (W waves per SIMD, 8 independent chains per lane).
// Used to turn the PMC instruction mix of path_kernel into a VALU-issue
// roofline (bench.py "roofline").
//
//   hipcc -O3 --offload-arch=gfx950 tools/valu_rates.hip -o tools/valu_rates && tools/valu_rates
//
// Output: one line per class: cycles per wave-instruction per SIMD (s_memtime
// shader cycles over the timed loop x waves on the SIMD / instructions per wave)
// and the effective clock (s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int kIters = 16384;  // loop trips; 8 instructions each

enum Op { FMA64, ADD64, MUL64, MAX64, RCP64, CMP64, FMA32, ADD32F, ADDU32, CNDMASK, MADU64, DIV64, SQRT64,
          LAT_FMA64, LAT_FMA32, LAT_RCP64,
          // round 4: the classes outside the f64 / int64 PMC counters ("other" in bench.py)
          MOV32, DPP, RFL, CVT64F32, CVT32F64, AND32, LSHL32, MULLO32, CMPU32, CMPCLS64, BFE32, ADDCO32,
          DIVSCALE64, DIVFMAS64, DIVFIXUP64, CNDMASK_VCC, XOR32, BITOP3, NOPS };
static const char* kName[NOPS] = {"v_fma_f64", "v_add_f64", "v_mul_f64", "v_max_f64", "v_rcp_f64",
                                  "v_cmp_lt_f64", "v_fma_f32", "v_add_f32", "v_add_u32", "v_cndmask_b32",
                                  "v_mad_u64_u32", "f64 x/y (compiled)", "f64 sqrt (compiled)",
                                  "dependent v_fma_f64", "dependent v_fma_f32", "dependent v_rcp_f64",
                                  "v_mov_b32", "v_mov_b32_dpp", "v_readfirstlane_b32", "v_cvt_f64_f32",
                                  "v_cvt_f32_f64", "v_and_b32", "v_lshlrev_b32", "v_mul_lo_u32", "v_cmp_gt_u32",
                                  "v_cmp_class_f64", "v_bfe_u32", "v_add_co_u32", "v_div_scale_f64",
                                  "v_div_fmas_f64", "v_div_fixup_f64", "v_cndmask_b32 (vcc)", "v_xor_b32",
                                  "v_bitop3_b32"};

#define R8(S) S S S S S S S S

template <int OP>
__global__ __launch_bounds__(256) void rate_kernel(double* out, unsigned long long* cyc, unsigned long long* rt,
                                                   double seed) {
    double a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7;
    const double m = 1.0000001, c = 1e-9;
    float f0 = (float)a0, f1 = f0 + 1, f2 = f0 + 2, f3 = f0 + 3, f4 = f0 + 4, f5 = f0 + 5, f6 = f0 + 6, f7 = f0 + 7;
    unsigned u0 = threadIdx.x, u1 = u0 + 1, u2 = u0 + 2, u3 = u0 + 3, u4 = u0 + 4, u5 = u0 + 5, u6 = u0 + 6,
             u7 = u0 + 7;
    const unsigned long long mask = __builtin_amdgcn_read_exec() & 0x5555555555555555ull;
    unsigned long long q0 = u0, q1 = u1, q2 = u2, q3 = u3, q4 = u4, q5 = u5, q6 = u6, q7 = u7;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < kIters; ++it) {
#define D8(INS) \
        asm volatile(INS : "+v"(a0) : "v"(m), "v"(c)); asm volatile(INS : "+v"(a1) : "v"(m), "v"(c)); \
        asm volatile(INS : "+v"(a2) : "v"(m), "v"(c)); asm volatile(INS : "+v"(a3) : "v"(m), "v"(c)); \
        asm volatile(INS : "+v"(a4) : "v"(m), "v"(c)); asm volatile(INS : "+v"(a5) : "v"(m), "v"(c)); \
        asm volatile(INS : "+v"(a6) : "v"(m), "v"(c)); asm volatile(INS : "+v"(a7) : "v"(m), "v"(c));
        if constexpr (OP == FMA64) { D8("v_fma_f64 %0, %0, %1, %2") }
#define L8(INS, X, ...) asm volatile(R8(INS "\n") : "+v"(X) : __VA_ARGS__);
        if constexpr (OP == LAT_FMA64) { L8("v_fma_f64 %0, %0, %1, %2", a0, "v"(m), "v"(c)) }
        if constexpr (OP == LAT_FMA32) { L8("v_fma_f32 %0, %0, %1, %1", f0, "v"((float)m)) }
        if constexpr (OP == LAT_RCP64) { L8("v_rcp_f64 %0, %0", a0, "v"(m)) }
        if constexpr (OP == ADD64) { D8("v_add_f64 %0, %0, %2") }
        if constexpr (OP == MUL64) { D8("v_mul_f64 %0, %0, %1") }
        if constexpr (OP == MAX64) { D8("v_max_f64 %0, %0, %2") }
        if constexpr (OP == RCP64) { D8("v_rcp_f64 %0, %0") }
        if constexpr (OP == CMP64) {
            // result to VCC then folded into a register so the chain stays live
            asm volatile(R8("v_cmp_lt_f64 vcc, %0, %1\n") : : "v"(a0), "v"(m) : "vcc");
        }
        if constexpr (OP == FMA32) {
#define F8(INS) \
            asm volatile(INS : "+v"(f0) : "v"((float)m)); asm volatile(INS : "+v"(f1) : "v"((float)m)); \
            asm volatile(INS : "+v"(f2) : "v"((float)m)); asm volatile(INS : "+v"(f3) : "v"((float)m)); \
            asm volatile(INS : "+v"(f4) : "v"((float)m)); asm volatile(INS : "+v"(f5) : "v"((float)m)); \
            asm volatile(INS : "+v"(f6) : "v"((float)m)); asm volatile(INS : "+v"(f7) : "v"((float)m));
            F8("v_fma_f32 %0, %0, %1, %1")
        }
        if constexpr (OP == ADD32F) { F8("v_add_f32 %0, %0, %1") }
        if constexpr (OP == ADDU32) {
#define U8(INS) \
            asm volatile(INS : "+v"(u0) : "v"(u7)); asm volatile(INS : "+v"(u1) : "v"(u7)); \
            asm volatile(INS : "+v"(u2) : "v"(u7)); asm volatile(INS : "+v"(u3) : "v"(u7)); \
            asm volatile(INS : "+v"(u4) : "v"(u0)); asm volatile(INS : "+v"(u5) : "v"(u0)); \
            asm volatile(INS : "+v"(u6) : "v"(u0)); asm volatile(INS : "+v"(u7) : "v"(u0));
            U8("v_add_u32 %0, %0, %1")
        }
        if constexpr (OP == CNDMASK) {
#define M8(INS) \
            asm volatile(INS : "+v"(u0) : "v"(u7), "s"(mask)); asm volatile(INS : "+v"(u1) : "v"(u7), "s"(mask)); \
            asm volatile(INS : "+v"(u2) : "v"(u7), "s"(mask)); asm volatile(INS : "+v"(u3) : "v"(u7), "s"(mask)); \
            asm volatile(INS : "+v"(u4) : "v"(u0), "s"(mask)); asm volatile(INS : "+v"(u5) : "v"(u0), "s"(mask)); \
            asm volatile(INS : "+v"(u6) : "v"(u0), "s"(mask)); asm volatile(INS : "+v"(u7) : "v"(u0), "s"(mask));
            M8("v_cndmask_b32_e64 %0, %0, %1, %2")
        }
        if constexpr (OP == MADU64) {
#define Q8(INS) \
            asm volatile(INS : "+v"(q0) : "v"(u1) : "vcc"); asm volatile(INS : "+v"(q1) : "v"(u1) : "vcc"); \
            asm volatile(INS : "+v"(q2) : "v"(u1) : "vcc"); asm volatile(INS : "+v"(q3) : "v"(u1) : "vcc"); \
            asm volatile(INS : "+v"(q4) : "v"(u1) : "vcc"); asm volatile(INS : "+v"(q5) : "v"(u1) : "vcc"); \
            asm volatile(INS : "+v"(q6) : "v"(u1) : "vcc"); asm volatile(INS : "+v"(q7) : "v"(u1) : "vcc");
            Q8("v_mad_u64_u32 %0, vcc, %1, %1, %0")
        }
        if constexpr (OP == MOV32) { U8("v_mov_b32 %0, %1") }
        if constexpr (OP == DPP) { U8("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf") }
        if constexpr (OP == RFL) {
            unsigned s0, s1, s2, s3, s4, s5, s6, s7;
            asm volatile(R8("v_readfirstlane_b32 %0, %8\n") "s_nop 0\n"
                         : "=s"(s0), "=s"(s1), "=s"(s2), "=s"(s3), "=s"(s4), "=s"(s5), "=s"(s6), "=s"(s7)
                         : "v"(u0));
            u0 += s0 ^ s7;
        }
        if constexpr (OP == CVT64F32) {
            asm volatile(R8("v_cvt_f64_f32 %0, %1\n") : "=v"(a0) : "v"(f0));
            a1 += a0;
        }
        if constexpr (OP == CVT32F64) {
            asm volatile(R8("v_cvt_f32_f64 %0, %1\n") : "=v"(f0) : "v"(a0));
            f1 += f0;
        }
        if constexpr (OP == AND32) { U8("v_and_b32 %0, %0, %1") }
        if constexpr (OP == LSHL32) { U8("v_lshlrev_b32 %0, 3, %1") }
        if constexpr (OP == MULLO32) { U8("v_mul_lo_u32 %0, %0, %1") }
        if constexpr (OP == CMPU32) { asm volatile(R8("v_cmp_gt_u32 vcc, %0, %1\n") : : "v"(u0), "v"(u1) : "vcc"); }
        if constexpr (OP == CMPCLS64) {
            asm volatile(R8("v_cmp_class_f64 vcc, %0, %1\n") : : "v"(a0), "v"(u1) : "vcc");
        }
        if constexpr (OP == BFE32) { U8("v_bfe_u32 %0, %0, 3, 7") }
        if constexpr (OP == XOR32) { U8("v_xor_b32 %0, %0, %1") }
        if constexpr (OP == BITOP3) { U8("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96") }
        if constexpr (OP == ADDCO32) {
            asm volatile(R8("v_add_co_u32 %0, vcc, %0, %1\n") : "+v"(u0) : "v"(u1) : "vcc");
        }
        if constexpr (OP == DIVSCALE64) { D8("v_div_scale_f64 %0, vcc, %1, %1, %0") }
        if constexpr (OP == DIVFMAS64) {
            asm volatile("s_mov_b64 vcc, 0" ::: "vcc");
            D8("v_div_fmas_f64 %0, %0, %1, %2")
        }
        if constexpr (OP == DIVFIXUP64) { D8("v_div_fixup_f64 %0, %0, %1, %2") }
        if constexpr (OP == CNDMASK_VCC) {
            asm volatile("s_mov_b64 vcc, %0" :: "s"(mask) : "vcc");
            U8("v_cndmask_b32 %0, %0, %1, vcc")
        }
        if constexpr (OP == DIV64) {
            a0 = m / a0; a1 = m / a1; a2 = m / a2; a3 = m / a3; a4 = m / a4; a5 = m / a5; a6 = m / a6; a7 = m / a7;
        }
        if constexpr (OP == SQRT64) {
            a0 = sqrt(a0 + c); a1 = sqrt(a1 + c); a2 = sqrt(a2 + c); a3 = sqrt(a3 + c);
            a4 = sqrt(a4 + c); a5 = sqrt(a5 + c); a6 = sqrt(a6 + c); a7 = sqrt(a7 + c);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    const double s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (double)(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7) +
                     (double)(u0 + u1 + u2 + u3 + u4 + u5 + u6 + u7) + (double)(q0 + q1 + q2 + q3 + q4 + q5 + q6 + q7);
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) {
        const unsigned w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        cyc[w] = t1 - t0;
        rt[w] = r1 - r0;
    }
}

static int cus = 0;
template <int OP>
static void run(int waves_per_simd, int /*unused*/) {
    const int blocks = cus * waves_per_simd;  // 256 threads = one wave per SIMD per block
    const int nw = blocks * 4;
    double* out; unsigned long long *cyc, *rt;
    CK(hipMalloc(&out, sizeof(double) * blocks * 256));
    CK(hipMalloc(&cyc, sizeof(unsigned long long) * nw));
    CK(hipMalloc(&rt, sizeof(unsigned long long) * nw));
    hipLaunchKernelGGL(rate_kernel<OP>, dim3(blocks), dim3(256), 0, 0, out, cyc, rt, 1.5);  // warm-up
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(rate_kernel<OP>, dim3(blocks), dim3(256), 0, 0, out, cyc, rt, 1.5);
    CK(hipEventRecord(e1));
    CK(hipDeviceSynchronize());
    float ms = 0; CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> c(nw), r(nw);
    CK(hipMemcpy(c.data(), cyc, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r.data(), rt, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost));
    double mc = 0, mr = 0;
    for (int i = 0; i < nw; ++i) { mc += (double)c[i]; mr += (double)r[i]; }
    mc /= nw; mr /= nw;
    const double per_wave = 8.0 * kIters;  // instructions (or operations) per wave
    const double ghz = mc / (mr * 10.0);                // s_memrealtime ticks at 100 MHz
    // chip-wide rate from wall time: wave-instructions per second; and the SIMD issue
    // cycles per wave-instruction it implies at the in-kernel clock (the waves of one
    // SIMD do not all run the whole launch side by side, so each wave's own s_memtime
    // span under-counts: the wall form is the issue cost, round 4)
    const double wall_rate = (double)nw * per_wave / (ms * 1e-3);
    const double cpi = ghz * 1e9 * (double)(cus * 4) / wall_rate;
    printf("%-22s waves/SIMD %d  cycles/wave-instr/SIMD %6.2f  clock %.3f GHz  wall %.3f ms  %.3e wave-instr/s\n",
           kName[OP], waves_per_simd, cpi, ghz, ms, wall_rate);
    CK(hipFree(out)); CK(hipFree(cyc)); CK(hipFree(rt));
}

int main(int argc, char** argv) {
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    printf("CUs %d\n", cus);
    if (argc > 1) {  // round 4: the full-load (8 waves/SIMD) table of every class, for bench.py's pricing
        run<FMA64>(8, cus); run<ADD64>(8, cus); run<MUL64>(8, cus); run<MAX64>(8, cus); run<RCP64>(8, cus);
        run<CMP64>(8, cus); run<FMA32>(8, cus); run<ADD32F>(8, cus); run<ADDU32>(8, cus); run<CNDMASK>(8, cus);
        run<MADU64>(8, cus); run<MOV32>(8, cus); run<DPP>(8, cus); run<RFL>(8, cus); run<CVT64F32>(8, cus);
        run<CVT32F64>(8, cus); run<AND32>(8, cus); run<LSHL32>(8, cus); run<MULLO32>(8, cus); run<CMPU32>(8, cus);
        run<CMPCLS64>(8, cus); run<BFE32>(8, cus); run<ADDCO32>(8, cus); run<DIVSCALE64>(8, cus);
        run<DIVFMAS64>(8, cus); run<DIVFIXUP64>(8, cus); run<CNDMASK_VCC>(8, cus); run<XOR32>(8, cus);
        run<BITOP3>(8, cus);
        for (int w : {4}) {
            run<FMA64>(w, cus); run<CMP64>(w, cus); run<CNDMASK>(w, cus); run<MOV32>(w, cus); run<DPP>(w, cus);
            run<RFL>(w, cus); run<CVT64F32>(w, cus); run<AND32>(w, cus); run<CMPU32>(w, cus);
        }
        return 0;
    }
    // dependent-chain latency: one chain, one wave per SIMD
    run<LAT_FMA64>(1, cus); run<LAT_FMA32>(1, cus); run<LAT_RCP64>(1, cus);
    for (int w : {1, 2, 4, 8}) {
        run<FMA64>(w, cus); run<ADD64>(w, cus); run<MUL64>(w, cus); run<MAX64>(w, cus); run<RCP64>(w, cus);
        run<CMP64>(w, cus); run<FMA32>(w, cus); run<ADD32F>(w, cus); run<ADDU32>(w, cus);
        run<CNDMASK>(w, cus); run<MADU64>(w, cus); run<DIV64>(w, cus); run<SQRT64>(w, cus);
    }
    return 0;
}
