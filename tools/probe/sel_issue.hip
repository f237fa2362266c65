// sel_issue.hip -- measurement tooling, not product. Follow-up to valu_issue.hip, whose v_cndmask
// case ran at ~23 SIMD cycles per instruction (64 consecutive v_cndmask_b32 reading VCC) while
// v_add_u32 ran at ~2.2 and VOP3 integer ops at ~4. Which selects are slow, and what to use
// instead, for k_gw_lane's select-heavy decode loop:
//   c_vcc      v_cndmask_b32 (e32, VCC mask), 64 consecutive
//   c_sgpr     v_cndmask_b32_e64 with an SGPR-pair mask (s[N:N+1] set before the loop), 64 consecutive
//   c_mix1     v_cndmask (VCC) and v_add_u32 alternating, 32 + 32
//   c_mix3     one v_cndmask (VCC) per three v_add_u32, 16 + 48
//   c_cmp      v_cmp_gt_u32 vcc + v_cndmask (VCC) pairs, 32 + 32 (a fresh mask per select)
//   c_salu     s_and_b64 vcc + v_cndmask (VCC) pairs (the compiler's pattern: SALU-built masks)
//   bfi        v_bfi_b32 with a VGPR mask (0 / ~0 per lane) as the select, 64 consecutive
//   andor      v_and_or_b32 (VOP3), 64 consecutive
//   add_s      v_add_u32 with an SGPR operand, 64 consecutive
//   c_vcc16    16 consecutive v_cndmask (VCC) then 49 v_add_u32
//   salu_vcc8  8 x (s_and_b64 vcc + v_cndmask VCC) + 48 v_add_u32 (the compiler's select pattern)
//   salu_sg8   8 x (s_and_b64 s[..] + v_cndmask_e64 s[..]) + 48 v_add_u32
//   cmp_vcc8   8 x (v_cmp vcc + v_cndmask VCC) + 48 v_add_u32
//   c_vcc32    32 consecutive v_cndmask (VCC) then 32 v_add_u32
//   c_vcc_e64  64 consecutive v_cndmask_b32_e64 naming VCC as an SGPR operand
//   addc_vcc   64 consecutive v_addc_co_u32 (VCC carry in and out)
// Output: one JSON line per (case, W) with SIMD cycles per instruction from the wall time
// (cycles of the slowest wave / (W x instructions per wave)).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
            std::exit(1);                                                          \
        }                                                                          \
    } while (0)

#define R2(X) X X
#define R4(X) R2(X) R2(X)
#define R8(X) R4(X) R4(X)
#define R16(X) R8(X) R8(X)
#define A8 "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)

template <int C>
__global__ __launch_bounds__(256) void sel(int iters, unsigned* __restrict__ sink, unsigned long long* __restrict__ cyc) {
    extern __shared__ unsigned lds[];
    unsigned a0 = threadIdx.x, a1 = a0 * 3u + 1, a2 = a0 ^ 0x55u, a3 = a0 + 7u, a4 = a0 * 5u, a5 = a0 + 11u,
             a6 = a0 ^ 0xa5u, a7 = a0 + 19u;
    const unsigned k1 = 3u + (sink[1] & 1u);
    const unsigned msk = (threadIdx.x & 1) ? ~0u : 0u;
    const unsigned long long sm = __builtin_amdgcn_readfirstlane(sink[3]) | 0x5555555555555555ull;
    asm volatile("v_cmp_gt_u32 vcc, %0, %1" ::"v"(a0), "v"(a1) : "vcc");
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (C == 0) {
            asm volatile(R8("v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n v_cndmask_b32 %3, %3, %8, vcc\n"
                            "v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc\n")
                         : A8 : "v"(k1) : "vcc");
        } else if (C == 1) {
            asm volatile(R8("v_cndmask_b32_e64 %0, %0, %8, %9\n v_cndmask_b32_e64 %1, %1, %8, %9\n v_cndmask_b32_e64 %2, %2, %8, %9\n v_cndmask_b32_e64 %3, %3, %8, %9\n"
                            "v_cndmask_b32_e64 %4, %4, %8, %9\n v_cndmask_b32_e64 %5, %5, %8, %9\n v_cndmask_b32_e64 %6, %6, %8, %9\n v_cndmask_b32_e64 %7, %7, %8, %9\n")
                         : A8 : "v"(k1), "s"(sm));
        } else if (C == 2) {
            asm volatile(R8("v_cndmask_b32 %0, %0, %8, vcc\n v_add_u32 %1, %1, %8\n v_cndmask_b32 %2, %2, %8, vcc\n v_add_u32 %3, %3, %8\n"
                            "v_cndmask_b32 %4, %4, %8, vcc\n v_add_u32 %5, %5, %8\n v_cndmask_b32 %6, %6, %8, vcc\n v_add_u32 %7, %7, %8\n")
                         : A8 : "v"(k1) : "vcc");
        } else if (C == 3) {
            asm volatile(R8("v_cndmask_b32 %0, %0, %8, vcc\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
                            "v_cndmask_b32 %4, %4, %8, vcc\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n")
                         : A8 : "v"(k1) : "vcc");
        } else if (C == 4) {
            asm volatile(R8("v_cmp_gt_u32 vcc, %0, %8\n v_cndmask_b32 %1, %1, %8, vcc\n v_cmp_gt_u32 vcc, %2, %8\n v_cndmask_b32 %3, %3, %8, vcc\n"
                            "v_cmp_gt_u32 vcc, %4, %8\n v_cndmask_b32 %5, %5, %8, vcc\n v_cmp_gt_u32 vcc, %6, %8\n v_cndmask_b32 %7, %7, %8, vcc\n")
                         : A8 : "v"(k1) : "vcc");
        } else if (C == 5) {
            // SALU-built masks: 32 s_and_b64 + 32 v_cndmask (VALU count 32)
            asm volatile(R8("s_and_b64 vcc, vcc, %9\n v_cndmask_b32 %0, %0, %8, vcc\n s_and_b64 vcc, vcc, %9\n v_cndmask_b32 %2, %2, %8, vcc\n"
                            "s_and_b64 vcc, vcc, %9\n v_cndmask_b32 %4, %4, %8, vcc\n s_and_b64 vcc, vcc, %9\n v_cndmask_b32 %6, %6, %8, vcc\n")
                         : A8 : "v"(k1), "s"(sm) : "vcc", "scc");
        } else if (C == 6) {
            asm volatile(R8("v_bfi_b32 %0, %9, %8, %0\n v_bfi_b32 %1, %9, %8, %1\n v_bfi_b32 %2, %9, %8, %2\n v_bfi_b32 %3, %9, %8, %3\n"
                            "v_bfi_b32 %4, %9, %8, %4\n v_bfi_b32 %5, %9, %8, %5\n v_bfi_b32 %6, %9, %8, %6\n v_bfi_b32 %7, %9, %8, %7\n")
                         : A8 : "v"(k1), "v"(msk));
        } else if (C == 7) {
            asm volatile(R8("v_and_or_b32 %0, %0, %9, %8\n v_and_or_b32 %1, %1, %9, %8\n v_and_or_b32 %2, %2, %9, %8\n v_and_or_b32 %3, %3, %9, %8\n"
                            "v_and_or_b32 %4, %4, %9, %8\n v_and_or_b32 %5, %5, %9, %8\n v_and_or_b32 %6, %6, %9, %8\n v_and_or_b32 %7, %7, %9, %8\n")
                         : A8 : "v"(k1), "v"(msk));
        } else if (C == 8) {
            asm volatile(R8("v_add_u32 %0, %8, %0\n v_add_u32 %1, %8, %1\n v_add_u32 %2, %8, %2\n v_add_u32 %3, %8, %3\n"
                            "v_add_u32 %4, %8, %4\n v_add_u32 %5, %8, %5\n v_add_u32 %6, %8, %6\n v_add_u32 %7, %8, %7\n")
                         : A8 : "s"(k1));
        } else if (C == 9) {
            asm volatile(R2("v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n v_cndmask_b32 %3, %3, %8, vcc\n"
                            "v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc\n")
                         R4(R2("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
                               "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n")) "v_add_u32 %0, %0, %8\n"
                         : A8 : "v"(k1) : "vcc");
        } else if (C == 10) {  // SALU-written VCC read by one v_cndmask, 8 pairs + 48 v_add
            asm volatile(R8("s_and_b64 vcc, vcc, %9\n v_cndmask_b32 %0, %0, %8, vcc\n"
                            "v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n v_add_u32 %4, %4, %8\n"
                            "v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n")
                         : A8 : "v"(k1), "s"(sm) : "vcc", "scc");
        } else if (C == 11) {  // SALU-written SGPR-pair mask read by one v_cndmask_e64, 8 pairs + 48 v_add
            unsigned long long m2 = sm;
            asm volatile(R8("s_and_b64 %8, %8, %10\n v_cndmask_b32_e64 %0, %0, %9, %8\n"
                            "v_add_u32 %1, %1, %9\n v_add_u32 %2, %2, %9\n v_add_u32 %3, %3, %9\n v_add_u32 %4, %4, %9\n"
                            "v_add_u32 %5, %5, %9\n v_add_u32 %6, %6, %9\n")
                         : A8, "+s"(m2) : "v"(k1), "s"(sm) : "scc");
        } else if (C == 12) {  // VALU-written VCC (v_cmp) read by a v_cndmask: 8 pairs + 48 v_add
            asm volatile(R8("v_cmp_gt_u32 vcc, %7, %8\n v_cndmask_b32 %0, %0, %8, vcc\n"
                            "v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n v_add_u32 %4, %4, %8\n"
                            "v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n")
                         : A8 : "v"(k1) : "vcc");
        } else if (C == 13) {  // 32 consecutive v_cndmask (VCC) + 32 v_add: where does "consecutive" turn slow
            asm volatile(R4("v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n v_cndmask_b32 %3, %3, %8, vcc\n"
                            "v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc\n")
                         R4("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
                            "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n")
                         : A8 : "v"(k1) : "vcc");
        } else if (C == 14) {  // 64 v_cndmask_e64 reading VCC as an SGPR operand (VOP3 form)
            asm volatile(R8("v_cndmask_b32_e64 %0, %0, %8, vcc\n v_cndmask_b32_e64 %1, %1, %8, vcc\n v_cndmask_b32_e64 %2, %2, %8, vcc\n v_cndmask_b32_e64 %3, %3, %8, vcc\n"
                            "v_cndmask_b32_e64 %4, %4, %8, vcc\n v_cndmask_b32_e64 %5, %5, %8, vcc\n v_cndmask_b32_e64 %6, %6, %8, vcc\n v_cndmask_b32_e64 %7, %7, %8, vcc\n")
                         : A8 : "v"(k1) : "vcc");
        } else if (C == 15) {  // 64 v_addc_co_u32 (VOP2 reading VCC as carry-in, writing VCC)
            asm volatile(R8("v_addc_co_u32 %0, vcc, %0, %8, vcc\n v_addc_co_u32 %1, vcc, %1, %8, vcc\n v_addc_co_u32 %2, vcc, %2, %8, vcc\n v_addc_co_u32 %3, vcc, %3, %8, vcc\n"
                            "v_addc_co_u32 %4, vcc, %4, %8, vcc\n v_addc_co_u32 %5, vcc, %5, %8, vcc\n v_addc_co_u32 %6, vcc, %6, %8, vcc\n v_addc_co_u32 %7, vcc, %7, %8, vcc\n")
                         : A8 : "v"(k1) : "vcc");
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (r == 0x9e3779b9u) sink[0] = r;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
    (void)lds;
}

// vector instructions per body (C5 also issues 32 SALU; C9 has one extra v_add)
static int valu(int c) { return c == 4 ? 64 : (c == 5 ? 32 : (c == 9 ? 65 : (c == 10 || c == 11 ? 56 : 64))); }

template <int C>
static void run(const char* name, int W, int cus, int iters, unsigned* sink, unsigned long long* cyc) {
    const int grid = cus * W;
    const size_t lds = (size_t)(160 * 1024 / W) & ~(size_t)1023;
    CK(hipFuncSetAttribute((const void*)sel<C>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(sel<C>, dim3(grid), dim3(256), lds, 0, 16, sink, cyc);
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(sel<C>, dim3(grid), dim3(256), lds, 0, iters, sink, cyc);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const int nw = grid * 4;
    unsigned long long* h = (unsigned long long*)std::malloc(sizeof(unsigned long long) * nw);
    CK(hipMemcpy(h, cyc, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost));
    double sum = 0, mx = 0;
    for (int i = 0; i < nw; ++i) {
        sum += (double)h[i];
        mx = h[i] > mx ? (double)h[i] : mx;
    }
    std::free(h);
    const double v = (double)valu(C) * iters;
    std::printf("{\"case\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"cyc_per_wave_avg\": %.0f, \"cyc_per_wave_max\": %.0f, "
                "\"valu_per_wave\": %.0f, \"simd_cyc_per_valu\": %.3f, \"one_wave_cyc_per_valu\": %.3f, \"clock_ghz\": %.3f}\n",
                name, W, ms, sum / nw, mx, v, mx / (W * v), sum / nw / v, mx / (ms * 1e6));
    std::fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int iters = argc > 1 ? std::atoi(argv[1]) : 4000;
    unsigned* sink = nullptr;
    unsigned long long* cyc = nullptr;
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(sink, 0, 64));
    CK(hipMalloc(&cyc, sizeof(unsigned long long) * cus * 8 * 4));
    const int Ws[] = {1, 2, 4, 8};
    for (int W : Ws) {
        run<0>("c_vcc", W, cus, iters, sink, cyc);
        run<1>("c_sgpr", W, cus, iters, sink, cyc);
        run<2>("c_mix1", W, cus, iters, sink, cyc);
        run<3>("c_mix3", W, cus, iters, sink, cyc);
        run<4>("c_cmp", W, cus, iters, sink, cyc);
        run<5>("c_salu", W, cus, iters, sink, cyc);
        run<6>("bfi", W, cus, iters, sink, cyc);
        run<7>("andor", W, cus, iters, sink, cyc);
        run<8>("add_s", W, cus, iters, sink, cyc);
        run<9>("c_vcc16", W, cus, iters, sink, cyc);
        run<10>("salu_vcc8", W, cus, iters, sink, cyc);
        run<11>("salu_sg8", W, cus, iters, sink, cyc);
        run<12>("cmp_vcc8", W, cus, iters, sink, cyc);
        run<13>("c_vcc32", W, cus, iters, sink, cyc);
        run<14>("c_vcc_e64", W, cus, iters, sink, cyc);
        run<15>("addc_vcc", W, cus, iters, sink, cyc);
    }
    CK(hipDeviceSynchronize());
    CK(hipFree(sink));
    CK(hipFree(cyc));
    return 0;
}
