// pmc_calib.hip -- calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE against known byte counts on
// this GPU (measurement tooling, not product). Each kernel moves an exact number of bytes of a
// 1 GiB buffer (4x the 256 MiB Infinity Cache, so nothing is served on-die twice):
//   calib_read16   16-byte loads per lane, every byte once        (the decoder's coefficient /
//   calib_read4    4-byte loads per lane, every byte once          U-stream read shapes)
//   calib_write16  16-byte stores per lane, every byte once
// tools/pmc_calib.py runs it under two separate --pmc passes and divides counter bytes by
// the bytes moved: the factor tools/pmc_traffic.py applies to FETCH_SIZE comes from here.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256) void calib_read16(const uint4* __restrict__ p, size_t n, unsigned* __restrict__ sink) {
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;  // keeps the loads; practically never stores
}

__global__ __launch_bounds__(256) void calib_read4(const unsigned* __restrict__ p, size_t n, unsigned* __restrict__ sink) {
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc ^= p[i];
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void calib_write16(uint4* __restrict__ p, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        p[i] = make_uint4((unsigned)i, 1u, 2u, 3u);
}

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
            return 1;                                                              \
        }                                                                          \
    } while (0)

int main() {
    const size_t bytes = (size_t)1 << 30;
    void *a = nullptr, *b = nullptr;
    unsigned* sink = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 0x5a, bytes));
    CK(hipMemset(b, 0x00, bytes));
    const int grid = 4096;
    // each kernel twice, with a 1 GiB write of the other buffer in between (evicts the caches)
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(calib_write16, dim3(grid), dim3(256), 0, 0, (uint4*)b, bytes / 16);
        hipLaunchKernelGGL(calib_read16, dim3(grid), dim3(256), 0, 0, (const uint4*)a, bytes / 16, sink);
        hipLaunchKernelGGL(calib_write16, dim3(grid), dim3(256), 0, 0, (uint4*)b, bytes / 16);
        hipLaunchKernelGGL(calib_read4, dim3(grid), dim3(256), 0, 0, (const unsigned*)a, bytes / 4, sink);
    }
    CK(hipDeviceSynchronize());
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(sink));
    std::printf("{\"bytes_per_launch\": %zu}\n", bytes);
    return 0;
}
