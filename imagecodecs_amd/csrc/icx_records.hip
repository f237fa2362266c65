// icx_records.hip -- per-image result records for the multi-GPU gather:
// {status, width, height, ncomp, checksum64} of each decoded image, computed on the device that
// decoded it, so ranks exchange 24 bytes per image instead of pixels.
//
// checksum64 = sum over the image's little-endian 32-bit words w_k (the last one zero-padded) of
// w_k * (2k + 1), mod 2^64. A weighted sum is order-independent to accumulate (wrap-around adds
// commute), so a grid of waves reduces it with 64-bit atomics, and numpy restates it in one line
// (tests/test_dist.py, tools/records.py).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "icx_internal.h"

namespace icx {

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// After k_records_init zeroed the sums (same stream). Grid (x: slices of the image, y: image). Aligned images take 16-byte loads (4 words per lane
// per round); an image at an address not a multiple of 16 (odd out_stride) assembles its words
// from byte loads.
__global__ __launch_bounds__(256) void k_records(int n, const uint8_t* __restrict__ out, uint64_t out_stride,
                                                 const int32_t* __restrict__ status, const int32_t* __restrict__ dims,
                                                 Record* __restrict__ rec) {
    const int i = blockIdx.y;
    if (i >= n) return;
    const int32_t st = status[i];
    const uint64_t nbytes = st == kOk ? (uint64_t)dims[3 * i] * dims[3 * i + 1] * dims[3 * i + 2] : 0;
    const uint8_t* p = out + (uint64_t)i * out_stride;
    const uint64_t nwords = (nbytes + 3) >> 2;
    uint64_t acc = 0;
    const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
    auto word_at = [&](uint64_t k) {  // byte-assembled word k (zero past the end)
        uint32_t w = 0;
        for (int b = 0; b < 4; ++b) {
            const uint64_t o = 4 * k + b;
            w |= (o < nbytes ? (uint32_t)p[o] : 0u) << (8 * b);
        }
        return w;
    };
    if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
        const uint64_t nq = nbytes >> 4;  // whole 16-byte units
        for (uint64_t q = t0; q < nq; q += nt) {
            const uint4 v = reinterpret_cast<const uint4*>(p)[q];
            const uint64_t k = 4 * q;
            acc += (uint64_t)v.x * (2 * k + 1) + (uint64_t)v.y * (2 * k + 3) + (uint64_t)v.z * (2 * k + 5) +
                   (uint64_t)v.w * (2 * k + 7);
        }
        for (uint64_t k = 4 * nq + t0; k < nwords; k += nt) acc += (uint64_t)word_at(k) * (2 * k + 1);
    } else {
        for (uint64_t k = t0; k < nwords; k += nt) acc += (uint64_t)word_at(k) * (2 * k + 1);
    }
    acc = wave_sum_u64(acc);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(reinterpret_cast<unsigned long long*>(&rec[i].checksum), acc);
}

__global__ void k_records_init(int n, const int32_t* __restrict__ status, const int32_t* __restrict__ dims,
                               Record* __restrict__ rec) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t st = status[i];
    Record r;
    r.status = st;
    r.w = st == kOk ? dims[3 * i] : 0;
    r.h = st == kOk ? dims[3 * i + 1] : 0;
    r.c = st == kOk ? dims[3 * i + 2] : 0;
    r.checksum = 0;
    rec[i] = r;
}

void launch_records(int n, const uint8_t* d_out, uint64_t out_stride, const int32_t* d_status, const int32_t* d_dims,
                    Record* d_rec, int max_w, int max_h, hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_records_init, dim3((n + 63) / 64), dim3(64), 0, st, n, d_status, d_dims, d_rec);
    // ~4K workgroups over the whole call; each image gets at least one
    const int64_t words = (int64_t)max_w * max_h * 3 / 4 + 1;
    const int gx = (int)std::max<int64_t>(1, std::min<int64_t>((words / 4 + 255) / 256, std::max(1, 4096 / n)));
    hipLaunchKernelGGL(k_records, dim3(gx, n), dim3(256), 0, st, n, d_out, out_stride, d_status, d_dims, d_rec);
}

}  // namespace icx
