// icx_exr.hip -- OpenEXR read on the MI355X: Image::readExr (codecs.cpp:464-493), i.e. tinyexr's
// LoadEXRFromMemory (/root/reference/tinyexr.h:6645-6860) -> RGBA float.
//
// The host parses the header and the offset table and checks every chunk header the way tinyexr
// does (a few hundred bytes of control data); the device does the pixel work:
//   k_exr_unpack   one workgroup per compressed chunk: lane 0 inflates (ZIP / ZIPS) or run-decodes
//                  (RLE) into the chunk's scratch, then the workgroup undoes the byte predictor
//                  with a prefix sum (tinyexr.h:1469-1479 / :1726-1736)
//   k_exr_convert  one thread per output pixel: the row / tile map names the chunk (and line) that
//                  wrote it last, the even / odd byte reorder (:1481-1500) is folded into the byte
//                  addressing, HALF -> FLOAT bit for bit (half_to_float :966-987), UINT bits copied
//                  as tinyexr's float** view does, RGBA assembled (:6685-6860).
// Scope (tinyexr returns otherwise): single-part scanline or one-level tiled
// images, NONE / RLE / ZIPS / ZIP. PIZ -> UNSUPPORTED_FORMAT (tinyexr built with
// TINYEXR_USE_PIZ 0), multi-part / deep / mip- or rip-mapped -> UNSUPPORTED_FEATURE. Pixels no
// chunk wrote (tinyexr: uninitialised memory) are 0.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "icx_exr_plan.h"
#include "icx_internal.h"

namespace icx {

// Per compressed chunk: decompress (lane 0), then the predictor as a workgroup prefix sum.
__global__ __launch_bounds__(256) void k_exr_unpack(const uint8_t* __restrict__ file, ExrChunk* __restrict__ ch,
                                                    const int32_t* __restrict__ list, uint8_t* __restrict__ scratch,
                                                    int32_t* __restrict__ fail) {
    __shared__ InfState st;
    __shared__ uint8_t win[kExrWin];
    __shared__ uint32_t part[256];
    __shared__ int64_t produced;
    ExrChunk& c = ch[list[blockIdx.x]];
    uint8_t* t = scratch + c.scratch;
    if (threadIdx.x == 0) {
        int64_t m = 0;
        bool ok;
        if (c.mode == 1) {
            ok = exr_inflate(file + c.src, c.len, t, c.out_len, &m, st, win);
        } else {
            ok = exr_unrle(file + c.src, c.len, t, c.out_len);
            m = c.out_len;
        }
        if (!ok) {
            atomicOr(fail, 1);
            m = 0;
        }
        produced = m;
        c.produced = m;
    }
    __syncthreads();
    const int64_t m = produced;
    if (m == 0) return;
    // t'[i] = t[0] + sum_{k=1..i} (t[k] - 128) mod 256: each thread one contiguous segment
    const int64_t seg = (m + 255) / 256;
    const int64_t a = min<int64_t>(m, (int64_t)threadIdx.x * seg), b = min<int64_t>(m, a + seg);
    uint32_t sum = 0;
    for (int64_t k = a; k < b; ++k) sum += k == 0 ? t[0] : (uint32_t)t[k] - 128u;
    part[threadIdx.x] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {  // (256 partial sums: a serial scan is cheap next to the inflate)
        uint32_t run = 0;
        for (int k = 0; k < 256; ++k) {
            const uint32_t v = part[k];
            part[k] = run;
            run += v;
        }
    }
    __syncthreads();
    uint32_t run = part[threadIdx.x];
    for (int64_t k = a; k < b; ++k) {
        run += k == 0 ? t[0] : (uint32_t)t[k] - 128u;
        t[k] = (uint8_t)run;
    }
}

__global__ __launch_bounds__(256) void k_exr_convert(const uint8_t* __restrict__ file, const uint8_t* __restrict__ scratch,
                                                     const ExrChunk* __restrict__ ch, const int2* __restrict__ map,
                                                     const int32_t* __restrict__ tile_h, const int32_t* __restrict__ ctype,
                                                     const int32_t* __restrict__ coffs, ExrConv cv, float* __restrict__ out) {
    const int64_t npx = (int64_t)cv.w * cv.h;
    for (int64_t px = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; px < npx; px += (int64_t)gridDim.x * blockDim.x)
        reinterpret_cast<uint4*>(out)[px] = exr_pixel(file, scratch, ch, map, tile_h, ctype, coffs, cv, px);
}

// The whole read: returns a tinyexr code; *out_rgba = malloc'd w*h*4 floats on success.
int exr_decode(hipStream_t st, const uint8_t* data, size_t size, float** out_rgba, int* width, int* height,
               std::string& err) {
    ExrPlan P;
    const int rc = exr_plan(data, (int64_t)size, P);
    if (rc != kExrOk) return rc;
    const int64_t npx = (int64_t)P.w * P.h;
    uint8_t *d_file = nullptr, *d_scr = nullptr;
    ExrChunk* d_ch = nullptr;
    int2* d_map = nullptr;
    int32_t *d_list = nullptr, *d_fail = nullptr, *d_th = nullptr, *d_ty = nullptr, *d_of = nullptr;
    float* d_out = nullptr;
    std::vector<int32_t> list;
    for (size_t k = 0; k < P.chunks.size(); ++k)
        if (P.chunks[k].mode != 0) list.push_back((int32_t)k);
    std::vector<int32_t> th = P.tile_h.empty() ? std::vector<int32_t>(1, 0) : P.tile_h;
    int res = -100;
    int32_t fail = 0;
    float* host = nullptr;
    const size_t nout = (size_t)npx * 4 * sizeof(float);
    auto ok = [&](hipError_t e) { return e == hipSuccess; };
    if (ok(hipMalloc(&d_file, size + 16)) && ok(hipMalloc(&d_scr, (size_t)std::max<int64_t>(16, P.scratch))) &&
        ok(hipMalloc(&d_ch, sizeof(ExrChunk) * std::max<size_t>(1, P.chunks.size()))) &&
        ok(hipMalloc(&d_map, sizeof(int2) * P.map.size())) &&
        ok(hipMalloc(&d_list, sizeof(int32_t) * std::max<size_t>(1, list.size()))) &&
        ok(hipMalloc(&d_fail, sizeof(int32_t))) && ok(hipMalloc(&d_th, sizeof(int32_t) * th.size())) &&
        ok(hipMalloc(&d_ty, sizeof(int32_t) * P.nch)) && ok(hipMalloc(&d_of, sizeof(int32_t) * P.nch)) &&
        ok(hipMalloc(&d_out, nout)) &&
        ok(hipMemcpyAsync(d_file, data, size, hipMemcpyHostToDevice, st)) &&
        ok(hipMemcpyAsync(d_ch, P.chunks.data(), sizeof(ExrChunk) * P.chunks.size(), hipMemcpyHostToDevice, st)) &&
        ok(hipMemcpyAsync(d_map, P.map.data(), sizeof(int2) * P.map.size(), hipMemcpyHostToDevice, st)) &&
        ok(hipMemcpyAsync(d_list, list.data(), sizeof(int32_t) * list.size(), hipMemcpyHostToDevice, st)) &&
        ok(hipMemcpyAsync(d_th, th.data(), sizeof(int32_t) * th.size(), hipMemcpyHostToDevice, st)) &&
        ok(hipMemcpyAsync(d_ty, P.type.data(), sizeof(int32_t) * P.nch, hipMemcpyHostToDevice, st)) &&
        ok(hipMemcpyAsync(d_of, P.offs.data(), sizeof(int32_t) * P.nch, hipMemcpyHostToDevice, st)) &&
        ok(hipMemsetAsync(d_fail, 0, sizeof(int32_t), st))) {
        if (!list.empty()) hipLaunchKernelGGL(k_exr_unpack, dim3((unsigned)list.size()), dim3(256), 0, st, d_file, d_ch, d_list, d_scr, d_fail);
        ExrConv cv{};
        cv.w = P.w; cv.h = P.h; cv.nch = P.nch; cv.pds = P.pds; cv.tiled = P.tiled; cv.tx = P.tx; cv.ty = P.ty;
        cv.ntx = P.ntx; cv.line_order = P.line_order;
        for (int k = 0; k < 4; ++k) cv.src[k] = P.src[k];
        const unsigned grid = (unsigned)std::min<int64_t>(8192, (npx + 255) / 256);
        hipLaunchKernelGGL(k_exr_convert, dim3(std::max(1u, grid)), dim3(256), 0, st, d_file, d_scr, d_ch, d_map, d_th, d_ty,
                           d_of, cv, d_out);
        if (ok(hipGetLastError()) && ok(hipMemcpyAsync(&fail, d_fail, sizeof(int32_t), hipMemcpyDeviceToHost, st)) &&
            ok(hipStreamSynchronize(st))) {
            if (fail) {
                res = kExrInvalidData;  // "Invalid/Corrupted data found when decoding pixels" (:5512-5524)
            } else {
                host = (float*)std::malloc(nout);
                if (host && ok(hipMemcpy(host, d_out, nout, hipMemcpyDeviceToHost))) {
                    *out_rgba = host;
                    *width = P.w;
                    *height = P.h;
                    host = nullptr;
                    res = kExrOk;
                } else {
                    err = "icx_exr_decode: host allocation or copy failed";
                }
            }
        } else {
            err = "icx_exr_decode: HIP failure";
        }
    } else {
        err = "icx_exr_decode: device allocation or copy failed";
    }
    std::free(host);
    for (void* q : {(void*)d_file, (void*)d_scr, (void*)d_ch, (void*)d_map, (void*)d_list, (void*)d_fail, (void*)d_th,
                    (void*)d_ty, (void*)d_of, (void*)d_out})
        if (q) (void)hipFree(q);
    return res;
}

int exr_probe(const uint8_t* data, size_t size, int* width, int* height) {
    ExrPlan P;
    const int rc = exr_plan(data, (int64_t)size, P);
    if (width) *width = rc == kExrOk ? P.w : 0;
    if (height) *height = rc == kExrOk ? P.h : 0;
    return rc;
}

}  // namespace icx
