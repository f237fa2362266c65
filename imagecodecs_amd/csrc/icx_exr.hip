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
//   k_exr_piz      one workgroup per PIZ chunk (TINYEXR_USE_PIZ is on in the reference build):
//                  Huffman tables in LDS, one thread walks the stream, the workgroup runs the
//                  wavelet levels and the range LUT (icx_exr_core.h PIZ section)
// Scope (tinyexr returns otherwise): single-part scanline images, and tiled ones
// with one level, mipmap or ripmap levels (every level is decoded and checked, level 0 is the
// output, as LoadEXRFromMemory does); NONE / RLE / ZIPS / ZIP / PIZ. Multi-part / deep ->
// UNSUPPORTED_FEATURE, PXR24 / B44 / ZFP -> UNSUPPORTED_FORMAT. Pixels no chunk wrote
// (tinyexr: uninitialised memory) are 0.
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

// One workgroup per PIZ chunk: the phases of icx_exr_core.h's PIZ section around barriers. The
// Huffman tables live in LDS (code lengths 64 KiB + the 14-bit direct table 64 KiB), then the same
// LDS holds the 64 Ki-entry range LUT; the channel planes and the long-code lists are the chunk's
// scratch. One thread walks the Huffman stream (a serial bit stream), the workgroup does the rest.
__global__ __launch_bounds__(256) void k_exr_piz(const uint8_t* __restrict__ file, int64_t fsize, ExrChunk* __restrict__ ch,
                                                 const int32_t* __restrict__ list, const int32_t* __restrict__ ctype, int nch,
                                                 uint8_t* __restrict__ scratch) {
    struct Tabs {
        uint8_t lens[kPizLens];
        uint32_t dec[kHufDecSize];
    };
    union PizLds {
        Tabs t;
        uint16_t lut[65536];
    };
    __shared__ PizLds L;
    __shared__ uint64_t nextc[59];
    __shared__ uint32_t ncnt[59];
    __shared__ uint32_t part[256];
    __shared__ PizHuf H;
    const int t = threadIdx.x, T = blockDim.x;
    ExrChunk& c = ch[list[blockIdx.x]];
    uint16_t* planes = reinterpret_cast<uint16_t*>(scratch + c.piz_work);
    PizWork& w = *reinterpret_cast<PizWork*>(scratch + c.piz_work + (c.out_len + 15) / 16 * 16);
    uint16_t* out = reinterpret_cast<uint16_t*>(scratch + c.scratch);
    const int64_t nus = c.out_len / 2;
    piz_init(t, T, L.t.lens, L.t.dec, w, planes, nus, ncnt);
    part[t] = piz_lut_count(file, c.piz_bitmap, c.piz_mnmx, t);
    __syncthreads();
    if (t == 0) {
        PizBytes F{file, fsize};
        H = piz_unpack(F, c.piz_huf, c.piz_len, L.t.lens);
    }
    __syncthreads();
    if (H.run) {  // (uniform)
        if (H.canon) piz_count(t, T, L.t.lens, ncnt);
        __syncthreads();
        if (t == 0) {
            for (int l = 0; l < 59; ++l) nextc[l] = ncnt[l];
            piz_first_codes(nextc);
            piz_build(H, L.t.lens, nextc, L.t.dec, w);
            PizBytes F{file, fsize};
            piz_decode(F, H, L.t.dec, L.t.lens, w, planes, nus);
        }
        __syncthreads();
    }
    // the LUT over the tables' LDS: thread t's values from the exclusive prefix of the counts
    uint32_t base = 0, total = 0;
    for (int k = 0; k < T; ++k) {
        const uint32_t v = part[k];
        base += k < t ? v : 0u;
        total += v;
    }
    piz_lut_fill(file, c.piz_bitmap, c.piz_mnmx, t, base, L.lut);
    piz_lut_tail(t, T, total, L.lut);
    const bool w14 = ((total - 1u) & 0xFFFFu) < (1u << 14);  // maxValue < 1 << 14
    int p2 = piz_top_p2(c.width, c.lines);
    for (int p = p2 >> 1; p >= 1; p2 = p, p >>= 1) {
        piz_wavelet_level(t, T, planes, ctype, nch, c.width, c.lines, w14, p, p2);
        __syncthreads();
    }
    __syncthreads();
    piz_interleave(t, T, planes, L.lut, ctype, nch, c.width, c.lines, out);
    if (t == 0) c.produced = c.out_len;
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
    int32_t *d_list = nullptr, *d_plist = nullptr, *d_fail = nullptr, *d_th = nullptr, *d_ty = nullptr, *d_of = nullptr;
    float* d_out = nullptr;
    std::vector<int32_t> list, plist;  // inflate / RLE chunks; PIZ chunks
    for (size_t k = 0; k < P.chunks.size(); ++k) {
        if (P.chunks[k].mode == 3) plist.push_back((int32_t)k);
        else if (P.chunks[k].mode != 0) list.push_back((int32_t)k);
    }
    std::vector<int32_t> th = P.tile_h.empty() ? std::vector<int32_t>(1, 0) : P.tile_h;
    int res = -100;
    int32_t fail = 0;
    float* host = nullptr;
    const size_t nout = (size_t)npx * 4 * sizeof(float);
    auto ok = [&](hipError_t e) { return e == hipSuccess; };
    // (the file + 16 zero bytes: the PIZ reader loads whole aligned 16-byte words)
    if (ok(hipMalloc(&d_file, size + 16)) && ok(hipMemsetAsync(d_file + size, 0, 16, st)) &&
        ok(hipMalloc(&d_scr, (size_t)std::max<int64_t>(16, P.scratch))) &&
        ok(hipMalloc(&d_ch, sizeof(ExrChunk) * std::max<size_t>(1, P.chunks.size()))) &&
        ok(hipMalloc(&d_map, sizeof(int2) * P.map.size())) &&
        ok(hipMalloc(&d_list, sizeof(int32_t) * std::max<size_t>(1, list.size()))) &&
        ok(hipMalloc(&d_plist, sizeof(int32_t) * std::max<size_t>(1, plist.size()))) &&
        ok(hipMalloc(&d_fail, sizeof(int32_t))) && ok(hipMalloc(&d_th, sizeof(int32_t) * th.size())) &&
        ok(hipMalloc(&d_ty, sizeof(int32_t) * P.nch)) && ok(hipMalloc(&d_of, sizeof(int32_t) * P.nch)) &&
        ok(hipMalloc(&d_out, nout)) &&
        ok(hipMemcpyAsync(d_file, data, size, hipMemcpyHostToDevice, st)) &&
        ok(hipMemcpyAsync(d_ch, P.chunks.data(), sizeof(ExrChunk) * P.chunks.size(), hipMemcpyHostToDevice, st)) &&
        ok(hipMemcpyAsync(d_map, P.map.data(), sizeof(int2) * P.map.size(), hipMemcpyHostToDevice, st)) &&
        ok(hipMemcpyAsync(d_list, list.data(), sizeof(int32_t) * list.size(), hipMemcpyHostToDevice, st)) &&
        ok(hipMemcpyAsync(d_plist, plist.data(), sizeof(int32_t) * plist.size(), hipMemcpyHostToDevice, st)) &&
        ok(hipMemcpyAsync(d_th, th.data(), sizeof(int32_t) * th.size(), hipMemcpyHostToDevice, st)) &&
        ok(hipMemcpyAsync(d_ty, P.type.data(), sizeof(int32_t) * P.nch, hipMemcpyHostToDevice, st)) &&
        ok(hipMemcpyAsync(d_of, P.offs.data(), sizeof(int32_t) * P.nch, hipMemcpyHostToDevice, st)) &&
        ok(hipMemsetAsync(d_fail, 0, sizeof(int32_t), st))) {
        if (!list.empty()) hipLaunchKernelGGL(k_exr_unpack, dim3((unsigned)list.size()), dim3(256), 0, st, d_file, d_ch, d_list, d_scr, d_fail);
        if (!plist.empty())
            hipLaunchKernelGGL(k_exr_piz, dim3((unsigned)plist.size()), dim3(256), 0, st, d_file, (int64_t)size, d_ch, d_plist,
                               d_ty, P.nch, d_scr);
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
    for (void* q : {(void*)d_file, (void*)d_scr, (void*)d_ch, (void*)d_map, (void*)d_list, (void*)d_plist, (void*)d_fail, (void*)d_th,
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
