// exr_emu.cpp -- TEST-ONLY CPU run of the OpenEXR read (icx_exr.hip): the same host plan
// (icx_exr_plan.h), chunk decompressors (icx_exr_core.h) and per-pixel gather the kernels use,
// with the predictor done serially. Never linked into libicx.so.
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "../../imagecodecs_amd/csrc/icx_exr_plan.h"

using namespace icx;

extern "C" {

// exr_inflate alone: 1 and *produced, or 0.
int emu_exr_inflate(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int64_t* produced) {
    auto st = std::make_unique<InfState>();
    std::vector<uint8_t> win(kExrWin);
    return exr_inflate(src, n, dst, cap, produced, *st, win.data()) ? 1 : 0;
}

// The whole read: the tinyexr code; on success w*h*4 float bits in out (cap_px pixels at most).
int emu_exr_decode(const uint8_t* data, int64_t size, uint32_t* out, int64_t cap_px, int* w, int* h) {
    ExrPlan P;
    *w = *h = 0;
    const int rc = exr_plan(data, size, P);
    if (rc != 0) return rc;
    if ((int64_t)P.w * P.h > cap_px) return -100;
    std::vector<uint8_t> scratch((size_t)std::max<int64_t>(16, P.scratch));
    auto st = std::make_unique<InfState>();
    std::vector<uint8_t> win(kExrWin);
    for (ExrChunk& c : P.chunks) {  // k_exr_unpack
        if (c.mode == 0) continue;
        uint8_t* t = scratch.data() + c.scratch;
        int64_t m = 0;
        const bool ok = c.mode == 1 ? exr_inflate(data + c.src, c.len, t, c.out_len, &m, *st, win.data())
                                    : (m = c.out_len, exr_unrle(data + c.src, c.len, t, c.out_len));
        if (!ok) return -4;
        for (int64_t k = 1; k < m; ++k) t[k] = (uint8_t)(t[k - 1] + t[k] - 128);
        c.produced = m;
    }
    ExrConv cv{};
    cv.w = P.w; cv.h = P.h; cv.nch = P.nch; cv.pds = P.pds; cv.tiled = P.tiled; cv.tx = P.tx; cv.ty = P.ty;
    cv.ntx = P.ntx; cv.line_order = P.line_order;
    for (int k = 0; k < 4; ++k) cv.src[k] = P.src[k];
    const int64_t npx = (int64_t)P.w * P.h;
    for (int64_t px = 0; px < npx; ++px) {  // k_exr_convert
        const uint4 v = exr_pixel(data, scratch.data(), P.chunks.data(), P.map.data(), P.tile_h.data(), P.type.data(),
                                  P.offs.data(), cv, px);
        out[4 * px] = v.x;
        out[4 * px + 1] = v.y;
        out[4 * px + 2] = v.z;
        out[4 * px + 3] = v.w;
    }
    *w = P.w;
    *h = P.h;
    return 0;
}
}
