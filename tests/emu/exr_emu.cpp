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

// One PIZ chunk, the kernel's phases in order (k_exr_piz), each phase's 256 threads one after the
// other. fpad: the file, 16-byte aligned with 16 bytes of zero slack (PizBytes' loads).
static void emu_piz(const uint8_t* fpad, int64_t size, ExrChunk& c, uint8_t* scratch, const ExrPlan& P) {
    const int T = 256;
    uint16_t* planes = reinterpret_cast<uint16_t*>(scratch + c.piz_work);
    static thread_local std::unique_ptr<PizWork> slot;  // (the kernel's pool slot: reused across chunks)
    if (!slot) slot.reset(new PizWork);
    PizWork& w = *slot;
    uint16_t* out = reinterpret_cast<uint16_t*>(scratch + c.scratch);
    const int64_t nus = c.out_len / 2;
    std::vector<uint8_t> lens(kPizLens);
    std::vector<uint32_t> dec(kHufDecSize);
    std::vector<uint16_t> lut(65536);
    uint32_t ncnt[59], part[256];
    for (int t = 0; t < T; ++t) piz_init(t, T, lens.data(), dec.data(), w, planes, nus, ncnt);
    for (int t = 0; t < T; ++t) part[t] = piz_lut_count(fpad, c.piz_bitmap, c.piz_mnmx, t);
    PizBytes F{fpad, size};
    const PizHuf H = piz_unpack(F, c.piz_huf, c.piz_len, lens.data());
    if (H.run) {
        if (H.canon)
            for (int t = 0; t < T; ++t) piz_count(t, T, lens.data(), ncnt);
        uint64_t nextc[59];
        for (int l = 0; l < 59; ++l) nextc[l] = ncnt[l];
        piz_first_codes(nextc);
        piz_build(H, lens.data(), nextc, dec.data(), w);
        piz_decode(F, H, dec.data(), lens.data(), w, planes, nus);
    }
    uint32_t total = 0;
    for (int t = 0; t < T; ++t) {
        piz_lut_fill(fpad, c.piz_bitmap, c.piz_mnmx, t, total, lut.data());
        total += part[t];
    }
    for (int t = 0; t < T; ++t) piz_lut_tail(t, T, total, lut.data());
    const bool w14 = ((total - 1) & 0xFFFFu) < (1u << 14);
    int p2 = piz_top_p2(c.width, c.lines);
    for (int p = p2 >> 1; p >= 1; p2 = p, p >>= 1)
        for (int t = 0; t < T; ++t) piz_wavelet_level(t, T, planes, P.type.data(), P.nch, c.width, c.lines, w14, p, p2);
    for (int t = 0; t < T; ++t) piz_interleave(t, T, planes, lut.data(), P.type.data(), P.nch, c.width, c.lines, out);
    c.produced = c.out_len;
}

extern "C" {

// exr_inflate alone: 1 and *produced, or 0.
int emu_exr_inflate(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int64_t* produced) {
    auto st = std::make_unique<InfState>();
    std::vector<uint8_t> win(kExrWin);
    return exr_inflate(src, n, dst, cap, produced, *st, win.data()) ? 1 : 0;
}

// The GPU's form: a 16 KiB ring, farther matches read back from dst (k_exr_unpack).
int emu_exr_inflate_ring(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int64_t* produced) {
    auto st = std::make_unique<InfState>();
    std::vector<uint8_t> win(16384);
    return exr_inflate<16384>(src, n, dst, cap, produced, *st, win.data()) ? 1 : 0;
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
    std::vector<uint4> fpad((size_t)(size + 16 + 15) / 16);  // (zero slack past the end)
    std::memcpy(fpad.data(), data, (size_t)size);
    for (ExrChunk& c : P.chunks) {  // k_exr_piz
        if (c.mode == 3) emu_piz(reinterpret_cast<const uint8_t*>(fpad.data()), size, c, scratch.data(), P);
    }
    for (ExrChunk& c : P.chunks) {  // k_exr_unpack
        if (c.mode == 0 || c.mode == 3) continue;
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
