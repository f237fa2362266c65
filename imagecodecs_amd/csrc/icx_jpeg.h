// icx_jpeg.h -- host/device core of the MI355X JPEG decoder (compiled by hipcc only).
//
// Everything here is __host__ __device__: the same header parser runs on the host for
// icx_jpeg_probe() and on the GPU (k_parse) for device-resident batches. Semantics follow
// NanoJPEG 1.3.5 as vendored by ImageCodecs (/root/reference/jpeg_dec.h); each function
// cites the lines it reproduces. Integer arithmetic that can overflow on hostile input is
// done in wrap-around uint32 form so results match the reference's two's-complement code.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ICX_HD __host__ __device__ __forceinline__

namespace icx {

// A 16-byte load that the compiler emits as global_load_dwordx4 whatever it knows about p.
// A pointer rebuilt from integers (readfirstlane'd bases, pointers carried through loop phis)
// loses its address space, and the load becomes flat_load_dwordx4. A flat load counts in BOTH
// vmcnt and lgkmcnt and completes out of order, so every s_waitcnt lgkmcnt(0) of a later LDS
// read then also waits for it: a prefetch issued ahead of its use turns into a full memory
// latency at the next LDS lookup.
typedef unsigned int icx_u32x4 __attribute__((ext_vector_type(4)));
ICX_HD uint4 gload16(const void* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    const icx_u32x4 v = *(const __attribute__((address_space(1))) icx_u32x4*)(p);
    return make_uint4(v.x, v.y, v.z, v.w);
#else
    return *reinterpret_cast<const uint4*>(p);
#endif
}
ICX_HD uint32_t gload4(const void* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return *(const __attribute__((address_space(1))) uint32_t*)(p);
#else
    return *reinterpret_cast<const uint32_t*>(p);
#endif
}

enum : int32_t {
    kOk = 0, kNoJpeg = 1, kUnsupported = 2, kOutOfMem = 3, kInternalErr = 4, kSyntaxError = 5,
    kPending = 6  // headers parsed, entropy-coded segment not yet decoded (internal)
};

// natural (row-major) index of zig-zag position k (jpeg_dec.h:334-337)
__constant__ static const uint8_t kNatOfZig[64] = {
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
static const uint8_t kNatOfZigHost[64] = {
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// zig-zag position of natural index n (inverse of the table above)
__constant__ static const uint8_t kZigOfNat[64] = {
    0, 1, 5, 6, 14, 15, 27, 28, 2, 4, 7, 13, 16, 26, 29, 42, 3, 8, 12, 17, 25, 30, 41, 43,
    9, 11, 18, 24, 31, 40, 44, 53, 10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
    21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};

ICX_HD int nat_of_zig(int k) {
#if defined(__HIP_DEVICE_COMPILE__)
    return kNatOfZig[k];
#else
    return kNatOfZigHost[k];
#endif
}

ICX_HD int32_t wadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
ICX_HD int32_t wsub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
ICX_HD int32_t wmul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
ICX_HD int32_t wshl(int32_t a, int k) { return (int32_t)((uint32_t)a << k); }
ICX_HD uint8_t clip8(int32_t v) { return v < 0 ? 0 : (v > 255 ? 255 : (uint8_t)v); }  // njClip :339

// ---------------------------------------------------------------------------------------
// Huffman table in canonical form. NanoJPEG fills a 64K direct table sequentially with
// left-justified codes (jpeg_dec.h:591-613); any valid lookup is identical to this one:
// a 16-bit window v has code length L = min{L : v < bound[L]}, symbol index
// first[L] + ((v - bound[L-1]) >> (16-L)); v >= bound[16] is an invalid code (bits == 0).
// fast[] resolves lengths <= kFastBits with one lookup.
// Codes longer than kFastBits: the 10-bit prefixes holding them are exactly
// [bound[10] >> 6, ceil(bound[16] / 64)) (bound[10] is a multiple of 64), and prefix p gets the
// 64-entry subtable p - (bound[10] >> 6), indexed by the next 6 bits: fast[p] = kSubFlag | offset.
// Tables needing more than kSubTabs subtables keep fast[p] = 0 and take the exact search.
constexpr int kFastBits = 10;
constexpr int kSubTabs = 8;
constexpr uint16_t kSubFlag = 0x8000;
struct Huff {
    uint16_t fast[1 << kFastBits];  // (len << 8) | sym, kSubFlag | subtable offset, or 0
    uint16_t sub[kSubTabs << (16 - kFastBits)];  // (len << 8) | sym, 0 = invalid
    uint32_t bound[17];
    int16_t first[17];
    uint8_t sym[256];
    uint8_t pad[2];
};

ICX_HD void huff_finalize(Huff& t, const uint8_t* count /*[17], count[0]=0*/) {
    uint32_t edge = 0;
    int idx = 0;
    t.bound[0] = 0;
    t.first[0] = 0;
    for (int L = 1; L <= 16; ++L) {
        t.first[L] = (int16_t)idx;
        edge += (uint32_t)count[L] << (16 - L);
        idx += count[L];
        t.bound[L] = edge;
    }
}

ICX_HD int huff_search(const Huff& t, uint32_t win, int from, int& sym) {  // canonical walk
    int L = from;
    while (L <= 16 && win >= t.bound[L]) ++L;
    if (L > 16) return 0;
    sym = t.sym[t.first[L] + (int)((win - t.bound[L - 1]) >> (16 - L))];
    return L;
}

// fast[p] and the subtables for entries lane, lane+step, ... (the GPU fills a table with a
// whole workgroup).
ICX_HD void huff_fill_fast(Huff& t, int lane, int step) {
    constexpr int kSubBits = 16 - kFastBits;
    const int p0 = (int)(t.bound[kFastBits] >> kSubBits);
    const int p1 = (int)((t.bound[16] + (1u << kSubBits) - 1) >> kSubBits);
    const int nsub = p1 - p0 <= kSubTabs ? p1 - p0 : 0;
    for (int p = lane; p < (1 << kFastBits); p += step) {
        const uint32_t v = (uint32_t)p << kSubBits;
        uint16_t e = 0;
        int s = 0;
        const int L = huff_search(t, v, 1, s);
        if (L && L <= kFastBits) e = (uint16_t)((L << 8) | s);
        else if (p >= p0 && p < p0 + nsub) e = (uint16_t)(kSubFlag | ((p - p0) << kSubBits));
        t.fast[p] = e;
    }
    for (int q = lane; q < (kSubTabs << kSubBits); q += step) {
        uint16_t e = 0;
        if (q < (nsub << kSubBits)) {
            const uint32_t v = ((uint32_t)(p0 + (q >> kSubBits)) << kSubBits) | (uint32_t)(q & ((1 << kSubBits) - 1));
            int s = 0;
            const int L = huff_search(t, v, kFastBits + 1, s);
            if (L) e = (uint16_t)((L << 8) | s);
        }
        t.sub[q] = e;
    }
}

// Decode one code from a 16-bit window. Returns length (0 = invalid) and symbol.
ICX_HD int huff_lookup(const Huff& t, uint32_t win, int& sym) {
    uint32_t e = t.fast[win >> (16 - kFastBits)];
    if (e & kSubFlag) e = t.sub[(e & ~kSubFlag) | (win & ((1u << (16 - kFastBits)) - 1))];
    if (e) { sym = (int)(e & 0xFF); return (int)(e >> 8); }
    return huff_search(t, win, kFastBits + 1, sym);
}

// ---------------------------------------------------------------------------------------
struct Comp {
    int32_t id, hs, vs;      // cid, ssx, ssy (jpeg_dec.h:302-311)
    int32_t w, h, stride;    // as set by njDecodeSOF (:563-566)
    int32_t tq, dc_tab, ac_tab;
    int32_t nblk;            // blocks of this component per MCU (hs*vs)
};

// Per-image descriptor: what njDecode knows when it reaches the entropy-coded data.
struct Desc {
    int32_t status;          // kPending after a successful header walk, else the final code
    int32_t W, H, nc;
    int32_t mbw, mbh, mbx_px, mby_px;
    int32_t restart;         // DRI interval (jpeg_dec.h:635-641)
    int32_t bpm;             // blocks per MCU
    int64_t scan_off;        // byte offset of the entropy-coded segment in the file
    int64_t size;            // file size (& 0x7FFFFFFF, jpeg_dec.h:883)
    Comp c[3];
    uint8_t q[4][64];        // DQT tables in zig-zag order (jpeg_dec.h:618-633)
    Huff huff[4];            // 0,1: DC tables; 2,3: AC tables ((Tc|Th>>3)&3, :587)
    // Where the image's coefficient blocks live in the group's pool (set by k_spec_plan):
    // block n at pool block acbase + n (mapped == 0), or at the pool block map[acbase + n]
    // names, with that entry's DC offset (mapped == 1: the guess-write path, icx_spec.hip)
    int64_t acbase;
    int32_t mapped, pad_;
};

// ---------------------------------------------------------------------------------------
// Header walk: njDecode's marker loop (jpeg_dec.h:880-903) through the SOS header of the
// first scan (:678-695). Returns the final code on any header error, kPending on success.
struct Cursor {
    const uint8_t* at;
    int32_t avail, seg, err;
};
ICX_HD int be16(const uint8_t* p) { return (p[0] << 8) | p[1]; }
ICX_HD void cskip(Cursor& c, int n) {  // njSkip :500-505
    c.at += n;
    c.avail -= n;
    c.seg -= n;
    if (c.avail < 0) c.err = kSyntaxError;
}
ICX_HD void copen(Cursor& c) {  // njDecodeLength :511-516
    if (c.avail < 2) { c.err = kSyntaxError; return; }
    c.seg = be16(c.at);
    if (c.seg > c.avail) { c.err = kSyntaxError; return; }
    cskip(c, 2);
}

ICX_HD int parse_sof(Cursor& cu, Desc& d) {  // njDecodeSOF :523-575
    copen(cu);
    if (cu.err) return cu.err;
    if (cu.seg < 9) return kSyntaxError;
    if (cu.at[0] != 8) return kUnsupported;
    d.H = be16(cu.at + 1);
    d.W = be16(cu.at + 3);
    if (!d.W || !d.H) return kSyntaxError;
    d.nc = cu.at[5];
    cskip(cu, 6);
    if (d.nc != 1 && d.nc != 3) return kUnsupported;
    if (cu.seg < d.nc * 3) return kSyntaxError;
    int hmax = 0, vmax = 0;
    for (int i = 0; i < d.nc; ++i) {
        Comp& c = d.c[i];
        c.id = cu.at[0];
        c.hs = cu.at[1] >> 4;
        if (!c.hs) return kSyntaxError;
        if (c.hs & (c.hs - 1)) return kUnsupported;
        c.vs = cu.at[1] & 15;
        if (!c.vs) return kSyntaxError;
        if (c.vs & (c.vs - 1)) return kUnsupported;
        c.tq = cu.at[2];
        if (c.tq & 0xFC) return kSyntaxError;
        cskip(cu, 3);
        hmax = c.hs > hmax ? c.hs : hmax;
        vmax = c.vs > vmax ? c.vs : vmax;
    }
    if (d.nc == 1) { d.c[0].hs = d.c[0].vs = hmax = vmax = 1; }
    d.mbx_px = hmax << 3;
    d.mby_px = vmax << 3;
    d.mbw = (d.W + d.mbx_px - 1) / d.mbx_px;
    d.mbh = (d.H + d.mby_px - 1) / d.mby_px;
    d.bpm = 0;
    for (int i = 0; i < d.nc; ++i) {
        Comp& c = d.c[i];
        c.w = (d.W * c.hs + hmax - 1) / hmax;
        c.h = (d.H * c.vs + vmax - 1) / vmax;
        c.stride = (d.mbw * c.hs) << 3;
        c.nblk = c.hs * c.vs;
        d.bpm += c.nblk;
        if ((c.w < 3 && c.hs != hmax) || (c.h < 3 && c.vs != vmax)) return kUnsupported;
        // NanoJPEG mallocs stride*rows here (:568); a plane beyond 2 GiB cannot be
        // represented by its int arithmetic and is reported as out of memory.
        if ((int64_t)c.stride * ((int64_t)(d.mbh * c.vs) << 3) > 0x7FFFFFFF) return kOutOfMem;
    }
    if (d.nc == 3 && (int64_t)d.W * d.H * 3 > 0x7FFFFFFF) return kOutOfMem;
    cskip(cu, cu.seg);
    return cu.err;
}

ICX_HD int parse_dht(Cursor& cu, Desc& d) {  // njDecodeDHT :577-616
    copen(cu);
    if (cu.err) return cu.err;
    while (cu.seg >= 17) {
        int tc = cu.at[0];
        if (tc & 0xEC) return kSyntaxError;
        if (tc & 0x02) return kUnsupported;
        Huff& t = d.huff[(tc | (tc >> 3)) & 3];
        uint8_t cnt[17];
        cnt[0] = 0;
        for (int L = 1; L <= 16; ++L) cnt[L] = cu.at[L];
        cskip(cu, 17);
        int32_t room = 65536, n = 0;
        for (int L = 1; L <= 16; ++L) {
            if (!cnt[L]) continue;
            if (cu.seg < cnt[L]) return kSyntaxError;
            room -= (int32_t)cnt[L] << (16 - L);
            if (room < 0) return kSyntaxError;
            for (int i = 0; i < cnt[L]; ++i) t.sym[n + i] = cu.at[i];
            n += cnt[L];
            cskip(cu, cnt[L]);
        }
        huff_finalize(t, cnt);
    }
    return cu.seg ? kSyntaxError : cu.err;
}

ICX_HD int parse_dqt(Cursor& cu, Desc& d) {  // njDecodeDQT :618-633
    copen(cu);
    if (cu.err) return cu.err;
    while (cu.seg >= 65) {
        int id = cu.at[0];
        if (id & 0xFC) return kSyntaxError;
        for (int i = 0; i < 64; ++i) d.q[id][i] = cu.at[1 + i];
        cskip(cu, 65);
    }
    return cu.seg ? kSyntaxError : cu.err;
}

ICX_HD int parse_sos(Cursor& cu, Desc& d) {  // njDecodeScan header :678-695
    copen(cu);
    if (cu.err) return cu.err;
    if (cu.seg < 4 + 2 * d.nc) return kSyntaxError;
    if (cu.at[0] != d.nc) return kUnsupported;
    cskip(cu, 1);
    for (int i = 0; i < d.nc; ++i) {
        Comp& c = d.c[i];
        if (cu.at[0] != c.id) return kSyntaxError;
        if (cu.at[1] & 0xEE) return kSyntaxError;
        c.dc_tab = cu.at[1] >> 4;
        c.ac_tab = (cu.at[1] & 1) | 2;
        cskip(cu, 2);
    }
    if (cu.at[0] || cu.at[1] != 63 || cu.at[2]) return kUnsupported;
    cskip(cu, cu.seg);
    return cu.err;
}

// Header walk into a descriptor; returns d.status. With zero = false the caller has already
// zeroed `d` (njInit, jpeg_dec.h:868-870). The fast[] lookup tables are NOT filled here: call
// huff_fill_fast on each table before decoding (k_parse does it with a whole workgroup).
ICX_HD int parse_headers(const uint8_t* file, int64_t size, Desc& d, bool zero = true) {
    if (zero) {
        uint8_t* raw = reinterpret_cast<uint8_t*>(&d);
        for (size_t i = 0; i < sizeof(Desc); ++i) raw[i] = 0;  // njInit :868-870
    }
    d.size = size & 0x7FFFFFFF;
    Cursor cu{file, (int32_t)d.size, 0, 0};
    if (cu.avail < 2 || file[0] != 0xFF || file[1] != 0xD8) return d.status = kNoJpeg;
    cskip(cu, 2);
    for (;;) {
        if (cu.avail < 2 || cu.at[0] != 0xFF) return d.status = kSyntaxError;
        cskip(cu, 2);
        int m = cu.at[-1], r;
        if (m == 0xC0) r = parse_sof(cu, d);
        else if (m == 0xC4) r = parse_dht(cu, d);
        else if (m == 0xDB) r = parse_dqt(cu, d);
        else if (m == 0xDD) {  // njDecodeDRI :635-641
            copen(cu);
            if (cu.err) r = cu.err;
            else if (cu.seg < 2) r = kSyntaxError;
            else { d.restart = be16(cu.at); cskip(cu, cu.seg); r = cu.err; }
        } else if (m == 0xDA) {
            r = parse_sos(cu, d);
            if (r) return d.status = r;
            d.scan_off = (int64_t)(cu.at - file);
            return d.status = kPending;
        } else if (m == 0xFE || (m & 0xF0) == 0xE0) {  // njSkipMarker :518-521
            copen(cu);
            cskip(cu, cu.seg);
            r = cu.err;
        } else {
            return d.status = kUnsupported;
        }
        if (r) return d.status = r;
    }
}

// Component of block r within an MCU, and its (bx, by) inside the component's MCU area.
ICX_HD int mcu_block_comp(const Desc& d, int r, int& sbx, int& sby) {
    int ci = 0;
    while (ci < 2 && r >= d.c[ci].nblk) { r -= d.c[ci].nblk; ++ci; }
    sby = r / d.c[ci].hs;
    sbx = r - sby * d.c[ci].hs;
    return ci;
}

// ---------------------------------------------------------------------------------------
// NanoJPEG bit reader over the raw entropy-coded bytes (njShowBits..njByteAlign,
// jpeg_dec.h:447-498), for the sequential decoder. Past the data (or after FF D9) the
// stream reads as 0xFF; FF 00 and FF FF give one FF data byte; FF Dn pushes both bytes;
// other FF xx, or an FF that ends the file, flags a syntax error.
struct RawBits {
    const uint8_t* at;
    int64_t avail;
    uint32_t acc;
    int32_t nacc, err;
};
ICX_HD void rb_fill(RawBits& b, int want) {
    while (b.nacc < want) {
        if (b.avail <= 0) { b.acc = (b.acc << 8) | 0xFFu; b.nacc += 8; continue; }
        uint32_t x = *b.at++;
        b.avail--;
        b.acc = (b.acc << 8) | x;
        b.nacc += 8;
        if (x != 0xFF) continue;
        if (!b.avail) { b.err = kSyntaxError; continue; }
        uint32_t m = *b.at++;
        b.avail--;
        if (m == 0x00 || m == 0xFF) continue;
        if (m == 0xD9) { b.avail = 0; continue; }
        if ((m & 0xF8) == 0xD0) { b.acc = (b.acc << 8) | m; b.nacc += 8; }
        else b.err = kSyntaxError;
    }
}
ICX_HD uint32_t rb_peek(RawBits& b, int n) {
    if (!n) return 0;
    rb_fill(b, n);
    return (b.acc >> (b.nacc - n)) & ((1u << n) - 1u);
}
ICX_HD void rb_drop(RawBits& b, int n) {
    if (b.nacc < n) rb_fill(b, n);
    b.nacc -= n;
}

// extend a magnitude of `nb` bits to a signed value (jpeg_dec.h:653-654)
ICX_HD int32_t extend(int32_t v, int nb) {
    return v < (1 << (nb - 1)) ? wadd(v, wadd(wshl(-1, nb), 1)) : v;
}

// ---------------------------------------------------------------------------------------
// Integer IDCT (njRowIDCT / njColIDCT, jpeg_dec.h:343-442) including the zero-AC
// shortcuts exactly as the reference tests them (on the shifted values).
enum { kW1 = 2841, kW2 = 2676, kW3 = 2408, kW5 = 1609, kW6 = 1108, kW7 = 565 };

// 24-bit multiply: the low 32 bits of the product of two operands that fit in signed 24 bits,
// i.e. exactly wmul for such operands (v_mul_i32_i24, full rate; v_mul_lo_u32 is quarter rate).
ICX_HD int32_t m24(int32_t a, int32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __mul24(a, b);
#else
    return (int32_t)(uint32_t)((int64_t)a * (int64_t)b);
#endif
}
template <bool F>
ICX_HD int32_t imul(int32_t a, int32_t b) { return F ? m24(a, b) : wmul(a, b); }
// The IDCT passes multiply constants by inputs and by pairwise sums of inputs (the 181 products
// of the last butterfly stay 32-bit): with every multiplied input below 2^22 in magnitude all
// those operands fit in 24 bits, so the F = true instantiation is exact.
ICX_HD bool idct_fast_ok(const int32_t (&v)[8]) {
    const uint32_t lim = 1u << 22;
    auto ok = [&](int32_t x) { return (uint32_t)(x + (int32_t)lim) < 2 * lim; };
    return ok(v[1]) && ok(v[2]) && ok(v[3]) && ok(v[5]) && ok(v[6]) && ok(v[7]);
}

template <bool F = false>
ICX_HD void idct_row(int32_t (&r)[8]) {
    int32_t a4 = wshl(r[4], 11);
    if (!(a4 | r[6] | r[2] | r[1] | r[7] | r[5] | r[3])) {
        int32_t v = wshl(r[0], 3);
        for (int i = 0; i < 8; ++i) r[i] = v;
        return;
    }
    int32_t x0 = wadd(wshl(r[0], 11), 128), x1 = a4, x2 = r[6], x3 = r[2];
    int32_t x4 = r[1], x5 = r[7], x6 = r[5], x7 = r[3], x8;
    x8 = imul<F>(kW7, wadd(x4, x5));
    x4 = wadd(x8, imul<F>(kW1 - kW7, x4));
    x5 = wsub(x8, imul<F>(kW1 + kW7, x5));
    x8 = imul<F>(kW3, wadd(x6, x7));
    x6 = wsub(x8, imul<F>(kW3 - kW5, x6));
    x7 = wsub(x8, imul<F>(kW3 + kW5, x7));
    x8 = wadd(x0, x1);
    x0 = wsub(x0, x1);
    x1 = imul<F>(kW6, wadd(x3, x2));
    x2 = wsub(x1, imul<F>(kW2 + kW6, x2));
    x3 = wadd(x1, imul<F>(kW2 - kW6, x3));
    x1 = wadd(x4, x6);
    x4 = wsub(x4, x6);
    x6 = wadd(x5, x7);
    x5 = wsub(x5, x7);
    x7 = wadd(x8, x3);
    x8 = wsub(x8, x3);
    x3 = wadd(x0, x2);
    x0 = wsub(x0, x2);
    x2 = wadd(wmul(181, wadd(x4, x5)), 128) >> 8;
    x4 = wadd(wmul(181, wsub(x4, x5)), 128) >> 8;
    r[0] = wadd(x7, x1) >> 8;
    r[1] = wadd(x3, x2) >> 8;
    r[2] = wadd(x0, x4) >> 8;
    r[3] = wadd(x8, x6) >> 8;
    r[4] = wsub(x8, x6) >> 8;
    r[5] = wsub(x0, x4) >> 8;
    r[6] = wsub(x3, x2) >> 8;
    r[7] = wsub(x7, x1) >> 8;
}

// Column pass: v[i] = coefficient row i of one column; writes 8 clipped samples.
template <bool F = false>
ICX_HD void idct_col(const int32_t (&v)[8], uint8_t (&out)[8]) {
    int32_t a4 = wshl(v[4], 8);
    if (!(a4 | v[6] | v[2] | v[1] | v[7] | v[5] | v[3])) {
        uint8_t s = clip8(wadd(wadd(v[0], 32) >> 6, 128));
        for (int i = 0; i < 8; ++i) out[i] = s;
        return;
    }
    int32_t x0 = wadd(wshl(v[0], 8), 8192), x1 = a4, x2 = v[6], x3 = v[2];
    int32_t x4 = v[1], x5 = v[7], x6 = v[5], x7 = v[3], x8;
    x8 = wadd(imul<F>(kW7, wadd(x4, x5)), 4);
    x4 = wadd(x8, imul<F>(kW1 - kW7, x4)) >> 3;
    x5 = wsub(x8, imul<F>(kW1 + kW7, x5)) >> 3;
    x8 = wadd(imul<F>(kW3, wadd(x6, x7)), 4);
    x6 = wsub(x8, imul<F>(kW3 - kW5, x6)) >> 3;
    x7 = wsub(x8, imul<F>(kW3 + kW5, x7)) >> 3;
    x8 = wadd(x0, x1);
    x0 = wsub(x0, x1);
    x1 = wadd(imul<F>(kW6, wadd(x3, x2)), 4);
    x2 = wsub(x1, imul<F>(kW2 + kW6, x2)) >> 3;
    x3 = wadd(x1, imul<F>(kW2 - kW6, x3)) >> 3;
    x1 = wadd(x4, x6);
    x4 = wsub(x4, x6);
    x6 = wadd(x5, x7);
    x5 = wsub(x5, x7);
    x7 = wadd(x8, x3);
    x8 = wsub(x8, x3);
    x3 = wadd(x0, x2);
    x0 = wsub(x0, x2);
    x2 = wadd(wmul(181, wadd(x4, x5)), 128) >> 8;
    x4 = wadd(wmul(181, wsub(x4, x5)), 128) >> 8;
    out[0] = clip8(wadd(wadd(x7, x1) >> 14, 128));
    out[1] = clip8(wadd(wadd(x3, x2) >> 14, 128));
    out[2] = clip8(wadd(wadd(x0, x4) >> 14, 128));
    out[3] = clip8(wadd(wadd(x8, x6) >> 14, 128));
    out[4] = clip8(wadd(wsub(x8, x6) >> 14, 128));
    out[5] = clip8(wadd(wsub(x0, x4) >> 14, 128));
    out[6] = clip8(wadd(wsub(x3, x2) >> 14, 128));
    out[7] = clip8(wadd(wsub(x7, x1) >> 14, 128));
}

// ---------------------------------------------------------------------------------------
// Bicubic chroma doubling taps (jpeg_dec.h:722-734): CF(x) = clip((x + 64) >> 7).
ICX_HD uint8_t cf(int32_t x) { return clip8((x + 64) >> 7); }
ICX_HD uint8_t tap2(int a, int b) { return cf(139 * a - 11 * b); }
ICX_HD uint8_t tap3x(int a, int b, int c) { return cf(104 * a + 27 * b - 3 * c); }
ICX_HD uint8_t tap3a(int a, int b, int c) { return cf(28 * a + 109 * b - 9 * c); }
ICX_HD uint8_t tap4(int a, int b, int c, int e) { return cf(-9 * a + 111 * b + 29 * c - 3 * e); }

// One output sample of a doubling pass along a line of n real samples. `at(i)` returns
// sample i; the edge samples (outputs n2-3..n2-1) come from `end(j)` = the j-th sample
// counted back from the line's end: for the horizontal pass that end is the row STRIDE
// (jpeg_dec.h:752-756), for the vertical pass the last real row (:782-785).
template <class At, class End>
ICX_HD uint8_t double_tap(int o, int n, At at, End end) {
    const int n2 = n << 1;
    if (o == 0) return tap2(at(0), at(1));
    if (o == 1) return tap3x(at(0), at(1), at(2));
    if (o == 2) return tap3a(at(0), at(1), at(2));
    if (o == n2 - 3) return tap3a(end(1), end(2), end(3));
    if (o == n2 - 2) return tap3x(end(1), end(2), end(3));
    if (o == n2 - 1) return tap2(end(1), end(2));
    const int x = (o - 3) >> 1;  // 4 taps on samples x..x+3
    return (o & 1) ? tap4(at(x), at(x + 1), at(x + 2), at(x + 3))
                   : tap4(at(x + 3), at(x + 2), at(x + 1), at(x));
}

// YCbCr -> RGB (jpeg_dec.h:843-848)
ICX_HD void ycc_to_rgb(int y, int cb, int cr, uint8_t* o) {
    const int32_t Y = y << 8, b = cb - 128, r = cr - 128;
    o[0] = clip8((Y + 359 * r + 128) >> 8);
    o[1] = clip8((Y - 88 * b - 183 * r + 128) >> 8);
    o[2] = clip8((Y + 454 * b + 128) >> 8);
}

}  // namespace icx
