// icx_hdr.hip -- Radiance .hdr (RGBE) decode on gfx950: Image::readHdr (codecs.cpp:706-777) with
// decrunchHDR (:662-703), oldDecrunchHDR (:630-660) and workOnRGBE (:617-628).
//
// The file is one serial byte stream: where scanline y starts depends on how every earlier
// scanline was coded. The common files are located in parallel and only the rest is walked:
//   k_hdr_parse      header walk (:713-750), one lane per image
//   k_hdr_scan       every byte of the pixel data: new-style scanline starts "2 2 w>>8 w&255"
//   k_hdr_candwalk   one lane per start found: walk that scanline to its end
//                    (their ends found by walking the 4 run-length coded components), and
//                    old-style run markers R=G=B=1 (:643-645)
//   k_hdr_flatcheck  flat files: is row y, at ds + 4*w*y, a plain RGBE row?
//   k_hdr_link       new-RLE files: sort the scanline starts, check that each one ends where the
//                    next begins, starting at the data start
//   k_hdr_walk       otherwise one lane replays the reference's scanline loop (exact, serial)
//   k_hdr_unpack     one wave per new-style scanline: the 4 component streams -> RGBE planes
//   k_hdr_convert    RGBE -> 4 floats per pixel, 16-byte stores
// convertComponent (:610-615) is (v / 256.0f) * (float)pow(2, e - 128): v has 8 significant bits,
// so the product v * 2^(e-136) is exact in binary32 (the smallest, 2^-136, is above the 2^-149
// subnormal floor) and ldexpf gives the same bits: epsilon = 0.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "icx_internal.h"

namespace icx {

constexpr int kHdrCandCap = 8192;  // new-style scanline starts sorted per image in k_hdr_link

ICX_HD bool hdr_space(int c) { return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r'; }

// strtol over [p, end): optional whitespace, sign, decimal digits. Returns false if no digits.
ICX_HD bool hdr_long(const char* p, const char* end, const char** next, int64_t* v) {
    while (p < end && hdr_space(*p)) ++p;
    bool neg = false;
    if (p < end && (*p == '+' || *p == '-')) { neg = *p == '-'; ++p; }
    const char* q = p;
    int64_t x = 0;
    while (p < end && *p >= '0' && *p <= '9') {
        if (x < (int64_t)1 << 40) x = x * 10 + (*p - '0');
        ++p;
    }
    if (p == q) return false;
    *v = neg ? -x : x;
    *next = p;
    return true;
}

// readHdr's header walk (codecs.cpp:713-750) -> kHdrOk and w, h, data start; else the error code.
// sscanf(reso, "-Y %ld +X %ld") (:745) must fill both fields (the reference reads w uninitialised
// when only h matches); sizes must be positive (w*h <= 2^30).
ICX_HD int hdr_parse(const uint8_t* d, int64_t n, int* w, int* h, int64_t* ds) {
    const char magic[10] = {'#', '?', 'R', 'A', 'D', 'I', 'A', 'N', 'C', 'E'};
    if (n < 10) return kHdrNotRadiance;
    for (int i = 0; i < 10; ++i)
        if (d[i] != (uint8_t)magic[i]) return kHdrNotRadiance;
    int64_t pos = 11;  // fseek(file, 1, SEEK_CUR) past the magic (:722)
    int c = 0, oldc;
    for (;;) {  // header lines up to an empty line (:727-734)
        oldc = c;
        if (pos >= n) return kHdrBadHeader;  // the reference loops forever at EOF
        c = d[pos++];
        if (c == 0xa && oldc == 0xa) break;
    }
    char reso[256];
    int k = 0;
    for (;;) {  // resolution line (:737-743)
        if (pos >= n || k >= 255) return kHdrBadHeader;
        reso[k] = (char)d[pos++];
        if (reso[k++] == 0xa) break;
    }
    const char* end = reso + k;
    const char* p = reso;
    int64_t hh, ww;
    if (k < 2 || p[0] != '-' || p[1] != 'Y') return kHdrBadHeader;
    if (!hdr_long(p + 2, end, &p, &hh)) return kHdrBadHeader;
    while (p < end && hdr_space(*p)) ++p;
    if (end - p < 2 || p[0] != '+' || p[1] != 'X') return kHdrBadHeader;
    if (!hdr_long(p + 2, end, &p, &ww)) return kHdrBadHeader;
    if (hh <= 0 || ww <= 0 || hh > (1 << 20) || ww > (1 << 20) || hh * ww > ((int64_t)1 << 30)) return kHdrBadHeader;
    *w = (int)ww;
    *h = (int)hh;
    *ds = pos;
    return kHdrOk;
}

// The 4 run-length coded components of a new-style scanline whose 4-byte header is at p
// (decrunchHDR :686-700). Returns the byte after it, or -1 (a run or literal overflows the
// scanline: undefined in the reference), -2 (the file ends first: decrunchHDR returns false),
// -3 (more than `cap` bytes: left to the serial walk).
ICX_HD int64_t hdr_walk_new(const uint8_t* d, int64_t n, int64_t p, int w, int64_t cap) {
    int64_t pos = p + 4;
    if (pos > n) return -2;
    const int64_t lim = cap > 0 ? p + cap : INT64_MAX;
    for (int c = 0; c < 4; ++c) {
        for (int j = 0; j < w;) {
            if (pos >= lim) return -3;
            if (pos >= n) return -2;
            int code = d[pos++];
            if (code > 128) {
                code &= 127;
                if (pos >= n) return -2;
                ++pos;  // the run value
                if (j + code > w) return -1;
                j += code;
            } else {
                if (j + code > w) return -1;
                if (pos + code > n) return -2;
                pos += code;
                j += code;
            }
        }
    }
    return pos;
}

enum : int32_t { kRowFlat = 0, kRowNew = 1, kRowStaged = 2 };

__device__ __forceinline__ void hdr_put_px(uint8_t* plane, int w, int x, const uint8_t* px) {
#pragma unroll
    for (int c = 0; c < 4; ++c) plane[(int64_t)c * w + x] = px[c];
}

__global__ void k_hdr_parse(int n, const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
                            const uint64_t* __restrict__ size, HdrDesc* __restrict__ desc, int max_w, int max_h) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    HdrDesc dd{};
    dd.size = (int64_t)size[i];
    int w = 0, h = 0;
    int64_t ds = 0;
    dd.status = hdr_parse(data + off[i], dd.size, &w, &h, &ds);
    if (dd.status == kHdrOk) {
        dd.status = (w > max_w || h > max_h) ? kHdrTooLarge : kHdrPending;
        dd.w = w;
        dd.h = h;
        dd.ds = ds;
    }
    desc[i] = dd;
}

// grid (x: byte chunks, y: image)
__global__ __launch_bounds__(256) void k_hdr_scan(const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
                                                  HdrDesc* __restrict__ desc, int32_t* __restrict__ cq,
                                                  int32_t* __restrict__ ce) {
    const int i = blockIdx.y;
    HdrDesc& dd = desc[i];
    if (dd.status != kHdrPending) return;
    const uint8_t* d = data + off[i];
    const int64_t n = dd.size, ds = dd.ds;
    const int w = dd.w;
    const bool newfmt = w >= 8 && w <= 0x7fff;
    bool marker = false;
    auto found = [&](int64_t qk) {  // a new-style scanline start at data offset qk
        const int s = atomicAdd(&dd.ncand, 1);  // its end: k_hdr_candwalk
        if (s < kHdrCandCap) cq[(int64_t)i * kHdrCandCap + s] = (int32_t)qk;
    };
    const uint32_t pat = 2u | 2u << 8 | (uint32_t)((w >> 8) & 255) << 16 | (uint32_t)(w & 255) << 24;
    // 16 positions per lane: six aligned dwords, realigned to p with alignbyte, give the 19 bytes
    // the four 4-byte groups and sixteen candidate windows need
    for (int64_t q = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; ds + q < n;
         q += (int64_t)gridDim.x * blockDim.x * 16) {
        const int64_t p = ds + q;
        if (p + 24 <= n) {
            const uintptr_t a = reinterpret_cast<uintptr_t>(d + p);
            const uint32_t mis = (uint32_t)(a & 3);
            const uint32_t* g = reinterpret_cast<const uint32_t*>(a - mis);
            uint32_t W[6], A[5];
#pragma unroll
            for (int k = 0; k < 6; ++k) W[k] = g[k];
#pragma unroll
            for (int k = 0; k < 5; ++k) A[k] = __builtin_amdgcn_alignbyte(W[k + 1], W[k], mis);  // bytes p+4k..
#pragma unroll
            for (int k = 0; k < 4; ++k) marker |= (A[k] & 0xFFFFFFu) == 0x010101u;  // aligned groups (:644)
            if (!newfmt) continue;
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const uint32_t v = (k & 3) ? __builtin_amdgcn_alignbyte(A[(k >> 2) + 1], A[k >> 2], (uint32_t)(k & 3))
                                           : A[k >> 2];
                if (v == pat) found(q + k);
            }
            continue;
        }
        for (int grp = 0; grp < 4; ++grp) {  // the file's last bytes, one at a time
            const int64_t qq = q + 4 * grp, pp = ds + qq;
            if (pp >= n) break;
            const int nb = (int)min<int64_t>(4, n - pp);
            uint8_t b[7];
#pragma unroll
            for (int k = 0; k < 7; ++k) b[k] = pp + k < n ? d[pp + k] : 0;
            marker |= nb == 4 && b[0] == 1 && b[1] == 1 && b[2] == 1;  // aligned groups (oldDecrunchHDR :644)
            if (!newfmt) continue;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (k < nb && pp + k + 3 < n && b[k] == 2 && b[k + 1] == 2 && b[k + 2] == (w >> 8) && b[k + 3] == (w & 255))
                    found(qq + k);
        }
    }
    if (__any(marker) && (threadIdx.x & 63) == 0) atomicOr(&dd.has_marker, 1);
}

// grid (x: candidate chunks, y: image): one lane per scanline start k_hdr_scan found walks that
// scanline's four run-length coded components to its end (hdr_walk_new). Walking in the scan
// itself left 63 of 64 lanes idle behind each walking lane; here every lane walks.
__global__ __launch_bounds__(256) void k_hdr_candwalk(const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
                                                      const HdrDesc* __restrict__ desc, const int32_t* __restrict__ cq,
                                                      int32_t* __restrict__ ce) {
    const int i = blockIdx.y;
    const HdrDesc& dd = desc[i];
    if (dd.status != kHdrPending) return;
    const int nc = min(dd.ncand, kHdrCandCap);
    const uint8_t* d = data + off[i];
    const int64_t n = dd.size, ds = dd.ds, cap = 16 * (int64_t)dd.w + 64;
    for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < nc; s += gridDim.x * blockDim.x) {
        const int64_t e = hdr_walk_new(d, n, ds + cq[(int64_t)i * kHdrCandCap + s], dd.w, cap);
        ce[(int64_t)i * kHdrCandCap + s] = e >= 0 ? (int32_t)(e - ds) : (int32_t)e;
    }
}

// grid (x: row chunks, y: image). Row y of a flat file starts at ds + 4*w*y; it is decoded as a
// plain row unless its first bytes select the new-style decoder (decrunchHDR :666-683).
__global__ __launch_bounds__(256) void k_hdr_flatcheck(const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
                                                       HdrDesc* __restrict__ desc) {
    const int i = blockIdx.y;
    HdrDesc& dd = desc[i];
    if (dd.status != kHdrPending) return;
    const uint8_t* d = data + off[i];
    const int64_t n = dd.size, rowb = 4 * (int64_t)dd.w;
    const bool newfmt = dd.w >= 8 && dd.w <= 0x7fff;
    if (blockIdx.x == 0 && threadIdx.x == 0 && dd.ds + rowb * dd.h > n) atomicOr(&dd.not_flat, 1);
    bool bad = false;
    for (int y = blockIdx.x * blockDim.x + threadIdx.x; y < dd.h; y += gridDim.x * blockDim.x) {
        const int64_t p = dd.ds + rowb * y;
        bad |= newfmt && p + 2 < n && d[p] == 2 && d[p + 1] == 2 && !(d[p + 2] & 128);
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(&dd.not_flat, 1);
}

// One workgroup per image: sort the new-style scanline starts found by k_hdr_scan and accept the
// chain if the first is at the data start and each scanline ends where the next one starts.
__global__ __launch_bounds__(1024) void k_hdr_link(HdrDesc* __restrict__ desc, const int32_t* __restrict__ cq,
                                                   const int32_t* __restrict__ ce, int64_t* __restrict__ start,
                                                   int max_h) {
    __shared__ uint64_t key[kHdrCandCap];
    __shared__ int s_ok;
    const int i = blockIdx.x;
    HdrDesc& dd = desc[i];
    if (dd.status != kHdrPending || dd.ncand < dd.h || dd.ncand > kHdrCandCap) return;
    const int nc = dd.ncand;
    int np = 1;
    while (np < nc) np <<= 1;
    for (int k = threadIdx.x; k < np; k += blockDim.x)
        key[k] = k < nc ? ((uint64_t)(uint32_t)cq[(int64_t)i * kHdrCandCap + k] << 32) |
                              (uint32_t)ce[(int64_t)i * kHdrCandCap + k]
                        : ~0ull;
    if (threadIdx.x == 0) s_ok = 1;
    __syncthreads();
    for (int kk = 2; kk <= np; kk <<= 1) {  // bitonic sort by position
        for (int j = kk >> 1; j > 0; j >>= 1) {
            for (int t = threadIdx.x; t < np; t += blockDim.x) {
                const int u = t ^ j;
                if (u > t) {
                    const uint64_t a = key[t], b = key[u];
                    const bool up = (t & kk) == 0;
                    if ((a > b) == up) { key[t] = b; key[u] = a; }
                }
            }
            __syncthreads();
        }
    }
    const int h = dd.h;
    for (int y = threadIdx.x; y < h; y += blockDim.x) {
        const int32_t q = (int32_t)(key[y] >> 32), e = (int32_t)(uint32_t)key[y];
        bool ok = e > 0 && (y > 0 || q == 0);
        if (y + 1 < h) ok = ok && e == (int32_t)(key[y + 1] >> 32);
        if (!ok) s_ok = 0;
    }
    __syncthreads();
    if (!s_ok) return;
    for (int y = threadIdx.x; y < h; y += blockDim.x) start[(int64_t)i * max_h + y] = dd.ds + (int64_t)(key[y] >> 32);
    if (threadIdx.x == 0) dd.new_ok = 1;
}

// oldDecrunchHDR (codecs.cpp:630-660) for pixels x0 .. x0+npix-1 of a row, into its RGBE planes.
// Returns 1, 0 (end of file: the reference's false), or -1 (undefined in the reference).
__device__ int hdr_old_serial(const uint8_t* d, int64_t n, int64_t& pos, uint8_t* plane, int w, int x0, int npix) {
    int rshift = 0, x = x0, len = npix;
    uint8_t prev[4] = {0, 0, 0, 0};
    if (x0 > 0)
#pragma unroll
        for (int c = 0; c < 4; ++c) prev[c] = plane[(int64_t)c * w + x0 - 1];
    while (len > 0) {
        uint8_t px[4];
        bool eof = false;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (pos < n) px[c] = d[pos++];
            else { px[c] = 0xFF; eof = true; }
        }
        if (eof) return 0;
        if (px[0] == 1 && px[1] == 1 && px[2] == 1) {
            if (rshift >= 32) return -1;  // an over-wide shift (:646)
            const int64_t cnt = (int64_t)px[3] << rshift;
            if (cnt > len || (cnt > 0 && x == 0)) return -1;  // past the scanline, or scanline[-1]
            for (int k = 0; k < cnt; ++k) hdr_put_px(plane, w, x++, prev);
            len -= cnt;
            rshift += 8;
        } else {
            hdr_put_px(plane, w, x++, px);
#pragma unroll
            for (int c = 0; c < 4; ++c) prev[c] = px[c];
            len -= 1;
            rshift = 0;
        }
    }
    return 1;
}

// One lane per image: all-flat and all-new-style files are already located; anything else is
// replayed scanline by scanline exactly as readHdr's loop (:765-776) reads it.
__global__ void k_hdr_walk(int n, const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
                           HdrDesc* __restrict__ desc, int64_t* __restrict__ start, uint8_t* __restrict__ kind,
                           uint8_t* __restrict__ planes, int max_w, int max_h) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    HdrDesc& dd = desc[i];
    if (dd.status != kHdrPending) return;
    const int w = dd.w, h = dd.h;
    if (!dd.has_marker && !dd.not_flat) { dd.mode = 1; dd.rows = h; dd.status = kHdrOk; return; }
    if (dd.new_ok) { dd.mode = 2; dd.rows = h; dd.status = kHdrOk; return; }
    dd.mode = 3;
    const uint8_t* d = data + off[i];
    const int64_t fsz = dd.size;
    int64_t* S = start + (int64_t)i * max_h;
    uint8_t* K = kind + (int64_t)i * max_h;
    const bool newfmt = w >= 8 && w <= 0x7fff;
    int64_t pos = dd.ds;
    int status = kHdrOk, y = 0;
    for (; y < h; ++y) {
        uint8_t* plane = planes + ((int64_t)i * max_h + y) * 4 * max_w;
        int r;
        int x0 = 0;
        int64_t row0 = pos;
        if (newfmt) {
            const int b0 = pos < fsz ? d[pos] : -1;
            if (pos < fsz) ++pos;
            if (b0 != 2) {
                pos -= 1;  // fseek(file, -1, SEEK_CUR) (:671), also at end of file
            } else {
                uint8_t px[4] = {2, 0xFF, 0xFF, 0xFF};
                for (int c = 1; c < 4; ++c)
                    if (pos < fsz) px[c] = d[pos++];
                if (px[1] == 2 && !(px[2] & 128)) {  // new-style scanline (:686-700)
                    const int64_t e = hdr_walk_new(d, fsz, row0, w, 0);
                    if (e < 0) { status = e == -1 ? kHdrMalformed : kHdrTruncated; break; }
                    S[y] = row0;
                    K[y] = kRowNew;
                    pos = e;
                    continue;
                }
                // (2, G, B, E) is pixel 0, then old-style from pixel 1 (:679-683); a read past
                // the end leaves the EOF flag set, so the next 4-byte read fails
                if (pos - row0 < 4) { status = kHdrTruncated; break; }
                hdr_put_px(plane, w, 0, px);
                x0 = 1;
            }
        }
        const int npix = w - x0;
        if (!dd.has_marker && ((pos - dd.ds) & 3) == 0 && pos + 4 * (int64_t)npix <= fsz) {
            S[y] = pos - 4 * x0;  // plain RGBE: pixel x at S + 4x (pixel 0 included)
            K[y] = kRowFlat;
            pos += 4 * (int64_t)npix;
            continue;
        }
        r = hdr_old_serial(d, fsz, pos, plane, w, x0, npix);
        if (r <= 0) { status = r < 0 ? kHdrMalformed : kHdrTruncated; break; }
        K[y] = kRowStaged;
    }
    dd.rows = y;
    dd.status = status;
}

// One wave per new-style row: the row's packet stream is staged through a 4 KB LDS window per wave
// (coalesced 16-byte loads), so the wave-uniform chain of packet headers runs at LDS latency
// instead of one dependent global load per packet; literal bytes and runs are written by the
// lanes into the row's 4 component planes. The window is refilled at the current packet whenever
// fewer than 129 bytes (the longest packet: code 128 + 128 literals) remain in it; bytes past the
// file end are never read. grid (x: row chunks of 4 waves, y: image)
constexpr int kHdrWin = 4096;
__global__ __launch_bounds__(256) void k_hdr_unpack(const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
                                                    const HdrDesc* __restrict__ desc, const int64_t* __restrict__ start,
                                                    const uint8_t* __restrict__ kind, uint8_t* __restrict__ planes,
                                                    int max_w, int max_h) {
    __shared__ __attribute__((aligned(16))) uint8_t win_all[4][kHdrWin];
    const int i = blockIdx.y;
    const HdrDesc& dd = desc[i];
    if (dd.mode != 2 && dd.mode != 3) return;
    const uint8_t* d = data + off[i];
    const int64_t fsize = dd.size;
    const int w = dd.w, lane = threadIdx.x & 63;
    uint8_t* win = win_all[threadIdx.x >> 6];
    for (int y = blockIdx.x * 4 + (threadIdx.x >> 6); y < dd.rows; y += gridDim.x * 4) {
        if (dd.mode == 3 && kind[(int64_t)i * max_h + y] != kRowNew) continue;
        int64_t pos = start[(int64_t)i * max_h + y] + 4;
        int64_t base = 0, lim = -1;  // window holds file bytes [base, base + kHdrWin); refill past lim
        uint8_t* plane = planes + ((int64_t)i * max_h + y) * 4 * max_w;
        for (int c = 0; c < 4; ++c) {
            uint8_t* pc = plane + (int64_t)c * w;
            for (int j = 0; j < w;) {
                if (pos > lim) {
                    // base: pos rounded down so that d + base is 16-byte aligned
                    base = pos - (int64_t)(reinterpret_cast<uintptr_t>(d + pos) & 15);
                    lim = base + kHdrWin - 129;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
#pragma unroll
                    for (int q = 0; q < kHdrWin / (64 * 16); ++q) {
                        const int o = (q * 64 + lane) * 16;
                        const int64_t a = base + o;
                        uint4 v = make_uint4(0, 0, 0, 0);
                        if (a >= 0 && a + 16 <= fsize) {
                            v = *reinterpret_cast<const uint4*>(d + a);
                        } else {
                            uint32_t t[4] = {0, 0, 0, 0};
                            for (int b = 0; b < 16; ++b)
                                if (a + b >= 0 && a + b < fsize) t[b >> 2] |= (uint32_t)d[a + b] << (8 * (b & 3));
                            v = make_uint4(t[0], t[1], t[2], t[3]);
                        }
                        *reinterpret_cast<uint4*>(win + o) = v;
                    }
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                }
                const uint8_t* p = win + (pos - base);
                int code = p[0];
                if (code > 128) {
                    code &= 127;
                    const uint8_t v = p[1];
                    for (int k = lane; k < code; k += 64) pc[j + k] = v;
                    pos += 2;
                } else {
                    for (int k = lane; k < code; k += 64) pc[j + k] = p[1 + k];
                    pos += 1 + code;
                }
                j += code;
            }
        }
    }
}

// The rows of one image, one pixel (16 bytes out) per lane. VEC: the image base is 16-byte
// aligned and each pixel leaves as one float4 store; otherwise four float stores (out_stride is
// any number of floats). Two instantiations, chosen once per image: a per-store branch on the
// alignment halved the kernel's rate (2.1 -> 4.1 ms per 32 images).
template <bool VEC>
__device__ __forceinline__ void hdr_convert_rows(const HdrDesc& dd, const uint8_t* d, int i, const int64_t* start,
                                                 const uint8_t* kind, const uint8_t* planes, float* fo, int max_w,
                                                 int max_h) {
    const int w = dd.w;
    float4* o = reinterpret_cast<float4*>(fo);
    auto put = [&](float4* p, const float4& v) {
        if (VEC) {
            *p = v;
        } else {
            float* q = reinterpret_cast<float*>(p);
            q[0] = v.x; q[1] = v.y; q[2] = v.z; q[3] = v.w;
        }
    };
    for (int y = blockIdx.x; y < dd.h; y += gridDim.x) {
        float4* orow = o + (int64_t)y * w;
        if (y >= dd.rows) {  // rows after a failed scanline (uninitialised in the reference)
            for (int x = threadIdx.x; x < w; x += blockDim.x) put(orow + x, make_float4(0.f, 0.f, 0.f, 0.f));
            continue;
        }
        int k = kRowFlat;
        int64_t s = dd.ds + 4 * (int64_t)w * y;
        if (dd.mode == 2) k = kRowNew;
        else if (dd.mode == 3) { k = kind[(int64_t)i * max_h + y]; s = start[(int64_t)i * max_h + y]; }
        const uint8_t* plane = planes + ((int64_t)i * max_h + y) * 4 * max_w;
        // flat rows: one aligned dword (two when the row is not 4-byte aligned, realigned with
        // alignbyte) per pixel instead of four byte loads; the row's last pixel may not read past
        // the file
        const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(d + s) & 3);
        const uint32_t* g4 = reinterpret_cast<const uint32_t*>(d + s - mis);
        const int xfast = mis && s + 4 * (int64_t)w + 4 > dd.size ? w - 1 : w;  // pixels with a safe 2nd dword
        for (int x = threadIdx.x; x < w; x += blockDim.x) {
            uint32_t r, g, b, e;
            if (k == kRowFlat) {
                uint32_t v;
                if (x < xfast) {
                    v = g4[x];
                    if (mis) v = __builtin_amdgcn_alignbyte(g4[x + 1], v, mis);
                } else {
                    const uint8_t* p = d + s + 4 * (int64_t)x;
                    v = (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
                }
                r = v & 255u; g = (v >> 8) & 255u; b = (v >> 16) & 255u; e = v >> 24;
            } else {
                r = plane[x]; g = plane[w + x]; b = plane[2 * w + x]; e = plane[3 * w + x];
            }
            const int ex = (int)e - 136;
            put(orow + x, make_float4(ldexpf((float)r, ex), ldexpf((float)g, ex), ldexpf((float)b, ex), (float)e));
        }
    }
}

// grid (x: row chunks, y: image); 256 lanes across a row, one pixel (16 bytes out) each.
__global__ __launch_bounds__(256) void k_hdr_convert(const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
                                                     const HdrDesc* __restrict__ desc, const int64_t* __restrict__ start,
                                                     const uint8_t* __restrict__ kind, const uint8_t* __restrict__ planes,
                                                     float* __restrict__ out, uint64_t out_stride, int max_w, int max_h) {
    const int i = blockIdx.y;
    const HdrDesc& dd = desc[i];
    if (dd.mode == 0) return;
    float* const fo = out + (int64_t)i * out_stride;
    if ((reinterpret_cast<uintptr_t>(fo) & 15) == 0)  // uniform per workgroup
        hdr_convert_rows<true>(dd, data + off[i], i, start, kind, planes, fo, max_w, max_h);
    else
        hdr_convert_rows<false>(dd, data + off[i], i, start, kind, planes, fo, max_w, max_h);
}

__global__ void k_hdr_finish(int n, HdrDesc* __restrict__ desc, int32_t* __restrict__ status, int32_t* __restrict__ dims) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const HdrDesc& dd = desc[i];
    status[i] = dd.status;
    const bool sized = dd.status == kHdrOk || dd.status == kHdrMalformed || dd.status == kHdrTruncated;
    dims[3 * i + 0] = sized ? dd.w : 0;
    dims[3 * i + 1] = sized ? dd.h : 0;
    dims[3 * i + 2] = sized ? dd.rows : 0;
}

// ------------------------------------------------------------------------------- host
int hdr_probe(const uint8_t* data, int64_t size, int* w, int* h) {
    int64_t ds;
    return hdr_parse(data, size, w, h, &ds);
}

int64_t hdr_ws_bytes(int max_images, int max_w, int max_h) {
    return (int64_t)max_images * ((int64_t)sizeof(HdrDesc) + 8LL * kHdrCandCap + 9LL * max_h +
                                  4LL * max_w * max_h);
}

bool hdr_ws_alloc(HdrWs& ws, int max_images, int max_w, int max_h) {
    ws.max_images = max_images;
    ws.max_w = max_w;
    ws.max_h = max_h;
    const size_t n = (size_t)max_images;
    return hipMalloc(&ws.desc, n * sizeof(HdrDesc)) == hipSuccess &&
           hipMalloc(&ws.cq, n * kHdrCandCap * 4) == hipSuccess && hipMalloc(&ws.ce, n * kHdrCandCap * 4) == hipSuccess &&
           hipMalloc(&ws.start, n * max_h * 8) == hipSuccess && hipMalloc(&ws.kind, n * max_h) == hipSuccess &&
           hipMalloc(&ws.planes, n * (size_t)max_h * 4 * max_w) == hipSuccess;
}

void hdr_ws_free(HdrWs& ws) {
    (void)hipFree(ws.desc);
    (void)hipFree(ws.cq);
    (void)hipFree(ws.ce);
    (void)hipFree(ws.start);
    (void)hipFree(ws.kind);
    (void)hipFree(ws.planes);
    ws = HdrWs{};
}

void launch_hdr_decode(const HdrWs& ws, int n, const uint8_t* d_data, const uint64_t* d_off, const uint64_t* d_size,
                       float* d_out, uint64_t out_stride, int32_t* d_status, int32_t* d_dims, hipStream_t st,
                       StageHook* hook) {
    if (n <= 0) return;
    auto B = [&](Stage s) { if (hook) hook->begin(s, st); };
    auto E = [&](Stage s) { if (hook) hook->end(s, st); };
    const int nb = (n + 63) / 64;
    const int gx = std::max(1, std::min(2048, 16384 / n));
    B(kStParse);
    hipLaunchKernelGGL(k_hdr_parse, dim3(nb), dim3(64), 0, st, n, d_data, d_off, d_size, ws.desc, ws.max_w, ws.max_h);
    E(kStParse);
    B(kStUnstuff);  // locating the scanlines
    hipLaunchKernelGGL(k_hdr_scan, dim3(gx, n), dim3(256), 0, st, d_data, d_off, ws.desc, ws.cq, ws.ce);
    hipLaunchKernelGGL(k_hdr_candwalk, dim3(kHdrCandCap / 256, n), dim3(256), 0, st, d_data, d_off, ws.desc, ws.cq,
                       ws.ce);
    hipLaunchKernelGGL(k_hdr_flatcheck, dim3(std::max(1, std::min(gx, (ws.max_h + 255) / 256)), n), dim3(256), 0, st,
                       d_data, d_off, ws.desc);
    hipLaunchKernelGGL(k_hdr_link, dim3(n), dim3(1024), 0, st, ws.desc, ws.cq, ws.ce, ws.start, ws.max_h);
    hipLaunchKernelGGL(k_hdr_walk, dim3(nb), dim3(64), 0, st, n, d_data, d_off, ws.desc, ws.start, ws.kind, ws.planes,
                       ws.max_w, ws.max_h);
    E(kStUnstuff);
    B(kStEntropy);  // run-length decoding
    hipLaunchKernelGGL(k_hdr_unpack, dim3(std::max(1, std::min(gx, (ws.max_h + 3) / 4)), n), dim3(256), 0, st, d_data,
                       d_off, ws.desc, ws.start, ws.kind, ws.planes, ws.max_w, ws.max_h);
    E(kStEntropy);
    B(kStConvert);
    hipLaunchKernelGGL(k_hdr_convert, dim3(std::max(1, std::min(gx, ws.max_h)), n), dim3(256), 0, st, d_data, d_off,
                       ws.desc, ws.start, ws.kind, ws.planes, d_out, out_stride, ws.max_w, ws.max_h);
    hipLaunchKernelGGL(k_hdr_finish, dim3(nb), dim3(64), 0, st, n, ws.desc, d_status, d_dims);
    E(kStConvert);
}

}  // namespace icx
