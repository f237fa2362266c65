// icx_png.hip -- gfx950 PNG encoder behind png_encoder::saveToFile (png_encoder.cpp:4474-4486).
//
// Parity contract: lodepng's colour-mode choice and filter bytes are
// reproduced exactly (lodepng_compute_color_stats :3357-3543, auto_choose_color :3552-3616,
// filter :3935-3983 with LFS_MINSUM and filter_palette_zero); the IDAT is a valid zlib stream
// that inflates to that identical filtered stream. The deflate is our own segment-parallel
// coder (lodepng's single shared hash chain, png_encoder.cpp:1840, is inherently serial).
//
//   k_png_stats      colour statistics: colored, alpha cases, grey bit needs, first transparent
//                    pixel, distinct colours (LDS set per workgroup -> global set, capped at 257)
//   k_png_keycheck   the colour-key cases (:3518-3528) once the key colour is known
//   k_png_convert    lodepng_convert to the chosen mode (palette index / grey bits / drop alpha),
//                    rows padded to whole bytes (preProcessScanlines)
//   k_png_filter     one workgroup per row: the five filters, MINSUM scores, strict-< choice,
//                    filtered row with its type byte
//   k_png_lz77       one wave per 4 KiB segment: lazy LZ77 over fixed candidate distances
//                    (1, pixel, 2 pixels, row above +-pixel), tokens + per-block histograms +
//                    Adler-32 partials; 64 segments = one 256 KiB deflate block
//   k_png_seam(_apply) join each segment's tokens to the previous segment's last match where
//                    it runs past the boundary (re-parsed head), and fix the counts
//   k_png_huff       one workgroup per block: length-limited Huffman codes (15/7 bits), the
//                    dynamic block header bits
//   k_png_segbits    bits per segment -> (scan) bit offsets
//   k_png_emit       one lane per segment: LSB-first bit packing of its tokens at its offset
//   k_png_crc*       CRC-32 of the IDAT chunk: per-segment table CRCs combined by x^(8n) shifts
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "icx_internal.h"

namespace icx {

namespace png {

#ifndef ICX_PNG_SEG
#define ICX_PNG_SEG 4096
#endif
constexpr int kSeg = ICX_PNG_SEG;     // LZ77 / emit segment (bytes of the filtered stream), one lane each
constexpr int kSlots = kSeg + 8;      // token slots per segment: up to kSeg - 1 literals + a match
                                      // overhanging the segment end (16-byte multiple)
constexpr int kSegPerBlock = 262144 / kSeg;  // 256 KiB deflate blocks (lodepng's size at this scale, :1830)
constexpr int kNLL = 286, kND = 30;   // literal/length and distance alphabets
constexpr int kHdrWords = 96;         // per-block header bit buffer (<= 3072 bits)
constexpr int kCrcSeg = 1024;         // CRC-32 segment, one lane each
constexpr uint32_t kAdlerMod = 65521;
enum { kGrey = 0, kRGB = 2, kPalette = 3, kGreyAlpha = 4, kRGBA = 6 };

struct Stats {
    uint32_t colored;    // some pixel with r != g or r != b
    uint32_t alpha_mid;  // some alpha not in {0, 255}
    uint32_t bits;       // max getValueRequiredBits(r)
    uint32_t any_a0;     // some alpha == 0
    unsigned long long first_a0;  // smallest pixel index with alpha == 0
    uint32_t ncolors;    // distinct RGBA colours inserted (saturates past 256)
    uint32_t overflow;   // > 256 distinct colours
    uint32_t a2, a3;     // key cases: transparent pixel of another colour / opaque key colour
};

constexpr int kSetSlots = 4096;  // global colour set: (colour | 1<<32) keys, min pixel index values

struct Mode {
    int colortype, bitdepth, bpp, bw;  // bpp in bits, bw = filter byte width
    int64_t lb;                        // bytes per (padded) row
    int npal;
    uint32_t pal[256];                 // RGBA packed r | g<<8 | b<<16 | a<<24
};

// ---- deflate tables (RFC 1951 3.2.5)
__constant__ uint16_t kLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                      35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769,
                                       1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
__constant__ uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

__device__ __forceinline__ int len_code(int len) {  // 3..258 -> 0..28
    int c = 0;
    while (c < 28 && kLenBase[c + 1] <= len) ++c;
    return c;
}
__device__ __forceinline__ int dist_code(int d) {  // 1..32768 -> 0..29
    int c = 0;
    while (c < 29 && kDistBase[c + 1] <= d) ++c;
    return c;
}

struct BlockCodes {
    uint16_t ll_code[kNLL];  // bit-reversed (LSB-first emission)
    uint8_t ll_len[kNLL];
    uint16_t d_code[kND];
    uint8_t d_len[kND];
    uint32_t hdr[kHdrWords];  // header bits, LSB-first
    uint32_t hdr_bits;
    uint32_t pad_;
};

__device__ __forceinline__ uint32_t required_bits(uint32_t v) {  // :3349-3355
    if (v == 0 || v == 255) return 1;
    if (v % 17 == 0) return v % 85 == 0 ? 2 : 4;
    return 8;
}

__device__ __forceinline__ uint32_t hash32(uint32_t c) { return (c * 2654435761u) >> 20; }

// ------------------------------------------------------------------------------- stats
// Grid-stride over pixels. Colours go through a per-workgroup LDS set first (one global insert
// per distinct colour per workgroup); > 256 distinct colours anywhere ends the counting.
__global__ __launch_bounds__(256) void k_png_stats(const uint8_t* __restrict__ px, int64_t np, int d,
                                                   Stats* __restrict__ st, unsigned long long* __restrict__ gset_key,
                                                   unsigned long long* __restrict__ gset_idx) {
    __shared__ uint32_t s_key[1024];
    __shared__ unsigned long long s_idx[1024];
    __shared__ uint32_t s_n, s_over;
    const int t = threadIdx.x;
    for (int i = t; i < 1024; i += 256) {
        s_key[i] = 0xFFFFFFFFu;
        s_idx[i] = ~0ull;
    }
    if (t == 0) {
        s_n = 0;
        s_over = 0;
    }
    __syncthreads();
    uint32_t colored = 0, amid = 0, bits = 1, any0 = 0;
    unsigned long long first0 = ~0ull;
    const bool count_colors = st->overflow == 0;
    // the LDS set reserves key 0xFFFFFFFF as empty: that colour (opaque white) uses slot s_white
    __shared__ unsigned long long s_white;
    if (t == 0) s_white = ~0ull;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * 256 + t; i < np; i += (int64_t)gridDim.x * 256) {
        const uint8_t* p = px + i * d;
        const uint32_t r = p[0], g = p[1], b = p[2], a = d == 4 ? p[3] : 255;
        colored |= (r != g) | (r != b);
        bits = max(bits, required_bits(r));
        if (d == 4) {
            amid |= a != 0 && a != 255;
            if (a == 0) {
                any0 = 1;
                first0 = min(first0, (unsigned long long)i);
            }
        }
        if (count_colors && !s_over) {
            const uint32_t c = r | g << 8 | b << 16 | a << 24;
            if (c == 0xFFFFFFFFu) {
                atomicMin(&s_white, (unsigned long long)i);
            } else {
                uint32_t h = hash32(c) & 1023;
                for (int probe = 0; probe < 1024; ++probe, h = (h + 1) & 1023) {
                    const uint32_t old = atomicCAS(&s_key[h], 0xFFFFFFFFu, c);
                    if (old == 0xFFFFFFFFu) {
                        if (atomicAdd(&s_n, 1u) >= 256) s_over = 1;
                    }
                    if (old == 0xFFFFFFFFu || old == c) {
                        atomicMin(&s_idx[h], (unsigned long long)i);
                        break;
                    }
                }
            }
        }
    }
    // workgroup reductions
    colored = __syncthreads_or(colored);
    amid = __syncthreads_or(amid);
    any0 = __syncthreads_or(any0);
    for (int o = 32; o > 0; o >>= 1) {
        bits = max(bits, (uint32_t)__shfl_xor((int)bits, o));
        first0 = min(first0, (unsigned long long)__shfl_xor((long long)first0, o));
    }
    __shared__ uint32_t s_bits;
    __shared__ unsigned long long s_first;
    if (t == 0) {
        s_bits = 1;
        s_first = ~0ull;
    }
    __syncthreads();
    if ((t & 63) == 0) {
        atomicMax(&s_bits, bits);
        atomicMin(&s_first, first0);
    }
    __syncthreads();
    if (t == 0) {
        if (colored) atomicOr(&st->colored, 1u);
        if (amid) atomicOr(&st->alpha_mid, 1u);
        if (any0) {
            atomicOr(&st->any_a0, 1u);
            atomicMin(&st->first_a0, s_first);
        }
        atomicMax(&st->bits, s_bits);
        if (s_over) atomicOr(&st->overflow, 1u);
    }
    if (!count_colors || s_over) return;
    // merge this workgroup's colours into the global set
    auto ginsert = [&](uint32_t c, unsigned long long idx) {
        const unsigned long long k = (unsigned long long)c | (1ull << 32);
        uint32_t h = hash32(c) & (kSetSlots - 1);
        for (int probe = 0; probe < kSetSlots; ++probe, h = (h + 1) & (kSetSlots - 1)) {
            const unsigned long long old = atomicCAS(&gset_key[h], 0ull, k);
            if (old == 0ull) {
                if (atomicAdd(&st->ncolors, 1u) >= 256) atomicOr(&st->overflow, 1u);
            }
            if (old == 0ull || old == k) {
                atomicMin(&gset_idx[h], idx);
                return;
            }
        }
        atomicOr(&st->overflow, 1u);
    };
    for (int i = t; i < 1024; i += 256)
        if (s_key[i] != 0xFFFFFFFFu) ginsert(s_key[i], s_idx[i]);
    if (t == 0 && s_white != ~0ull) ginsert(0xFFFFFFFFu, s_white);
}

// The colour-key cases once the first transparent pixel's colour K is known (d == 4, no alpha
// yet): a transparent pixel of another colour, or a non-transparent pixel of colour K.
__global__ __launch_bounds__(256) void k_png_keycheck(const uint8_t* __restrict__ px, int64_t np, uint32_t key,
                                                      Stats* __restrict__ st) {
    uint32_t a2 = 0, a3 = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < np; i += (int64_t)gridDim.x * 256) {
        const uint8_t* p = px + i * 4;
        const uint32_t rgb = p[0] | p[1] << 8 | p[2] << 16;
        a2 |= p[3] == 0 && rgb != key;
        a3 |= p[3] != 0 && rgb == key;
    }
    a2 = __syncthreads_or(a2);
    a3 = __syncthreads_or(a3);
    if (threadIdx.x == 0) {
        if (a2) atomicOr(&st->a2, 1u);
        if (a3) atomicOr(&st->a3, 1u);
    }
}

// ----------------------------------------------------------------------------- convert
// One output byte per thread: lodepng_convert (rgba8ToPixel :2781-2835) + row padding.
__global__ __launch_bounds__(256) void k_png_convert(const uint8_t* __restrict__ px, int w, int h, int d,
                                                     const Mode* __restrict__ mode, uint8_t* __restrict__ out) {
    __shared__ uint32_t s_used[512], s_col[512];
    __shared__ uint8_t s_val[512];
    const Mode& M = *mode;
    if (M.colortype == kPalette) {  // colour -> palette index (color_tree_get)
        for (int i = threadIdx.x; i < 512; i += 256) s_used[i] = 0;
        __syncthreads();
        if (threadIdx.x == 0)
            for (int k = 0; k < M.npal; ++k) {
                const uint32_t c = M.pal[k];
                uint32_t hh = hash32(c) & 511;
                while (s_used[hh]) hh = (hh + 1) & 511;
                s_used[hh] = 1;
                s_col[hh] = c;
                s_val[hh] = (uint8_t)k;
            }
        __syncthreads();
    }
    auto pixel = [&](int64_t y, int64_t x, uint32_t& r, uint32_t& g, uint32_t& b, uint32_t& a) {
        const uint8_t* p = px + (y * w + x) * d;
        r = p[0];
        g = p[1];
        b = p[2];
        a = d == 4 ? p[3] : 255;
    };
    auto index_of = [&](int64_t y, int64_t x) -> uint32_t {
        uint32_t r, g, b, a;
        pixel(y, x, r, g, b, a);
        const uint32_t c = r | g << 8 | b << 16 | a << 24;
        uint32_t hh = hash32(c) & 511;
        for (int probe = 0; probe < 512; ++probe, hh = (hh + 1) & 511) {
            if (!s_used[hh]) return 0;
            if (s_col[hh] == c) return s_val[hh];
        }
        return 0;
    };
    const int64_t total = M.lb * h;
    for (int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x; o < total; o += (int64_t)gridDim.x * 256) {
        const int64_t y = o / M.lb, xb = o - y * M.lb;
        uint32_t v = 0;
        if (M.bitdepth == 8) {
            const int ch = M.bpp / 8;
            const int64_t x = xb / ch;
            const int c = (int)(xb - x * ch);
            uint32_t r, g, b, a;
            pixel(y, x, r, g, b, a);
            switch (M.colortype) {
                case kRGBA: v = c == 0 ? r : c == 1 ? g : c == 2 ? b : a; break;
                case kRGB: v = c == 0 ? r : c == 1 ? g : b; break;
                case kGreyAlpha: v = c == 0 ? r : a; break;
                case kGrey: v = r; break;
                default: v = index_of(y, x); break;
            }
        } else {  // 1/2/4-bit grey or palette, MSB-first (addColorBits :2706-2714), zero pad
            const int per = 8 / M.bitdepth;
            for (int k = 0; k < per; ++k) {
                const int64_t x = xb * per + k;
                uint32_t s = 0;
                if (x < w) {
                    if (M.colortype == kGrey) {
                        uint32_t r, g, b, a;
                        pixel(y, x, r, g, b, a);
                        s = (r >> (8 - M.bitdepth)) & ((1u << M.bitdepth) - 1u);
                    } else {
                        s = index_of(y, x) & ((1u << M.bitdepth) - 1u);
                    }
                }
                v |= s << (M.bitdepth * (per - 1 - k));
            }
        }
        out[o] = (uint8_t)v;
    }
}

// ------------------------------------------------------------------------------ filter
__device__ __forceinline__ uint32_t paeth(uint32_t a, uint32_t b, uint32_t c) {  // :3621-3631
    int pa = abs((int)b - (int)c), pb = abs((int)a - (int)c), pc = abs((int)a + (int)b - 2 * (int)c);
    if (pb < pa) {
        a = b;
        pa = pb;
    }
    return pc < pa ? c : a;
}
__device__ __forceinline__ uint32_t filt(int type, uint32_t s, uint32_t left, uint32_t up, uint32_t ul) {
    switch (type) {
        case 1: return (s - left) & 255;
        case 2: return (s - up) & 255;
        case 3: return (s - ((left + up) >> 1)) & 255;
        case 4: return (s - paeth(left, up, ul)) & 255;
        default: return s;
    }
}

// Bytes [s, s+4) of row R packed little-endian (bytes before the row start read 0): the left
// (or upper-left) neighbours of 4 consecutive positions at filter byte width bw.
__device__ __forceinline__ uint32_t row_bytes4(const uint32_t* R, int64_t s) {
    if (s >= 0) {
        const int64_t j = s >> 2;
        const int o = (int)(s & 3);
        const uint32_t lo = R[j];
        return o ? __builtin_amdgcn_alignbyte(R[j + 1], lo, (uint32_t)o) : lo;  // byte shift o
    }
    uint32_t v = 0;
    for (int b = 0; b < 4; ++b)
        if (s + b >= 0) v |= ((R[(s + b) >> 2] >> (8 * ((s + b) & 3))) & 255u) << (8 * b);
    return v;
}

// One workgroup per row (grid-stride): MINSUM over the five filters, ties to the lower type
// (`sum < smallest`, :3968), type 0 scored unsigned; palette / < 8 bits: type 0 (:3950).
// Rows of whole dwords (lb % 4 == 0, the RGBA / 16-bit cases) are read a dword per lane:
// the pixel, the pixel above and the left / upper-left neighbours (one alignbyte each).
__global__ __launch_bounds__(256) void k_png_filter(const uint8_t* __restrict__ img, int h, const Mode* __restrict__ mode,
                                                    uint8_t* __restrict__ out) {
    const Mode& M = *mode;
    const int64_t lb = M.lb;
    const int bw = M.bw;
    const bool zero = M.colortype == kPalette || M.bitdepth < 8;
    const bool wide = (lb & 3) == 0 && (reinterpret_cast<uintptr_t>(img) & 3) == 0;
    __shared__ uint32_t s_sum[5][4];
    for (int y = blockIdx.x; y < h; y += gridDim.x) {
        const uint8_t* cur = img + (int64_t)y * lb;
        const uint8_t* prv = y ? cur - lb : nullptr;
        const uint32_t* C4 = reinterpret_cast<const uint32_t*>(cur);
        const uint32_t* P4 = reinterpret_cast<const uint32_t*>(prv);
        int best = 0;
        if (!zero) {
            uint32_t sum[5] = {0, 0, 0, 0, 0};
            auto score = [&](uint32_t s, uint32_t left, uint32_t up, uint32_t ul) {
                sum[0] += s;
#pragma unroll
                for (int tt = 1; tt < 5; ++tt) {
                    const uint32_t f = filt(tt, s, left, up, ul);
                    sum[tt] += f < 128 ? f : 255u - f;
                }
            };
            if (wide) {
                for (int64_t i = 4 * (int64_t)threadIdx.x; i < lb; i += 1024) {
                    const uint32_t s4 = C4[i >> 2], l4 = row_bytes4(C4, i - bw);
                    const uint32_t u4 = prv ? P4[i >> 2] : 0u, ul4 = prv ? row_bytes4(P4, i - bw) : 0u;
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        score((s4 >> (8 * b)) & 255u, (l4 >> (8 * b)) & 255u, (u4 >> (8 * b)) & 255u, (ul4 >> (8 * b)) & 255u);
                }
            } else {
                for (int64_t i = threadIdx.x; i < lb; i += 256) {
                    const uint32_t s = cur[i], left = i >= bw ? cur[i - bw] : 0, up = prv ? prv[i] : 0,
                                   ul = (prv && i >= bw) ? prv[i - bw] : 0;
                    score(s, left, up, ul);
                }
            }
#pragma unroll
            for (int tt = 0; tt < 5; ++tt)
                for (int o = 32; o > 0; o >>= 1) sum[tt] += (uint32_t)__shfl_xor((int)sum[tt], o);
            if ((threadIdx.x & 63) == 0)
                for (int tt = 0; tt < 5; ++tt) s_sum[tt][threadIdx.x >> 6] = sum[tt];
            __syncthreads();
            uint32_t smallest = 0;
            for (int tt = 0; tt < 5; ++tt) {
                const uint32_t v = s_sum[tt][0] + s_sum[tt][1] + s_sum[tt][2] + s_sum[tt][3];
                if (tt == 0 || v < smallest) {
                    best = tt;
                    smallest = v;
                }
            }
            __syncthreads();
        }
        uint8_t* o = out + (int64_t)y * (lb + 1);
        if (threadIdx.x == 0) o[0] = (uint8_t)best;
        if (wide) {
            for (int64_t i = 4 * (int64_t)threadIdx.x; i < lb; i += 1024) {
                const uint32_t s4 = C4[i >> 2];
                if (best == 0) {
#pragma unroll
                    for (int b = 0; b < 4; ++b) o[1 + i + b] = (uint8_t)(s4 >> (8 * b));
                    continue;
                }
                const uint32_t l4 = row_bytes4(C4, i - bw);
                const uint32_t u4 = prv ? P4[i >> 2] : 0u, ul4 = prv ? row_bytes4(P4, i - bw) : 0u;
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    o[1 + i + b] = (uint8_t)filt(best, (s4 >> (8 * b)) & 255u, (l4 >> (8 * b)) & 255u,
                                                 (u4 >> (8 * b)) & 255u, (ul4 >> (8 * b)) & 255u);
            }
        } else {
            for (int64_t i = threadIdx.x; i < lb; i += 256) {
                const uint32_t s = cur[i], left = i >= bw ? cur[i - bw] : 0, up = prv ? prv[i] : 0,
                               ul = (prv && i >= bw) ? prv[i - bw] : 0;
                o[1 + i] = (uint8_t)filt(best, s, left, up, ul);
            }
        }
    }
}

// ------------------------------------------------------------------------------- LZ77
// Token slots (uint16): a literal is its byte value (< 256); a match is a length slot
// 0x4000 | (len - 3) followed by a distance slot 0x8000 | (dist - 1).
// A segment's matches start inside it but may run past its end (the overhang, < 258 bytes): the
// stream is then parsed as one serial parse would, without the short match every segment
// boundary would otherwise cost (k_png_seam joins the next segment's tokens to the overhang).
// A wave's view of the filtered stream around its segment, staged in LDS: `near` covers
// [s0 - kNear, s1 + kOver) (the segment, its overhang and the short candidate distances), `far`
// covers [s0 - rowlen - kNear, s1 + kOver - rowlen + kNear) (the row above +- one pixel). Both
// start at a 16-byte-aligned stream index so the staging is 16-byte loads. Every source byte a
// candidate can compare (q - d + l with q + l < s1 + 258) lies in one of them: indices
// >= s0 - kNear in `near`, the others (distances rowlen - bw .. rowlen + bw only) in `far`.
constexpr int kNear = 16;                               // >= 2 * bw (bw <= 8)
constexpr int kOver = 272;                              // >= 258: a match past the segment end
constexpr int kStage = kSeg + kOver + 2 * kNear + 32;   // bytes per staged view, 16-byte multiple (dword-read slack)
struct SegView {
    const uint8_t* nearp;  // LDS base, = stream index nb0
    const uint8_t* farp;   // LDS base, = stream index fb0
    int64_t nb0, fb0, nlo; // nlo = s0 - kNear: lowest index served by `near`
    __device__ __forceinline__ uint8_t at(int64_t i) const {
        return i >= nlo ? nearp[i - nb0] : farp[i - fb0];
    }
    // bytes i .. i+3, byte i lowest (a far-view read never crosses the end of that view: far
    // candidates compare below s1 + 258 - rowlen + bw, and the view runs past it by more than
    // kNear + 16)
    __device__ __forceinline__ uint32_t dword(int64_t i) const {
        const bool nr = i >= nlo;
        const int64_t o = nr ? i - nb0 : i - fb0;
        const uint32_t* w = reinterpret_cast<const uint32_t*>(nr ? nearp : farp) + (o >> 2);
        return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(o & 3));
    }
};
__device__ __forceinline__ void stage_view(const uint8_t* __restrict__ F, int64_t N, int64_t b0, uint8_t* lds, int lane,
                                           int nbytes = kStage) {
    for (int k = lane; k < nbytes / 16; k += 64) {
        const int64_t g = b0 + 16 * k;
        uint4 v;
        if (g >= 0 && g + 16 <= N) {
            v = *reinterpret_cast<const uint4*>(F + g);
        } else {
            uint8_t t[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) t[j] = (g + j >= 0 && g + j < N) ? F[g + j] : 0;
            __builtin_memcpy(&v, t, 16);
        }
        *reinterpret_cast<uint4*>(lds + 16 * k) = v;
    }
}
// A lane's value at a wave-uniform lane index: v_readlane into a scalar register (__shfl is an LDS
// permute, and its round trip sat on the parse's serial chain)
__device__ __forceinline__ int rdl(int v, int i) { return __builtin_amdgcn_readlane(v, i); }

// Length of the match at p against p - dist, at most maxlen: four bytes per step, the first
// differing byte from the lowest set bit of the XOR.
__device__ __forceinline__ int match_len(const SegView& V, int64_t p, int64_t dist, int maxlen) {
    int l = 0;
    while (l < maxlen) {
        const uint32_t x = V.dword(p + l) ^ V.dword(p - dist + l);
        if (x) return min(l + (int)(__builtin_ctz(x) >> 3), maxlen);
        l += 4;
    }
    return maxlen;
}

// One workgroup (4 waves) per 256 KiB block; each wave takes a 4 KiB segment at a time, stages
// its two views in LDS, and walks it in 64-position windows: every lane scores the position
// under it against the six structural candidates (left pixel, up to two pixels back, the pixel
// above and its two neighbours), then the wave parses the window with ballots -- the literal
// run up to the first position with a match is emitted by all lanes at once, the match by one.
// The tokens are those of a serial parse with one-step lazy evaluation (a match of length >= 3
// per position, longest over the candidates; a match whose next position in the window has a
// longer one is deferred to it, as zlib's lazy matching does). The last match may run past the
// segment end; its overhang goes to seam[4 seg] for k_png_seam.
__global__ __launch_bounds__(256) void k_png_lz77(const uint8_t* __restrict__ F, int64_t N, int64_t nseg, int64_t rowlen,
                                                  int bw, uint16_t* __restrict__ tok, uint32_t* __restrict__ ntok,
                                                  uint32_t* __restrict__ hist, uint32_t* __restrict__ adl,
                                                  uint16_t* __restrict__ seghist, uint32_t* __restrict__ segx,
                                                  uint32_t* __restrict__ seam, uint32_t* __restrict__ blksym) {
    __shared__ uint32_t h_ll[kNLL], h_d[kND], s_sym;
    __shared__ uint32_t s_h[4][kNLL + kND];  // per wave: the current segment's symbol counts
    __shared__ __attribute__((aligned(16))) uint8_t views[4][2][kStage];
    const int64_t blk = blockIdx.x;
    for (int i = threadIdx.x; i < kNLL; i += 256) h_ll[i] = 0;
    if (threadIdx.x < kND) h_d[threadIdx.x] = 0;
    if (threadIdx.x == 0) s_sym = 1;  // + EOB
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int64_t cand[6] = {1, bw, 2 * bw, rowlen, rowlen - bw, rowlen + bw};
#pragma unroll
    for (int k = 0; k < 6; ++k)
        if (cand[k] <= 0 || cand[k] > 32768) cand[k] = 0;
    for (int sl = wave; sl < kSegPerBlock; sl += 4) {
        const int64_t seg = blk * kSegPerBlock + sl;
        if (seg >= nseg) break;  // wave-uniform
        const int64_t s0 = seg * kSeg, s1 = min(N, s0 + kSeg);
        uint16_t* T = tok + seg * kSlots;
        uint32_t* SH = s_h[wave];
        for (int i = lane; i < kNLL + kND; i += 64) SH[i] = 0;
        uint32_t xbits = 0;  // length / distance extra bits of the segment's matches (lane 0)
        SegView V;
        V.nlo = s0 - kNear;
        V.nb0 = V.nlo & ~(int64_t)15;
        V.fb0 = (s0 - rowlen - kNear) & ~(int64_t)15;
        V.nearp = views[wave][0];
        V.farp = views[wave][1];
        __builtin_amdgcn_wave_barrier();
        stage_view(F, N, V.nb0, views[wave][0], lane);
        stage_view(F, N, V.fb0, views[wave][1], lane);
        __builtin_amdgcn_wave_barrier();
        // Adler-32 partials: sum b, sum (N - g) b (reduced mod 65521 at the end)
        uint64_t a1 = 0, a2 = 0;
        for (int64_t q = s0 + lane; q < s1; q += 64) {
            const uint32_t b = V.nearp[q - V.nb0];
            a1 += b;
            a2 += (uint64_t)(N - q) * b;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            a1 += __shfl_xor(a1, o);
            a2 += __shfl_xor(a2, o);
        }
        if (lane == 0) {
            adl[2 * seg] = (uint32_t)(a1 % kAdlerMod);
            adl[2 * seg + 1] = (uint32_t)(a2 % kAdlerMod);
        }
        uint32_t nt = 0, nm = 0;  // token slots, matches
        int64_t pos = s0;  // first position not yet covered by a token
        for (int64_t p0 = s0; p0 < s1; p0 += 64) {
            const int64_t q = p0 + lane;
            int best = 0, bd = 0;
            uint32_t lit = 0;
            if (q < s1) {
                const uint32_t t4 = V.dword(q);
                lit = t4 & 255u;
                const int maxlen = (int)min((int64_t)258, N - q);
                if (maxlen >= 3 && q >= pos) {  // positions under a previous match need no score
#pragma unroll
                    for (int k = 0; k < 6; ++k) {
                        const int64_t dd = cand[k];
                        if (dd == 0 || dd > q) continue;
                        if (((V.dword(q - dd) ^ t4) & 0xFFFFFFu) != 0) continue;  // first three bytes
                        const int l = 3 + match_len(V, q + 3, dd, maxlen - 3);
                        if (l > best) {
                            best = l;
                            bd = (int)dd;
                        }
                    }
                }
            }
            const uint64_t cmask = __ballot(best >= 3);
            const int wend = (int)min((int64_t)64, s1 - p0);  // live lanes of this window
            while (pos < p0 + wend) {  // wave-uniform
                const int li = (int)(pos - p0);
                uint64_t m = cmask & (~0ull << li);
                int mi = m ? __ffsll((unsigned long long)m) - 1 : 64;
                // lazy evaluation (zlib's deflate_slow): a match start whose successor has a
                // longer match becomes a literal, and the successor is considered in turn
                while (mi + 1 < wend && rdl(best, mi + 1) > rdl(best, mi)) {
                    m &= m - 1;
                    mi = __ffsll((unsigned long long)m) - 1;
                }
                const int le = min(mi, wend);
                if (lane >= li && lane < le) {  // the literal run li .. le-1
                    T[nt + (lane - li)] = (uint16_t)lit;
                    atomicAdd(&SH[lit], 1u);
                }
                nt += (uint32_t)(le - li);
                pos = p0 + le;
                if (mi < wend) {  // the match at lane mi
                    const int len = rdl(best, mi), dist = rdl(bd, mi);
                    if (lane == 0) {
                        T[nt] = (uint16_t)(0x4000u | (uint32_t)(len - 3));    // match: length slot,
                        T[nt + 1] = (uint16_t)(0x8000u | (uint32_t)(dist - 1));  // then distance slot
                        const int lc = len_code(len), dc = dist_code(dist);
                        SH[257 + lc] += 1u;
                        SH[kNLL + dc] += 1u;
                        xbits += kLenExtra[lc] + kDistExtra[dc];
                    }
                    nt += 2;
                    nm += 1;
                    pos += len;
                }
            }
        }
        if (lane == 0) {
            ntok[seg] = nt;
            segx[seg] = xbits;
            seam[4 * seg] = (uint32_t)(pos - s1);  // the overhang
            atomicAdd(&s_sym, nt - nm);
        }
        __builtin_amdgcn_wave_barrier();
        // the segment's counts: to HBM for k_png_segbits, into the block histogram for k_png_huff
        uint16_t* G = seghist + seg * (kNLL + kND);
        for (int i = lane; i < kNLL + kND; i += 64) {
            const uint32_t c = SH[i];
            G[i] = (uint16_t)c;
            if (c) atomicAdd(i < kNLL ? &h_ll[i] : &h_d[i - kNLL], c);
        }
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    uint32_t* H = hist + blk * (kNLL + kND);
    for (int i = threadIdx.x; i < kNLL; i += 256) H[i] = h_ll[i] + (i == 256 ? 1u : 0u);  // + EOB
    if (threadIdx.x < kND) H[kNLL + threadIdx.x] = h_d[threadIdx.x];
    if (threadIdx.x == 0) blksym[blk] = s_sym;
}

// ------------------------------------------------------------------------------ seams
// Segment B's tokens were parsed from its first byte, but the previous segment A's last match
// may already cover B's first o bytes (A's overhang). k_png_seam re-parses B from s0 + o, the
// same way (longest structural candidate, one-step lazy), until it reaches the start of one of
// B's own tokens -- greedy parses resynchronise within a few tokens -- and B's tokens before that
// are replaced by the re-parsed head (at most kHead slots). If no such join is found before B's
// last token (which fixes B's own overhang), A's last match is cut back to A's end instead and B
// keeps its tokens. seam[4 s + 0..3]: overhang, head skip (B's slots dropped), head slots, A cut.
constexpr int kHead = 32;
// Longest candidate match at q (lanes 0..5: candidate k at q; lanes 6..11: candidate k at q + 1)
// in the segment's staged views, the candidate order deciding ties as in k_png_lz77;
// -> (len, dist) at q and len at q + 1.
__device__ __forceinline__ void seam_score(const SegView& V, int64_t N, int64_t q, const int64_t* cand, int lane,
                                           int& len0, int& dist0, int& len1) {
    int l = 0, d = 0;
    if (lane < 12) {
        const int64_t p = q + (lane >= 6), dd = cand[lane % 6];
        const int maxlen = (int)min((int64_t)258, N - p);
        if (dd && dd <= p && maxlen >= 3) {
            l = match_len(V, p, dd, maxlen);
            if (l < 3) l = 0;
            d = (int)dd;
        }
    }
    len0 = dist0 = len1 = 0;
    for (int k = 0; k < 6; ++k) {
        const int a = rdl(l, k), b = rdl(l, 6 + k);
        if (a > len0) {
            len0 = a;
            dist0 = rdl(d, k);
        }
        len1 = max(len1, b);
    }
}
__device__ __forceinline__ void tok_counts(uint16_t* G, uint32_t* H, uint32_t& xbits, uint32_t t, uint32_t tnext, int sgn) {
    if (t < 256) {
        G[t] = (uint16_t)(G[t] + sgn);
        atomicAdd(&H[t], (uint32_t)sgn);
        return;
    }
    const int len = (int)(t & 255) + 3, dist = (int)(tnext & 0x7FFFu) + 1;
    const int lc = len_code(len), dc = dist_code(dist);
    G[257 + lc] = (uint16_t)(G[257 + lc] + sgn);
    G[kNLL + dc] = (uint16_t)(G[kNLL + dc] + sgn);
    atomicAdd(&H[257 + lc], (uint32_t)sgn);
    atomicAdd(&H[kNLL + dc], (uint32_t)sgn);
    xbits += (uint32_t)(sgn * (int)(kLenExtra[lc] + kDistExtra[dc]));
}
// One wave per segment B (the seam before it): B's two views staged as in k_png_lz77, then
// the wave walks B's tokens while 12 lanes score each re-parse position.
// The re-parse may run over the whole of B (a highly compressible segment joins only after a few
// 258-byte matches); it walks B's first kSeamToks token slots from LDS. (Views of B's first KiB
// only, cutting A's match where the head had not joined by then, were tried: C5 +1%, but the
// reference's test.bmp with alpha went 1.042 -> 1.049 of zlib -6.)
constexpr int kSeamStage = kStage;
constexpr int kSeamReach = kSeg + kOver;  // (no limit inside the segment)
constexpr int kSeamToks = 256;
__global__ __launch_bounds__(256) void k_png_seam(const uint8_t* __restrict__ F, int64_t N, int64_t nseg, int64_t rowlen,
                                                  int bw, const uint16_t* __restrict__ tok,
                                                  const uint32_t* __restrict__ ntok, uint32_t* __restrict__ seam,
                                                  uint16_t* __restrict__ head, int join) {
    __shared__ __attribute__((aligned(16))) uint8_t views[4][2][kSeamStage];
    __shared__ uint16_t toks[4][kSeamToks];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + wave;
    if (b >= nseg) return;  // wave-uniform; no block barriers below
    if (b == nseg - 1 && lane == 0) seam[4 * b + 3] = 0;  // no seam after the last segment
    const uint32_t o = b > 0 ? seam[4 * (b - 1)] : 0u;
    uint32_t skip = 0, nh = 0, cut = 0;
    if (o) {
        int64_t cand[6] = {1, bw, 2 * bw, rowlen, rowlen - bw, rowlen + bw};
        for (int k = 0; k < 6; ++k)
            if (cand[k] <= 0 || cand[k] > 32768) cand[k] = 0;
        const int64_t s0 = b * kSeg;
        SegView V;
        V.nlo = s0 - kNear;
        V.nb0 = V.nlo & ~(int64_t)15;
        V.fb0 = (s0 - rowlen - kNear) & ~(int64_t)15;
        V.nearp = views[wave][0];
        V.farp = views[wave][1];
        stage_view(F, N, V.nb0, views[wave][0], lane, kSeamStage);
        stage_view(F, N, V.fb0, views[wave][1], lane, kSeamStage);
        const uint16_t* T = tok + b * kSlots;
        const uint32_t nt = ntok[b];
        for (int k = lane; k < kSeamToks; k += 64) toks[wave][k] = k < (int)nt ? T[k] : 0;
        __builtin_amdgcn_wave_barrier();
        auto tokat = [&](uint32_t i) { return i < (uint32_t)kSeamToks ? (uint32_t)toks[wave][i] : (uint32_t)T[i]; };
        const uint32_t last = (nt >= 2 && (T[nt - 1] & 0x8000u)) ? nt - 2 : nt - 1;  // B's last token slot
        const bool final_seg = b == nseg - 1;
        uint16_t* Hd = head + b * kHead;
        uint32_t si = 0;      // B's token slot under consideration ...
        int64_t bp = s0;      // ... and the stream position it starts at
        int64_t q = s0 + o;   // the re-parse position
        bool joined = false;
        for (;;) {  // wave-uniform: every lane walks the same tokens
            while (si <= last && bp < q) {
                const uint32_t t = tokat(si);
                if (t < 256) {
                    bp += 1;
                    si += 1;
                } else {
                    bp += (t & 255) + 3;
                    si += 2;
                }
            }
            if (si <= last && bp == q) {  // join B's own parse at slot si
                joined = true;
                break;
            }
            if (final_seg && q >= N) {  // the whole final segment re-parsed
                si = nt;
                joined = true;
                break;
            }
            if ((si > last && !final_seg) || nh + 2 > kHead || !join || q >= s0 + kSeamReach) break;  // no join: cut A
            int len0, dist0, len1;
            seam_score(V, N, q, cand, lane, len0, dist0, len1);
            if (len0 >= 3 && !(q + 1 < N && len1 > len0)) {
                if (lane == 0) {
                    Hd[nh] = (uint16_t)(0x4000u | (uint32_t)(len0 - 3));
                    Hd[nh + 1] = (uint16_t)(0x8000u | (uint32_t)(dist0 - 1));
                }
                nh += 2;
                q += len0;
            } else {
                if (lane == 0) Hd[nh] = V.at(q);
                nh += 1;
                q += 1;
            }
        }
        if (joined) skip = si;
        else {
            nh = 0;
            cut = 1;
        }
    }
    if (lane == 0) {
        seam[4 * b + 1] = skip;
        seam[4 * b + 2] = nh;
        if (b > 0) seam[4 * (b - 1) + 3] = cut;
    }
}
// One lane per segment: the symbol counts (segment, block) and extra bits follow the seams --
// the dropped head slots out, the re-parsed head in, and a cut last match shortened (or, under
// three bytes, turned into its literals, in place).
__global__ __launch_bounds__(256) void k_png_seam_apply(const uint8_t* __restrict__ F, int64_t N, int64_t nseg,
                                                        uint16_t* __restrict__ tok, uint32_t* __restrict__ ntok,
                                                        const uint32_t* __restrict__ seam, const uint16_t* __restrict__ head,
                                                        uint16_t* __restrict__ seghist, uint32_t* __restrict__ segx,
                                                        uint32_t* __restrict__ hist) {
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= nseg) return;
    const uint32_t o = seam[4 * s], skip = seam[4 * s + 1], nh = seam[4 * s + 2], cut = seam[4 * s + 3];
    if (!skip && !nh && !cut) return;
    uint16_t* T = tok + s * kSlots;
    uint16_t* G = seghist + s * (kNLL + kND);
    uint32_t* H = hist + (s / kSegPerBlock) * (kNLL + kND);
    uint32_t nt = ntok[s], xbits = segx[s];
    for (uint32_t i = 0; i < skip;) {
        const uint32_t t = T[i];
        tok_counts(G, H, xbits, t, i + 1 < nt ? T[i + 1] : 0u, -1);
        i += t < 256 ? 1 : 2;
    }
    const uint16_t* Hd = head + s * kHead;
    for (uint32_t i = 0; i < nh;) {
        const uint32_t t = Hd[i];
        tok_counts(G, H, xbits, t, i + 1 < nh ? Hd[i + 1] : 0u, +1);
        i += t < 256 ? 1 : 2;
    }
    if (cut) {  // the last token is a match ending o bytes past the segment end
        const uint32_t t = T[nt - 2], d = T[nt - 1];
        tok_counts(G, H, xbits, t, d, -1);
        const int len = (int)(t & 255) + 3 - (int)o;
        const int64_t p = min(N, (s + 1) * kSeg) - len;  // its start
        if (len >= 3) {
            T[nt - 2] = (uint16_t)(0x4000u | (uint32_t)(len - 3));
            tok_counts(G, H, xbits, T[nt - 2], d, +1);
        } else {
            for (int k = 0; k < len; ++k) {
                T[nt - 2 + k] = F[p + k];
                tok_counts(G, H, xbits, F[p + k], 0u, +1);
            }
            nt -= 2 - len;
        }
    }
    ntok[s] = nt;
    segx[s] = xbits;
}

// ------------------------------------------------------------------------------ Huffman
// Code lengths for freq[0..n) limited to maxbits (Huffman by sorting + JPEG Annex K.3
// "adjust bits" length limiting, which keeps the code complete). Single thread; scratch in LDS.
// The used symbols of freq[0..n) in (freq, symbol) ascending order, by rank counting over all
// lanes of the workgroup (blockDim.x lanes; the caller synchronises before and after).
__device__ void rank_order(const uint32_t* freq, int n, uint16_t* order) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t f = freq[i];
        if (!f) continue;
        int r = 0;
        for (int j = 0; j < n; ++j) {
            const uint32_t g = freq[j];
            r += g && (g < f || (g == f && j < i));
        }
        order[r] = (uint16_t)i;
    }
}

// presorted: order[] already holds the used symbols sorted (rank_order).
__device__ void huff_lengths(const uint32_t* freq, int n, int maxbits, uint8_t* len, uint16_t* order, uint32_t* wt,
                             int16_t* parent, int* nused_out, bool presorted = false) {
    int m = 0;
    for (int i = 0; i < n; ++i) {
        len[i] = 0;
        if (freq[i]) {
            if (!presorted) order[m] = (uint16_t)i;
            ++m;
        }
    }
    *nused_out = m;
    if (m == 0) return;
    if (m == 1) {
        len[order[0]] = 1;
        return;
    }
    // insertion sort by (freq, symbol) ascending
    for (int a = 1; a < m && !presorted; ++a) {
        const uint16_t v = order[a];
        int b = a - 1;
        while (b >= 0 && (freq[order[b]] > freq[v] || (freq[order[b]] == freq[v] && order[b] > v))) {
            order[b + 1] = order[b];
            --b;
        }
        order[b + 1] = v;
    }
    // two-queue Huffman: leaves 0..m-1 (sorted), internal nodes m..2m-2
    for (int i = 0; i < m; ++i) wt[i] = freq[order[i]];
    int li = 0, ii = m, in_end = m;
    for (int k = 0; k < m - 1; ++k) {
        int pick[2];
        for (int q = 0; q < 2; ++q) {
            if (li < m && (ii >= in_end || wt[li] <= wt[ii])) pick[q] = li++;
            else pick[q] = ii++;
        }
        wt[in_end] = wt[pick[0]] + wt[pick[1]];
        parent[pick[0]] = (int16_t)in_end;
        parent[pick[1]] = (int16_t)in_end;
        ++in_end;
    }
    // depths top-down (a parent always has a larger index than its children); wt is reused
    uint32_t* dep = wt;
    dep[in_end - 1] = 0;
    for (int k = in_end - 2; k >= 0; --k) dep[k] = dep[parent[k]] + 1;
    int bl[40];
    for (int i = 0; i < 40; ++i) bl[i] = 0;
    int maxd = 0;
    for (int i = 0; i < m; ++i) {
        const int dd = dep[i] > 39 ? 39 : (int)dep[i];
        ++bl[dd];
        maxd = dd > maxd ? dd : maxd;
    }
    for (int i = maxd; i > maxbits; --i) {  // Annex K.3 Adjust_BITS
        while (bl[i] > 0) {
            int j = i - 2;
            while (j > 1 && bl[j] == 0) --j;
            bl[i] -= 2;
            bl[i - 1] += 1;
            bl[j + 1] += 2;
            bl[j] -= 1;
        }
    }
    // most frequent symbols get the shortest codes: walk sorted order from the top
    int k = m - 1;
    for (int l = 1; l <= maxbits; ++l)
        for (int c = 0; c < bl[l]; ++c) len[order[k--]] = (uint8_t)l;
}

__device__ void canon_codes(const uint8_t* len, int n, uint16_t* code) {  // RFC 1951 3.2.2, bit-reversed
    int bl[16] = {0};
    for (int i = 0; i < n; ++i) ++bl[len[i]];
    bl[0] = 0;
    int next[16];
    int c = 0;
    for (int b = 1; b < 16; ++b) {
        c = (c + bl[b - 1]) << 1;
        next[b] = c;
    }
    for (int i = 0; i < n; ++i) {
        const int l = len[i];
        code[i] = 0;
        if (!l) continue;
        const uint32_t v = (uint32_t)next[l]++;
        code[i] = (uint16_t)(__brev(v) >> (32 - l));
    }
}

struct BitW {
    uint32_t* w;
    uint32_t n = 0;  // bits written
    __device__ void put(uint32_t v, int nb) {
        if (!nb) return;
        const uint32_t s = n & 31;
        w[n >> 5] |= v << s;
        if (s + nb > 32) w[(n >> 5) + 1] |= v >> (32 - s);
        n += nb;
    }
};

// Deflate blocks: k_png_lz77 counts symbols per 256 KiB base block; consecutive base blocks
// with few tokens between them share one deflate block (one header), as zlib's blocks end at
// kBlockTokens symbols (lit_bufsize at memLevel 8) -- highly compressible input would otherwise
// pay a code-table header per 256 KiB. plan[2 b], plan[2 b + 1] = the first / last base block
// of b's deflate block. One workgroup; thread 0 groups greedily over the base blocks' symbol
// counts (k_png_lz77's, before the seams move a few tokens: the grouping only needs their size).
constexpr uint32_t kBlockTokens = 16384;
// Counts staged in LDS when they fit (kPlanLds base blocks = 4 GiB of filtered bytes); past that
// the one walking thread reads them from global memory (slower, still exact).
constexpr int64_t kPlanLds = 16384;
__global__ __launch_bounds__(256) void k_png_blockplan(const uint32_t* __restrict__ blksym, int64_t nblk,
                                                       uint32_t* __restrict__ plan, int64_t lds_max) {
    extern __shared__ uint32_t cnt[];  // min(nblk, lds_max) symbol counts
    const bool lds = nblk <= lds_max;
    if (lds)
        for (int64_t b = threadIdx.x; b < nblk; b += 256) cnt[b] = blksym[b];
    __syncthreads();
    if (threadIdx.x != 0) return;
    int64_t first = 0;
    uint32_t acc = 0;
    for (int64_t b = 0; b <= nblk; ++b) {
        const uint32_t cb = b < nblk ? (lds ? cnt[b] : blksym[b]) : 0u;
        if (b == nblk || (acc && acc + cb > kBlockTokens)) {
            for (int64_t k = first; k < b; ++k) {
                plan[2 * k] = (uint32_t)first;
                plan[2 * k + 1] = (uint32_t)(b - 1);
            }
            first = b;
            acc = 0;
        }
        acc += cb;
    }
}

// One workgroup per base block, thread 0 builds everything (deterministic, tiny); the base
// blocks of one deflate block compute the same codes from the same summed counts.
__global__ __launch_bounds__(64) void k_png_huff(const uint32_t* __restrict__ hist, int64_t nblk,
                                                 const uint32_t* __restrict__ plan, BlockCodes* __restrict__ bc) {
    __shared__ uint32_t f_ll[kNLL], f_d[kND];
    __shared__ uint16_t order[kNLL], order_d[kND];
    __shared__ uint32_t wt[2 * kNLL];
    __shared__ int16_t parent[2 * kNLL];
    __shared__ uint8_t l_ll[kNLL], l_d[kND];
    __shared__ uint8_t rle_sym[kNLL + kND];
    __shared__ uint8_t rle_ext[kNLL + kND];
    const int64_t blk = blockIdx.x, gfirst = plan[2 * blk], glast = plan[2 * blk + 1];
    for (int i = threadIdx.x; i < kNLL + kND; i += 64) {
        uint32_t f = 0;
        for (int64_t b = gfirst; b <= glast; ++b) f += hist[b * (kNLL + kND) + i];
        if (i == 256) f -= (uint32_t)(glast - gfirst);  // one EOB per deflate block
        if (i < kNLL) f_ll[i] = f;
        else f_d[i - kNLL] = f;
    }
    BlockCodes& B = bc[blk];
    for (int i = threadIdx.x; i < kHdrWords; i += 64) B.hdr[i] = 0;
    __syncthreads();
    if (threadIdx.x == 0) {  // at least two codes per tree keeps every code complete
        int u = 0;
        for (int i = 0; i < kNLL; ++i) u += f_ll[i] != 0;
        if (u < 2) f_ll[f_ll[0] ? 1 : 0] = 1;
        u = 0;
        for (int i = 0; i < kND; ++i) u += f_d[i] != 0;
        if (u < 2) {
            if (!f_d[0]) f_d[0] = 1;
            if (!f_d[1]) f_d[1] = 1;
        }
    }
    __syncthreads();
    rank_order(f_ll, kNLL, order);
    rank_order(f_d, kND, order_d);
    __syncthreads();
    if (threadIdx.x != 0) return;
    int used;
    huff_lengths(f_ll, kNLL, 15, l_ll, order, wt, parent, &used, true);
    huff_lengths(f_d, kND, 15, l_d, order_d, wt, parent, &used, true);
    canon_codes(l_ll, kNLL, B.ll_code);
    canon_codes(l_d, kND, B.d_code);
    for (int i = 0; i < kNLL; ++i) B.ll_len[i] = l_ll[i];
    for (int i = 0; i < kND; ++i) B.d_len[i] = l_d[i];
    int hlit = kNLL;
    while (hlit > 257 && l_ll[hlit - 1] == 0) --hlit;
    int hdist = kND;
    while (hdist > 1 && l_d[hdist - 1] == 0) --hdist;
    // run-length code the concatenated lengths (16: repeat 3-6, 17: zeros 3-10, 18: zeros 11-138)
    int ns = 0;
    const int tot = hlit + hdist;
    auto L = [&](int i) { return i < hlit ? l_ll[i] : l_d[i - hlit]; };
    for (int i = 0; i < tot;) {
        const int cur = L(i);
        int run = 1;
        while (i + run < tot && L(i + run) == cur) ++run;
        int left = run;
        if (cur == 0) {
            while (left >= 11) {
                const int r = min(left, 138);
                rle_sym[ns] = 18;
                rle_ext[ns++] = (uint8_t)(r - 11);
                left -= r;
            }
            if (left >= 3) {
                rle_sym[ns] = 17;
                rle_ext[ns++] = (uint8_t)(left - 3);
                left = 0;
            }
            while (left > 0) {
                rle_sym[ns] = 0;
                rle_ext[ns++] = 0;
                --left;
            }
        } else {
            rle_sym[ns] = (uint8_t)cur;
            rle_ext[ns++] = 0;
            --left;
            while (left >= 3) {
                const int r = min(left, 6);
                rle_sym[ns] = 16;
                rle_ext[ns++] = (uint8_t)(r - 3);
                left -= r;
            }
            while (left > 0) {
                rle_sym[ns] = (uint8_t)cur;
                rle_ext[ns++] = 0;
                --left;
            }
        }
        i += run;
    }
    uint32_t f_cl[19];
    for (int i = 0; i < 19; ++i) f_cl[i] = 0;
    for (int i = 0; i < ns; ++i) ++f_cl[rle_sym[i]];
    {
        int u = 0;
        for (int i = 0; i < 19; ++i) u += f_cl[i] != 0;
        if (u < 2) {
            if (!f_cl[0]) f_cl[0] = 1;
            else f_cl[1] = 1;
        }
    }
    uint8_t l_cl[19];
    uint16_t c_cl[19];
    huff_lengths(f_cl, 19, 7, l_cl, order, wt, parent, &used);
    canon_codes(l_cl, 19, c_cl);
    int hclen = 19;
    while (hclen > 4 && l_cl[kClOrder[hclen - 1]] == 0) --hclen;
    BitW bw{B.hdr};
    bw.put(glast == nblk - 1 ? 1u : 0u, 1);  // BFINAL
    bw.put(2u, 2);                          // BTYPE = dynamic
    bw.put((uint32_t)(hlit - 257), 5);
    bw.put((uint32_t)(hdist - 1), 5);
    bw.put((uint32_t)(hclen - 4), 4);
    for (int i = 0; i < hclen; ++i) bw.put(l_cl[kClOrder[i]], 3);
    for (int i = 0; i < ns; ++i) {
        const int s = rle_sym[i];
        bw.put(c_cl[s], l_cl[s]);
        if (s == 16) bw.put(rle_ext[i], 2);
        else if (s == 17) bw.put(rle_ext[i], 3);
        else if (s == 18) bw.put(rle_ext[i], 7);
    }
    B.hdr_bits = bw.n;
}

// The workgroup's block code tables -> LDS (every lane reaches the barrier).
__device__ __forceinline__ void stage_codes(const BlockCodes* __restrict__ bc, BlockCodes& B) {
    static_assert(sizeof(BlockCodes) % 4 == 0 && kSegPerBlock % 4 == 0, "staging layout");
    const uint32_t* src = reinterpret_cast<const uint32_t*>(bc + (int64_t)blockIdx.x * 4 / kSegPerBlock);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&B);
    for (int i = threadIdx.x; i < (int)(sizeof(BlockCodes) / 4); i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

// One wave per segment: the segment's symbol counts (from k_png_lz77) times the block's code
// lengths, plus the extra bits of its matches -- no pass over the tokens.
// A segment opens its deflate block (header) / closes it (EOB).
__device__ __forceinline__ bool seg_opens(int64_t seg, const uint32_t* plan) {
    return seg % kSegPerBlock == 0 && plan[2 * (seg / kSegPerBlock)] == (uint32_t)(seg / kSegPerBlock);
}
__device__ __forceinline__ bool seg_closes(int64_t seg, int64_t nseg, const uint32_t* plan) {
    return seg == nseg - 1 ||
           (seg % kSegPerBlock == kSegPerBlock - 1 && plan[2 * (seg / kSegPerBlock) + 1] == (uint32_t)(seg / kSegPerBlock));
}
__global__ __launch_bounds__(256) void k_png_segbits(int64_t nseg, const uint16_t* __restrict__ seghist,
                                                     const uint32_t* __restrict__ segx, const BlockCodes* __restrict__ bc,
                                                     const uint32_t* __restrict__ plan, unsigned long long* __restrict__ bits) {
    __shared__ BlockCodes B;  // the four waves' segments share one block (kSegPerBlock % 4 == 0)
    stage_codes(bc, B);
    const int64_t seg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (seg >= nseg) return;  // wave-uniform
    const uint16_t* G = seghist + seg * (kNLL + kND);
    uint32_t b = 0;
    for (int i = lane; i < kNLL + kND; i += 64) b += (uint32_t)G[i] * (i < kNLL ? B.ll_len[i] : B.d_len[i - kNLL]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) b += __shfl_xor(b, o);
    if (lane == 0) {
        unsigned long long t = (unsigned long long)b + segx[seg];
        if (seg_opens(seg, plan)) t += B.hdr_bits;
        if (seg_closes(seg, nseg, plan)) t += B.ll_len[256];  // EOB
        bits[seg] = t;
    }
}

// Token slot i -> (bits, count), LSB-first: a literal; or, at a match's length slot, code, length
// extra, distance code, distance extra (at most 15 + 5 + 15 + 13 = 48 bits); a distance slot
// emits nothing (its match's length slot took it).
__device__ __forceinline__ uint64_t token_code(const BlockCodes& B, uint32_t t, uint32_t tnext, int& nb) {
    if (t < 256) {
        nb = B.ll_len[t];
        return B.ll_code[t];
    }
    if (t & 0x8000u) {
        nb = 0;
        return 0;
    }
    const int len = (int)(t & 255) + 3, dist = (int)(tnext & 0x7FFFu) + 1;
    const int lc = len_code(len), dc = dist_code(dist);
    uint64_t v = B.ll_code[257 + lc];
    int n = B.ll_len[257 + lc];
    v |= (uint64_t)(len - kLenBase[lc]) << n;
    n += kLenExtra[lc];
    v |= (uint64_t)B.d_code[dc] << n;
    n += B.d_len[dc];
    v |= (uint64_t)(dist - kDistBase[dc]) << n;
    nb = n + kDistExtra[dc];
    return v;
}

// One wave per segment: each round of 64 tokens gets bit offsets from a wave prefix sum and is
// OR-ed into the wave's LDS image of the segment's output words (aligned to the output's word
// grid), which then leaves with coalesced stores -- the two boundary words (shared with the
// neighbouring segments) with atomicOr. Segments whose bits exceed the LDS image (pathological
// token mixes only) OR their words straight into the output.
constexpr int kEmitWords = 2048;  // 64 Kbit per wave (a 4 KiB segment averages ~22 Kbit)
__device__ __forceinline__ void or_bits(uint32_t* w, unsigned long long bitpos, uint64_t v, int nb) {
    if (!nb) return;
    const unsigned long long wi = bitpos >> 5;
    const int sh = (int)(bitpos & 31);
    const uint64_t hi = sh ? (v >> (32 - sh)) : (v >> 32);  // the bits above word wi
    atomicOr(w + wi, (uint32_t)(v << sh));
    if (sh + nb > 32) atomicOr(w + wi + 1, (uint32_t)hi);
    if (sh + nb > 64) atomicOr(w + wi + 2, (uint32_t)(hi >> 32));
}
// The segment's bits into W (word 0 = output word w0; zeroed), starting at bit `pos`: its nh
// re-parsed head slots Hd, then its own slots T[0 .. nt).
__device__ __forceinline__ void emit_segment(uint32_t* W, unsigned long long pos, const BlockCodes& B,
                                             const uint16_t* Hd, uint32_t nh, const uint16_t* T, uint32_t nt,
                                             bool head, bool eob, int lane) {
    if (head) {  // the block header: its words, shifted into place
        const uint32_t hb = B.hdr_bits;
        for (uint32_t i = lane; i * 32 < hb; i += 64) {
            const int n = (int)min(32u, hb - i * 32);
            or_bits(W, pos + i * 32, n == 32 ? B.hdr[i] : (B.hdr[i] & ((1u << n) - 1u)), n);
        }
        pos += hb;
    }
    const uint32_t n = nh + nt;
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
        const uint32_t i = i0 + lane;
        int nb = 0;
        uint64_t v = 0;
        if (i < nh) v = token_code(B, Hd[i], i + 1 < nh ? Hd[i + 1] : 0u, nb);
        else if (i < n) v = token_code(B, T[i - nh], i + 1 < n ? T[i + 1 - nh] : 0u, nb);
        uint32_t inc;  // inclusive scan of nb over the wave (rocprim's DPP cross-lane scan)
        using WScan = rocprim::warp_scan<uint32_t, 64>;
        typename WScan::storage_type wst;  // empty for the cross-lane implementation
        WScan().inclusive_scan((uint32_t)nb, inc, wst);
        or_bits(W, pos + inc - nb, v, nb);
        pos += (uint32_t)rdl((int)inc, 63);
    }
    if (eob && lane == 0) or_bits(W, pos, B.ll_code[256], B.ll_len[256]);
}
// emit_segment for the wave's LDS image (round 6): each lane takes kRun consecutive token slots,
// one wave prefix sum of the lanes' bit totals places them, and each lane packs its slots into
// whole words in a register -- the words it fills alone are plain stores, only its first and last
// (shared with the neighbouring lanes) are atomicOr. (One slot per lane OR-ed every token into LDS
// with up to three atomics, several lanes on each word.)
constexpr int kRun = 8;
__device__ __forceinline__ void emit_segment_runs(uint32_t* W, unsigned long long pos, const BlockCodes& B,
                                                  const uint16_t* Hd, uint32_t nh, const uint16_t* T, uint32_t nt,
                                                  bool head, bool eob, int lane) {
    if (head) {  // the block header: its words, shifted into place
        const uint32_t hb = B.hdr_bits;
        for (uint32_t i = lane; i * 32 < hb; i += 64) {
            const int n = (int)min(32u, hb - i * 32);
            or_bits(W, pos + i * 32, n == 32 ? B.hdr[i] : (B.hdr[i] & ((1u << n) - 1u)), n);
        }
        pos += hb;
    }
    const uint32_t n = nh + nt;
    auto slot = [&](uint32_t i) -> uint32_t { return i < nh ? (uint32_t)Hd[i] : (uint32_t)T[i - nh]; };
    for (uint32_t i0 = 0; i0 < n; i0 += 64 * kRun) {
        const uint32_t ib = i0 + (uint32_t)lane * kRun;
        uint64_t v[kRun];
        int nb[kRun];
        uint32_t tot = 0;
#pragma unroll
        for (int r = 0; r < kRun; ++r) {
            const uint32_t i = ib + r;
            nb[r] = 0;
            v[r] = i < n ? token_code(B, slot(i), i + 1 < n ? slot(i + 1) : 0u, nb[r]) : 0;
            tot += (uint32_t)nb[r];
        }
        uint32_t inc;  // inclusive scan of the lanes' bit totals (rocprim's DPP cross-lane scan)
        using WScan = rocprim::warp_scan<uint32_t, 64>;
        typename WScan::storage_type wst;
        WScan().inclusive_scan(tot, inc, wst);
        const unsigned long long s0 = pos + inc - tot;
        uint32_t wi = (uint32_t)(s0 >> 5);
        int an = (int)(s0 & 31);
        uint64_t acc = 0;
        bool first = true;
        auto put = [&](uint32_t piece, int k) {  // k <= 32 bits; an < 32 before
            acc |= (uint64_t)piece << an;
            an += k;
            if (an >= 32) {
                if (first) atomicOr(W + wi, (uint32_t)acc);  // (shared with the lane before)
                else W[wi] = (uint32_t)acc;
                first = false;
                ++wi;
                acc >>= 32;
                an -= 32;
            }
        };
#pragma unroll
        for (int r = 0; r < kRun; ++r) {
            if (nb[r] > 32) {
                put((uint32_t)v[r], 32);
                put((uint32_t)(v[r] >> 32), nb[r] - 32);
            } else if (nb[r] > 0) {
                put((uint32_t)v[r], nb[r]);
            }
        }
        if (tot && an > 0) atomicOr(W + wi, (uint32_t)acc);  // (shared with the lane after)
        pos += (uint32_t)rdl((int)inc, 63);
    }
    if (eob && lane == 0) or_bits(W, pos, B.ll_code[256], B.ll_len[256]);
}

// The file's layout once the deflate stream's length is known, on the device (k_png_size): the
// rest of the encode reads it there, so no host read-back sits between the deflate and the file.
struct PngTail {
    unsigned long long dbytes;  // deflate stream bytes (zero-padded to a byte)
    unsigned long long zlen;    // zlib stream: 2 + dbytes + 4 (Adler-32)
    unsigned long long total;   // file bytes
    unsigned long long fits;    // total <= cap: only then is anything written to the output
};
__device__ __forceinline__ bool png_fits(const PngTail* t) { return t->fits != 0; }

__global__ __launch_bounds__(256) void k_png_emit(int64_t nseg, const uint16_t* __restrict__ tok,
                                                  const uint32_t* __restrict__ ntok, const uint32_t* __restrict__ seam,
                                                  const uint16_t* __restrict__ hbuf, const BlockCodes* __restrict__ bc,
                                                  const uint32_t* __restrict__ plan,
                                                  const unsigned long long* __restrict__ off,
                                                  const unsigned long long* __restrict__ bits, uint32_t* __restrict__ out,
                                                  unsigned long long base_bits, const struct PngTail* __restrict__ tl) {
    __shared__ uint32_t img[4][kEmitWords];
    __shared__ BlockCodes B;  // the four waves' segments share one block
    stage_codes(bc, B);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t seg = (int64_t)blockIdx.x * 4 + wave;
    if (seg >= nseg || !png_fits(tl)) return;  // wave-uniform; no block barriers below
    const uint32_t skip = seam[4 * seg + 1], nh = seam[4 * seg + 2];
    const uint16_t* T = tok + seg * kSlots + skip;
    const uint16_t* Hd = hbuf + seg * kHead;
    const uint32_t nt = ntok[seg] - skip;
    const unsigned long long o0 = base_bits + off[seg], o1 = o0 + bits[seg];
    if (o1 == o0) return;
    const unsigned long long w0 = o0 >> 5, wl = (o1 - 1) >> 5;  // first / last output word
    const int nw = (int)(wl - w0 + 1);
    const bool head = seg_opens(seg, plan), eob = seg_closes(seg, nseg, plan);
    if (nw > kEmitWords) {  // straight into the (zeroed) output
        emit_segment(out + w0, o0 & 31, B, Hd, nh, T, nt, head, eob, lane);
        return;
    }
    uint32_t* W = img[wave];
    for (int i = lane; i < nw; i += 64) W[i] = 0;
    __builtin_amdgcn_wave_barrier();
    emit_segment_runs(W, o0 & 31, B, Hd, nh, T, nt, head, eob, lane);
    __builtin_amdgcn_wave_barrier();
    for (int i = lane; i < nw; i += 64) {
        const uint32_t v = W[i];
        if (i == 0 || i == nw - 1) atomicOr(out + w0 + i, v);  // shared with the neighbours
        else out[w0 + i] = v;
    }
}

// ------------------------------------------------------------------------------- CRC-32
__device__ __forceinline__ uint32_t crc_table(uint32_t i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = c & 1 ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    return c;
}
// The raw CRC (register starting at 0, no final xor) is linear and leading zero bytes leave it
// at 0, so the range is cut into kCrcSeg-byte segments aligned to its END (the first one padded
// with zeros in front): raw(range) = sum_r raw(seg_r) * X^r over r = segments after seg_r,
// X = x^(8 kCrcSeg) mod P. One lane per segment (slicing-by-4 tables in LDS, dword loads);
// k_png_crc_reduce folds 256 consecutive r at a time (X -> X^256 per pass).
__global__ __launch_bounds__(256) void k_png_crc_seg(const uint8_t* __restrict__ p, const PngTail* __restrict__ tl,
                                                     int64_t nseg, uint32_t* __restrict__ part) {
    __shared__ uint32_t tab[4][256];
    uint32_t t = crc_table(threadIdx.x);
    tab[0][threadIdx.x] = t;
    __syncthreads();
#pragma unroll
    for (int k = 1; k < 4; ++k) {
        t = (t >> 8) ^ tab[0][t & 255];
        tab[k][threadIdx.x] = t;
    }
    __syncthreads();
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;  // segments after this one
    if (r >= nseg) return;
    // (nseg covers the largest stream that fits; segments before the real one's start are 0)
    const int64_t n = png_fits(tl) ? (int64_t)tl->zlen + 4 : 0;  // "IDAT" + the zlib stream
    const int64_t b = n - r * kCrcSeg, a = max((int64_t)0, b - kCrcSeg);
    uint32_t c = 0;
    int64_t i = a;
    // (the range's first 4 bytes enter complemented: that is the 0xFFFFFFFF register start)
    for (; i < b && (i < 4 || (reinterpret_cast<uintptr_t>(p + i) & 3)); ++i)
        c = tab[0][(c ^ (i < 4 ? (uint8_t)~p[i] : p[i])) & 255] ^ (c >> 8);
    for (; i + 4 <= b; i += 4) {
        c ^= *reinterpret_cast<const uint32_t*>(p + i);
        c = tab[3][c & 255] ^ tab[2][(c >> 8) & 255] ^ tab[1][(c >> 16) & 255] ^ tab[0][c >> 24];
    }
    for (; i < b; ++i) c = tab[0][(c ^ p[i]) & 255] ^ (c >> 8);
    part[r] = c;
}
// a(x) * b(x) mod P(x), reflected (bit 31 = x^0)
__device__ __host__ inline uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = b & 1 ? (b >> 1) ^ 0xEDB88320u : b >> 1;
    }
    return p;
}
__device__ __host__ inline uint32_t x8n(uint64_t n) {  // x^(8n) mod P
    uint32_t r = 1u << 31, sq = 1u << 23;            // x^0 ; x^8
    while (n) {
        if (n & 1) r = multmodp(sq, r);
        sq = multmodp(sq, sq);
        n >>= 1;
    }
    return r;
}
// One pass of the fold: out[j] = sum_{k<256} in[256 j + k] * X^k (entries past `n` are 0).
__global__ __launch_bounds__(256) void k_png_crc_reduce(const uint32_t* __restrict__ in, int64_t n, uint32_t X,
                                                        uint32_t* __restrict__ out) {
    __shared__ uint32_t v[256];
    __shared__ uint32_t xp[8];  // X^(2^k)
    if (threadIdx.x == 0) {
        uint32_t x = X;
        for (int k = 0; k < 8; ++k) {
            xp[k] = x;
            x = multmodp(x, x);
        }
    }
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    v[threadIdx.x] = i < n ? in[i] : 0u;
    __syncthreads();
    for (int k = 0; k < 8; ++k) {
        const int s = 1 << k;
        if ((threadIdx.x & (2 * s - 1)) == 0) v[threadIdx.x] ^= multmodp(xp[k], v[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = v[0];
}

__global__ void k_png_adler(const uint32_t* __restrict__ adl, int64_t nseg, uint32_t* __restrict__ out) {
    // two sums over segment partials, one lane each (nseg is small: N / 4 KiB)
    __shared__ unsigned long long s[2][256];
    unsigned long long a = 0, b = 0;
    for (int64_t i = threadIdx.x; i < nseg; i += 256) {
        a += adl[2 * i];
        b += adl[2 * i + 1];
    }
    s[0][threadIdx.x] = a;
    s[1][threadIdx.x] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long A = 0, B = 0;
        for (int i = 0; i < 256; ++i) {
            A += s[0][i];
            B += s[1][i];
        }
        out[0] = (uint32_t)(A % kAdlerMod);
        out[1] = (uint32_t)(B % kAdlerMod);
    }
}

// ---- the file's tail on the device (png_encoder.cpp:1888-1952 zlib, :2277 chunk CRC) -------
__device__ __forceinline__ void be32_dev(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}
// Stream length from the last segment's bit offset -> the file layout (one thread).
__global__ void k_png_size(const unsigned long long* __restrict__ off, const unsigned long long* __restrict__ bits,
                           int64_t nseg, unsigned long long data_at, unsigned long long cap, PngTail* __restrict__ tl) {
    const unsigned long long dbytes = (off[nseg - 1] + bits[nseg - 1] + 7) / 8;  // zero-padded to a byte
    const unsigned long long zlen = 2 + dbytes + 4;
    const unsigned long long total = data_at + zlen + 4 + 12;  // + IDAT CRC + IEND chunk
    tl->dbytes = dbytes;
    tl->zlen = zlen;
    tl->total = total;
    tl->fits = total <= cap ? 1ull : 0ull;
}
// Zeroes the words k_png_emit ORs into (from the 4-aligned word before the deflate data to one
// word past it), when the file fits, with 16-byte stores over that range widened to 16-byte
// bounds: the widening stays inside the file (the zlib header before it and the Adler-32, CRC
// and IEND after it are written afterwards).
__global__ __launch_bounds__(256) void k_png_zero(uint32_t* __restrict__ w, unsigned long long mis,
                                                  const PngTail* __restrict__ tl) {
    if (!png_fits(tl)) return;
    const unsigned long long nb = ((tl->dbytes + mis + 3) & ~3ull) + 4;  // bytes from w
    const uintptr_t a = reinterpret_cast<uintptr_t>(w), a16 = a & ~(uintptr_t)15, e16 = (a + nb + 15) & ~(uintptr_t)15;
    uint4* q = reinterpret_cast<uint4*>(a16);
    const unsigned long long n16 = (e16 - a16) / 16;
    for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (unsigned long long)gridDim.x * 256)
        q[i] = make_uint4(0, 0, 0, 0);
}
// After the emit: the header bytes (signature .. IDAT type + zlib header 78 01, built on the host
// and staged in device memory), the IDAT length and the Adler-32 (s1 = 1 + sum of bytes,
// s2 = N + the weighted sum, both mod 65521; the segment sums are in ad[0..1]).
__global__ __launch_bounds__(256) void k_png_head(uint8_t* __restrict__ out, const uint8_t* __restrict__ pre, int npre,
                                                  unsigned long long idat_at, unsigned long long dstart,
                                                  const uint32_t* __restrict__ ad, long long N,
                                                  const PngTail* __restrict__ tl) {
    if (!png_fits(tl)) return;
    for (int i = threadIdx.x; i < npre; i += 256) out[i] = pre[i];
    __syncthreads();
    if (threadIdx.x == 0) {
        be32_dev(out + idat_at, (uint32_t)tl->zlen);
        const uint32_t s1 = (1 + ad[0]) % kAdlerMod, s2 = (uint32_t)(((unsigned long long)N + ad[1]) % kAdlerMod);
        be32_dev(out + dstart + tl->dbytes, s2 << 16 | s1);
    }
}
// The IDAT chunk's CRC-32 (k_png_crc_seg's raw CRC over "IDAT" and the zlib stream with the
// first 4 bytes complemented = the standard register start; the final complement here) and the
// IEND chunk.
__global__ void k_png_tail(uint8_t* __restrict__ out, unsigned long long data_at, const uint32_t* __restrict__ crc_sum,
                           const PngTail* __restrict__ tl) {
    if (!png_fits(tl)) return;
    uint8_t* t = out + data_at + tl->zlen;
    be32_dev(t, ~crc_sum[0]);
    const uint8_t iend[12] = {0, 0, 0, 0, 'I', 'E', 'N', 'D', 0xAE, 0x42, 0x60, 0x82};
    for (int i = 0; i < 12; ++i) t[4 + i] = iend[i];
}

}  // namespace png

// =============================================================================== host side
using namespace png;

struct PngWs {
    Stats* st = nullptr;
    unsigned long long *set_key = nullptr, *set_idx = nullptr;
    Mode* mode = nullptr;
    uint8_t *conv = nullptr, *filt = nullptr;
    size_t conv_cap = 0, filt_cap = 0;
    uint16_t* tok = nullptr;  // token slots: literal byte, or a match's length slot + distance slot
    uint32_t *ntok = nullptr, *hist = nullptr, *adl = nullptr, *crc = nullptr, *small = nullptr;
    size_t tok_cap = 0, seg_cap = 0, blk_cap = 0, hist_cap = 0, crc_cap = 0;
    BlockCodes* bc = nullptr;
    unsigned long long *bits = nullptr, *off = nullptr;
    uint16_t* seghist = nullptr;  // per segment: literal/length and distance symbol counts
    uint32_t* segx = nullptr;     // per segment: extra bits of its matches
    uint32_t* seam = nullptr;     // per segment: overhang, head skip, head slots, cut (k_png_seam)
    uint16_t* head = nullptr;     // per segment: kHead re-parsed head slots
    uint32_t* plan = nullptr;     // per base block: first / last base block of its deflate block
    uint32_t* blksym = nullptr;   // per base block: symbols k_png_lz77 counted (+ EOB)
    size_t seghist_cap = 0, segx_cap = 0, seam_cap = 0, head_cap = 0, plan_cap = 0, blksym_cap = 0;
    void* tmp = nullptr;
    size_t tmp_cap = 0;
    struct PngHost* host = nullptr;  // pinned read-back buffer (PngJob)
    png::PngTail* tl = nullptr;      // device: the file layout (k_png_size)
    uint8_t* predev = nullptr;       // device copy of the header bytes (k_png_head)
    hipEvent_t done = nullptr;       // a job's statistics event
    // per-stage HIP events (icx_png_encoder_stage_times): stage i spans ev[s][2i] .. ev[s][2i+1],
    // two sets used by alternate images, so one image's times are read once the next image's
    // statistics are in (its kernels are done by then); ms[] accumulates until read
    static constexpr int kStages = 6;
    hipEvent_t ev[2][2 * kStages] = {};
    int evset = 0;          // the set the next image records into
    bool ev_pending = false;  // the other set holds an image's events not yet read
    float ms[kStages] = {};
    void read_times(int set) {
        for (int i = 0; i < kStages; ++i) {
            float t = 0.f;
            if (hipEventElapsedTime(&t, ev[set][2 * i], ev[set][2 * i + 1]) == hipSuccess) ms[i] += t;
        }
    }
    ~PngWs() {
        for (auto& set : ev)
            for (hipEvent_t e : set)
                if (e) (void)hipEventDestroy(e);
        if (done) (void)hipEventDestroy(done);
        if (host) (void)hipHostFree(host);
        for (void* p : {(void*)tl, (void*)predev, (void*)st, (void*)set_key, (void*)set_idx, (void*)mode, (void*)conv, (void*)filt, (void*)tok,
                        (void*)ntok, (void*)hist, (void*)adl, (void*)crc, (void*)small, (void*)bc, (void*)bits,
                        (void*)off, (void*)seghist, (void*)segx, (void*)seam, (void*)head, (void*)plan, (void*)blksym, tmp})
            if (p) (void)hipFree(p);
    }
};
PngWs* png_ws_create() {
    PngWs* ws = new PngWs();
    for (auto& set : ws->ev)
        for (hipEvent_t& e : set)
            if (hipEventCreate(&e) != hipSuccess) e = nullptr;
    return ws;
}
static const char* const kPngStageNames[PngWs::kStages] = {"stats", "filter", "lz77", "huff", "emit", "crc"};
int png_ws_stage_times(PngWs* ws, const char** names, float* ms, int cap) {
    if (ws->ev_pending && hipEventQuery(ws->ev[ws->evset ^ 1][2 * PngWs::kStages - 1]) == hipSuccess) {
        ws->read_times(ws->evset ^ 1);  // (the last image encoded)
        ws->ev_pending = false;
    }
    const int k = cap < PngWs::kStages ? cap : PngWs::kStages;
    for (int i = 0; i < k; ++i) {
        if (names) names[i] = kPngStageNames[i];
        if (ms) ms[i] = ws->ms[i];
    }
    for (float& m : ws->ms) m = 0.f;
    return k;
}
void png_ws_destroy(PngWs* ws) { delete ws; }

#define PNG_HIP(call)                               \
    do {                                            \
        if ((call) != hipSuccess) return -1;        \
    } while (0)

// ICX_PNG_SEAM=0: cut every overhanging match back to its segment end (no re-parsed heads).
static int seam_join() {
    const char* e = std::getenv("ICX_PNG_SEAM");
    return !(e && e[0] == '0');
}
template <class T>
static bool pgrow(T*& p, size_t bytes, size_t& cap) {
    if (p && bytes <= cap) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, std::max<size_t>(bytes, 64)) != hipSuccess) return false;
    cap = bytes;
    return true;
}

static void be32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}
static uint32_t crc32_host(uint32_t c, const uint8_t* p, size_t n) {  // standard CRC-32, running
    c = ~c;
    for (size_t i = 0; i < n; ++i) {
        c ^= p[i];
        for (int k = 0; k < 8; ++k) c = c & 1 ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    }
    return ~c;
}
static void chunk(std::vector<uint8_t>& o, const char* type, const uint8_t* data, uint32_t n) {
    uint8_t h[8];
    be32(h, n);
    std::memcpy(h + 4, type, 4);
    o.insert(o.end(), h, h + 8);
    if (n) o.insert(o.end(), data, data + n);
    uint8_t c[4];
    be32(c, crc32_host(0, o.data() + o.size() - n - 4, n + 4));
    o.insert(o.end(), c, c + 4);
}

// Host-visible results of one encode, read back between its phases (pinned: the copies into it
// are asynchronous and the host waits on an event, not on the stream).
struct PngHost {
    Stats S;
    uint8_t pre[2048];  // signature + IHDR / PLTE / tRNS + IDAT header + zlib header
    png::PngTail tl;    // png_encode_device's layout read-back (pinned with the rest: no per-call allocation)
};

// One image's encode as two issue phases with one host read between them (png_encode_device
// runs them back to back; png_encode_device_batch keeps several images in flight on their own
// workspaces and streams, so one image's kernels run while the host reads another's statistics):
//   A  colour statistics                                                        -> Stats (host)
//   B  (host: colour mode, palette, header bytes) convert, filter, LZ77, Huffman, bit offsets;
//      then on the device: the file layout (k_png_size), emit, header / IDAT length / Adler-32
//      (k_png_head), the IDAT CRC-32 and IEND (k_png_tail) -- written only when the file fits;
//      the layout goes to `out_tl` (pinned) with the image's other work, read after the stream
struct PngJob {
    PngWs* ws = nullptr;
    PngHost* hb = nullptr;
    png::PngTail* out_tl = nullptr;  // pinned: where the image's layout lands
    hipStream_t st = nullptr;
    hipEvent_t ev = nullptr;  // recorded after phase A's read-back
    int w = 0, h = 0, d = 0;
    const uint8_t* d_src = nullptr;
    uint8_t* d_out = nullptr;
    uint64_t cap = 0;
    Mode M{};
    std::vector<uint8_t> head;
    int64_t N = 0, nseg = 0, nblk = 0;
    unsigned gwave = 0;
    bool timed = false;
    int set = 0;
    void mark(int i) {  // event i: stage i/2 begins (even) or ends (odd)
        if (timed) (void)hipEventRecord(ws->ev[set][i], st);
    }
    int issue_a();
    int issue_b();  // after ev of A: everything else, no further host read
};

int PngJob::issue_a() {
    const int64_t np = (int64_t)w * h;
    set = ws->evset;
    timed = ws->ev[set][2 * PngWs::kStages - 1] != nullptr;
    size_t c1 = ws->st ? sizeof(Stats) : 0, c2 = ws->set_key ? kSetSlots * 8 : 0, c3 = c2, c4 = ws->mode ? sizeof(Mode) : 0;
    if (!pgrow(ws->st, sizeof(Stats), c1) || !pgrow(ws->set_key, kSetSlots * 8, c2) ||
        !pgrow(ws->set_idx, kSetSlots * 8, c3) || !pgrow(ws->mode, sizeof(Mode), c4))
        return -1;
    // ---- P1: colour statistics (lodepng_compute_color_stats) and auto_choose_color
    Stats zero{};
    zero.bits = 1;
    zero.first_a0 = ~0ull;
    hb->S = zero;
    PNG_HIP(hipMemcpyAsync(ws->st, &hb->S, sizeof zero, hipMemcpyHostToDevice, st));
    PNG_HIP(hipMemsetAsync(ws->set_key, 0, kSetSlots * 8, st));
    PNG_HIP(hipMemsetAsync(ws->set_idx, 0xFF, kSetSlots * 8, st));
    mark(0);
    const int gs = (int)std::max<int64_t>(1, std::min<int64_t>((np + 255) / 256, 4096));
    if (np) hipLaunchKernelGGL(k_png_stats, dim3(gs), dim3(256), 0, st, d_src, np, d, ws->st, ws->set_key, ws->set_idx);
    mark(1);
    PNG_HIP(hipMemcpyAsync(&hb->S, ws->st, sizeof(Stats), hipMemcpyDeviceToHost, st));
    PNG_HIP(hipEventRecord(ev, st));
    return 0;
}

int PngJob::issue_b() {
    const int64_t np = (int64_t)w * h;
    if (ws->ev_pending) {  // the previous image on this workspace ran before this one's statistics
        ws->read_times(set ^ 1);
        ws->ev_pending = false;
    }
    const int gs = (int)std::max<int64_t>(1, std::min<int64_t>((np + 255) / 256, 4096));
    Stats S = hb->S;
    uint32_t kr = 0, kg = 0, kb = 0;
    bool alpha = S.alpha_mid != 0, key = false;
    if (d == 4 && !alpha && S.any_a0) {  // (rare: a colour key candidate; read back synchronously)
        uint8_t kp[4];
        PNG_HIP(hipMemcpyAsync(kp, d_src + S.first_a0 * 4, 4, hipMemcpyDeviceToHost, st));
        PNG_HIP(hipStreamSynchronize(st));
        kr = kp[0];
        kg = kp[1];
        kb = kp[2];
        hipLaunchKernelGGL(k_png_keycheck, dim3(gs), dim3(256), 0, st, d_src, np, kr | kg << 8 | kb << 16, ws->st);
        PNG_HIP(hipMemcpyAsync(&hb->S, ws->st, sizeof S, hipMemcpyDeviceToHost, st));
        PNG_HIP(hipStreamSynchronize(st));
        S = hb->S;
        alpha = S.a2 || S.a3;
        key = !alpha;
    }
    uint32_t bits = S.bits;
    const bool colored = S.colored != 0;
    if (colored || alpha) bits = std::max(bits, 8u);  // :3480, :3491, :3503
    const uint32_t ncol = S.overflow ? 257u : std::min(S.ncolors, 257u);
    // auto_choose_color (:3552-3616)
    if (key && np <= 16) {
        alpha = true;
        key = false;
        bits = std::max(bits, 8u);
    }
    const bool gray_ok = !colored;
    if (!gray_ok && bits < 8) bits = 8;
    const uint32_t palettebits = ncol <= 2 ? 1 : (ncol <= 4 ? 2 : (ncol <= 16 ? 4 : 8));
    bool palette_ok = ncol <= 256 && bits <= 8 && ncol != 0;
    if ((uint64_t)np < (uint64_t)ncol * 2) palette_ok = false;
    if (gray_ok && !alpha && bits <= palettebits) palette_ok = false;
    std::memset(&M, 0, sizeof M);
    bool key_defined = false;
    uint32_t key16[3] = {kr + (kr << 8), kg + (kg << 8), kb + (kb << 8)};
    if (palette_ok) {
        M.colortype = kPalette;
        M.bitdepth = (int)palettebits;
        std::vector<unsigned long long> keys(kSetSlots), idx(kSetSlots);
        PNG_HIP(hipMemcpyAsync(keys.data(), ws->set_key, kSetSlots * 8, hipMemcpyDeviceToHost, st));
        PNG_HIP(hipMemcpyAsync(idx.data(), ws->set_idx, kSetSlots * 8, hipMemcpyDeviceToHost, st));
        PNG_HIP(hipStreamSynchronize(st));
        std::vector<std::pair<unsigned long long, uint32_t>> cols;
        for (int i = 0; i < kSetSlots; ++i)
            if (keys[i]) cols.push_back({idx[i], (uint32_t)keys[i]});
        std::sort(cols.begin(), cols.end());  // first-seen order (lodepng's palette order, :3500-3509)
        M.npal = (int)cols.size();
        for (int i = 0; i < M.npal; ++i) M.pal[i] = cols[i].second;
    } else {
        M.bitdepth = (int)bits;
        M.colortype = alpha ? (gray_ok ? kGreyAlpha : kRGBA) : (gray_ok ? kGrey : kRGB);
        if (key) {
            const uint32_t mask = (1u << M.bitdepth) - 1u;
            key_defined = true;
            for (uint32_t& k : key16) k &= mask;
        }
    }
    const int ch = M.colortype == kRGB ? 3 : M.colortype == kRGBA ? 4 : M.colortype == kGreyAlpha ? 2 : 1;
    M.bpp = ch * M.bitdepth;
    M.bw = (M.bpp + 7) / 8;
    M.lb = ((int64_t)w * M.bpp + 7) / 8;
    PNG_HIP(hipMemcpyAsync(ws->mode, &M, sizeof M, hipMemcpyHostToDevice, st));

    // ---- header bytes (host; tiny)
    head.assign({137, 80, 78, 71, 13, 10, 26, 10});
    uint8_t ihdr[13];
    be32(ihdr, (uint32_t)w);
    be32(ihdr + 4, (uint32_t)h);
    ihdr[8] = (uint8_t)M.bitdepth;
    ihdr[9] = (uint8_t)M.colortype;
    ihdr[10] = ihdr[11] = ihdr[12] = 0;
    chunk(head, "IHDR", ihdr, 13);
    if (M.colortype == kPalette) {
        uint8_t pl[768];
        for (int i = 0; i < M.npal; ++i) {
            pl[3 * i] = (uint8_t)M.pal[i];
            pl[3 * i + 1] = (uint8_t)(M.pal[i] >> 8);
            pl[3 * i + 2] = (uint8_t)(M.pal[i] >> 16);
        }
        chunk(head, "PLTE", pl, (uint32_t)M.npal * 3);
        uint32_t ntr = (uint32_t)M.npal;
        while (ntr && (M.pal[ntr - 1] >> 24) == 255) --ntr;
        uint8_t tr[256];
        for (uint32_t i = 0; i < ntr; ++i) tr[i] = (uint8_t)(M.pal[i] >> 24);
        if (ntr) chunk(head, "tRNS", tr, ntr);
    } else if (key_defined && M.colortype == kGrey) {
        uint8_t tr[2] = {(uint8_t)(key16[0] >> 8), (uint8_t)key16[0]};
        chunk(head, "tRNS", tr, 2);
    } else if (key_defined && M.colortype == kRGB) {
        uint8_t tr[6];
        for (int i = 0; i < 3; ++i) {
            tr[2 * i] = (uint8_t)(key16[i] >> 8);
            tr[2 * i + 1] = (uint8_t)key16[i];
        }
        chunk(head, "tRNS", tr, 6);
    }

    // ---- P2: convert (unless the input already is the chosen mode) and filter
    N = (int64_t)h * (1 + M.lb);
    const bool identity = (M.colortype == kRGBA && d == 4) || (M.colortype == kRGB && d == 3);
    const uint8_t* img = d_src;
    mark(2);
    if (!identity) {
        if (!pgrow(ws->conv, (size_t)(M.lb * h), ws->conv_cap)) return -1;
        const int gc = (int)std::max<int64_t>(1, std::min<int64_t>((M.lb * h + 255) / 256, 16384));
        hipLaunchKernelGGL(k_png_convert, dim3(gc), dim3(256), 0, st, d_src, w, h, d, ws->mode, ws->conv);
        img = ws->conv;
    }
    if (!pgrow(ws->filt, (size_t)N, ws->filt_cap)) return -1;
    hipLaunchKernelGGL(k_png_filter, dim3(std::max(1, std::min(h, 16384))), dim3(256), 0, st, img, h, ws->mode, ws->filt);
    mark(3);

    // ---- P3/P4: deflate
    nseg = (N + kSeg - 1) / kSeg;
    nblk = (nseg + kSegPerBlock - 1) / kSegPerBlock;
    size_t c5 = ws->seg_cap, c6 = ws->seg_cap, c7 = ws->seg_cap, c8 = ws->seg_cap;
    if (!pgrow(ws->tok, (size_t)nseg * kSlots * 2, ws->tok_cap)) return -1;
    if ((size_t)nseg * 8 > ws->seg_cap || !ws->ntok) {
        if (!pgrow(ws->ntok, (size_t)nseg * 8, c5) || !pgrow(ws->adl, (size_t)nseg * 8, c6) ||
            !pgrow(ws->bits, (size_t)nseg * 8, c7) || !pgrow(ws->off, (size_t)nseg * 8, c8))
            return -1;
        ws->seg_cap = (size_t)nseg * 8;
    }
    if (!pgrow(ws->hist, (size_t)nblk * (kNLL + kND) * 4, ws->hist_cap) ||
        !pgrow(ws->bc, (size_t)nblk * sizeof(BlockCodes), ws->blk_cap))
        return -1;
    size_t c11 = ws->small ? 64 : 0;
    if (!pgrow(ws->small, 64, c11)) return -1;
    mark(4);
    if (!pgrow(ws->seghist, (size_t)nseg * (kNLL + kND) * 2, ws->seghist_cap) ||
        !pgrow(ws->segx, (size_t)nseg * 4, ws->segx_cap) || !pgrow(ws->seam, (size_t)nseg * 16, ws->seam_cap) ||
        !pgrow(ws->head, (size_t)nseg * kHead * 2, ws->head_cap) || !pgrow(ws->plan, (size_t)nblk * 8, ws->plan_cap) ||
        !pgrow(ws->blksym, (size_t)nblk * 4, ws->blksym_cap))
        return -1;
    hipLaunchKernelGGL(k_png_lz77, dim3((unsigned)nblk), dim3(256), 0, st, ws->filt, N, nseg, 1 + M.lb, M.bw, ws->tok,
                       ws->ntok, ws->hist, ws->adl, ws->seghist, ws->segx, ws->seam, ws->blksym);
    gwave = (unsigned)((nseg + 3) / 4);  // one wave per segment
    hipLaunchKernelGGL(k_png_seam, dim3(gwave), dim3(256), 0, st, ws->filt, N, nseg, 1 + M.lb, M.bw, ws->tok, ws->ntok,
                       ws->seam, ws->head, seam_join());
    hipLaunchKernelGGL(k_png_seam_apply, dim3((unsigned)((nseg + 255) / 256)), dim3(256), 0, st, ws->filt, N, nseg,
                       ws->tok, ws->ntok, ws->seam, ws->head, ws->seghist, ws->segx, ws->hist);
    mark(5);
    mark(6);
    // (ICX_PNG_PLAN_LDS lowers the LDS limit so tests reach the global-memory walk)
    const char* pl = std::getenv("ICX_PNG_PLAN_LDS");
    const int64_t lds_max = pl ? std::max<int64_t>(0, std::min<int64_t>(kPlanLds, std::atoll(pl))) : kPlanLds;
    hipLaunchKernelGGL(k_png_blockplan, dim3(1), dim3(256), (size_t)std::max<int64_t>(1, std::min<int64_t>(nblk, lds_max)) * 4,
                       st, ws->blksym, nblk, ws->plan, lds_max);
    hipLaunchKernelGGL(k_png_huff, dim3((unsigned)nblk), dim3(64), 0, st, ws->hist, nblk, ws->plan, ws->bc);
    hipLaunchKernelGGL(k_png_segbits, dim3(gwave), dim3(256), 0, st, nseg, ws->seghist, ws->segx, ws->bc, ws->plan,
                       ws->bits);
    size_t tb = 0;
    PNG_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, ws->bits, ws->off, (int)nseg, st));
    if (!pgrow(ws->tmp, tb, ws->tmp_cap)) return -1;
    PNG_HIP(hipcub::DeviceScan::ExclusiveSum(ws->tmp, tb, ws->bits, ws->off, (int)nseg, st));
    hipLaunchKernelGGL(k_png_adler, dim3(1), dim3(256), 0, st, ws->adl, nseg, ws->small);
    mark(7);
    // ---- P5: the file (png_encoder.cpp:1888-1952, 2277), laid out on the device
    size_t c13 = ws->tl ? sizeof(png::PngTail) : 0, c14 = ws->predev ? sizeof hb->pre : 0;
    if (!pgrow(ws->tl, sizeof(png::PngTail), c13) || !pgrow(ws->predev, sizeof hb->pre, c14)) return -1;
    const uint64_t idat_at = head.size();  // IDAT chunk header position
    const uint64_t data_at = idat_at + 8;  // zlib stream position
    const uint64_t dstart = data_at + 2;   // deflate data
    hipLaunchKernelGGL(k_png_size, dim3(1), dim3(1), 0, st, ws->off, ws->bits, nseg, (unsigned long long)data_at,
                       (unsigned long long)cap, ws->tl);
    // The deflate bits go to a 4-byte aligned word view of d_out starting at dstart rounded down
    // -- aligned as an address, since a batch slot may start anywhere (k_png_emit's atomics on the
    // words two segments share need it) -- and the few bytes before it (zlib header) are
    // rewritten afterwards.
    const uint64_t mis = (reinterpret_cast<uintptr_t>(d_out) + dstart) & 3u;
    uint32_t* wv = reinterpret_cast<uint32_t*>(d_out + dstart - mis);
    mark(8);
    hipLaunchKernelGGL(k_png_zero, dim3(1024), dim3(256), 0, st, wv, (unsigned long long)mis, ws->tl);
    hipLaunchKernelGGL(k_png_emit, dim3(gwave), dim3(256), 0, st, nseg, ws->tok, ws->ntok, ws->seam, ws->head, ws->bc,
                       ws->plan, ws->off, ws->bits, wv, (unsigned long long)(mis * 8), ws->tl);
    mark(9);
    // signature + IHDR/PLTE/tRNS + IDAT length (k_png_head) / type + zlib header (78 01, :1932-1941)
    std::vector<uint8_t> pre = head;
    const uint8_t ih[8] = {0, 0, 0, 0, 'I', 'D', 'A', 'T'};
    pre.insert(pre.end(), ih, ih + 8);
    pre.push_back(0x78);
    pre.push_back(0x01);
    if (pre.size() > sizeof hb->pre) return -1;
    std::memcpy(hb->pre, pre.data(), pre.size());
    PNG_HIP(hipMemcpyAsync(ws->predev, hb->pre, pre.size(), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_png_head, dim3(1), dim3(256), 0, st, d_out, ws->predev, (int)pre.size(),
                       (unsigned long long)idat_at, (unsigned long long)dstart, ws->small, (long long)N, ws->tl);
    // CRC-32 over "IDAT" + zlib stream: segment CRCs aligned to the stream's end (the device
    // knows its length; the grid covers the longest stream that fits), folded 256:1 per pass
    // (bounded by the longest stream this image can produce -- at most 16 bits per filtered byte
    // (a length-3 match with 15-bit codes and 5 + 13 extra bits), plus every block's dynamic
    // header (< 600 bytes: 17 + 19 x 3 bits + 316 code lengths of at most 7 + 7 bits) and EOB,
    // and the zlib framing -- not by the caller's capacity, which may be far larger)
    const uint64_t zworst = 2 + 2 * (uint64_t)N + (uint64_t)nblk * 1024 + 1024;
    const uint64_t zcap = cap > data_at + 16 ? cap - data_at - 16 : 0;
    const uint64_t zmax = std::min(zcap, zworst) + 4;  // ("IDAT" + stream)
    const int64_t ncs = std::max<int64_t>(1, (int64_t)((zmax + kCrcSeg - 1) / kCrcSeg));
    size_t c12 = ws->crc_cap;
    const size_t crc_need = (size_t)(ncs + (ncs + 255) / 256 + 64) * 4;
    if (crc_need > ws->crc_cap || !ws->crc) {
        if (!pgrow(ws->crc, crc_need, c12)) return -1;
        ws->crc_cap = crc_need;
    }
    mark(10);
    hipLaunchKernelGGL(k_png_crc_seg, dim3((unsigned)((ncs + 255) / 256)), dim3(256), 0, st, d_out + idat_at + 4,
                       ws->tl, ncs, ws->crc);
    uint32_t X = x8n(kCrcSeg);
    uint32_t* cur = ws->crc;
    int64_t m = ncs;
    while (m > 1) {
        const int64_t nb = (m + 255) / 256;
        uint32_t* nxt = cur + m;
        hipLaunchKernelGGL(k_png_crc_reduce, dim3((unsigned)nb), dim3(256), 0, st, cur, m, X, nxt);
        for (int k = 0; k < 8; ++k) X = multmodp(X, X);
        cur = nxt;
        m = nb;
    }
    hipLaunchKernelGGL(k_png_tail, dim3(1), dim3(1), 0, st, d_out, (unsigned long long)data_at, cur, ws->tl);
    mark(11);
    PNG_HIP(hipMemcpyAsync(out_tl, ws->tl, sizeof(png::PngTail), hipMemcpyDeviceToHost, st));
    PNG_HIP(hipGetLastError());
    if (timed) {
        ws->ev_pending = true;
        ws->evset = set ^ 1;
    }
    return 0;
}

static bool png_job_init(PngJob& j, PngWs* ws, hipStream_t st, int w, int h, int d, const uint8_t* d_src, uint8_t* d_out,
                         uint64_t cap, png::PngTail* out_tl) {
    if (!ws->host && hipHostMalloc(reinterpret_cast<void**>(&ws->host), sizeof(PngHost)) != hipSuccess) return false;
    if (!ws->done && hipEventCreateWithFlags(&ws->done, hipEventDisableTiming) != hipSuccess) return false;
    j.ws = ws;
    j.hb = ws->host;
    j.st = st;
    j.ev = ws->done;
    j.w = w;
    j.h = h;
    j.d = d;
    j.d_src = d_src;
    j.d_out = d_out;
    j.cap = cap;
    j.out_tl = out_tl;
    return true;
}

// Encode the device image d_src (w*h*d bytes, d = 3 RGB8 / 4 RGBA8) into a whole PNG file at
// d_out. Returns 0 ok, 1 d_out too small (*size = bytes needed), -1 HIP failure.
int png_encode_device(hipStream_t st, PngWs* ws, int w, int h, int d, const uint8_t* d_src, uint8_t* d_out,
                      uint64_t cap, uint64_t* size) {
    // (the layout lands in the workspace's pinned PngHost: no per-call pinned allocation, whose
    // hipHostFree would synchronise the device)
    PngJob j;
    int rc = png_job_init(j, ws, st, w, h, d, d_src, d_out, cap, nullptr) ? 0 : -1;
    png::PngTail* tl = rc == 0 ? &ws->host->tl : nullptr;
    if (rc == 0) {
        *tl = png::PngTail{};
        j.out_tl = tl;
        rc = j.issue_a();
    }
    if (rc == 0) rc = hipEventSynchronize(j.ev) == hipSuccess ? j.issue_b() : -1;
    if (rc == 0) rc = hipStreamSynchronize(st) == hipSuccess ? (tl->fits ? 0 : 1) : -1;
    *size = rc >= 0 ? tl->total : 0;
    return rc;
}

// n images of w x h x d at d_srcs[i] into d_out + i * stride (sizes[i], status[i]: 0 ok, 1 the
// slot is too small: nothing written, -1 failure). k jobs in flight on (ws[j], st[j]): the host
// reads one image's colour statistics (the only read-back per image) while the others' kernels
// run; every size is read once, after the last image. Returns -1 on a HIP failure.
int png_encode_device_batch(int k, hipStream_t* sts, PngWs** wss, int n, int w, int h, int d,
                            const uint8_t* const* d_srcs, uint8_t* d_out, uint64_t stride, uint64_t* sizes,
                            int32_t* status) {
    png::PngTail* tl = nullptr;
    if (hipHostMalloc(reinterpret_cast<void**>(&tl), sizeof(png::PngTail) * std::max(n, 1)) != hipSuccess) return -1;
    std::memset(tl, 0, sizeof(png::PngTail) * std::max(n, 1));
    std::vector<PngJob> job(k);
    std::vector<int> img(k, -1);
    // -1 until the image's whole work is issued (an image no job reached, or whose issue failed,
    // reports -1, never a stale layout)
    std::vector<int32_t> rc(std::max(n, 1), -1);
    int next = 0, live = 0;
    auto start = [&](int j) {
        img[j] = -1;
        if (next >= n) return;
        img[j] = next++;
        job[j] = PngJob{};
        if (!png_job_init(job[j], wss[j], sts[j], w, h, d, d_srcs[img[j]], d_out + (uint64_t)img[j] * stride, stride,
                          tl + img[j]) ||
            job[j].issue_a() != 0) {
            rc[img[j]] = -1;
            img[j] = -1;
        }
    };
    for (int j = 0; j < k; ++j) start(j);
    for (int j = 0; j < k; ++j) live += img[j] >= 0;
    // round robin over the jobs: wait for one job's statistics, issue the rest of its image and
    // its next image's statistics (measured a little faster than taking whichever is ready first)
    for (int j = 0; live > 0; j = (j + 1) % k) {
        if (img[j] < 0) continue;
        PngJob& J = job[j];
        rc[img[j]] = hipEventSynchronize(J.ev) != hipSuccess || J.issue_b() != 0 ? -1 : 0;
        start(j);
        if (img[j] < 0) --live;
    }
    // per-image failures are in status[] (-1); the call fails only when a stream itself did
    bool stream_fail = false;
    for (int j = 0; j < k; ++j)
        if (hipStreamSynchronize(sts[j]) != hipSuccess) stream_fail = true;
    for (int i = 0; i < n; ++i) {
        const bool bad = rc[i] < 0 || stream_fail;
        sizes[i] = bad ? 0 : tl[i].total;
        status[i] = bad ? -1 : (tl[i].fits ? 0 : 1);
    }
    (void)hipHostFree(tl);
    return stream_fail ? -1 : 0;
}

bool png_encode_gpu(hipStream_t st, int w, int h, int d, const uint8_t* src, std::vector<uint8_t>& out) {
    PngWs ws;
    const size_t srcb = (size_t)w * h * d;
    uint8_t *d_src = nullptr, *d_out = nullptr;
    bool ok = hipMalloc(&d_src, std::max<size_t>(srcb, 1)) == hipSuccess &&
              hipMemcpyAsync(d_src, src, srcb, hipMemcpyHostToDevice, st) == hipSuccess;
    uint64_t cap = srcb + srcb / 64 + (1 << 20), n = 0;
    int rc = -1;
    if (ok) {
        ok = hipMalloc(&d_out, cap) == hipSuccess;
        if (ok) rc = png_encode_device(st, &ws, w, h, d, d_src, d_out, cap, &n);
        if (rc == 1) {
            (void)hipFree(d_out);
            d_out = nullptr;
            cap = n;
            ok = hipMalloc(&d_out, cap) == hipSuccess;
            if (ok) rc = png_encode_device(st, &ws, w, h, d, d_src, d_out, cap, &n);
        }
        ok = ok && rc == 0;
        if (ok) {
            out.resize(n);
            ok = hipMemcpy(out.data(), d_out, n, hipMemcpyDeviceToHost) == hipSuccess;
        }
    }
    if (d_src) (void)hipFree(d_src);
    if (d_out) (void)hipFree(d_out);
    return ok;
}

}  // namespace icx
