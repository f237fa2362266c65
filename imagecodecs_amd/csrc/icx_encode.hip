// icx_encode.hip -- gfx950 JPEG encoder: tiny_jpeg-exact (jpeg_enc.h:786-1175) and the C4
// extension (4:2:0 / 4:4:4, IJG quality; defined by oracle/tje_oracle.c or_jpeg_encode).
//
//   k_enc_units   gather + float RGB->YCbCr (+ 2x2 chroma mean for 4:2:0) staged in LDS per
//                 512-pixel run, then one lane per data unit: AAN float FDCT + quantize + the
//                 AC bit length (jpeg_enc.h:1094-1126, 656-817, 851-887)
//   k_enc_count   adds the DC code length of every unit       (jpeg_enc.h:831-849)
//   (scan)        exclusive prefix sum of unit bit lengths -> bit offsets (hipCUB)
//   k_enc_emit    pack each unit's codes at its bit offset    (jpeg_enc.h:613-643)
//   k_stuff_*     FF -> FF 00 byte stuffing by count/scan/copy (jpeg_enc.h:634-638)
// Built with -ffp-contract=off: every float op rounds exactly like the reference build.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstring>
#include <vector>

#include "icx_internal.h"

namespace icx {

struct EncTables {
    float pq[2][64];          // 1/(8*aan[x]*aan[y]*q), natural order (jpeg_enc.h:980-986)
    uint16_t code[4][256];    // 0 luma DC, 1 luma AC, 2 chroma DC, 3 chroma AC
    uint8_t len[4][256];
};

// Data units in stream order: MCU m (raster), unit k of upm in the MCU. tiny_jpeg: 8x8 MCUs of
// (Y, Cb, Cr); 4:2:0 extension: 16x16 MCUs of (Y0 Y1 Y2 Y3 Cb Cr), chroma = 2x2 pixel means.
struct EncLayout {
    int upm;                 // units per MCU
    int ms;                  // MCU size in pixels (8 or 16)
    int mbw;                 // MCUs per row
    int sub;                 // chroma units average 2x2 pixels
    int8_t comp[6], bx[6], by[6];
    int8_t prevk[6];         // previous unit of the same component in the MCU, or -1
    int8_t lastk[3];         // last unit of each component in an MCU
};
__device__ __forceinline__ int64_t pred_unit(const EncLayout& L, int64_t u) {  // DC predictor source
    const int64_t m = u / L.upm;
    const int k = (int)(u - m * L.upm);
    if (L.prevk[k] >= 0) return m * L.upm + L.prevk[k];
    return m > 0 ? (m - 1) * L.upm + L.lastk[L.comp[k]] : -1;
}

// AAN float FDCT on 8 samples at stride S (tjei_fdct, jpeg_enc.h:667-712), in registers.
template <int S>
__device__ __forceinline__ void fdct8(float* p) {
    const float t0 = p[0] + p[7 * S], t7 = p[0] - p[7 * S];
    const float t1 = p[S] + p[6 * S], t6 = p[S] - p[6 * S];
    const float t2 = p[2 * S] + p[5 * S], t5 = p[2 * S] - p[5 * S];
    const float t3 = p[3 * S] + p[4 * S], t4 = p[3 * S] - p[4 * S];
    const float e10 = t0 + t3, e13 = t0 - t3, e11 = t1 + t2, e12 = t1 - t2;
    p[0] = e10 + e11;
    p[4 * S] = e10 - e11;
    const float z1 = (e12 + e13) * ((float)0.707106781);
    p[2 * S] = e13 + z1;
    p[6 * S] = e13 - z1;
    const float o10 = t4 + t5, o11 = t5 + t6, o12 = t6 + t7;
    const float z5 = (o10 - o12) * ((float)0.382683433);
    const float z2 = ((float)0.541196100) * o10 + z5;
    const float z4 = ((float)1.306562965) * o12 + z5;
    const float z3 = o11 * ((float)0.707106781);
    const float z11 = t7 + z3, z13 = t7 - z3;
    p[5 * S] = z13 + z2;
    p[3 * S] = z13 - z2;
    p[S] = z11 + z4;
    p[7 * S] = z11 - z4;
}

// Zig-zag position of natural index i as a compile-time function: after unrolling, every block
// store index is a constant and the quantised block stays in registers.
constexpr int zig_of_nat(int i) {
    constexpr uint8_t t[64] = {0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
                               3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
                               10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
                               21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};
    return t[i];
}

__device__ __forceinline__ void vli(int v, int& nb, uint32_t& bits) {  // jpeg_enc.h:598-610
    int mag = v < 0 ? -v : v;
    if (v < 0) --v;
    nb = mag ? 32 - __clz(mag) : 1;
    bits = (uint32_t)v & ((1u << nb) - 1u);
}

// A workgroup owns a 512-pixel run of one MCU row (64 MCUs at 4:4:4, 32 at 4:2:0; 192 data units
// either way). Phase 1: all lanes read the run's pixels (coalesced, edge-clamped as
// jpeg_enc.h:1106-1111) and write the samples the units use to LDS -- Y per pixel, Cb/Cr per pixel
// (4:4:4) or per 2x2 mean (4:2:0), each with the reference's float expression and order
// (:1118-1120). Phase 2: one lane per data unit: 8x8 samples from LDS, AAN FDCT, quantise
// (:806-817), the zig-zag block as eight 16-byte stores, and the AC part of its Huffman bit length
// (the DC part needs the previous unit's DC: k_enc_count adds it).
constexpr int kRunPx = 512;
__global__ __launch_bounds__(256) void k_enc_units(const uint8_t* __restrict__ src, int w, int h, int comps,
                                                   EncLayout L, int runs_per_row, const EncTables* __restrict__ T,
                                                   int16_t* __restrict__ zz, uint64_t* __restrict__ nbits) {
    __shared__ float S[3 * 8 * kRunPx];  // 4:4:4: Y|Cb|Cr, 8 x 512 each; 4:2:0: Y 16 x 512 | Cb|Cr 8 x 256
    __shared__ float pq[2][64];
    __shared__ uint8_t aclen[2][256];
    const int t = threadIdx.x;
    if (t < 128) pq[t >> 6][t & 63] = T->pq[t >> 6][t & 63];
    aclen[0][t] = T->len[1][t];
    aclen[1][t] = T->len[3][t];
    const int my = blockIdx.x / runs_per_row, rx = blockIdx.x - my * runs_per_row;
    const int x0 = rx * kRunPx, y0 = my * L.ms;
    const int mcu0 = x0 / L.ms, nm = min(kRunPx / L.ms, L.mbw - mcu0), wpx = nm * L.ms;
    auto pix = [&](int x, int y) { return src + ((int64_t)min(y, h - 1) * w + min(x, w - 1)) * comps; };
    auto ycc = [](const uint8_t* p, int c) {  // jpeg_enc.h:1118-1120, evaluated left to right
        const uint8_t r = p[0], g = p[1], b = p[2];
        if (c == 0) return 0.299f * r + 0.587f * g + 0.114f * b - 128;
        if (c == 1) return -0.1687f * r - 0.3313f * g + 0.5f * b;
        return 0.5f * r - 0.4187f * g - 0.0813f * b;
    };
    constexpr int kHalf = kRunPx / 2;
    // RGB rows 4-byte aligned (3 bytes per pixel, w % 4 == 0, src aligned): a thread takes two
    // quads (4 x 2 pixels) with three dword loads per row instead of 12 byte loads
    const bool rows4 = comps == 3 && (w & 3) == 0 && (reinterpret_cast<uintptr_t>(src) & 3) == 0;
    if (L.sub && rows4) {
        for (int pr = t; pr < kHalf * 4; pr += 256) {
            const int qy = pr / (kHalf / 2), qx = 2 * (pr - qy * (kHalf / 2));
            if (2 * qx >= wpx) continue;
            const int x = x0 + 2 * qx, y = y0 + 2 * qy;
            uint32_t rw[2][3];  // rows y, y + 1: pixels x .. x + 3 (edge-clamped past the image)
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                if (x + 3 < w && y + r < h) {
                    const uint32_t* q = reinterpret_cast<const uint32_t*>(src + ((int64_t)(y + r) * w + x) * 3);
                    rw[r][0] = q[0]; rw[r][1] = q[1]; rw[r][2] = q[2];
                } else {
                    uint8_t b[12];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const uint8_t* pp = pix(x + k, y + r);
                        b[3 * k] = pp[0]; b[3 * k + 1] = pp[1]; b[3 * k + 2] = pp[2];
                    }
#pragma unroll
                    for (int d = 0; d < 3; ++d)
                        rw[r][d] = (uint32_t)b[4 * d] | (uint32_t)b[4 * d + 1] << 8 | (uint32_t)b[4 * d + 2] << 16 | (uint32_t)b[4 * d + 3] << 24;
                }
            }
            const uint8_t* B0 = reinterpret_cast<const uint8_t*>(rw[0]);
            const uint8_t* B1 = reinterpret_cast<const uint8_t*>(rw[1]);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (2 * (qx + j) >= wpx) break;
                const uint8_t *p00 = B0 + 6 * j, *p10 = B0 + 6 * j + 3, *p01 = B1 + 6 * j, *p11 = B1 + 6 * j + 3;
                float* Y = S + 2 * qy * kRunPx + 2 * (qx + j);
                Y[0] = ycc(p00, 0);
                Y[1] = ycc(p10, 0);
                Y[kRunPx] = ycc(p01, 0);
                Y[kRunPx + 1] = ycc(p11, 0);
#pragma unroll
                for (int c = 1; c < 3; ++c) {
                    const float a = ycc(p00, c), b = ycc(p10, c), cc = ycc(p01, c), d = ycc(p11, c);
                    S[16 * kRunPx + (c - 1) * 8 * kHalf + qy * kHalf + qx + j] = ((a + b) + (cc + d)) * 0.25f;
                }
            }
        }
    } else if (L.sub) {  // 2x2 quads; chroma = ((a + b) + (c + d)) * 0.25f of the per-pixel values
        for (int qd = t; qd < kHalf * 8; qd += 256) {
            const int qy = qd / kHalf, qx = qd - qy * kHalf;
            if (2 * qx >= wpx) continue;
            const int x = x0 + 2 * qx, y = y0 + 2 * qy;
            const uint8_t *p00 = pix(x, y), *p10 = pix(x + 1, y), *p01 = pix(x, y + 1), *p11 = pix(x + 1, y + 1);
            float* Y = S + 2 * qy * kRunPx + 2 * qx;
            Y[0] = ycc(p00, 0);
            Y[1] = ycc(p10, 0);
            Y[kRunPx] = ycc(p01, 0);
            Y[kRunPx + 1] = ycc(p11, 0);
#pragma unroll
            for (int c = 1; c < 3; ++c) {
                const float a = ycc(p00, c), b = ycc(p10, c), cc = ycc(p01, c), d = ycc(p11, c);
                S[16 * kRunPx + (c - 1) * 8 * kHalf + qy * kHalf + qx] = ((a + b) + (cc + d)) * 0.25f;
            }
        }
    } else if (rows4) {  // 4:4:4, aligned RGB rows: four pixels per thread, three dword loads
        for (int i = t; i < kRunPx * 2; i += 256) {
            const int yy = i / (kRunPx / 4), xx = 4 * (i - yy * (kRunPx / 4));
            if (xx >= wpx) continue;
            const int x = x0 + xx, y = y0 + yy;
            uint32_t rw[3];
            if (x + 3 < w && y < h) {
                const uint32_t* q = reinterpret_cast<const uint32_t*>(src + ((int64_t)y * w + x) * 3);
                rw[0] = q[0]; rw[1] = q[1]; rw[2] = q[2];
            } else {
                uint8_t b[12];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint8_t* pp = pix(x + k, y);
                    b[3 * k] = pp[0]; b[3 * k + 1] = pp[1]; b[3 * k + 2] = pp[2];
                }
#pragma unroll
                for (int d = 0; d < 3; ++d)
                    rw[d] = (uint32_t)b[4 * d] | (uint32_t)b[4 * d + 1] << 8 | (uint32_t)b[4 * d + 2] << 16 | (uint32_t)b[4 * d + 3] << 24;
            }
            const uint8_t* B = reinterpret_cast<const uint8_t*>(rw);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (xx + k >= wpx) break;
#pragma unroll
                for (int c = 0; c < 3; ++c) S[c * 8 * kRunPx + yy * kRunPx + xx + k] = ycc(B + 3 * k, c);
            }
        }
    } else {
        for (int i = t; i < kRunPx * 8; i += 256) {
            const int yy = i / kRunPx, xx = i - yy * kRunPx;
            if (xx >= wpx) continue;
            const uint8_t* p = pix(x0 + xx, y0 + yy);
#pragma unroll
            for (int c = 0; c < 3; ++c) S[c * 8 * kRunPx + yy * kRunPx + xx] = ycc(p, c);
        }
    }
    __syncthreads();
    if (t >= nm * L.upm) return;
    const int ml = t / L.upm, k = t - ml * L.upm, c = L.comp[k];
    const float* base;
    int pitch = kRunPx;
    if (!L.sub) base = S + c * 8 * kRunPx + ml * 8;
    else if (c == 0) base = S + L.by[k] * 8 * kRunPx + ml * 16 + L.bx[k] * 8;
    else { base = S + 16 * kRunPx + (c - 1) * 8 * kHalf + ml * 8; pitch = kHalf; }
    float f[64];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const float4 lo = *reinterpret_cast<const float4*>(base + r * pitch);
        const float4 hi = *reinterpret_cast<const float4*>(base + r * pitch + 4);
        f[8 * r + 0] = lo.x; f[8 * r + 1] = lo.y; f[8 * r + 2] = lo.z; f[8 * r + 3] = lo.w;
        f[8 * r + 4] = hi.x; f[8 * r + 5] = hi.y; f[8 * r + 6] = hi.z; f[8 * r + 7] = hi.w;
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) fdct8<1>(f + 8 * r);
#pragma unroll
    for (int q = 0; q < 8; ++q) fdct8<8>(f + q);
    const float* pqc = pq[c ? 1 : 0];
    int o[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) {  // jpeg_enc.h:806-817
        float v = f[i];
        v *= pqc[i];
        v = floorf(v + 1024 + 0.5f);
        v -= 1024;
        o[zig_of_nat(i)] = (int)v;
    }
    const int64_t u = ((int64_t)my * L.mbw + mcu0 + ml) * L.upm + k;
    int4* dst = reinterpret_cast<int4*>(zz + u * 64);
    auto pk = [](int a, int b) { return (int)(((uint32_t)a & 0xFFFFu) | ((uint32_t)b << 16)); };
#pragma unroll
    for (int q = 0; q < 8; ++q)
        dst[q] = make_int4(pk(o[8 * q], o[8 * q + 1]), pk(o[8 * q + 2], o[8 * q + 3]), pk(o[8 * q + 4], o[8 * q + 5]),
                           pk(o[8 * q + 6], o[8 * q + 7]));
    // AC codes (jpeg_enc.h:851-887): a ZRL per 16 zeros before a nonzero coefficient, (run, size)
    // symbol + amplitude bits, EOB unless coefficient 63 is nonzero
    const uint8_t* al = aclen[c ? 1 : 0];
    uint32_t bits = 0;
    int run = 0;
#pragma unroll
    for (int i = 1; i < 64; ++i) {
        const int v = (int16_t)o[i];
        if (v) {
            const int mag = v < 0 ? -v : v, nb = 32 - __clz(mag);
            bits += (uint32_t)((run >> 4) * al[0xF0] + al[((run & 15) << 4) | nb] + nb);
            run = 0;
        } else {
            ++run;
        }
    }
    if (!(int16_t)o[63]) bits += al[0];
    nbits[u] = bits;
}

// Adds the DC code length (jpeg_enc.h:834-849) to the AC bits k_enc_units stored.
__global__ __launch_bounds__(256) void k_enc_count(const int16_t* __restrict__ zz, int64_t nunits, EncLayout L,
                                                   const EncTables* __restrict__ T, uint64_t* __restrict__ nbits) {
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= nunits) return;
    const int c = L.comp[u % L.upm], td = c ? 2 : 0;
    const int64_t pu = pred_unit(L, u);
    const int pred = pu >= 0 ? zz[pu * 64] : 0;  // DC predictor never resets (:834-835)
    const int diff = zz[u * 64] - pred;
    int nb = 0;
    uint32_t bits;
    if (diff) vli(diff, nb, bits);
    nbits[u] += (uint64_t)(T->len[td][nb] + nb);
}

// Stream words hold bits MSB-first: word k covers stream bits [32k, 32k+32). One lane per unit:
// its zig-zag block is loaded once (eight 16-byte loads) and walked with a fully unrolled
// coefficient loop, so every coefficient is a register; code tables come from LDS. Codes are
// appended to a 64-bit accumulator and every completed word is stored; only words shared with a
// neighbouring unit (the first, when the unit starts mid-word, and the last) use atomicOr.
// Code order as tjei_encode_and_write_MCU (jpeg_enc.h:831-887): DC diff (never reset), then per
// nonzero AC coefficient a ZRL per 16 preceding zeros, the (run, size) symbol and its amplitude
// bits, and EOB unless coefficient 63 is nonzero.
__global__ __launch_bounds__(256) void k_enc_emit(const int16_t* __restrict__ zz, int64_t nunits, EncLayout L,
                                                  const EncTables* __restrict__ T, const uint64_t* __restrict__ off,
                                                  const uint64_t* __restrict__ nbits, uint64_t cap_bits,
                                                  uint32_t* __restrict__ words) {
    __shared__ uint32_t tab[4][256];  // code << 8 | len
    for (int i = threadIdx.x; i < 4 * 256; i += 256) tab[i >> 8][i & 255] = (uint32_t)T->code[i >> 8][i & 255] << 8 | T->len[i >> 8][i & 255];
    __syncthreads();
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= nunits || off[u] + nbits[u] + 32 > cap_bits) return;  // past the words buffer: host re-runs
    const int c = L.comp[u % L.upm];
    const int64_t pu = pred_unit(L, u);
    const int pred = pu >= 0 ? zz[pu * 64] : 0;
    const int4* src = reinterpret_cast<const int4*>(zz + u * 64);
    uint32_t w[32];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int4 v = src[q];
        w[4 * q] = (uint32_t)v.x; w[4 * q + 1] = (uint32_t)v.y; w[4 * q + 2] = (uint32_t)v.z; w[4 * q + 3] = (uint32_t)v.w;
    }
    auto coef = [&](int i) { return (int)(int16_t)(w[i >> 1] >> (16 * (i & 1))); };
    const uint32_t* td = tab[c ? 2 : 0];
    const uint32_t* ta = tab[c ? 3 : 1];
    const uint64_t pos = off[u];
    uint32_t* wp = words + (pos >> 5);
    const int o0 = (int)(pos & 31);
    uint64_t acc = 0;
    int nacc = o0;        // the first o0 bits of the first word belong to the previous unit (zeros here)
    bool first = true;
    auto put = [&](int n, uint32_t v) {
        acc = (acc << n) | (v & ((1u << n) - 1u));
        nacc += n;
        if (nacc >= 32) {
            const uint32_t word = (uint32_t)(acc >> (nacc - 32));
            if (first && o0) atomicOr(wp, word);
            else *wp = word;
            first = false;
            ++wp;
            nacc -= 32;
        }
    };
    auto code = [&](uint32_t e) { put((int)(e & 255), e >> 8); };
    int nb;
    uint32_t bits;
    const int diff = coef(0) - pred;
    if (diff) {
        vli(diff, nb, bits);
        code(td[nb]);
        put(nb, bits);
    } else {
        code(td[0]);
    }
    int run = 0;
#pragma unroll
    for (int i = 1; i < 64; ++i) {
        const int v = coef(i);
        if (v) {
            for (int z = run >> 4; z > 0; --z) code(ta[0xF0]);
            vli(v, nb, bits);
            code(ta[((run & 15) << 4) | nb]);
            put(nb, bits);
            run = 0;
        } else {
            ++run;
        }
    }
    if (!coef(63)) code(ta[0]);
    if (nacc > 0) atomicOr(wp, (uint32_t)(acc << (32 - nacc)));  // shared with the next unit
}

// 16 stream bytes (4 words, one 16-byte load) per lane: adjacent lanes write adjacent output.
constexpr int kStuffChunk = 16;
__device__ __forceinline__ void chunk_words(const uint32_t* words, int64_t t, uint64_t nbytes, uint32_t (&w)[4]) {
    const uint64_t b0 = (uint64_t)t * kStuffChunk;
    if (b0 + kStuffChunk <= nbytes) {
        const uint4 v = *reinterpret_cast<const uint4*>(words + (b0 >> 2));
        w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) w[q] = b0 + 4 * q < nbytes ? words[(b0 >> 2) + q] : 0u;
    }
}

// info[0] = stream bytes (k_enc_size), info[1] = stuffed bytes (k_stuff_total)
__global__ void k_enc_size(const uint64_t* __restrict__ off, const uint64_t* __restrict__ nbits, int64_t nunits,
                           uint64_t* __restrict__ info) {
    info[0] = (off[nunits - 1] + nbits[nunits - 1] + 7) / 8;  // final partial byte zero-padded (:1161-1165)
}
__global__ __launch_bounds__(256) void k_zero_words(uint32_t* __restrict__ words, uint64_t cap_words,
                                                    const uint64_t* __restrict__ info) {
    const uint64_t n = min<uint64_t>(cap_words, (info[0] + 3) / 4 + 1);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        words[i] = 0;
}
__global__ __launch_bounds__(256) void k_stuff_count(const uint32_t* __restrict__ words, const uint64_t* __restrict__ info,
                                                     uint32_t* __restrict__ cnt, int64_t nchunks) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nchunks) return;
    const uint64_t nbytes = info[0];
    const uint64_t b0 = (uint64_t)t * kStuffChunk;
    if (b0 >= nbytes) { cnt[t] = 0; return; }
    const int nb = (int)min<uint64_t>(kStuffChunk, nbytes - b0);
    uint32_t w[4];
    chunk_words(words, t, nbytes, w);
    uint32_t n = 0;
#pragma unroll
    for (int i = 0; i < kStuffChunk; ++i) n += (i < nb && ((w[i >> 2] >> (24 - 8 * (i & 3))) & 255u) == 255u);
    cnt[t] = n;
}

__global__ void k_stuff_total(const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ base, int64_t nchunks,
                              uint64_t* __restrict__ info) {
    info[1] = info[0] + base[nchunks - 1] + cnt[nchunks - 1];
}
// The file header (SOI .. SOS, < 1 KiB) as a kernel argument: written with the stream, only when
// the whole file fits, without a host sync.
struct HdrArg {
    uint8_t b[1024];
    int n;
};
__global__ void k_put_header(HdrArg h, uint8_t* __restrict__ file, const uint64_t* __restrict__ info, uint64_t cap_e,
                             int eoi, uint64_t wbytes) {
    if (info[1] + (eoi ? 2 : 0) > cap_e || info[0] + 4 > wbytes) return;
    for (int i = threadIdx.x; i < h.n; i += blockDim.x) file[i] = h.b[i];
}
// Writes the stuffed stream only when it fits in `cap` bytes (and, with eoi, the EOI marker after it).
__global__ __launch_bounds__(256) void k_stuff_write(const uint32_t* __restrict__ words, const uint64_t* __restrict__ info,
                                                     const uint32_t* __restrict__ base, int64_t nchunks, uint64_t cap,
                                                     int eoi, uint8_t* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nbytes = info[0], total = info[1];
    // nothing is written unless the whole stream fits in cap and every unit was emitted
    if (t >= nchunks || total + (eoi ? 2 : 0) > cap || nbytes + 4 > (uint64_t)nchunks * kStuffChunk) return;
    if (eoi && t == 0) { out[total] = 0xFF; out[total + 1] = 0xD9; }
    const uint64_t b0 = (uint64_t)t * kStuffChunk;
    if (b0 >= nbytes) return;
    const int nb = (int)min<uint64_t>(kStuffChunk, nbytes - b0);
    uint32_t w[4];
    chunk_words(words, t, nbytes, w);
    uint8_t* o = out + b0 + base[t];
#pragma unroll
    for (int i = 0; i < kStuffChunk; ++i) {
        if (i >= nb) break;
        const uint8_t v = (uint8_t)(w[i >> 2] >> (24 - 8 * (i & 3)));
        *o++ = v;
        if (v == 0xFF) *o++ = 0;  // jpeg_enc.h:634-638
    }
}

// ------------------------------------------------------------------------------ host
static const uint8_t kLumaQ[64] = {
    16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55, 14, 13, 16, 24, 40, 57, 69, 56,
    14, 17, 22, 29, 51, 87, 80, 62, 18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};  // jpeg_enc.h:266-276
static const uint8_t kChromaQ[64] = {
    16, 12, 14, 14, 18, 24, 49, 72, 11, 10, 16, 24, 40, 51, 61, 12, 13, 17, 22, 35, 64, 92, 14, 16,
    22, 37, 55, 78, 95, 19, 24, 29, 56, 64, 87, 98, 26, 40, 51, 68, 81, 103, 112, 58, 57, 87, 109, 104,
    121, 100, 60, 69, 80, 103, 113, 120, 103, 55, 56, 62, 77, 92, 101, 99};  // jpeg_enc.h:294-305
static const uint8_t kDcLB[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
static const uint8_t kDcCB[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
static const uint8_t kDcV[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
static const uint8_t kAcLB[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
static const uint8_t kAcCB[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
static const uint8_t kAcLV[162] = {  // jpeg_enc.h:336-349
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22, 0x71,
    0x14, 0x32, 0x81, 0x91, 0xA1, 0x08, 0x23, 0x42, 0xB1, 0xC1, 0x15, 0x52, 0xD1, 0xF0, 0x24, 0x33, 0x62, 0x72,
    0x82, 0x09, 0x0A, 0x16, 0x17, 0x18, 0x19, 0x1A, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2A, 0x34, 0x35, 0x36, 0x37,
    0x38, 0x39, 0x3A, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4A, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59,
    0x5A, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6A, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7A, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8A, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9A, 0xA2, 0xA3,
    0xA4, 0xA5, 0xA6, 0xA7, 0xA8, 0xA9, 0xAA, 0xB2, 0xB3, 0xB4, 0xB5, 0xB6, 0xB7, 0xB8, 0xB9, 0xBA, 0xC2, 0xC3,
    0xC4, 0xC5, 0xC6, 0xC7, 0xC8, 0xC9, 0xCA, 0xD2, 0xD3, 0xD4, 0xD5, 0xD6, 0xD7, 0xD8, 0xD9, 0xDA, 0xE1, 0xE2,
    0xE3, 0xE4, 0xE5, 0xE6, 0xE7, 0xE8, 0xE9, 0xEA, 0xF1, 0xF2, 0xF3, 0xF4, 0xF5, 0xF6, 0xF7, 0xF8, 0xF9, 0xFA};
static const uint8_t kAcCV[162] = {  // jpeg_enc.h:355-368
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13, 0x22,
    0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xA1, 0xB1, 0xC1, 0x09, 0x23, 0x33, 0x52, 0xF0, 0x15, 0x62, 0x72, 0xD1,
    0x0A, 0x16, 0x24, 0x34, 0xE1, 0x25, 0xF1, 0x17, 0x18, 0x19, 0x1A, 0x26, 0x27, 0x28, 0x29, 0x2A, 0x35, 0x36,
    0x37, 0x38, 0x39, 0x3A, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4A, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58,
    0x59, 0x5A, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6A, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7A,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8A, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9A,
    0xA2, 0xA3, 0xA4, 0xA5, 0xA6, 0xA7, 0xA8, 0xA9, 0xAA, 0xB2, 0xB3, 0xB4, 0xB5, 0xB6, 0xB7, 0xB8, 0xB9, 0xBA,
    0xC2, 0xC3, 0xC4, 0xC5, 0xC6, 0xC7, 0xC8, 0xC9, 0xCA, 0xD2, 0xD3, 0xD4, 0xD5, 0xD6, 0xD7, 0xD8, 0xD9, 0xDA,
    0xE2, 0xE3, 0xE4, 0xE5, 0xE6, 0xE7, 0xE8, 0xE9, 0xEA, 0xF2, 0xF3, 0xF4, 0xF5, 0xF6, 0xF7, 0xF8, 0xF9, 0xFA};
static const uint8_t kZigOfNatH[64] = {
    0, 1, 5, 6, 14, 15, 27, 28, 2, 4, 7, 13, 16, 26, 29, 42, 3, 8, 12, 17, 25, 30, 41, 43,
    9, 11, 18, 24, 31, 40, 44, 53, 10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
    21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};

static void huff_codes(uint16_t* code, uint8_t* len, const uint8_t* bits, const uint8_t* vals) {  // C.2
    unsigned cd = 0;
    int k = 0;
    for (int L = 1; L <= 16; ++L) {
        for (int i = 0; i < bits[L - 1]; ++i, ++k) { code[vals[k]] = (uint16_t)cd++; len[vals[k]] = (uint8_t)L; }
        cd <<= 1;
    }
}

// Header bytes of tje_encode_main (jpeg_enc.h:989-1077) for quality tables ql/qc.
static void tje_header(std::vector<uint8_t>& o, int w, int h, const uint8_t* ql, const uint8_t* qc) {
    auto u8 = [&](int v) { o.push_back((uint8_t)v); };
    auto be = [&](int v) { u8(v >> 8); u8(v & 255); };
    static const uint8_t jfif[] = {0xFF, 0xD8, 0xFF, 0xE0, 0x00, 0x10, 'J', 'F', 'I', 'F', 0,
                                   0x01, 0x02, 0x01, 0x00, 0x60, 0x00, 0x60, 0x00, 0x00};
    o.insert(o.end(), jfif, jfif + sizeof jfif);
    static const char com[] = "Created by Tiny JPEG Encoder";
    be(0xFFFE);
    be(2 + (int)sizeof(com) - 1);
    o.insert(o.end(), com, com + sizeof(com) - 1);
    be(0xFFDB); be(0x43); u8(0); o.insert(o.end(), ql, ql + 64);
    be(0xFFDB); be(0x43); u8(1); o.insert(o.end(), qc, qc + 64);
    be(0xFFC0); be(17); u8(8); be(h); be(w); u8(3);
    for (int i = 0; i < 3; ++i) { u8(i + 1); u8(0x11); u8(i ? 1 : 0); }
    const uint8_t* hb[4] = {kDcLB, kAcLB, kDcCB, kAcCB};
    const uint8_t* hv[4] = {kDcV, kAcLV, kDcV, kAcCV};
    const int id[4] = {0x00, 0x10, 0x01, 0x11};
    for (int t = 0; t < 4; ++t) {
        int n = 0;
        for (int i = 0; i < 16; ++i) n += hb[t][i];
        be(0xFFC4); be(2 + 1 + 16 + n); u8(id[t]);
        o.insert(o.end(), hb[t], hb[t] + 16);
        o.insert(o.end(), hv[t], hv[t] + n);
    }
    be(0xFFDA); be(12); u8(3);
    u8(1); u8(0x00); u8(2); u8(0x11); u8(3); u8(0x11);
    u8(0); u8(63); u8(0);
}

static const uint8_t kK2Chroma[64] = {  // JPEG spec table K.2, natural order (C4 extension)
    17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99, 24, 26, 56, 99, 99, 99, 99, 99,
    47, 66, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};

// Quantizer reciprocals for per-natural-position tables qnl/qnc (jpeg_enc.h:980-986) + Huffman.
static void build_tables(EncTables& T, const uint8_t* qnl, const uint8_t* qnc) {
    std::memset(&T, 0, sizeof T);
    static const float aan[8] = {1.0f, 1.387039845f, 1.306562965f, 1.175875602f,
                                 1.0f, 0.785694958f, 0.541196100f, 0.275899379f};
    for (int y = 0; y < 8; ++y)
        for (int x = 0; x < 8; ++x) {
            const int i = y * 8 + x;
            T.pq[0][i] = 1.0f / (8 * aan[x] * aan[y] * qnl[i]);
            T.pq[1][i] = 1.0f / (8 * aan[x] * aan[y] * qnc[i]);
        }
    huff_codes(T.code[0], T.len[0], kDcLB, kDcV);
    huff_codes(T.code[1], T.len[1], kAcLB, kAcLV);
    huff_codes(T.code[2], T.len[2], kDcCB, kDcV);
    huff_codes(T.code[3], T.len[3], kAcCB, kAcCV);
}

static EncLayout make_layout(int subsampling, int w) {
    EncLayout L;
    std::memset(&L, 0, sizeof L);
    if (subsampling == 420) {
        L.upm = 6;
        L.ms = 16;
        L.sub = 1;
        const int8_t comp[6] = {0, 0, 0, 0, 1, 2}, bx[6] = {0, 1, 0, 1, 0, 0}, by[6] = {0, 0, 1, 1, 0, 0};
        const int8_t prevk[6] = {-1, 0, 1, 2, -1, -1};
        for (int k = 0; k < 6; ++k) { L.comp[k] = comp[k]; L.bx[k] = bx[k]; L.by[k] = by[k]; L.prevk[k] = prevk[k]; }
        L.lastk[0] = 3; L.lastk[1] = 4; L.lastk[2] = 5;
    } else {  // 4:4:4 (tiny_jpeg's only layout)
        L.upm = 3;
        L.ms = 8;
        for (int k = 0; k < 3; ++k) { L.comp[k] = (int8_t)k; L.prevk[k] = -1; L.lastk[k] = (int8_t)k; }
    }
    L.mbw = (w + L.ms - 1) / L.ms;
    return L;
}

// C4 extension header: tiny_jpeg's layout with zig-zag DQT and the sampling in SOF0.
static void ext_header(std::vector<uint8_t>& o, int w, int h, const uint8_t* qnl, const uint8_t* qnc, int subsampling) {
    auto u8 = [&](int v) { o.push_back((uint8_t)v); };
    auto be = [&](int v) { u8(v >> 8); u8(v & 255); };
    static const uint8_t jfif[] = {0xFF, 0xD8, 0xFF, 0xE0, 0x00, 0x10, 'J', 'F', 'I', 'F', 0,
                                   0x01, 0x02, 0x01, 0x00, 0x60, 0x00, 0x60, 0x00, 0x00};
    o.insert(o.end(), jfif, jfif + sizeof jfif);
    static const char com[] = "icx JPEG encoder";
    be(0xFFFE);
    be(2 + (int)sizeof(com) - 1);
    o.insert(o.end(), com, com + sizeof(com) - 1);
    uint8_t zq[64];
    for (int k = 0; k < 64; ++k) zq[kZigOfNatH[k]] = qnl[k];
    be(0xFFDB); be(0x43); u8(0); o.insert(o.end(), zq, zq + 64);
    for (int k = 0; k < 64; ++k) zq[kZigOfNatH[k]] = qnc[k];
    be(0xFFDB); be(0x43); u8(1); o.insert(o.end(), zq, zq + 64);
    be(0xFFC0); be(17); u8(8); be(h); be(w); u8(3);
    for (int i = 0; i < 3; ++i) { u8(i + 1); u8(i == 0 && subsampling == 420 ? 0x22 : 0x11); u8(i ? 1 : 0); }
    const uint8_t* hb[4] = {kDcLB, kAcLB, kDcCB, kAcCB};
    const uint8_t* hv[4] = {kDcV, kAcLV, kDcV, kAcCV};
    const int id[4] = {0x00, 0x10, 0x01, 0x11};
    for (int t = 0; t < 4; ++t) {
        int n = 0;
        for (int i = 0; i < 16; ++i) n += hb[t][i];
        be(0xFFC4); be(2 + 1 + 16 + n); u8(id[t]);
        o.insert(o.end(), hb[t], hb[t] + 16);
        o.insert(o.end(), hv[t], hv[t] + n);
    }
    be(0xFFDA); be(12); u8(3);
    u8(1); u8(0x00); u8(2); u8(0x11); u8(3); u8(0x11);
    u8(0); u8(63); u8(0);
}

static void ijg_table(const uint8_t* base, int q, uint8_t* out) {  // IJG jpeg_quality_scaling
    const int scale = q < 50 ? 5000 / q : 200 - 2 * q;
    for (int i = 0; i < 64; ++i) {
        const int v = (base[i] * scale + 50) / 100;
        out[i] = (uint8_t)(v < 1 ? 1 : v > 255 ? 255 : v);
    }
}

// ----------------------------------------------------------------------- device pipeline
struct EncWs {
    EncTables* T = nullptr;
    int16_t* zz = nullptr;
    uint64_t *nb = nullptr, *off = nullptr;
    int64_t units_cap = 0;
    uint32_t* words = nullptr;
    uint64_t words_cap = 0;  // bytes
    uint32_t *cnt = nullptr, *base = nullptr;
    int64_t chunks_cap = 0;
    uint64_t* info = nullptr;  // device: stream bytes, stuffed bytes
    uint64_t* hinfo = nullptr; // pinned host copy of info, valid when `fin` completes
    hipEvent_t fin = nullptr;
    uint64_t est_bytes = 0;    // words-buffer estimate from the images so far
    uint64_t wbytes = 0;       // words buffer of the job in flight
    int64_t nunits = 0;        // data units of the job in flight
    void* tmp = nullptr;
    size_t tmp_cap = 0;
    // per-stage HIP events of the last entropy pass (icx_encoder_stage_times): units, count,
    // scan, emit, stuff; ms[] accumulates over calls until read
    hipEvent_t ev[10] = {};  // stage i spans ev[2i] .. ev[2i+1]
    float ms[5] = {};
    ~EncWs() {
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
        for (void* p : {(void*)T, (void*)zz, (void*)nb, (void*)off, (void*)words, (void*)cnt, (void*)base, (void*)info, tmp})
            if (p) (void)hipFree(p);
        if (hinfo) (void)hipHostFree(hinfo);
        if (fin) (void)hipEventDestroy(fin);
    }
};
EncWs* enc_ws_create() {
    EncWs* ws = new EncWs();
    for (hipEvent_t& e : ws->ev)
        if (hipEventCreate(&e) != hipSuccess) e = nullptr;
    return ws;
}
const char* const kEncStageNames[5] = {"units", "count", "scan", "emit", "stuff"};
int enc_ws_stage_times(EncWs* ws, const char** names, float* ms, int cap) {
    const int k = cap < 5 ? cap : 5;
    for (int i = 0; i < k; ++i) {
        if (names) names[i] = kEncStageNames[i];
        if (ms) ms[i] = ws->ms[i];
    }
    for (float& m : ws->ms) m = 0.f;
    return k;
}
void enc_ws_destroy(EncWs* ws) { delete ws; }

#define ENC_HIP(call)                                  \
    do {                                               \
        if ((call) != hipSuccess) return false;        \
    } while (0)

template <class Ptr>
static bool grow(Ptr*& p, size_t need, size_t& cap_bytes) {
    if (need <= cap_bytes && p) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap_bytes = 0;
    if (hipMalloc(&p, need) != hipSuccess) return false;
    cap_bytes = need;
    return true;
}

// One image's entropy-coded data is produced in two launches-only phases and one collect:
//   enc_front  units, bit counts, scan, stream size (info[0], device)
//   enc_tail   words (sized from the images before: the stream's size is known on the device
//              only), emit, stuffing, stuffed size (info[1]); writes d_out only when the whole
//              result fits in cap (and, with hdr / eoi, the header before it and EOI after it);
//              info -> pinned host memory, event `fin`
//   enc_collect  waits for `fin`: 1 = done (*n = stuffed bytes), 0 = the stream outgrew the words
//              buffer (nothing written; run enc_tail again: est_bytes now holds its size), -1 = HIP
//              failure
// So an image costs one host wait, and a caller with two workspaces on two streams can issue
// image i+1 before waiting for image i.
static bool enc_front(hipStream_t st, EncWs& ws, const EncLayout& L, const EncTables* T, const uint8_t* d_src, int w,
                      int h, int comps) {
    const int64_t mbh = (h + L.ms - 1) / L.ms;
    const int64_t nunits = (int64_t)L.mbw * mbh * L.upm;
    ws.nunits = nunits;
    size_t c0 = ws.units_cap * 128, c1 = ws.units_cap * 8, c2 = c1;
    if (nunits > ws.units_cap) {
        if (!grow(ws.zz, (size_t)nunits * 128, c0) || !grow(ws.nb, (size_t)nunits * 8, c1) ||
            !grow(ws.off, (size_t)nunits * 8, c2))
            return false;
        ws.units_cap = nunits;
    }
    if (!ws.T) ENC_HIP(hipMalloc(&ws.T, sizeof(EncTables)));
    if (!ws.info) ENC_HIP(hipMalloc(&ws.info, 4 * sizeof(uint64_t)));
    if (!ws.hinfo) ENC_HIP(hipHostMalloc(&ws.hinfo, 4 * sizeof(uint64_t)));
    if (!ws.fin) ENC_HIP(hipEventCreateWithFlags(&ws.fin, hipEventDisableTiming));
    if (T) ENC_HIP(hipMemcpyAsync(ws.T, T, sizeof *T, hipMemcpyHostToDevice, st));
    const int TB = 256;
    const int gu = (int)((nunits + TB - 1) / TB);
    const bool ev = ws.ev[9] != nullptr;
    auto mark = [&](int i) {
        if (ev) (void)hipEventRecord(ws.ev[i], st);
    };
    mark(0);
    const int runs_per_row = (L.mbw * L.ms + kRunPx - 1) / kRunPx;
    hipLaunchKernelGGL(k_enc_units, dim3((unsigned)(runs_per_row * mbh)), dim3(TB), 0, st, d_src, w, h, comps, L,
                       runs_per_row, ws.T, ws.zz, ws.nb);
    mark(1);
    mark(2);
    hipLaunchKernelGGL(k_enc_count, dim3(gu), dim3(TB), 0, st, ws.zz, nunits, L, ws.T, ws.nb);
    mark(3);
    mark(4);
    size_t tmp_b = 0;
    ENC_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_b, ws.nb, ws.off, (int)nunits, st));
    if (!grow(ws.tmp, tmp_b, ws.tmp_cap)) return false;
    ENC_HIP(hipcub::DeviceScan::ExclusiveSum(ws.tmp, tmp_b, ws.nb, ws.off, (int)nunits, st));
    mark(5);
    hipLaunchKernelGGL(k_enc_size, dim3(1), dim3(1), 0, st, ws.off, ws.nb, nunits, ws.info);
    return hipGetLastError() == hipSuccess;
}

static bool enc_tail(hipStream_t st, EncWs& ws, const EncLayout& L, int w, int h, int comps, uint8_t* d_out,
                     uint64_t cap, bool eoi, const HdrArg* hdr) {
    const int TB = 256;
    const int64_t nunits = ws.nunits;
    const int gu = (int)((nunits + TB - 1) / TB);
    const bool ev = ws.ev[9] != nullptr;
    auto mark = [&](int i) {
        if (ev) (void)hipEventRecord(ws.ev[i], st);
    };
    const uint64_t est = ws.est_bytes ? ws.est_bytes : std::max<uint64_t>(65536, (uint64_t)w * h * comps / 4);
    const uint64_t wbytes = (est + 4 + 15) / 16 * 16;
    if (!grow(ws.words, wbytes, ws.words_cap)) return false;
    ws.wbytes = wbytes;
    const int64_t nchunks = (int64_t)(wbytes / kStuffChunk);
    size_t cc = ws.chunks_cap * 4, cb = cc;
    if (nchunks > ws.chunks_cap) {
        if (!grow(ws.cnt, (size_t)nchunks * 4, cc) || !grow(ws.base, (size_t)nchunks * 4, cb)) return false;
        ws.chunks_cap = nchunks;
    }
    hipLaunchKernelGGL(k_zero_words, dim3(1024), dim3(TB), 0, st, ws.words, (uint64_t)(wbytes / 4), ws.info);
    mark(6);
    hipLaunchKernelGGL(k_enc_emit, dim3(gu), dim3(TB), 0, st, ws.zz, nunits, L, ws.T, ws.off, ws.nb,
                       (uint64_t)wbytes * 8, ws.words);
    mark(7);
    mark(8);
    const int gc = (int)((nchunks + TB - 1) / TB);
    hipLaunchKernelGGL(k_stuff_count, dim3(gc), dim3(TB), 0, st, ws.words, ws.info, ws.cnt, nchunks);
    size_t tmp_b2 = 0;
    ENC_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_b2, ws.cnt, ws.base, (int)nchunks, st));
    if (!grow(ws.tmp, tmp_b2, ws.tmp_cap)) return false;
    ENC_HIP(hipcub::DeviceScan::ExclusiveSum(ws.tmp, tmp_b2, ws.cnt, ws.base, (int)nchunks, st));
    hipLaunchKernelGGL(k_stuff_total, dim3(1), dim3(1), 0, st, ws.cnt, ws.base, nchunks, ws.info);
    hipLaunchKernelGGL(k_stuff_write, dim3(gc), dim3(TB), 0, st, ws.words, ws.info, ws.base, nchunks, cap,
                       eoi ? 1 : 0, d_out);
    if (hdr)
        hipLaunchKernelGGL(k_put_header, dim3(1), dim3(256), 0, st, *hdr, d_out - hdr->n, ws.info, cap, eoi ? 1 : 0,
                           (uint64_t)wbytes);
    mark(9);
    ENC_HIP(hipGetLastError());
    ENC_HIP(hipMemcpyAsync(ws.hinfo, ws.info, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    ENC_HIP(hipEventRecord(ws.fin, st));
    return true;
}

static int enc_collect(EncWs& ws, uint64_t* n) {
    if (hipEventSynchronize(ws.fin) != hipSuccess) return -1;
    const uint64_t nbytes = ws.hinfo[0];
    if (nbytes + 4 > ws.wbytes) {  // the stream outgrew the words buffer: nothing was written
        ws.est_bytes = nbytes + nbytes / 4;
        return 0;
    }
    ws.est_bytes = std::max(ws.est_bytes, nbytes + nbytes / 4);
    *n = ws.hinfo[1];
    if (ws.ev[9]) {
        for (int i = 0; i < 5; ++i) {
            float t = 0.f;
            if (hipEventElapsedTime(&t, ws.ev[2 * i], ws.ev[2 * i + 1]) == hipSuccess) ws.ms[i] += t;
        }
    }
    return 1;
}

// Entropy-coded data of the image at d_src (device) -> d_out[0 .. *n) (stuffed bytes); with eoi,
// FF D9 follows it, with hdr the header precedes it (all only when they fit in cap). Returns false
// on a HIP failure.
static bool encode_entropy(hipStream_t st, EncWs& ws, const EncLayout& L, const EncTables& T, const uint8_t* d_src,
                           int w, int h, int comps, uint8_t* d_out, uint64_t cap, uint64_t* n, bool eoi = false,
                           const HdrArg* hdr = nullptr) {
    *n = 0;
    const int64_t mbh = (h + L.ms - 1) / L.ms;
    if ((int64_t)L.mbw * mbh * L.upm == 0 || w == 0 || h == 0) return true;
    if (!enc_front(st, ws, L, &T, d_src, w, h, comps)) return false;
    for (int attempt = 0; attempt < 2; ++attempt) {
        if (!enc_tail(st, ws, L, w, h, comps, d_out, cap, eoi, hdr)) return false;
        const int rc = enc_collect(ws, n);
        if (rc < 0) return false;
        if (rc > 0) return true;
    }
    return false;
}

bool encode_host_image(hipStream_t st, const EncLayout& L, const EncTables& T, int w, int h, int comps,
                       const uint8_t* src, std::vector<uint8_t>& out);

// tiny_jpeg-exact encode (quality 1..3, 4:4:4) of a host image; `out` receives the whole file.
bool tje_encode_gpu(hipStream_t st, int quality, int w, int h, int comps, const uint8_t* src,
                    std::vector<uint8_t>& out) {
    uint8_t ql[64], qc[64];
    for (int i = 0; i < 64; ++i) {  // jpeg_enc.h:1231-1256
        if (quality == 3) { ql[i] = qc[i] = 1; continue; }
        const int div = quality == 2 ? 10 : 1;
        ql[i] = (uint8_t)(kLumaQ[i] / div);
        if (!ql[i]) ql[i] = 1;
        qc[i] = (uint8_t)(kChromaQ[i] / div);
        if (!qc[i]) qc[i] = 1;
    }
    uint8_t qnl[64], qnc[64];  // tiny_jpeg indexes its tables through the zig-zag map (:983-984)
    for (int i = 0; i < 64; ++i) { qnl[i] = ql[kZigOfNatH[i]]; qnc[i] = qc[kZigOfNatH[i]]; }
    EncTables T;
    build_tables(T, qnl, qnc);
    out.clear();
    tje_header(out, w, h, ql, qc);
    return encode_host_image(st, make_layout(444, w), T, w, h, comps, src, out);
}

// Shared tail of the host entry points: upload, encode, download, EOI.
bool encode_host_image(hipStream_t st, const EncLayout& L, const EncTables& T, int w, int h, int comps,
                       const uint8_t* src, std::vector<uint8_t>& out) {
    EncWs ws;
    const size_t srcb = (size_t)w * h * comps;
    uint8_t *d_src = nullptr, *d_out = nullptr;
    bool ok = true;
    uint64_t n = 0;
    if (srcb) {
        ok = hipMalloc(&d_src, srcb) == hipSuccess &&
             hipMemcpyAsync(d_src, src, srcb, hipMemcpyHostToDevice, st) == hipSuccess;
        // first pass sizes the output, the second (only when it did not fit) writes it
        uint64_t cap = srcb + 65536;
        ok = ok && hipMalloc(&d_out, cap) == hipSuccess && encode_entropy(st, ws, L, T, d_src, w, h, comps, d_out, cap, &n);
        if (ok && n > cap) {
            (void)hipFree(d_out);
            d_out = nullptr;
            cap = n;
            ok = hipMalloc(&d_out, cap) == hipSuccess && encode_entropy(st, ws, L, T, d_src, w, h, comps, d_out, cap, &n);
        }
        if (ok && n) {
            const size_t h0 = out.size();
            out.resize(h0 + n);
            ok = hipMemcpyAsync(out.data() + h0, d_out, n, hipMemcpyDeviceToHost, st) == hipSuccess &&
                 hipStreamSynchronize(st) == hipSuccess;
        }
    }
    if (d_src) (void)hipFree(d_src);
    if (d_out) (void)hipFree(d_out);
    out.push_back(0xFF);
    out.push_back(0xD9);
    return ok;
}

// C4 extension, host image -> whole file.
bool jpeg_encode_gpu(hipStream_t st, int quality, int subsampling, int w, int h, int comps, const uint8_t* src,
                     std::vector<uint8_t>& out) {
    uint8_t qnl[64], qnc[64];
    ijg_table(kLumaQ, quality, qnl);
    ijg_table(kK2Chroma, quality, qnc);
    EncTables T;
    build_tables(T, qnl, qnc);
    out.clear();
    ext_header(out, w, h, qnl, qnc, subsampling);
    return encode_host_image(st, make_layout(subsampling, w), T, w, h, comps, src, out);
}

// C4 extension, device image -> whole file in d_out (device). Returns 0 ok, 1 d_out too small
// (*size = bytes needed), -1 HIP failure.
int jpeg_encode_device(hipStream_t st, EncWs* ws, int quality, int subsampling, int w, int h, int comps,
                       const uint8_t* d_src, uint8_t* d_out, uint64_t cap, uint64_t* size) {
    uint8_t qnl[64], qnc[64];
    ijg_table(kLumaQ, quality, qnl);
    ijg_table(kK2Chroma, quality, qnc);
    EncTables T;
    build_tables(T, qnl, qnc);
    std::vector<uint8_t> head;
    ext_header(head, w, h, qnl, qnc, subsampling);
    const uint64_t hn = head.size();
    if (hn > sizeof(HdrArg::b)) return -1;
    HdrArg ha;
    std::memcpy(ha.b, head.data(), hn);
    ha.n = (int)hn;
    if (w == 0 || h == 0) {  // no data units: header + EOI only
        *size = hn + 2;
        if (*size > cap) return 1;
        static const uint8_t eoi[2] = {0xFF, 0xD9};
        if (hipMemcpyAsync(d_out, head.data(), hn, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(d_out + hn, eoi, 2, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return -1;
        return 0;
    }
    uint64_t n = 0;
    // the whole file (header, stuffed stream, EOI) is written on the device, only if it fits
    if (!encode_entropy(st, *ws, make_layout(subsampling, w), T, d_src, w, h, comps, d_out + hn, cap > hn ? cap - hn : 0,
                        &n, true, &ha))
        return -1;
    *size = hn + n + 2;
    return *size > cap ? 1 : 0;
}

// A batch of device images, same geometry and settings: image i -> d_out + i*stride. Images
// alternate between two workspaces on two streams, so image i+1's kernels are issued before the
// host waits for image i. Per image: sizes[i] and status[i] (0 ok, 1 did not fit: nothing
// written). Returns 0, or -1 on a HIP failure. Synchronous.
int jpeg_encode_device_batch(hipStream_t st0, hipStream_t st1, EncWs* w0, EncWs* w1, int n, int quality,
                             int subsampling, int w, int h, int comps, const uint8_t* const* d_srcs, uint8_t* d_out,
                             uint64_t stride, uint64_t* sizes, int32_t* status) {
    if (n <= 0) return 0;
    if (w == 0 || h == 0) {
        for (int i = 0; i < n; ++i) {
            const int rc = jpeg_encode_device(st0, w0, quality, subsampling, w, h, comps, d_srcs[i],
                                              d_out + (uint64_t)i * stride, stride, &sizes[i]);
            if (rc < 0) return -1;
            status[i] = rc;
        }
        return 0;
    }
    uint8_t qnl[64], qnc[64];
    ijg_table(kLumaQ, quality, qnl);
    ijg_table(kK2Chroma, quality, qnc);
    EncTables T;
    build_tables(T, qnl, qnc);
    std::vector<uint8_t> head;
    ext_header(head, w, h, qnl, qnc, subsampling);
    const uint64_t hn = head.size();
    if (hn > sizeof(HdrArg::b)) return -1;
    HdrArg ha;
    std::memcpy(ha.b, head.data(), hn);
    ha.n = (int)hn;
    const EncLayout L = make_layout(subsampling, w);
    EncWs* W[2] = {w0, w1};
    hipStream_t S[2] = {st0, st1};
    const uint64_t cap = stride > hn ? stride - hn : 0;
    hipEvent_t fork = nullptr;
    if (hipEventCreateWithFlags(&fork, hipEventDisableTiming) != hipSuccess) return -1;
    bool ok = hipEventRecord(fork, st0) == hipSuccess && hipStreamWaitEvent(st1, fork, 0) == hipSuccess;
    auto finish = [&](int i) {  // wait for image i; re-run its tail once if its stream outgrew the buffer
        EncWs& ws = *W[i & 1];
        uint64_t nn = 0;
        int rc = enc_collect(ws, &nn);
        if (rc == 0) {
            rc = enc_tail(S[i & 1], ws, L, w, h, comps, d_out + (uint64_t)i * stride + hn, cap, true, &ha) ? enc_collect(ws, &nn)
                                                                                                       : -1;
        }
        if (rc <= 0) return false;
        sizes[i] = hn + nn + 2;
        status[i] = sizes[i] > stride ? 1 : 0;
        return true;
    };
    for (int i = 0; ok && i < n + 2; ++i) {
        if (i >= 2) ok = finish(i - 2);
        if (ok && i < n) {
            EncWs& ws = *W[i & 1];
            ok = enc_front(S[i & 1], ws, L, i < 2 ? &T : nullptr, d_srcs[i], w, h, comps) &&
                 enc_tail(S[i & 1], ws, L, w, h, comps, d_out + (uint64_t)i * stride + hn, cap, true, &ha);
        }
    }
    // The caller's stream (st0) resumes after both -- on the error path too: an image may still
    // be running on st1, writing d_out and ws2, and a caller that reuses d_out on st0 must not
    // overtake it. If the join itself cannot be recorded, wait for st1 on the host.
    const bool joined = hipEventRecord(fork, st1) == hipSuccess && hipStreamWaitEvent(st0, fork, 0) == hipSuccess;
    if (!joined) (void)hipStreamSynchronize(st1);
    (void)hipEventDestroy(fork);
    return ok && joined ? 0 : -1;
}

}  // namespace icx
