// icx_encode.hip -- gfx950 JPEG encoder: tiny_jpeg-exact (jpeg_enc.h:786-1175) and the C4
// extension (4:2:0 / 4:4:4, IJG quality; defined by oracle/tje_oracle.c or_jpeg_encode).
//
//   k_enc_run        one workgroup per 512-pixel run of an MCU row, any number of images per
//                    launch: gather + float RGB->YCbCr (+ 2x2 chroma mean for 4:2:0) staged in LDS,
//                    one lane per data unit: AAN float FDCT, quantise, code lengths (jpeg_enc.h
//                    :1094-1126, 656-817, 831-887); a decoupled look-back over the image's earlier
//                    runs gives the run's bit offset and the DC predictors across runs; every lane
//                    then packs its unit's codes at its offset (:613-643)
//   k_stuff_count_b  FF -> FF 00 byte stuffing by count / scan (hipCUB, one per batch) / copy
//   k_stuff_write_b  (:634-638), the header and EOI written with the stream
// Built with -ffp-contract=off: every float op rounds exactly like the reference build.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
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
    int8_t firstk[3];        // first unit of each component in an MCU
    int8_t lastk[3];         // last unit of each component in an MCU
};
// AAN float FDCT on 8 samples at stride S (tjei_fdct, jpeg_enc.h:667-712), in registers.
typedef float f2 __attribute__((ext_vector_type(2)));  // packed FP32 (v_pk_add_f32 / v_pk_mul_f32)

// AAN float FDCT on 8 samples at stride S (tjei_fdct, jpeg_enc.h:667-712), in registers. T is
// float, or a packed pair of floats (two independent transforms per v_pk instruction: the same
// operations in the same order, each rounded as the reference rounds it).
template <int S, class T>
__device__ __forceinline__ void fdct8(T* p) {
    const T t0 = p[0] + p[7 * S], t7 = p[0] - p[7 * S];
    const T t1 = p[S] + p[6 * S], t6 = p[S] - p[6 * S];
    const T t2 = p[2 * S] + p[5 * S], t5 = p[2 * S] - p[5 * S];
    const T t3 = p[3 * S] + p[4 * S], t4 = p[3 * S] - p[4 * S];
    const T e10 = t0 + t3, e13 = t0 - t3, e11 = t1 + t2, e12 = t1 - t2;
    p[0] = e10 + e11;
    p[4 * S] = e10 - e11;
    const T z1 = (e12 + e13) * T((float)0.707106781);
    p[2 * S] = e13 + z1;
    p[6 * S] = e13 - z1;
    const T o10 = t4 + t5, o11 = t5 + t6, o12 = t6 + t7;
    const T z5 = (o10 - o12) * T((float)0.382683433);
    const T z2 = T((float)0.541196100) * o10 + z5;
    const T z4 = T((float)1.306562965) * o12 + z5;
    const T z3 = o11 * T((float)0.707106781);
    const T z11 = t7 + z3, z13 = t7 - z3;
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

// One workgroup per run: 512 pixels of one MCU row (64 MCUs at 4:4:4, 32 at 4:2:0; 192 data
// units either way), runs in stream order within an image, taken by ticket so a run's
// predecessors are always resident. The whole entropy-coded stream of the run is produced here:
//   1. all lanes read the run's pixels (coalesced, edge-clamped as jpeg_enc.h:1106-1111) and write
//      the samples the units use to LDS -- Y per pixel, Cb/Cr per pixel (4:4:4) or per 2x2 mean
//      (4:2:0), each with the reference's float expression and order (:1118-1120);
//   2. one lane per data unit: 8x8 samples from LDS, AAN FDCT, quantise (:806-817), the AC part of
//      its Huffman bit length (:851-887) and its DC value;
//   3. the DC code lengths (:831-849) of every unit whose predecessor (the previous unit of its
//      component in stream order) is in the run, the run's bit count without its first units'
//      DC codes (A), and its first / last DC of each component, published as look-back records;
//   4. decoupled look-back (wave 0) over earlier runs of the image for the stream bits before the
//      run, whose last DCs also give the first units' DC codes; the run's inclusive count is
//      published at once;
//   5. a block scan of the unit bit lengths, and every lane packs its unit's codes (DC diff, then
//      per nonzero AC coefficient a ZRL per 16 preceding zeros, the (run, size) symbol and the
//      amplitude bits, EOB unless coefficient 63 is nonzero: tjei_encode_and_write_MCU,
//      :831-887) at its bit offset (:613-643) from registers: no coefficient round trip.
// The coefficients never leave registers, and the count / scan / emit passes are this one launch.
constexpr int kRunPx = 512;
struct EncBatch {
    const uint8_t* const* srcs;  // device array: image i's RGB pixels
    int w, h, comps;
    int runs_per_row, runs;      // per image
    uint64_t wwords;             // words per image in `words` (its stride)
};
// Look-back records, one per run of an image: three 8-byte granules, each written once by one
// agent-scope (sc1) 8-byte store with its own valid bit, so readers need no ordering
// (MI355X_MICROARCH.md, inter-workgroup visibility: self-tagged granules).
struct RunRec {
    unsigned long long agg;   // [63] valid, [62:42] A, [41:0] first DC per component (14-bit, +8192)
    unsigned long long last;  // [63] valid, [41:0] last DC per component
    unsigned long long inc;   // [63] valid, [62:0] stream bits up to and including the run
};
constexpr unsigned long long kGValid = 1ull << 63;
#ifndef ICX_LB_SLEEP  // s_sleep units (64 clocks) between polls of a look-back record
#define ICX_LB_SLEEP 8
#endif
__device__ __forceinline__ unsigned long long g_load(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_store(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Waits for a record another (earlier, hence resident) workgroup publishes; bounded (about a
// second), so a defect cannot hang the GPU: on expiry it raises *fail (the host reports a HIP
// failure) and returns a valid, wrong record.
__device__ __forceinline__ unsigned long long g_wait(const unsigned long long* p, unsigned* fail) {
    unsigned long long v;
    for (int it = 0; !((v = g_load(p)) & kGValid); ++it) {
        if (it == (1 << 22)) {
            atomicOr(fail, 1u);
            return kGValid | ((8192ull << 28) | (8192ull << 14) | 8192ull);
        }
        __builtin_amdgcn_s_sleep(ICX_LB_SLEEP);
    }
    return v;
}
__device__ __forceinline__ int dc_field(unsigned long long g, int c) { return (int)((g >> (14 * c)) & 0x3FFFu) - 8192; }
__device__ __forceinline__ int dc_bits(const uint8_t (&dcl)[2][16], int c, int diff) {  // jpeg_enc.h:834-849
    const int mag = diff < 0 ? -diff : diff;
    const int nb = mag ? 32 - __clz(mag) : 0;
    return dcl[c ? 1 : 0][nb] + nb;
}
__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor((unsigned long long)v, o);
    return v;
}

__global__ __launch_bounds__(256) void k_enc_run(EncBatch B, EncLayout L, const EncTables* __restrict__ T,
                                                 RunRec* __restrict__ recs, unsigned* __restrict__ ticket,  // [0] ticket, [1] look-back expired
                                                 uint32_t* __restrict__ words, uint64_t* __restrict__ info) {
    // the run's samples (4:4:4: Y|Cb|Cr, 8 x 512 each; 4:2:0: Y 16 x 512 | Cb|Cr 8 x 256), then
    // (once every lane holds its unit) the code tables and each unit's AC codes
    constexpr int kSlotW = 58;  // words per unit: 63 AC codes of at most 16 + 11 bits < 58 x 32
    __shared__ union {
        float S[3 * 8 * kRunPx];
        struct {
            uint32_t slot[192][kSlotW];  // a unit's AC codes, MSB first
            uint32_t tab[4][256];        // code << 8 | length
        } E;
    } U;
    static_assert(sizeof(U.E) <= sizeof(U.S), "the codes fit the samples' LDS");
    __shared__ float pq[2][64];
    __shared__ uint8_t dcl[2][16];
    __shared__ int32_t dcs[256];
    __shared__ uint32_t wsum[4];
    __shared__ int s_tk;
    __shared__ unsigned long long s_excl;
    __shared__ int32_t s_lprev[3];
    float* S = U.S;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (t == 0) s_tk = (int)atomicAdd(ticket, 1u);
    if (t < 128) pq[t >> 6][t & 63] = T->pq[t >> 6][t & 63];
    if (t < 32) dcl[t >> 4][t & 15] = (t & 15) < 12 ? T->len[(t >> 4) ? 2 : 0][t & 15] : 0;
    __syncthreads();
    // (the grid is exactly one workgroup per run of the batch; the ticket is made wave-uniform so
    // the run's geometry and source pointer stay in SGPRs)
    const int tk = __builtin_amdgcn_readfirstlane(s_tk);
    const int img = tk / B.runs, run = tk - img * B.runs;
    const uint8_t* src = B.srcs[img];
    const int w = B.w, h = B.h, comps = B.comps;
    RunRec* R = recs + (int64_t)img * B.runs;
    const int my = run / B.runs_per_row, rx = run - my * B.runs_per_row;
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
    // 1. RGB rows 4-byte aligned (3 bytes per pixel, w % 4 == 0, src aligned): a thread takes two
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
            // The thread's two quads (j = 0, 1; both inside the run: wpx is a multiple of 16 and qx
            // even) as the two halves of packed-FP32 vectors: every colour expression below is the
            // reference's, in its order, evaluated for both quads by one v_pk instruction.
            const uint8_t* B0 = reinterpret_cast<const uint8_t*>(rw[0]);
            const uint8_t* B1 = reinterpret_cast<const uint8_t*>(rw[1]);
            auto ld = [](const uint8_t* p, int o) { return f2{(float)p[o], (float)p[6 + o]}; };
            // pixel (dx, dy) of both quads: bytes 3 dx (+6 for quad 1) of row dy
            f2 Yv[2][2], Cb[2][2], Cr[2][2];
#pragma unroll
            for (int dy = 0; dy < 2; ++dy)
#pragma unroll
                for (int dx = 0; dx < 2; ++dx) {
                    const uint8_t* p = (dy ? B1 : B0) + 3 * dx;
                    const f2 r = ld(p, 0), g = ld(p, 1), b = ld(p, 2);
                    Yv[dy][dx] = f2(0.299f) * r + f2(0.587f) * g + f2(0.114f) * b - f2(128.f);
                    Cb[dy][dx] = f2(-0.1687f) * r - f2(0.3313f) * g + f2(0.5f) * b;
                    Cr[dy][dx] = f2(0.5f) * r - f2(0.4187f) * g - f2(0.0813f) * b;
                }
#pragma unroll
            for (int dy = 0; dy < 2; ++dy)  // Y: pixels x .. x + 3 of the row, one 16-byte store
                *reinterpret_cast<float4*>(S + (2 * qy + dy) * kRunPx + 2 * qx) =
                    make_float4(Yv[dy][0].x, Yv[dy][1].x, Yv[dy][0].y, Yv[dy][1].y);
            const f2 mb = ((Cb[0][0] + Cb[0][1]) + (Cb[1][0] + Cb[1][1])) * f2(0.25f);
            const f2 mr = ((Cr[0][0] + Cr[0][1]) + (Cr[1][0] + Cr[1][1])) * f2(0.25f);
            *reinterpret_cast<f2*>(S + 16 * kRunPx + qy * kHalf + qx) = mb;
            *reinterpret_cast<f2*>(S + 16 * kRunPx + 8 * kHalf + qy * kHalf + qx) = mr;
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
            const uint8_t* Bq = reinterpret_cast<const uint8_t*>(rw);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (xx + k >= wpx) break;
#pragma unroll
                for (int c = 0; c < 3; ++c) S[c * 8 * kRunPx + yy * kRunPx + xx + k] = ycc(Bq + 3 * k, c);
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
    // 2. one lane per data unit (lanes past the run's units idle to the barriers)
    const int nunits = nm * L.upm;
    const bool act = t < nunits;
    const int ml = act ? t / L.upm : 0, k = act ? t - ml * L.upm : 0, c = L.comp[k];
    float f[64];
    {
        const float* base;
        int pitch = kRunPx;
        if (!L.sub) base = S + c * 8 * kRunPx + ml * 8;
        else if (c == 0) base = S + L.by[k] * 8 * kRunPx + ml * 16 + L.bx[k] * 8;
        else { base = S + 16 * kRunPx + (c - 1) * 8 * kHalf + ml * 8; pitch = kHalf; }
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const float4 lo = *reinterpret_cast<const float4*>(base + r * pitch);
            const float4 hi = *reinterpret_cast<const float4*>(base + r * pitch + 4);
            f[8 * r + 0] = lo.x; f[8 * r + 1] = lo.y; f[8 * r + 2] = lo.z; f[8 * r + 3] = lo.w;
            f[8 * r + 4] = hi.x; f[8 * r + 5] = hi.y; f[8 * r + 6] = hi.z; f[8 * r + 7] = hi.w;
        }
    }
    __syncthreads();  // every lane holds its samples: the code tables and AC codes take their LDS
    for (int i = t; i < 4 * 256; i += 256) U.E.tab[i >> 8][i & 255] = (uint32_t)T->code[i >> 8][i & 255] << 8 | T->len[i >> 8][i & 255];
    // rows in pairs (P[8k + c] = rows 2k, 2k+1 of column c), then columns in pairs (Q[4r + m] =
    // columns 2m, 2m+1 of row r): the reference's row pass, then its column pass
    f2 P[32], Q[32];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int cc = 0; cc < 8; ++cc) P[8 * k + cc] = f2{f[16 * k + cc], f[16 * k + 8 + cc]};
#pragma unroll
    for (int k = 0; k < 4; ++k) fdct8<1>(P + 8 * k);
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const f2 a = P[8 * (r >> 1) + 2 * m], b = P[8 * (r >> 1) + 2 * m + 1];
            Q[4 * r + m] = (r & 1) ? f2{a.y, b.y} : f2{a.x, b.x};
        }
#pragma unroll
    for (int m = 0; m < 4; ++m) fdct8<4>(Q + m);
    uint32_t cw[32];  // the quantised block, zig-zag order, two coefficients per word
    {
        const float* pqc = pq[c ? 1 : 0];
        int o[64];
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int m = 0; m < 4; ++m) {  // jpeg_enc.h:806-817, natural indices 8r + 2m, + 1
                f2 v = Q[4 * r + m];
                v = v * *reinterpret_cast<const f2*>(pqc + 8 * r + 2 * m);
                v = v + f2(1024.f);
                v = v + f2(0.5f);
                v = f2{floorf(v.x), floorf(v.y)};
                v = v - f2(1024.f);
                o[zig_of_nat(8 * r + 2 * m)] = (int)v.x;
                o[zig_of_nat(8 * r + 2 * m + 1)] = (int)v.y;
            }
#pragma unroll
        for (int q = 0; q < 32; ++q) cw[q] = ((uint32_t)o[2 * q] & 0xFFFFu) | ((uint32_t)o[2 * q + 1] << 16);
    }
    // (the whole block is quantised before the code loop reads it: left alone, the compiler
    // interleaves the FDCT with that loop and keeps the unpacked coefficients alive, 250+ VGPRs)
#pragma unroll
    for (int q = 0; q < 32; ++q) asm volatile("" : "+v"(cw[q]));
    auto coef = [&](int i) { return (int)(int16_t)(cw[i >> 1] >> (16 * (i & 1))); };
    const int dc = coef(0);
    dcs[t] = act ? dc : 0;
    __syncthreads();  // code tables and DCs in LDS
    // 3. the unit's AC codes into its LDS slot (jpeg_enc.h:851-887): a ZRL per 16 zeros before a
    // nonzero coefficient, then the (run, size) code and the amplitude bits as one piece of up to
    // 27 bits (code << size | amplitude), EOB unless coefficient 63 is nonzero. Its bit count is
    // the unit's AC length, before any offset is known.
    uint32_t bits_ac = 0;
    uint32_t* const sl = U.E.slot[act ? t : 0];
    if (act) {
        const uint32_t* ta = U.E.tab[c ? 3 : 1];
        uint64_t acc = 0;
        int nacc = 0, widx = 0;
        auto put = [&](int n, uint32_t v) {  // v < 2^n, n <= 27
            acc = (acc << n) | v;
            nacc += n;
            if (nacc >= 32) {
                nacc -= 32;
                sl[widx++] = (uint32_t)(acc >> nacc);
            }
        };
        int zr = 0;
#pragma unroll
        for (int i = 1; i < 64; ++i) {
            const int v = coef(i);
            if (v) {
                if (i > 16 && zr >= 16) {  // (a run of 16+ zeros needs 16 coefficients before it)
                    const uint32_t z = ta[0xF0];
                    for (int q = zr >> 4; q > 0; --q) put((int)(z & 255), z >> 8);
                }
                int nb;
                uint32_t vb;
                vli(v, nb, vb);
                const uint32_t e = ta[((zr & 15) << 4) | nb];
                put((int)(e & 255) + nb, (e >> 8) << nb | vb);
                zr = 0;
            } else {
                ++zr;
            }
        }
        if (!coef(63)) put((int)(ta[0] & 255), ta[0] >> 8);
        if (nacc) sl[widx] = (uint32_t)(acc << (32 - nacc));
        bits_ac = (uint32_t)widx * 32 + (uint32_t)nacc;
    }
    // 4. the DC code (:834-849: the predictor never resets) as one piece, once its predictor is
    // known: the previous unit of its component in the run, or (the run's first units) the last
    // DC of the run before, from the look-back
    const uint32_t* td = U.E.tab[c ? 2 : 0];
    auto dc_piece = [&](int pred, int& n, uint32_t& v) {
        int nb = 0;
        uint32_t vb = 0;
        const int diff = dc - pred;
        if (diff) vli(diff, nb, vb);
        const uint32_t e = td[nb];
        n = (int)(e & 255) + nb;
        v = (e >> 8) << nb | vb;
    };
    const bool first = L.prevk[k] < 0 && ml == 0;  // the run's first unit of its component
    const int pt = L.prevk[k] >= 0 ? ml * L.upm + L.prevk[k] : (ml - 1) * L.upm + L.lastk[c];
    int dcn = 0;
    uint32_t dcv = 0;
    if (act && !first) dc_piece(dcs[pt], dcn, dcv);
    uint32_t bits = act ? bits_ac + (uint32_t)dcn : 0u;  // (first units: AC only so far)
    {
        const uint32_t sa = wave_sum32(bits);
        if (lane == 0) wsum[wv] = sa;
    }
    __syncthreads();
    // 5. look-back (wave 0): the run's A, first and last DCs go out first
    if (wv == 0) {
        const uint32_t A = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        unsigned long long F = 0, Lr = 0;
#pragma unroll
        for (int cc = 0; cc < 3; ++cc) {
            F |= (unsigned long long)(dcs[L.firstk[cc]] + 8192) << (14 * cc);
            Lr |= (unsigned long long)(dcs[(nm - 1) * L.upm + L.lastk[cc]] + 8192) << (14 * cc);
        }
        if (lane == 0) {
            g_store(&R[run].agg, kGValid | (unsigned long long)A << 42 | F);
            g_store(&R[run].last, kGValid | Lr);
        }
        // bits before the run: sum the T of the runs back to the nearest inclusive one, where
        // T(j) = A(j) + the DC codes of j's first units, predicted from run j - 1's last DCs
        unsigned long long excl = 0;
        for (int hi = run - 1;; hi -= 64) {
            const int j = hi - lane;
            unsigned long long gi = 0;
            bool inc = j < 0;  // (before the image: an inclusive count of 0)
            if (!inc) {
                gi = g_load(&R[j].inc);
                inc = (gi & kGValid) != 0;
            }
            const uint64_t m = __ballot(inc);
            const int stop = m ? __ffsll((unsigned long long)m) - 1 : 64;
            unsigned long long v = 0;
            if (lane < stop) {
                const unsigned long long ga = g_wait(&R[j].agg, ticket + 1);
                const unsigned long long gl = j > 0 ? g_wait(&R[j - 1].last, ticket + 1) : kGValid | ((8192ull << 28) | (8192ull << 14) | 8192ull);
                v = (ga >> 42) & 0x1FFFFFull;
#pragma unroll
                for (int cc = 0; cc < 3; ++cc) v += (unsigned long long)dc_bits(dcl, cc, dc_field(ga, cc) - dc_field(gl, cc));
            } else if (lane == stop) {
                v = j < 0 ? 0 : gi & ~kGValid;
            }
            excl += wave_sum64(v);
            if (m) break;
        }
        if (lane == 0) {
            const unsigned long long gl = run > 0 ? g_wait(&R[run - 1].last, ticket + 1) : kGValid | ((8192ull << 28) | (8192ull << 14) | 8192ull);
            unsigned long long Tr = A;
#pragma unroll
            for (int cc = 0; cc < 3; ++cc) {
                s_lprev[cc] = dc_field(gl, cc);
                Tr += (unsigned long long)dc_bits(dcl, cc, dc_field(F, cc) - dc_field(gl, cc));
            }
            g_store(&R[run].inc, kGValid | (excl + Tr));
            s_excl = excl;
            if (run == B.runs - 1) info[(int64_t)img * 4] = (excl + Tr + 7) / 8;  // stream bytes (:1161-1165)
        }
    }
    __syncthreads();
    if (act && first) {
        dc_piece(s_lprev[c], dcn, dcv);
        bits += (uint32_t)dcn;
    }
    // 6. block exclusive scan of the unit lengths -> bit offsets
    uint32_t incl = bits;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[wv] = incl;  // (wave 0 read the A sums before the barrier above)
    __syncthreads();
    uint32_t before = incl - bits;
    for (int q = 0; q < wv; ++q) before += wsum[q];
    const uint64_t pos = s_excl + before;
    const uint64_t cap_bits = B.wwords * 32;
    if (!act || pos + bits + 32 > cap_bits) return;  // past the words buffer: the host runs it again
    // 7. the unit's DC piece and its AC codes at its bit offset (jpeg_enc.h:613-643)
    uint32_t* wp = words + (int64_t)img * B.wwords + (pos >> 5);
    uint32_t* const wp0 = wp;
    const int o0 = (int)(pos & 31);
    uint64_t acc = 0;
    int nacc = o0;  // the first o0 bits of the first word belong to the previous unit (zeros here)
    // A word shared with the previous unit (o0 != 0: the first) is kept in a register and OR-ed
    // in at the end, so the word check stores plainly or not at all.
    bool firstw = o0 != 0;
    uint32_t wfirst = 0;
    auto put = [&](int n, uint32_t v) {  // v < 2^n, n <= 32
        acc = (acc << n) | v;
        nacc += n;
        if (nacc >= 32) {
            nacc -= 32;
            const uint32_t word = (uint32_t)(acc >> nacc);
            wfirst = firstw ? word : wfirst;
            if (!firstw) *wp = word;
            firstw = false;
            ++wp;
        }
    };
    put(dcn, dcv);
    const int nfull = (int)(bits_ac >> 5), rem = (int)(bits_ac & 31);
    for (int q = 0; q < nfull; ++q) put(32, sl[q]);
    if (rem) put(rem, sl[nfull] >> (32 - rem));
    if (o0 && wp != wp0) atomicOr(wp0, wfirst);                    // shared with the previous unit
    if (nacc > 0) atomicOr(wp, (uint32_t)(acc << (32 - nacc)));  // shared with the next unit
}

// FF -> FF 00 byte stuffing (jpeg_enc.h:634-638) of a batch's streams: 16 stream bytes (4 words,
// one 16-byte load) per lane, a workgroup per 4 KB; k_stuff_count_b counts each workgroup's FF
// bytes, one scan over the batch gives every workgroup's stuffed offset, k_stuff_write_b recounts
// per lane, scans in the workgroup and copies.
constexpr int kStuffChunk = 16;
constexpr int kStuffWg = 256 * kStuffChunk;
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
__device__ __forceinline__ uint32_t chunk_ff(const uint32_t (&w)[4], int nb) {
    uint32_t n = 0;
#pragma unroll
    for (int i = 0; i < kStuffChunk; ++i) n += (i < nb && ((w[i >> 2] >> (24 - 8 * (i & 3))) & 255u) == 255u);
    return n;
}
// the image's stream bytes, clamped to its words buffer (an image past it is encoded again)
__device__ __forceinline__ uint64_t stream_bytes(const uint64_t* info, int img, uint64_t wwords) {
    return min<uint64_t>(info[(int64_t)img * 4], wwords * 4);
}
__global__ __launch_bounds__(256) void k_stuff_count_b(const uint32_t* __restrict__ words, uint64_t wwords,
                                                       const uint64_t* __restrict__ info, int nwg,
                                                       uint32_t* __restrict__ wsum) {
    __shared__ uint32_t s[4];
    const int img = blockIdx.y, t = threadIdx.x;
    const uint64_t nbytes = stream_bytes(info, img, wwords);
    const int64_t ch = (int64_t)blockIdx.x * 256 + t;
    const uint64_t b0 = (uint64_t)ch * kStuffChunk;
    uint32_t n = 0;
    if (b0 < nbytes) {
        uint32_t w[4];
        chunk_words(words + (int64_t)img * wwords, ch, nbytes, w);
        n = chunk_ff(w, (int)min<uint64_t>(kStuffChunk, nbytes - b0));
    }
    n = wave_sum32(n);
    if ((t & 63) == 0) s[t >> 6] = n;
    __syncthreads();
    if (t == 0) {
        wsum[(int64_t)img * nwg + blockIdx.x] = s[0] + s[1] + s[2] + s[3];
        if (img == (int)gridDim.y - 1 && (int)blockIdx.x == nwg - 1) wsum[(int64_t)gridDim.y * nwg] = 0;  // scan tail
    }
}
// The file header (SOI .. SOS, < 1 KiB) as a kernel argument.
struct HdrArg {
    uint8_t b[1024];
    int n;
};
// Writes image img's stuffed stream (after its header when hdr.n > 0, and EOI after it with eoi)
// only when the whole file fits in cap bytes past out + img * stride; info[4 img + 1] = stuffed
// bytes either way.
__global__ __launch_bounds__(256) void k_stuff_write_b(const uint32_t* __restrict__ words, uint64_t wwords,
                                                       uint64_t* __restrict__ info, int nwg,
                                                       const uint32_t* __restrict__ wbase, HdrArg hdr,
                                                       uint8_t* __restrict__ out, uint64_t stride, uint64_t cap, int eoi) {
    __shared__ uint32_t s[4];
    const int img = blockIdx.y, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint64_t nbytes_raw = info[(int64_t)img * 4];
    const uint64_t nbytes = min<uint64_t>(nbytes_raw, wwords * 4);
    const uint32_t* base = wbase + (int64_t)img * nwg;
    const uint64_t total = nbytes + (uint32_t)(base[nwg] - base[0]);
    if (blockIdx.x == 0 && t == 0) info[(int64_t)img * 4 + 1] = total;
    const uint64_t need = (uint64_t)hdr.n + total + (eoi ? 2 : 0);
    if (need > cap || nbytes_raw + 4 > wwords * 4) return;  // (uniform per workgroup)
    uint8_t* o0 = out + (int64_t)img * stride;
    if (blockIdx.x == 0) {
        for (int i = t; i < hdr.n; i += 256) o0[i] = hdr.b[i];
        if (eoi && t == 0) { o0[hdr.n + total] = 0xFF; o0[hdr.n + total + 1] = 0xD9; }
    }
    const int64_t ch = (int64_t)blockIdx.x * 256 + t;
    const uint64_t b0 = (uint64_t)ch * kStuffChunk;
    uint32_t w[4] = {0, 0, 0, 0};
    int nb = 0;
    if (b0 < nbytes) {
        chunk_words(words + (int64_t)img * wwords, ch, nbytes, w);
        nb = (int)min<uint64_t>(kStuffChunk, nbytes - b0);
    }
    // the workgroup's stuffed bytes are assembled in LDS at the destination's dword phase, then
    // leave as aligned dword stores (bytes only at the two ends, shared with the neighbours)
    __shared__ uint32_t ob[(2 * kStuffWg + 8) / 4];
    uint8_t* obb = reinterpret_cast<uint8_t*>(ob);
    const uint32_t n = chunk_ff(w, nb);
    const uint32_t mine = (uint32_t)nb + n;  // this lane's output bytes
    uint32_t incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) s[wv] = incl;
    __syncthreads();
    uint32_t lo = incl - mine;
    for (int q = 0; q < wv; ++q) lo += s[q];
    const uint32_t wg_len = s[0] + s[1] + s[2] + s[3];
    if (!wg_len) return;  // (uniform: a workgroup past the stream)
    uint8_t* gdst = o0 + hdr.n + (uint64_t)blockIdx.x * kStuffWg + (base[blockIdx.x] - base[0]);
    const int al = (int)(reinterpret_cast<uintptr_t>(gdst) & 3);
    {
        uint8_t* q = obb + al + lo;
#pragma unroll
        for (int i = 0; i < kStuffChunk; ++i) {
            if (i >= nb) break;
            const uint8_t v = (uint8_t)(w[i >> 2] >> (24 - 8 * (i & 3)));
            *q++ = v;
            if (v == 0xFF) *q++ = 0;  // jpeg_enc.h:634-638
        }
    }
    __syncthreads();
    uint32_t* gw = reinterpret_cast<uint32_t*>(gdst - al);
    const int end = al + (int)wg_len, nd = (end + 3) >> 2;
    for (int d = t; d < nd; d += 256) {
        const int b0d = 4 * d;
        if (b0d >= al && b0d + 4 <= end) {
            gw[d] = ob[d];
        } else {
            for (int j = max(b0d, al); j < min(b0d + 4, end); ++j) (gdst - al)[j] = obb[j];
        }
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
        L.firstk[0] = 0; L.firstk[1] = 4; L.firstk[2] = 5;
        L.lastk[0] = 3; L.lastk[1] = 4; L.lastk[2] = 5;
    } else {  // 4:4:4 (tiny_jpeg's only layout)
        L.upm = 3;
        L.ms = 8;
        for (int k = 0; k < 3; ++k) { L.comp[k] = (int8_t)k; L.prevk[k] = -1; L.firstk[k] = L.lastk[k] = (int8_t)k; }
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
// A batch of images (same geometry and settings) is encoded by one fused launch and the stuffing
// pair, whatever the batch size:
//   memset     the words buffers (image i's at words + i * wwords), look-back records, ticket
//   k_enc_run  every run of every image (units, DC chain, look-back scan, emit); info[4i] = stream
//              bytes
//   k_stuff_count_b, one scan over the batch, k_stuff_write_b: stuffed stream (with header and EOI
//              when asked) at out + i * stride, only when it fits; info[4i + 1] = stuffed bytes
//   info -> pinned host memory, one host wait per batch
// An image whose stream outgrew its words buffer (sized from the images before) is encoded again
// with a buffer of its measured size.
struct EncWs {
    EncTables* T = nullptr;
    RunRec* recs = nullptr;
    size_t recs_cap = 0;
    unsigned* ticket = nullptr;
    uint32_t* words = nullptr;
    size_t words_cap = 0;        // bytes
    uint32_t *wsum = nullptr, *wbase = nullptr;
    size_t wsum_cap = 0, wbase_cap = 0;
    uint64_t* info = nullptr;    // device: 4 per image (stream bytes, stuffed bytes)
    uint64_t* hinfo = nullptr;   // pinned host copy
    size_t info_cap = 0;         // images
    const uint8_t** srcs = nullptr;  // device array of source pointers
    size_t srcs_cap = 0;
    uint64_t est_bytes = 0;      // words-buffer estimate per image from the images so far
    void* tmp = nullptr;
    size_t tmp_cap = 0;
    // per-stage HIP events of the last batch (icx_encoder_stage_times): encode, stuff; ms[]
    // accumulates over calls until read
    hipEvent_t ev[4] = {};
    float ms[2] = {};
    ~EncWs() {
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
        for (void* p : {(void*)T, (void*)recs, (void*)ticket, (void*)words, (void*)wsum, (void*)wbase, (void*)info,
                        (void*)srcs, tmp})
            if (p) (void)hipFree(p);
        if (hinfo) (void)hipHostFree(hinfo);
    }
};
EncWs* enc_ws_create() {
    EncWs* ws = new EncWs();
    for (hipEvent_t& e : ws->ev)
        if (hipEventCreate(&e) != hipSuccess) e = nullptr;
    return ws;
}
const char* const kEncStageNames[2] = {"encode", "stuff"};
int enc_ws_stage_times(EncWs* ws, const char** names, float* ms, int cap) {
    const int k = cap < 2 ? cap : 2;
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

// Images per launch: the words buffers of one launch stay within this many bytes.
constexpr uint64_t kEncWordsBudget = 4ull << 30;

// Encodes n images (device sources srcs[i], w x h x comps) into out + i * stride: hdr (if any),
// the stuffed stream, EOI (with eoi), only when all of it fits in `cap` bytes; nbytes[i] = stream
// bytes, total[i] = stuffed bytes. wbytes: words buffer per image. Returns false on a HIP failure.
static bool enc_launch(hipStream_t st, EncWs& ws, const EncLayout& L, const EncTables& T, int n,
                       const uint8_t* const* srcs, int w, int h, int comps, uint64_t wbytes, uint8_t* out,
                       uint64_t stride, uint64_t cap, bool eoi, const HdrArg& hdr, uint64_t* nbytes, uint64_t* total) {
    const int64_t mbh = (h + L.ms - 1) / L.ms;
    const int runs_per_row = (L.mbw * L.ms + kRunPx - 1) / kRunPx;
    const int64_t runs = (int64_t)runs_per_row * mbh;
    const uint64_t wwords = wbytes / 4;
    const int nwg = (int)((wbytes + kStuffWg - 1) / kStuffWg);
    if (!ws.T) ENC_HIP(hipMalloc(&ws.T, sizeof(EncTables)));
    if (!ws.ticket) ENC_HIP(hipMalloc(&ws.ticket, 2 * sizeof(unsigned)));
    if (!grow(ws.recs, sizeof(RunRec) * runs * n, ws.recs_cap) || !grow(ws.words, wbytes * n, ws.words_cap) ||
        !grow(ws.wsum, sizeof(uint32_t) * ((size_t)nwg * n + 1), ws.wsum_cap) ||
        !grow(ws.wbase, sizeof(uint32_t) * ((size_t)nwg * n + 1), ws.wbase_cap))
        return false;
    if (!grow(ws.srcs, sizeof(uint8_t*) * n, ws.srcs_cap)) return false;
    if ((size_t)n > ws.info_cap) {
        if (ws.info) (void)hipFree(ws.info);
        if (ws.hinfo) (void)hipHostFree(ws.hinfo);
        ws.info = nullptr;
        ws.hinfo = nullptr;
        ws.info_cap = 0;
        ENC_HIP(hipMalloc(&ws.info, sizeof(uint64_t) * 4 * n));
        ENC_HIP(hipHostMalloc(&ws.hinfo, sizeof(uint64_t) * (4 * n + 1)));
        ws.info_cap = n;
    }
    ENC_HIP(hipMemcpyAsync(ws.T, &T, sizeof T, hipMemcpyHostToDevice, st));
    ENC_HIP(hipMemcpyAsync(ws.srcs, srcs, sizeof(uint8_t*) * n, hipMemcpyHostToDevice, st));
    const bool ev = ws.ev[3] != nullptr;
    if (ev) ENC_HIP(hipEventRecord(ws.ev[0], st));
    ENC_HIP(hipMemsetAsync(ws.words, 0, wbytes * n, st));
    ENC_HIP(hipMemsetAsync(ws.recs, 0, sizeof(RunRec) * runs * n, st));
    ENC_HIP(hipMemsetAsync(ws.ticket, 0, 2 * sizeof(unsigned), st));
    EncBatch B;
    B.srcs = ws.srcs;
    B.w = w;
    B.h = h;
    B.comps = comps;
    B.runs_per_row = runs_per_row;
    B.runs = (int)runs;
    B.wwords = wwords;
    hipLaunchKernelGGL(k_enc_run, dim3((unsigned)(runs * n)), dim3(256), 0, st, B, L, ws.T, ws.recs, ws.ticket, ws.words,
                       ws.info);
    if (ev) ENC_HIP(hipEventRecord(ws.ev[1], st));
    if (ev) ENC_HIP(hipEventRecord(ws.ev[2], st));
    hipLaunchKernelGGL(k_stuff_count_b, dim3(nwg, n), dim3(256), 0, st, ws.words, wwords, ws.info, nwg, ws.wsum);
    size_t tmp_b = 0;
    const int ns = nwg * n + 1;
    ENC_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_b, ws.wsum, ws.wbase, ns, st));
    if (!grow(ws.tmp, tmp_b, ws.tmp_cap)) return false;
    ENC_HIP(hipcub::DeviceScan::ExclusiveSum(ws.tmp, tmp_b, ws.wsum, ws.wbase, ns, st));
    hipLaunchKernelGGL(k_stuff_write_b, dim3(nwg, n), dim3(256), 0, st, ws.words, wwords, ws.info, nwg, ws.wbase, hdr, out,
                       stride, cap, eoi ? 1 : 0);
    if (ev) ENC_HIP(hipEventRecord(ws.ev[3], st));
    ENC_HIP(hipGetLastError());
    ENC_HIP(hipMemcpyAsync(ws.hinfo, ws.info, sizeof(uint64_t) * 4 * n, hipMemcpyDeviceToHost, st));
    ENC_HIP(hipMemcpyAsync(ws.hinfo + 4 * n, ws.ticket + 1, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    ENC_HIP(hipStreamSynchronize(st));
    if (*reinterpret_cast<const unsigned*>(ws.hinfo + 4 * n)) return false;  // a look-back wait expired
    for (int i = 0; i < n; ++i) {
        nbytes[i] = ws.hinfo[4 * i];
        total[i] = ws.hinfo[4 * i + 1];
    }
    if (ev) {
        for (int i = 0; i < 2; ++i) {
            float t = 0.f;
            if (hipEventElapsedTime(&t, ws.ev[2 * i], ws.ev[2 * i + 1]) == hipSuccess) ws.ms[i] += t;
        }
    }
    return true;
}

// The batch encode behind every entry point: images in launches of at most kEncWordsBudget bytes
// of words buffers; an image whose stream did not fit its words buffer is encoded again alone.
// sizes[i] = header + stuffed bytes (+ 2 with eoi); fits[i] = it was written.
static bool enc_batch(hipStream_t st, EncWs& ws, const EncLayout& L, const EncTables& T, int n,
                      const uint8_t* const* srcs, int w, int h, int comps, uint8_t* out, uint64_t stride, uint64_t cap,
                      bool eoi, const HdrArg& hdr, uint64_t* sizes, bool* fits) {
    const uint64_t est = ws.est_bytes ? ws.est_bytes : std::max<uint64_t>(65536, (uint64_t)w * h * comps / 4);
    const uint64_t wbytes = (est + 4 + kStuffWg - 1) / kStuffWg * kStuffWg;
    int per = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)n, kEncWordsBudget / wbytes));
    if (const char* e = std::getenv("ICX_ENC_BATCH")) per = std::max(1, std::min(per, std::atoi(e)));  // (tests)
    std::vector<uint64_t> nb(per), tot(per);
    for (int i0 = 0; i0 < n; i0 += per) {
        const int k = std::min(per, n - i0);
        if (!enc_launch(st, ws, L, T, k, srcs + i0, w, h, comps, wbytes, out + (uint64_t)i0 * stride, stride, cap, eoi, hdr,
                        nb.data(), tot.data()))
            return false;
        for (int i = 0; i < k; ++i) {
            uint64_t nbytes = nb[i], stuffed = tot[i];
            if (nbytes + 4 > wbytes) {  // the stream outgrew the words buffer: nothing was written
                const uint64_t wb2 = (nbytes + nbytes / 4 + 4 + kStuffWg - 1) / kStuffWg * kStuffWg;
                uint64_t nb2 = 0, tot2 = 0;
                if (!enc_launch(st, ws, L, T, 1, srcs + i0 + i, w, h, comps, wb2, out + (uint64_t)(i0 + i) * stride, stride,
                                cap, eoi, hdr, &nb2, &tot2))
                    return false;
                if (nb2 + 4 > wb2) return false;  // (cannot happen: same image, same size)
                nbytes = nb2;
                stuffed = tot2;
            }
            ws.est_bytes = std::max(ws.est_bytes, nbytes + nbytes / 4);
            sizes[i0 + i] = hdr.n + stuffed + (eoi ? 2 : 0);
            fits[i0 + i] = sizes[i0 + i] <= cap;
        }
    }
    return true;
}

static HdrArg make_hdr(const std::vector<uint8_t>& head) {
    HdrArg ha;
    std::memcpy(ha.b, head.data(), head.size());
    ha.n = (int)head.size();
    return ha;
}

// Upload, encode, download: the whole file of one host image into `out` (header built on the host).
static bool encode_host_image(hipStream_t st, const EncLayout& L, const EncTables& T, int w, int h, int comps,
                              const uint8_t* src, std::vector<uint8_t>& out) {
    const size_t srcb = (size_t)w * h * comps;
    if (!srcb) {
        out.push_back(0xFF);
        out.push_back(0xD9);
        return true;
    }
    EncWs ws;
    uint8_t *d_src = nullptr, *d_out = nullptr;
    HdrArg none;
    none.n = 0;
    bool ok = hipMalloc(&d_src, srcb) == hipSuccess && hipMemcpyAsync(d_src, src, srcb, hipMemcpyHostToDevice, st) == hipSuccess;
    // first pass sizes the output, the second (only when it did not fit) writes it
    uint64_t cap = srcb + 65536, size = 0;
    bool fit = false;
    const uint8_t* srcs[1] = {d_src};
    ok = ok && hipMalloc(&d_out, cap) == hipSuccess && enc_batch(st, ws, L, T, 1, srcs, w, h, comps, d_out, cap, cap, false, none, &size, &fit);
    if (ok && !fit) {
        (void)hipFree(d_out);
        d_out = nullptr;
        cap = size;
        ok = hipMalloc(&d_out, cap) == hipSuccess && enc_batch(st, ws, L, T, 1, srcs, w, h, comps, d_out, cap, cap, false, none, &size, &fit) && fit;
    }
    if (ok && size) {
        const size_t h0 = out.size();
        out.resize(h0 + size);
        ok = hipMemcpyAsync(out.data() + h0, d_out, size, hipMemcpyDeviceToHost, st) == hipSuccess &&
             hipStreamSynchronize(st) == hipSuccess;
    }
    if (d_src) (void)hipFree(d_src);
    if (d_out) (void)hipFree(d_out);
    out.push_back(0xFF);
    out.push_back(0xD9);
    return ok;
}

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

// A batch of device images, same geometry and settings: image i's whole file (header, stuffed
// stream, EOI) -> d_out + i*stride, written only when it fits in stride bytes. Per image:
// sizes[i] (the file's bytes, also when it did not fit) and status[i] (0 ok, 1 did not fit:
// nothing written). Returns 0, or -1 on a HIP failure. Synchronous (one host wait per launch).
int jpeg_encode_device_batch(hipStream_t st, EncWs* ws, int n, int quality, int subsampling, int w, int h, int comps,
                             const uint8_t* const* d_srcs, uint8_t* d_out, uint64_t stride, uint64_t* sizes,
                             int32_t* status) {
    if (n <= 0) return 0;
    uint8_t qnl[64], qnc[64];
    ijg_table(kLumaQ, quality, qnl);
    ijg_table(kK2Chroma, quality, qnc);
    EncTables T;
    build_tables(T, qnl, qnc);
    std::vector<uint8_t> head;
    ext_header(head, w, h, qnl, qnc, subsampling);
    const uint64_t hn = head.size();
    if (hn > sizeof(HdrArg::b)) return -1;
    if (w == 0 || h == 0) {  // no data units: header + EOI only
        static const uint8_t eoi[2] = {0xFF, 0xD9};
        for (int i = 0; i < n; ++i) {
            sizes[i] = hn + 2;
            status[i] = sizes[i] > stride ? 1 : 0;
            uint8_t* o = d_out + (uint64_t)i * stride;
            if (!status[i] && (hipMemcpyAsync(o, head.data(), hn, hipMemcpyHostToDevice, st) != hipSuccess ||
                               hipMemcpyAsync(o + hn, eoi, 2, hipMemcpyHostToDevice, st) != hipSuccess))
                return -1;
        }
        return hipStreamSynchronize(st) == hipSuccess ? 0 : -1;
    }
    const HdrArg ha = make_hdr(head);
    std::unique_ptr<bool[]> fit(new bool[n]);
    if (!enc_batch(st, *ws, make_layout(subsampling, w), T, n, d_srcs, w, h, comps, d_out, stride, stride, true, ha, sizes,
                   fit.get()))
        return -1;
    for (int i = 0; i < n; ++i) status[i] = fit[i] ? 0 : 1;
    return 0;
}

// C4 extension, device image -> whole file in d_out (device). Returns 0 ok, 1 d_out too small
// (*size = bytes needed), -1 HIP failure.
int jpeg_encode_device(hipStream_t st, EncWs* ws, int quality, int subsampling, int w, int h, int comps,
                       const uint8_t* d_src, uint8_t* d_out, uint64_t cap, uint64_t* size) {
    const uint8_t* srcs[1] = {d_src};
    int32_t stt = 0;
    const int rc = jpeg_encode_device_batch(st, ws, 1, quality, subsampling, w, h, comps, srcs, d_out, cap, size, &stt);
    return rc < 0 ? -1 : stt;
}

}  // namespace icx
