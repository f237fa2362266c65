// icx_decode.hip -- gfx950 kernels for batched JPEG decode (NanoJPEG-exact).
//
// Pipeline per group of images (one slot per image, all kernels cover the whole group):
//   k_parse          header walk per image on the GPU            (jpeg_dec.h:880-903)
//   k_entropy_seq    sequential Huffman decode, one lane/image   (jpeg_dec.h:643-718)
//   k_idct           dequant + integer IDCT, 8 lanes per block   (jpeg_dec.h:343-442,658-676)
//   k_upsample       one bicubic doubling pass per launch        (jpeg_dec.h:736-791,817-833)
//   k_convert        YCbCr->RGB / gray stride removal            (jpeg_dec.h:834-865)
// All integer math reproduces the reference bit for bit (icx_jpeg.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "icx_internal.h"

namespace icx {

const char* const kStageNames[kStCount] = {"parse", "unstuff", "entropy", "write", "idct", "upsample", "convert"};

int64_t ws_coef_cap(int w, int h) {  // any power-of-two sampling: MCU <= 64 px
    int64_t wp = ((int64_t)w + 63) / 64 * 64, hp = ((int64_t)h + 63) / 64 * 64;
    return 3 * (wp / 8) * (hp / 8);
}
int64_t ws_plane_cap(int w, int h) { return ws_coef_cap(w, h) * 64; }
int64_t ws_tmp_cap(int w, int h) { return ((int64_t)w + 8) * ((int64_t)h + 8); }

// ------------------------------------------------------------------------------ parse
__device__ __forceinline__ bool fused420_shape(const Desc& d);  // (the 4:2:0 back half, below)
// One 64-lane workgroup per image: zero the descriptor together, lane 0 walks the markers,
// then all lanes fill the four 1024-entry fast Huffman tables. `layout` (pinned memory, zeroed by
// the host before the launch): set when an image that will be decoded is not 4:2:0 in the fused
// layout -- the host reads it once the group's planning has run and launches the other
// samplings' back-half kernels only then.
__global__ __launch_bounds__(64) void k_parse(int n, const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
                                              const uint64_t* __restrict__ size, Desc* __restrict__ desc, int max_w,
                                              int max_h, uint64_t out_stride, int32_t* __restrict__ layout) {
    const int i = blockIdx.x;
    if (i >= n) return;
    Desc& d = desc[i];
    uint32_t* raw = reinterpret_cast<uint32_t*>(&d);
    for (size_t k = threadIdx.x; k < sizeof(Desc) / 4; k += blockDim.x) raw[k] = 0;
    __syncthreads();
    if (threadIdx.x == 0) {
        const int st = parse_headers(data + off[i], (int64_t)size[i], d, false);
        if (st == kPending) {
            // capacity of this batch's workspace / output slot (the reference allocates here, :568-572)
            const int64_t out_bytes = (int64_t)d.W * d.H * (d.nc == 1 ? 1 : d.nc);
            if (d.W > max_w || d.H > max_h || out_bytes > (int64_t)out_stride) d.status = kOutOfMem;
        }
        if (layout && d.status == kPending && !fused420_shape(d)) *layout = 1;
    }
    __syncthreads();
    if (d.status != kPending) return;
    for (int t = 0; t < 4; ++t) huff_fill_fast(d.huff[t], threadIdx.x, blockDim.x);
}

// ---------------------------------------------------------------- entropy (sequential)
// One wave per image that neither parallel path takes (a stream whose restart markers NanoJPEG
// reads where no lane starts, more than kSpecMaxBpm blocks per MCU -- beyond the JPEG limit of 10,
// so non-conforming --, an exhausted workspace, a repair walk that never resynchronises). Lane 0
// walks the entropy-coded segment exactly like njDecodeScan (jpeg_dec.h:643-718). The wave keeps
// the image's four Huffman tables in LDS and the stream's next bytes in an LDS ring, refilled a KiB
// at a time by all 64 lanes with 16-byte loads, so the serial walk runs at LDS latency instead of
// a dependent global load per byte and per table lookup.
// ICX_SEQ_LDS=0 (default): the tables and the stream are read from global memory (L1/L2) instead.
// The LDS form walks ~10% faster, but a kernel holding ~14 KB of LDS per workgroup cannot be
// dispatched while the other pipeline's entropy kernels fill every CU's LDS, and it sits in the
// stream before the back half even when it has nothing to do (every group, every call): at C2 it
// waited ~0.16 ms per group for LDS it then did not use.
#ifndef ICX_SEQ_LDS
#define ICX_SEQ_LDS 0
#endif
constexpr int kSeqRing = 4096;  // 4 quarters of 1 KiB; lane 0 always has >= 2 KiB loaded ahead
struct RingBits {                // rb_fill's byte rules (icx_jpeg.h) over the ring
    const uint8_t* ring;
    int64_t pos, end;            // next byte, stream end (relative to the aligned ring origin)
    uint32_t acc;
    int32_t nacc, err;
    __device__ uint32_t byte() { return ring[(pos++) & (ICX_SEQ_LDS ? kSeqRing - 1 : ~(int64_t)0)]; }
    __device__ void fill(int want) {
        while (nacc < want) {
            if (pos >= end) { acc = (acc << 8) | 0xFFu; nacc += 8; continue; }
            const uint32_t x = byte();
            acc = (acc << 8) | x;
            nacc += 8;
            if (x != 0xFF) continue;
            if (pos >= end) { err = kSyntaxError; continue; }
            const uint32_t m = byte();
            if (m == 0x00 || m == 0xFF) continue;
            if (m == 0xD9) { end = pos; continue; }
            if ((m & 0xF8) == 0xD0) { acc = (acc << 8) | m; nacc += 8; }
            else err = kSyntaxError;
        }
    }
    __device__ uint32_t peek(int n) {
        if (!n) return 0;
        fill(n);
        return (acc >> (nacc - n)) & ((1u << n) - 1u);
    }
    __device__ void drop(int n) {
        if (nacc < n) fill(n);
        nacc -= n;
    }
};
__global__ __launch_bounds__(64) void k_entropy_seq(int n, const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
                                                    Desc* __restrict__ desc, int16_t* __restrict__ ac, int32_t* __restrict__ dcv) {
    const int i = blockIdx.x;
    if (i >= n) return;
    Desc& d = desc[i];
    if (d.status != kPending) return;  // (uniform)
    const int lane = threadIdx.x;
    const uint8_t* S = data + off[i] + d.scan_off;
    const int mis = (int)(reinterpret_cast<uintptr_t>(S) & 15);
    const uint8_t* S0 = S - mis;
    const int64_t end = (int64_t)(d.size - d.scan_off) + mis;
#if !ICX_SEQ_LDS
    const Huff* HT = d.huff;
    RingBits b{S0, mis, end, 0u, 0, 0};  // (fill never reads at or past `end`)
    auto refill = [&](int64_t) {};
#else
    __shared__ Huff HT[4];
    __shared__ uint4 ring4[kSeqRing / 16];
    {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(d.huff);
        uint32_t* dst = reinterpret_cast<uint32_t*>(HT);
        for (int k = lane; k < (int)(sizeof(HT) / 4); k += 64) dst[k] = src[k];
    }
    // the ring holds the stream from a 16-byte aligned origin: quarter q of the ring = stream KiB qi
    // with qi % 4 == q; quarters qlo .. qlo+3 are loaded
    auto fill_quarter = [&](int64_t qi) {  // all lanes (bytes past the end read as FF, never used)
        const int64_t at = qi * 1024 + lane * 16;
        uint4 v = make_uint4(~0u, ~0u, ~0u, ~0u);
        if (at + 16 <= end) {
            v = *reinterpret_cast<const uint4*>(S0 + at);
        } else if (at < end) {
            uint8_t tb[16];
            for (int k = 0; k < 16; ++k) tb[k] = at + k < end ? S0[at + k] : 0xFF;
            __builtin_memcpy(&v, tb, 16);
        }
        ring4[(qi & 3) * 64 + lane] = v;
    };
    int64_t qlo = 0;
    for (int q = 0; q < 4; ++q) fill_quarter(q);
    __syncthreads();
    RingBits b{reinterpret_cast<const uint8_t*>(ring4), mis, end, 0u, 0, 0};
    auto refill = [&](int64_t pos) {
        while (pos >= (qlo + 2) * 1024) {
            fill_quarter(qlo + 4);
            ++qlo;
        }
    };
#endif
    int16_t* A = ac + d.acbase * 64;  // (in place: the pool region k_spec_plan gave the image)
    int32_t* D = dcv + d.acbase;
    int32_t pred[3] = {0, 0, 0};
    int left = d.restart, expect = 0;
    const int64_t nmcu = (int64_t)d.mbw * d.mbh;
    int64_t blk = 0;
    int err = 0;
    for (int64_t m = 0; m < (nmcu > 0 ? nmcu : 1) && !err; ++m) {
        for (int r = 0; r < d.bpm && !err; ++r, ++blk) {
            // wave-uniform: keep >= 2 KiB loaded past lane 0's position (a block reads < 600 bytes)
            const int64_t pos = __builtin_amdgcn_readfirstlane((int)b.pos) |
                                ((int64_t)__builtin_amdgcn_readfirstlane((int)(b.pos >> 32)) << 32);
            refill(pos);
            __builtin_amdgcn_wave_barrier();  // (one wave: its LDS accesses stay in order)
            if (lane == 0) {
                int sbx, sby;
                const int ci = mcu_block_comp(d, r, sbx, sby);
                const Comp& c = d.c[ci];
                int16_t* row = A + blk * 64;
#pragma unroll
                for (int q = 0; q < 8; ++q) reinterpret_cast<int4*>(row)[q] = make_int4(0, 0, 0, 0);
                // DC (jpeg_dec.h:662-663)
                int sym = 0;
                int len = huff_lookup(HT[c.dc_tab], b.peek(16), sym);
                if (!len) {
                    err = kSyntaxError;
                } else {
                    b.drop(len);
                    int nb = sym & 15;
                    int32_t v = 0;
                    if (nb) { v = extend((int32_t)b.peek(nb), nb); b.drop(nb); }
                    pred[ci] = wadd(pred[ci], v);
                    row[0] = dc_cell(pred[ci]);
                    if (row[0] == kDcEscape) D[blk] = pred[ci];
                    // AC (jpeg_dec.h:664-671)
                    int k = 0;
                    do {
                        len = huff_lookup(HT[c.ac_tab], b.peek(16), sym);
                        if (!len) { err = kSyntaxError; break; }
                        b.drop(len);
                        if (!sym) break;  // EOB
                        if (!(sym & 0x0F) && sym != 0xF0) { err = kSyntaxError; break; }
                        nb = sym & 15;
                        v = 0;
                        if (nb) { v = extend((int32_t)b.peek(nb), nb); b.drop(nb); }
                        k += (sym >> 4) + 1;
                        if (k > 63) { err = kSyntaxError; break; }
                        row[k] = (int16_t)v;  // blocks are kept in zig-zag order (k_idct reorders)
                    } while (k < 63);
                    if (b.err) err = b.err;
                }
            }
            err = __builtin_amdgcn_readfirstlane(err);
        }
        if (err) break;
        if (d.restart && m + 1 < nmcu && !(--left)) {  // jpeg_dec.h:707-715 (uniform control)
            if (lane == 0) {
                b.nacc &= 0xF8;
                const int mk = (int)b.peek(16);
                b.drop(16);
                if ((mk & 0xFFF8) != 0xFFD0 || (mk & 7) != expect) err = kSyntaxError;
            }
            err = __builtin_amdgcn_readfirstlane(err);
            if (err) break;
            expect = (expect + 1) & 7;
            left = d.restart;
            pred[0] = pred[1] = pred[2] = 0;
        }
    }
    if (lane == 0) d.status = err ? kSyntaxError : kOk;
}

// ----------------------------------------------------------------------- plane layout
__device__ __forceinline__ int64_t comp_plane_off(const Desc& d, int ci) {
    int64_t o = 0;
    for (int j = 0; j < ci; ++j) o += (int64_t)d.c[j].stride * ((int64_t)d.mbh * d.c[j].vs * 8);
    return o;
}

// --------------------------------------------------------------------------------- IDCT
// Every wave works alone on octets of 8 consecutive blocks: lane (b, r) dequantizes and
// row-transforms natural row r of block b, then column-transforms column r, then stores row r
// of the 8x8 pixel tile (8 bytes). The row->column and column->row exchanges go through the
// wave's own LDS area, ordered by wave barriers only (a wave's LDS operations execute in issue
// order), so the four waves of a workgroup never wait for each other. Each wave loads kIdctU
// octets (kIdctU 16-byte chunks per lane) before transforming the first: more bytes in flight
// per wave is what the HBM needs (the old 32-block, 3-__syncthreads loop sat at ~2.4 TB/s).
// Multiplies are 24-bit whenever every multiplied operand fits (always for dequantisation;
// per row / column for the transforms, with the exact 32-bit wrap path otherwise).
struct IdctGeo {
    int64_t off;     // plane offset of the block's component
    int32_t stride;  // plane stride
    int32_t dx, dy;  // pixel offset of the block inside the MCU
    int32_t mx, my;  // MCU pitch in pixels in this plane (8*hs, 8*vs)
    int32_t ci;
};
constexpr int kIdctU = 4;
constexpr int kIdctUnitBlocks = 64;
__global__ __launch_bounds__(256) void k_idct_any(const Desc* __restrict__ desc, const int16_t* __restrict__ ac,
                                              const int32_t* __restrict__ dcv, const uint2* __restrict__ map,
                                              uint8_t* __restrict__ planes, int64_t plane_cap) {
    const int img = blockIdx.y;
    const Desc& d = desc[img];
    if (d.status != kOk || d.bpm <= kIdctUnitBlocks) return;  // k_idct takes those
    __shared__ int32_t qn[3][64];          // natural-order dequant table per component
    __shared__ IdctGeo geo[kSpecMaxBpm];   // per block-in-MCU
    __shared__ int4 zzb[4][8][8];          // per wave: the octet's blocks as stored (zig-zag order)
    __shared__ int32_t rows[4][8][8][9];   // per wave: row-pass output, padded
    __shared__ uint2 pix[4][8][8];         // per wave: 8x8 pixel tiles, one 8-byte row per entry
    const int t = threadIdx.x;
    if (t < 3 * 64) {
        const int ci = t >> 6, n = t & 63;
        qn[ci][n] = ci < d.nc ? d.q[d.c[ci].tq][kZigOfNat[n]] : 0;
    }
    const int bpm = d.bpm, mbw = d.mbw;
    if (t < kSpecMaxBpm && t < bpm) {
        int sbx, sby;
        const int ci = mcu_block_comp(d, t, sbx, sby);
        const Comp& c = d.c[ci];
        geo[t] = IdctGeo{comp_plane_off(d, ci), c.stride, sbx * 8, sby * 8, c.hs * 8, c.vs * 8, ci};
    }
    __syncthreads();
    const uint32_t nblocks = (uint32_t)((int64_t)d.mbw * d.mbh * bpm);
    const uint32_t noct = (nblocks + 7) >> 3;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63, lb = lane >> 3, r = lane & 7;
    // natural row r = zig-zag positions kZigOfNat[8r .. 8r+7] of the staged block (byte offsets)
    uint32_t zo[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) zo[j] = 2u * kZigOfNat[r * 8 + j];
    const uint8_t* zrow = reinterpret_cast<const uint8_t*>(&zzb[wave][lb][0]);
    uint8_t* P = planes + (int64_t)img * plane_cap;
    const bool small_mcu = bpm <= kSpecMaxBpm;
    // XCD-aware order: workgroups dispatched to one XCD (linear id % 8, gridDim.x a multiple of
    // 8) take adjacent octet ranges, so the partial plane lines they write merge in that XCD's L2
    const uint32_t chunk0 = (gridDim.x & 7) ? blockIdx.x : (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    const uint32_t wid = chunk0 * 4 + wave, nw = gridDim.x * 4;
    for (uint32_t o0 = wid * kIdctU; o0 < noct; o0 += nw * kIdctU) {
        int4 c[kIdctU];
        BlkLoc loc[kIdctU];
#pragma unroll
        for (int u = 0; u < kIdctU; ++u) {
            const uint32_t n = (o0 + u) * 8 + lb;
            loc[u] = blk_loc(d, map, n < nblocks ? n : 0);
            c[u] = n < nblocks ? *reinterpret_cast<const int4*>(ac + loc[u].blk * 64 + r * 8) : make_int4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < kIdctU; ++u) {
            const uint32_t n = (o0 + u) * 8 + lb;
            const bool live = n < nblocks;
            zzb[wave][lb][r] = c[u];
            __builtin_amdgcn_wave_barrier();
            const uint32_t mcu = n / (uint32_t)bpm, k = n - mcu * (uint32_t)bpm;
            const uint32_t mby = mcu / (uint32_t)mbw, mbx = mcu - mby * (uint32_t)mbw;
            IdctGeo g;
            if (small_mcu) {
                g = geo[k];
            } else {  // > 16 blocks per MCU: walk the component list
                int sbx = 0, sby = 0;
                const int ci = mcu_block_comp(d, (int)k, sbx, sby);
                const Comp& cc = d.c[ci];
                g = IdctGeo{comp_plane_off(d, ci), cc.stride, sbx * 8, sby * 8, cc.hs * 8, cc.vs * 8, ci};
            }
            int16_t s[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) s[j] = *reinterpret_cast<const int16_t*>(zrow + zo[j]);
            int32_t v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = m24(s[j], qn[g.ci][r * 8 + j]);  // int16 x 8-bit: exact
            if (r == 0 && live) v[0] = wmul(blk_dc(s[0], dcv, loc[u]), qn[g.ci][0]);  // absolute DC (pool cell + offset)
            if (idct_fast_ok(v)) idct_row<true>(v);
            else idct_row<false>(v);
#pragma unroll
            for (int j = 0; j < 8; ++j) rows[wave][lb][r][j] = v[j];
            __builtin_amdgcn_wave_barrier();
            int32_t col[8];
            uint8_t o[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) col[j] = rows[wave][lb][j][r];
            if (idct_fast_ok(col)) idct_col<true>(col, o);
            else idct_col<false>(col, o);
            uint8_t* pb = reinterpret_cast<uint8_t*>(&pix[wave][lb][0]);
#pragma unroll
            for (int j = 0; j < 8; ++j) pb[j * 8 + r] = o[j];
            __builtin_amdgcn_wave_barrier();
            if (live) {
                const int64_t y = (int64_t)mby * g.my + g.dy + r, x = (int64_t)mbx * g.mx + g.dx;
                *reinterpret_cast<uint2*>(P + g.off + y * g.stride + x) = pix[wave][lb][r];
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}


// Lane-pair IDCT helpers (k_idct420c, k_fused420): a block is transformed by two lanes in
// registers -- lane h takes natural rows 4h..4h+3 in the row pass and columns 4h..4h+3 in the
// column pass, the 4x4 quadrants changing hands by DPP. Full row / column formulas (no zero-AC
// shortcuts) with 24-bit multiplies: exact whenever every dequantized coefficient is below 2^14
// in magnitude (then no row output reaches 2^21); otherwise the reference code (idct_row /
// idct_col, shortcuts and 32-bit wrap included) runs.
namespace {
constexpr uint8_t kZigOfNatC[64] = {
    0, 1, 5, 6, 14, 15, 27, 28, 2, 4, 7, 13, 16, 26, 29, 42, 3, 8, 12, 17, 25, 30, 41, 43,
    9, 11, 18, 24, 31, 40, 44, 53, 10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
    21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};
}
// Full row / column formulas (no shortcuts): 24-bit multiplies of the inputs and their pairwise
// sums (below 2^23 on the fast path), 32-bit multiplies for the last butterfly's 181 products,
// whose operands x4 +- x5 are not (a dequantized AC of 2500 puts 8.5M there).
// The three rotations as packed 16-bit dot products (round 6): over the integers
// W7(x4 + x5) + (W1 - W7)x4 = W1 x4 + W7 x5 and W7(x4 + x5) - (W1 + W7)x5 = W7 x4 - W1 x5 (likewise
// for (x6, x7) and (x2, x3)), with no rounding between, so one v_dot2_i32_i16 of the packed pair
// gives each output exactly. The inputs are dequantized coefficients, below 2^14 on this path
// (block_transform's vote), so the pairs pack into int16 and no sum leaves int32 (< 2^27).
// (v_dot2_i32_i16 written out: the builtin became the VOP2 v_dot2c, whose accumulator is its
// destination, plus a v_mov of the zero into it -- more issue cycles than the multiplies it replaced)
__device__ __forceinline__ uint32_t pk16(int32_t lo, int32_t hi) {  // (lo, hi) low halves, one v_perm
    return __builtin_amdgcn_perm((uint32_t)hi, (uint32_t)lo, 0x05040100u);
}
__device__ __forceinline__ int32_t rdot2(uint32_t a, uint32_t w, int32_t zero) {
    int32_t r;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(w), "v"(zero));
    return r;
}
constexpr uint32_t kw16(int lo, int hi) { return ((uint32_t)lo & 0xFFFFu) | ((uint32_t)hi << 16); }
__device__ __forceinline__ void idct_row_full(int32_t (&r)[8]) {
    const int32_t z = __builtin_amdgcn_readfirstlane(0);  // (a zero accumulator the compiler keeps in a register)
    const uint32_t p17 = pk16(r[1], r[7]), p53 = pk16(r[5], r[3]), p26 = pk16(r[2], r[6]);
    int32_t x0 = (r[0] << 11) + 128, x1 = r[4] << 11;
    int32_t x4 = rdot2(p17, kw16(kW1, kW7), z), x5 = rdot2(p17, kw16(kW7, -kW1), z);  // W1 r1 + W7 r7, W7 r1 - W1 r7
    int32_t x6 = rdot2(p53, kw16(kW5, kW3), z), x7 = rdot2(p53, kw16(kW3, -kW5), z);  // W5 r5 + W3 r3, W3 r5 - W5 r3
    int32_t x3 = rdot2(p26, kw16(kW2, kW6), z), x2 = rdot2(p26, kw16(kW6, -kW2), z);  // W2 r2 + W6 r6, W6 r2 - W2 r6
    int32_t x8 = x0 + x1;
    x0 -= x1;
    x1 = x4 + x6;
    x4 -= x6;
    x6 = x5 + x7;
    x5 -= x7;
    x7 = x8 + x3;
    x8 -= x3;
    x3 = x0 + x2;
    x0 -= x2;
    // (x4 +- x5 reaches ~2^27 here: the 181 products stay 32-bit, as in idct_row)
    x2 = (wmul(181, x4 + x5) + 128) >> 8;
    x4 = (wmul(181, x4 - x5) + 128) >> 8;
    r[0] = (x7 + x1) >> 8;
    r[1] = (x3 + x2) >> 8;
    r[2] = (x0 + x4) >> 8;
    r[3] = (x8 + x6) >> 8;
    r[4] = (x8 - x6) >> 8;
    r[5] = (x0 - x4) >> 8;
    r[6] = (x3 - x2) >> 8;
    r[7] = (x7 - x1) >> 8;
}
__device__ __forceinline__ void idct_col_full(const int32_t (&v)[8], int32_t (&o)[8]) {
    int32_t x0 = (v[0] << 8) + 8192, x1 = v[4] << 8, x2 = v[6], x3 = v[2];
    int32_t x4 = v[1], x5 = v[7], x6 = v[5], x7 = v[3], x8;
    x8 = m24(kW7, x4 + x5) + 4;
    x4 = (x8 + m24(kW1 - kW7, x4)) >> 3;
    x5 = (x8 - m24(kW1 + kW7, x5)) >> 3;
    x8 = m24(kW3, x6 + x7) + 4;
    x6 = (x8 - m24(kW3 - kW5, x6)) >> 3;
    x7 = (x8 - m24(kW3 + kW5, x7)) >> 3;
    x8 = x0 + x1;
    x0 -= x1;
    x1 = m24(kW6, x3 + x2) + 4;
    x2 = (x1 - m24(kW2 + kW6, x2)) >> 3;
    x3 = (x1 + m24(kW2 - kW6, x3)) >> 3;
    x1 = x4 + x6;
    x4 -= x6;
    x6 = x5 + x7;
    x5 -= x7;
    x7 = x8 + x3;
    x8 -= x3;
    x3 = x0 + x2;
    x0 -= x2;
    x2 = (wmul(181, x4 + x5) + 128) >> 8;  // (32-bit: as in idct_col)
    x4 = (wmul(181, x4 - x5) + 128) >> 8;
    auto cl = [](int32_t x) { return min(max((x >> 14) + 128, 0), 255); };
    o[0] = cl(x7 + x1);
    o[1] = cl(x3 + x2);
    o[2] = cl(x0 + x4);
    o[3] = cl(x8 + x6);
    o[4] = cl(x8 - x6);
    o[5] = cl(x0 - x4);
    o[6] = cl(x3 - x2);
    o[7] = cl(x7 - x1);
}
// idct_col_full before its clip: o[r] = the value whose clip8(o >> 14) is the pixel, the +128
// level shift folded into x0's rounding constant (every output holds x0's constant exactly once:
// (x >> 14) + 128 == (x + (128 << 14)) >> 14), so sat4<14> packs four of them with the clip.
__device__ __forceinline__ void idct_col_raw(const int32_t (&v)[8], int32_t (&o)[8]) {
    int32_t x0 = (v[0] << 8) + 8192 + (128 << 14), x1 = v[4] << 8, x2 = v[6], x3 = v[2];
    int32_t x4 = v[1], x5 = v[7], x6 = v[5], x7 = v[3], x8;
    x8 = m24(kW7, x4 + x5) + 4;
    x4 = (x8 + m24(kW1 - kW7, x4)) >> 3;
    x5 = (x8 - m24(kW1 + kW7, x5)) >> 3;
    x8 = m24(kW3, x6 + x7) + 4;
    x6 = (x8 - m24(kW3 - kW5, x6)) >> 3;
    x7 = (x8 - m24(kW3 + kW5, x7)) >> 3;
    x8 = x0 + x1;
    x0 -= x1;
    x1 = m24(kW6, x3 + x2) + 4;
    x2 = (x1 - m24(kW2 + kW6, x2)) >> 3;
    x3 = (x1 + m24(kW2 - kW6, x3)) >> 3;
    x1 = x4 + x6;
    x4 -= x6;
    x6 = x5 + x7;
    x5 -= x7;
    x7 = x8 + x3;
    x8 -= x3;
    x3 = x0 + x2;
    x0 -= x2;
    x2 = (wmul(181, x4 + x5) + 128) >> 8;  // (32-bit: as in idct_col)
    x4 = (wmul(181, x4 - x5) + 128) >> 8;
    o[0] = x7 + x1;
    o[1] = x3 + x2;
    o[2] = x0 + x4;
    o[3] = x8 + x6;
    o[4] = x8 - x6;
    o[5] = x0 - x4;
    o[6] = x3 - x2;
    o[7] = x7 - x1;
}
__device__ __forceinline__ int32_t pair_swap(int32_t x) {  // the other lane of the pair (DPP quad_perm [1,0,3,2])
    return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ bool fused420(const Desc& d);  // (k_fused420 below)

// The main IDCT kernel, for MCUs of up to kIdctUnitBlocks blocks (every sampling but the
// exotic 8x-subsampled ones). A wave's unit of work is kUM horizontally adjacent MCUs of one MCU
// row (kUM = the largest power of two with kUM * bpm <= 64: 8 MCUs = 48 blocks at 4:2:0). Its
// blocks are transformed an octet at a time as in k_idct_any, but the pixel tiles land in the
// wave's LDS copy of the unit's plane rectangles; the wave then writes those rectangles row by
// row with 8-byte stores of consecutive lanes (128-byte luma rows at 4:2:0) instead of one
// 8-byte piece per block row: the scattered pieces cost 2x their bytes in HBM writes (PMC).
struct IdctComp {
    int64_t off;
    int32_t stride, mx, my, cpr;  // plane stride, MCU pitch (px), 8-byte chunks per unit row
};
__global__ __launch_bounds__(256) void k_idct(const Desc* __restrict__ desc, const int16_t* __restrict__ ac,
                                              const int32_t* __restrict__ dcv, const uint2* __restrict__ map,
                                              uint8_t* __restrict__ planes, int64_t plane_cap, int fuse) {
    const int img = blockIdx.y;
    const Desc& d = desc[img];
    // (bpm is 0 for a descriptor without a frame header: nothing to transform)
    if (d.status != kOk || d.bpm <= 0 || d.bpm > kIdctUnitBlocks || (fuse && fused420(d))) return;
    __shared__ int32_t qn[3][64];                // natural-order dequant table per component
    __shared__ uint32_t bgeo[kIdctUnitBlocks];   // unit block q -> ci | LDS offset of its tile << 2
    __shared__ IdctComp cg[3];
    __shared__ int32_t roff[4];                  // LDS offset of each component's rectangle
    // per wave: row-pass output (padded); the octet's blocks as stored (zig-zag) share its space:
    // they are read before the row pass writes (a wave's LDS accesses complete in order), and
    // the 4 KB saved fits six workgroups per CU (6 waves/SIMD) instead of five
    __shared__ __attribute__((aligned(16))) int32_t rows[4][8][8][9];
    __shared__ uint2 pixu[4][kIdctUnitBlocks * 8];  // per wave: the unit's pixels (64 B per block)
    const int t = threadIdx.x;
    const int bpm = d.bpm, mbw = d.mbw, nc = d.nc;
    int kum = 1;
    while (kum * 2 * bpm <= kIdctUnitBlocks) kum *= 2;
    if (t < 3 * 64) {
        const int ci = t >> 6, n = t & 63;
        qn[ci][n] = ci < nc ? d.q[d.c[ci].tq][kZigOfNat[n]] : 0;
    }
    if (t < 3) {
        const int ci = t < nc ? t : 0;
        const Comp& c = d.c[ci];
        cg[t] = IdctComp{comp_plane_off(d, ci), c.stride, c.hs * 8, c.vs * 8, kum * c.hs};
    }
    if (t == 0) {  // rectangles: component c is (kum * 8 hs) x (8 vs) bytes
        int o = 0;
        for (int ci = 0; ci < 3; ++ci) {
            roff[ci] = o;
            if (ci < nc) o += kum * d.c[ci].hs * 8 * d.c[ci].vs * 8;
        }
        roff[3] = o;
    }
    __syncthreads();
    if (t < kum * bpm) {
        const int m = t / bpm, k = t - m * bpm;
        int sbx, sby;
        const int ci = mcu_block_comp(d, k, sbx, sby);
        const int wc = kum * d.c[ci].hs * 8;
        bgeo[t] = (uint32_t)ci | (uint32_t)(roff[ci] + sby * 8 * wc + m * d.c[ci].hs * 8 + sbx * 8) << 2;
    }
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63, lb = lane >> 3, r = lane & 7;
    uint32_t zo[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) zo[j] = 2u * kZigOfNat[r * 8 + j];
    static_assert(sizeof(rows[0]) % 16 == 0 && sizeof(rows[0]) >= sizeof(int4) * 64, "zig-zag stage fits");
    int4* zzw = reinterpret_cast<int4*>(&rows[wave][0][0][0]);  // this wave's [8][8] stage
    const uint8_t* zrow = reinterpret_cast<const uint8_t*>(zzw + lb * 8);
    uint8_t* pb = reinterpret_cast<uint8_t*>(&pixu[wave][0]);
    uint8_t* P = planes + (int64_t)img * plane_cap;
    const uint32_t ucols = (uint32_t)((mbw + kum - 1) / kum), nunits = ucols * (uint32_t)d.mbh;
    const uint32_t chunk0 = (gridDim.x & 7) ? blockIdx.x : (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    const uint32_t wid = chunk0 * 4 + wave, nw = gridDim.x * 4;
    for (uint32_t u = wid; u < nunits; u += nw) {
        const uint32_t mby = u / ucols, mbx0 = (u - mby * ucols) * (uint32_t)kum;
        const int cnt = min(kum, mbw - (int)mbx0);            // MCUs in this unit
        const int nb = cnt * bpm, noct = (nb + 7) >> 3;        // blocks, octets
        const uint32_t b0 = ((uint32_t)mby * (uint32_t)mbw + mbx0) * (uint32_t)bpm;  // first block
        for (int o0 = 0; o0 < noct; o0 += kIdctU) {
            int4 c[kIdctU];
            BlkLoc loc[kIdctU];
#pragma unroll
            for (int k = 0; k < kIdctU; ++k) {
                const int q = (o0 + k) * 8 + lb;
                loc[k] = blk_loc(d, map, b0 + (q < nb ? q : 0));
                c[k] = q < nb ? *reinterpret_cast<const int4*>(ac + loc[k].blk * 64 + r * 8) : make_int4(0, 0, 0, 0);
            }
#pragma unroll
            for (int k = 0; k < kIdctU; ++k) {
                if (o0 + k >= noct) break;  // wave-uniform
                const int q = (o0 + k) * 8 + lb;
                const bool live = q < nb;
                zzw[lb * 8 + r] = c[k];
                __builtin_amdgcn_wave_barrier();
                const uint32_t bg = bgeo[live ? q : 0];
                const int ci = (int)(bg & 3);
                int16_t s[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) s[j] = *reinterpret_cast<const int16_t*>(zrow + zo[j]);
                int32_t v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = m24(s[j], qn[ci][r * 8 + j]);  // int16 x 8-bit: exact
                if (r == 0 && live) v[0] = wmul(blk_dc(s[0], dcv, loc[k]), qn[ci][0]);  // absolute DC (pool cell + offset)
                if (idct_fast_ok(v)) idct_row<true>(v);
                else idct_row<false>(v);
#pragma unroll
                for (int j = 0; j < 8; ++j) rows[wave][lb][r][j] = v[j];
                __builtin_amdgcn_wave_barrier();
                int32_t col[8];
                uint8_t ob[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) col[j] = rows[wave][lb][j][r];
                if (idct_fast_ok(col)) idct_col<true>(col, ob);
                else idct_col<false>(col, ob);
                if (live) {
                    const int wc = cg[ci].cpr * 8;
                    uint8_t* dst = pb + (bg >> 2) + r;
#pragma unroll
                    for (int j = 0; j < 8; ++j) dst[j * wc] = ob[j];
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
        // the unit's rectangles -> planes: consecutive lanes store consecutive 8-byte chunks
        for (int ci = 0; ci < nc; ++ci) {
            const IdctComp g = cg[ci];
            const int cpr = cnt * (g.mx >> 3);  // live chunks per row (partial unit at a row end)
            const int total = cpr * g.my;
            uint8_t* base = P + g.off + (int64_t)mby * g.my * g.stride + (int64_t)mbx0 * g.mx;
            const uint2* src = &pixu[wave][roff[ci] >> 3];
            for (int i = lane; i < total; i += 64) {
                const int row = i / cpr, col = i - row * cpr;
                *reinterpret_cast<uint2*>(base + (int64_t)row * g.stride + col * 8) = src[row * g.cpr + col];
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ----------------------------------------------------------------------------- upsample
// The doubling program of one component: njConvert's loop (jpeg_dec.h:822-827).
struct Plane {
    const uint8_t* p;
    int w, h, stride;
};
__device__ __forceinline__ int comp_program(const Desc& d, int ci, uint8_t (&ops)[6]) {
    int w = d.c[ci].w, h = d.c[ci].h, n = 0;
    while ((w < d.W || h < d.H) && n < 6) {
        if (w < d.W) { ops[n++] = 'H'; w <<= 1; }
        if (h < d.H && n < 6) { ops[n++] = 'V'; h <<= 1; }
    }
    return n;
}
// Buffer holding the output of pass p (p < 0: the IDCT plane) of component ci.
__device__ __forceinline__ Plane pass_plane(const Desc& d, int ci, int p, const uint8_t* plane_slot,
                                            const uint8_t* tmp_slot, int64_t tmp_cap, const uint8_t (&ops)[6]) {
    const Comp& c = d.c[ci];
    Plane pl{plane_slot + comp_plane_off(d, ci), c.w, c.h, c.stride};
    for (int k = 0; k <= p; ++k) {
        if (ops[k] == 'H') pl.w <<= 1; else pl.h <<= 1;
        pl.stride = pl.w;
        pl.p = tmp_slot + ((int64_t)ci * 2 + (k & 1)) * tmp_cap;
    }
    return pl;
}

__device__ __forceinline__ bool fused_ok(const Desc& d);
__device__ __forceinline__ int stream_kind(const Desc& d);
// grid: (x: pixel tiles, y: slot*3 + comp). Pass `p` of every component that has one.
__global__ __launch_bounds__(256) void k_upsample(const Desc* __restrict__ desc, const uint8_t* __restrict__ planes,
                                                  uint8_t* __restrict__ tmp, int64_t plane_cap, int64_t tmp_cap, int p) {
    const int img = blockIdx.y / 3, ci = blockIdx.y % 3;
    const Desc& d = desc[img];
    if (d.status != kOk || ci >= d.nc || fused_ok(d)) return;
    uint8_t ops[6];
    const int nops = comp_program(d, ci, ops);
    if (p >= nops) return;
    const uint8_t* pslot = planes + (int64_t)img * plane_cap;
    uint8_t* tslot = tmp + (int64_t)img * 3 * 2 * tmp_cap;
    const Plane in = pass_plane(d, ci, p - 1, pslot, tslot, tmp_cap, ops);
    const Plane out = pass_plane(d, ci, p, pslot, tslot, tmp_cap, ops);
    uint8_t* o = const_cast<uint8_t*>(out.p);
    const int64_t total = (int64_t)out.w * out.h;
    for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
        const int y = (int)(idx / out.w), x = (int)(idx - (int64_t)y * out.w);
        uint8_t v;
        if (ops[p] == 'H') {
            const uint8_t* row = in.p + (int64_t)y * in.stride;
            v = double_tap(x, in.w, [&](int i) { return (int)row[i]; },
                           [&](int j) { return (int)row[in.stride - j]; });
        } else {
            const uint8_t* col = in.p + x;
            v = double_tap(y, in.h, [&](int i) { return (int)col[(int64_t)i * in.stride]; },
                           [&](int j) { return (int)col[(int64_t)(in.h - j) * in.stride]; });
        }
        o[idx] = v;
    }
}

// ------------------------------------------------------------------------------ convert
__global__ __launch_bounds__(256) void k_convert(const Desc* __restrict__ desc, const uint8_t* __restrict__ planes,
                                                 const uint8_t* __restrict__ tmp, int64_t plane_cap, int64_t tmp_cap,
                                                 uint8_t* __restrict__ out, uint64_t out_stride) {
    const int img = blockIdx.y;
    const Desc& d = desc[img];
    if (d.status != kOk || fused_ok(d)) return;
    const uint8_t* pslot = planes + (int64_t)img * plane_cap;
    const uint8_t* tslot = tmp + (int64_t)img * 3 * 2 * tmp_cap;
    Plane pl[3];
    for (int ci = 0; ci < d.nc; ++ci) {
        uint8_t ops[6];
        const int nops = comp_program(d, ci, ops);
        pl[ci] = pass_plane(d, ci, nops - 1, pslot, tslot, tmp_cap, ops);
    }
    uint8_t* o = out + (int64_t)img * out_stride;
    const int64_t total = (int64_t)d.W * d.H;
    for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
        const int y = (int)(idx / d.W), x = (int)(idx - (int64_t)y * d.W);
        if (d.nc == 3) {
            ycc_to_rgb(pl[0].p[(int64_t)y * pl[0].stride + x], pl[1].p[(int64_t)y * pl[1].stride + x],
                       pl[2].p[(int64_t)y * pl[2].stride + x], o + idx * 3);
        } else {
            o[idx] = pl[0].p[(int64_t)y * pl[0].stride + x];
        }
    }
}

// ------------------------------------------------------------- fused upsample + convert
// For the samplings that need at most one doubling per direction per chroma component
// (4:4:4, 4:2:2, 4:4:0, 4:2:0, ...) and an un-resampled luma plane, njConvert's H/V passes
// (jpeg_dec.h:736-791) and the YCbCr->RGB step (:834-853) are evaluated per 64x16 output
// tile straight from the IDCT planes: no intermediate planes, one RGB write per pixel.
// kind: bit 0 = horizontal doubling, bit 1 = vertical doubling, -1 = not covered.
__device__ __forceinline__ int fused_kind(const Desc& d, int ci) {
    uint8_t ops[6];
    const int n = comp_program(d, ci, ops);
    if (n == 0) return 0;
    if (n == 1) return ops[0] == 'H' ? 1 : 2;
    if (n == 2 && ops[0] == 'H' && ops[1] == 'V') return 3;
    return -1;
}
__device__ __forceinline__ bool fused_ok(const Desc& d) {
    if (d.nc == 1) return true;
    if (d.nc != 3 || fused_kind(d, 0) != 0) return false;
    return fused_kind(d, 1) >= 0 && fused_kind(d, 2) >= 0;
}

// Horizontal doubling of row r of a plane (w real samples, stride s; right edge from the
// stride end, jpeg_dec.h:752-756), output column x.
__device__ __forceinline__ int hval(const uint8_t* P, int w, int s, int r, int x) {
    const uint8_t* row = P + (int64_t)r * s;
    return double_tap(x, w, [&](int i) { return (int)row[i]; }, [&](int j) { return (int)row[s - j]; });
}

constexpr int kTW = 64, kTH = 16, kHR = 12, kCW = 40;  // tile, staged H rows, staged chroma cols

// Interior 4-tap doubling (jpeg_dec.h:749-750) of samples a..e at output parity odd/even.
__device__ __forceinline__ int tap_mid(int o, int a, int b, int c, int e) {
    return (o & 1) ? tap4(a, b, c, e) : tap4(e, c, b, a);
}

__global__ __launch_bounds__(256) void k_convert_fused(const Desc* __restrict__ desc, const uint8_t* __restrict__ planes,
                                                       int64_t plane_cap, uint8_t* __restrict__ out, uint64_t out_stride) {
    const int img = blockIdx.y;
    const Desc& d = desc[img];
    if (d.status != kOk || !fused_ok(d) || stream_kind(d) >= 0) return;
    __shared__ uint8_t sC[2][kHR][kCW];      // raw chroma window
    __shared__ uint8_t sH[2][kHR][kTW];      // horizontally doubled chroma rows
    __shared__ uint32_t sRGB[kTH][kTW * 3 / 4];
    const uint8_t* pslot = planes + (int64_t)img * plane_cap;
    uint8_t* o = out + (int64_t)img * out_stride;
    const int W = d.W, H = d.H, t = threadIdx.x;
    const uint8_t* P0 = pslot;
    const int s0 = d.c[0].stride;
    const int ntx = (W + kTW - 1) / kTW, nty = (H + kTH - 1) / kTH;
    const int ntiles = ntx * nty;
    const uint8_t* P[3] = {P0, P0 + comp_plane_off(d, 1), P0 + comp_plane_off(d, 2)};
    const int kind[2] = {fused_kind(d, 1), fused_kind(d, 2)};
    // dword stores need 4-byte aligned rows: the row pitch and the image base (out_stride may be odd)
    const bool aligned_out = ((W * 3) & 3) == 0 && (reinterpret_cast<uintptr_t>(o) & 3) == 0;
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int ty = tile / ntx, tx = tile - ty * ntx;
        const int X0 = tx * kTW, Y0 = ty * kTH;
        const int R0 = max(0, (Y0 >> 1) - 2), CX0 = max(0, (X0 >> 1) - 2);
        // 1) raw chroma window + 2) horizontally doubled rows, for components doubled both ways
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if (kind[c] != 3) continue;
            const Comp& cc = d.c[c + 1];
            const uint8_t* C = P[c + 1];
            const int R1 = min(cc.h - 1, (Y0 >> 1) + 9);
            for (int k = t; k < kHR * kCW; k += 256) {
                const int rr = k / kCW, xx = k - rr * kCW;
                const int r = R0 + rr, x = CX0 + xx;
                if (r <= R1 && x < cc.stride) sC[c][rr][xx] = C[r * cc.stride + x];
            }
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if (kind[c] != 3) continue;
            const Comp& cc = d.c[c + 1];
            const uint8_t* C = P[c + 1];
            const int R1 = min(cc.h - 1, (Y0 >> 1) + 9), n2 = cc.w << 1;
            for (int k = t; k < kHR * kTW; k += 256) {
                const int rr = k / kTW, xx = k - rr * kTW;
                const int r = R0 + rr, x = X0 + xx;
                if (r > R1 || x >= W) continue;
                int v;
                if (x >= 3 && x < n2 - 3) {
                    const int q = ((x - 3) >> 1) - CX0;
                    v = tap_mid(x, sC[c][rr][q], sC[c][rr][q + 1], sC[c][rr][q + 2], sC[c][rr][q + 3]);
                } else {
                    v = hval(C, cc.w, cc.stride, r, x);  // image edges (stride-end right taps)
                }
                sH[c][rr][xx] = (uint8_t)v;
            }
        }
        __syncthreads();
        // 3) per pixel: vertical doubling from sH (or the single-direction forms), YCbCr->RGB
        {
            const int ly = t >> 4, lx0 = (t & 15) * 4, y = Y0 + ly;
            uint8_t rgb[12];
            if (y < H) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int lx = lx0 + q, x = X0 + lx;
                    if (x >= W) break;
                    int ch[2];
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const Comp& cc = d.c[c + 1];
                        const uint8_t* C = P[c + 1];
                        int v;
                        if (kind[c] == 3) {
                            const int h2 = cc.h << 1;
                            if (y >= 3 && y < h2 - 3) {
                                const int rr = ((y - 3) >> 1) - R0;
                                v = tap_mid(y, sH[c][rr][lx], sH[c][rr + 1][lx], sH[c][rr + 2][lx], sH[c][rr + 3][lx]);
                            } else {
                                v = double_tap(y, cc.h, [&](int i) { return (int)sH[c][i - R0][lx]; },
                                               [&](int j) { return (int)sH[c][cc.h - j - R0][lx]; });
                            }
                        } else if (kind[c] == 0) {
                            v = C[y * cc.stride + x];
                        } else if (kind[c] == 1) {
                            v = hval(C, cc.w, cc.stride, y, x);
                        } else {  // vertical only: the component's own stride (jpeg_dec.h:765)
                            v = double_tap(y, cc.h, [&](int i) { return (int)C[i * cc.stride + x]; },
                                           [&](int j) { return (int)C[(cc.h - j) * cc.stride + x]; });
                        }
                        ch[c] = v;
                    }
                    ycc_to_rgb(P0[y * s0 + x], ch[0], ch[1], &rgb[3 * q]);
                }
                uint8_t* srow = reinterpret_cast<uint8_t*>(&sRGB[ly][0]);
#pragma unroll
                for (int k = 0; k < 12; ++k) srow[lx0 * 3 + k] = rgb[k];
            }
        }
        __syncthreads();
        const int wpx = min(kTW, W - X0), rowb = wpx * 3;
        if (aligned_out && rowb == kTW * 3) {  // full tile row, 4-byte aligned: dword stores
            for (int k = t; k < kTH * kTW * 3 / 4; k += 256) {
                const int ly = k / (kTW * 3 / 4), wd = k - ly * (kTW * 3 / 4);
                const int y = Y0 + ly;
                if (y < H) reinterpret_cast<uint32_t*>(o + ((int64_t)y * W + X0) * 3)[wd] = sRGB[ly][wd];
            }
        } else {
            for (int k = t; k < kTH * kTW * 3; k += 256) {
                const int ly = k / (kTW * 3), bx = k - ly * (kTW * 3);
                const int y = Y0 + ly;
                if (y < H && bx < rowb)
                    o[((int64_t)y * W + X0) * 3 + bx] = reinterpret_cast<const uint8_t*>(&sRGB[ly][0])[bx];
            }
        }
        __syncthreads();
    }
}


// Wave index as a wave-uniform (SGPR) value: threadIdx.x >> 6 is uniform per wave, but the
// compiler's divergence analysis cannot see it, so loops and branches on values derived from it
// were compiled as divergent -- loads under exec masks, and an s_waitcnt vmcnt(0) at every join.
__device__ __forceinline__ int wave_index() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

// ------------------------------------------------------------ streaming upsample + convert
// The common layouts -- gray, and 3 components whose luma is full size and whose two chroma
// components take the same doubling program (4:4:4, 4:2:2, 4:4:0, 4:2:0) -- are converted by
// register streaming: one wave owns a 256-pixel-wide, kSH-row strip, each lane owns 4 adjacent
// columns and walks down the strip. Horizontally doubled chroma rows (jpeg_dec.h:736-760) are
// made from two dword loads per row; the vertical pass (:762-791) slides a 5-row window held in
// registers; YCbCr->RGB (:834-853) is stored as one 12-byte write per lane. No LDS, no barriers.
// Vertical edge rows are wave-uniform branches; horizontal edge lanes take the generic taps.
#ifndef ICX_KSH
#define ICX_KSH 64
#endif
constexpr int kSH = ICX_KSH;
// rows (row pairs) whose loads are in flight ahead of the one being converted: one row pair per
// wave left ~30 KB of loads in flight per CU, below what the HBM latency needs
#ifndef ICX_CONV_PD
#define ICX_CONV_PD 2
#endif
constexpr int kPD = ICX_CONV_PD;

// 4 = gray; 0..3 = the shared chroma kind; -1 = left to k_convert_fused / the generic passes.
__device__ __forceinline__ int stream_kind(const Desc& d) {
    if (d.nc == 1) return 4;
    if (d.nc != 3 || fused_kind(d, 0) != 0) return -1;
    const int k = fused_kind(d, 1);
    if (k < 0 || fused_kind(d, 2) != k) return -1;
    if ((k & 1) && min(d.c[1].w, d.c[2].w) < 4) return -1;
    if ((k & 2) && min(d.c[1].h, d.c[2].h) < 4) return -1;
    return k;
}

struct CPl {
    const uint8_t* p;
    int w, h, s;
};
// Timing experiment ICX_NT_BACK (bit 0: plane and coefficient loads, bit 1: IDCT plane stores)
// marked non-temporal (streamed past L2, so the other pipeline's entropy lanes keep their U lines).
#ifndef ICX_NT_BACK
#define ICX_NT_BACK 0
#endif
template <class T>
__device__ __forceinline__ T nt_ld(const T* p) {
#if ICX_NT_BACK & 1
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
template <class T>
__device__ __forceinline__ void nt_st(T v, T* p) {
#if ICX_NT_BACK & 2
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}
__device__ __forceinline__ int4 nt_ld(const int4* p) {
#if ICX_NT_BACK & 1
    typedef int v4i __attribute__((ext_vector_type(4)));
    const v4i v = __builtin_nontemporal_load(reinterpret_cast<const v4i*>(p));
    return int4{v.x, v.y, v.z, v.w};
#else
    return *p;
#endif
}
__device__ __forceinline__ uint32_t ld4(const uint8_t* p) { return nt_ld(reinterpret_cast<const uint32_t*>(p)); }
__device__ __forceinline__ int bt(uint32_t v, int i) { return (v >> (8 * i)) & 255; }
// Packs four 0..255 values with v_perm_b32. (A shift/or pack of clamped taps lets the compiler
// form gfx950's v_ashr_pk_u8_i32, whose result's upper half was observed to leak into the
// neighbouring bytes; the explicit byte permutes avoid that pattern.)
__device__ __forceinline__ uint32_t pack4(uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3) {
    const uint32_t lo = __builtin_amdgcn_perm(t1, t0, 0x0c0c0400u);
    const uint32_t hi = __builtin_amdgcn_perm(t3, t2, 0x0c0c0400u);
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}
template <class F>
__device__ __forceinline__ uint32_t pmap(F f) {
    return pack4((uint32_t)f(0), (uint32_t)f(1), (uint32_t)f(2), (uint32_t)f(3));
}

// Chroma samples for output columns 4M..4M+3 of real row r: the horizontally doubled row when
// KH, else the raw samples. `fast` = all four outputs use interior taps and stay inside the row.
// Split into the loads (chroma_fetch, issued one row pair ahead) and the taps (chroma_make).
struct CRaw {
    uint32_t d0, d1;
};
// (The loads are unconditional -- edge lanes read the row start and ignore it: a load under a
// per-lane branch gets an s_waitcnt vmcnt(0) at the join, which serialised every row fetch.)
template <bool KH>
__device__ __forceinline__ CRaw chroma_fetch(const CPl& c, int r, int M, bool fast) {
    const uint8_t* row = c.p + (int64_t)r * c.s;  // (uniform row base + 32-bit lane offset, as put3)
    if (!KH) return CRaw{ld4(row + (uint32_t)(4 * M)), 0u};
    const uint32_t base = fast ? (uint32_t)((2 * M - 2) & ~3) : 0u;  // edge lanes load inside chroma_make
    return CRaw{ld4(row + base), ld4(row + (base + 4))};
}
// The 4-tap kernel as one v_dot4 on four packed samples: samples are biased to int8 (x ^ 0x80
// = x - 128) and, since the taps sum to 128, sum(k*x) + 64 = dot(k, x - 128) + 128*128 + 64.
// kTapFwd weighs bytes (s0..s3) as tap4(s0, s1, s2, s3); kTapRev as tap4(s3, s2, s1, s0).
constexpr uint32_t kBias8 = 0x80808080u;
constexpr int32_t kTapFwd = (int32_t)((uint32_t)(uint8_t)-9 | (111u << 8) | (29u << 16) | ((uint32_t)(uint8_t)-3 << 24));
constexpr int32_t kTapRev = (int32_t)((uint32_t)(uint8_t)-3 | (29u << 8) | (111u << 16) | ((uint32_t)(uint8_t)-9 << 24));
// The VOP3P dot products, whose accumulator is a source operand. The builtins compile to the
// VOP2 v_dot4c_i32_i8 / v_dot2c_i32_i16, whose accumulator is the destination, so every dot with
// a constant bias spent a v_mov re-loading it: a quarter of each tap, 3 VALU per converted pixel.
// (The weights -- wave-uniform constants -- in an SGPR, the one a VOP3 may read; the biases in
// VGPRs. Both are loop-invariant, so they are set up once.)
__device__ __forceinline__ int32_t dot4_i8(uint32_t a, int32_t b, int32_t acc) {
    int32_t r;
    asm("v_dot4_i32_i8 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(acc));
    return r;
}
__device__ __forceinline__ int32_t dot2_i16(uint32_t a, uint32_t b, int32_t acc) {
    int32_t r;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(acc));
    return r;
}
__device__ __forceinline__ uint32_t dtap(uint32_t biased, int32_t k) {
    const int32_t v = dot4_i8(biased, k, 128 * 128 + 64) >> 7;
    return (uint32_t)min(max(v, 0), 255);
}
// Four clipped bytes in one dword from four int32 values: byte i = clip8(v_i >> SH), by gfx950's
// v_ashr_pk_u8_i32 (D[7:0] = sat_u8(S0 >> S2), D[15:8] = sat_u8(S1 >> S2)). It writes only the
// low half of D and keeps the high half, and with op_sel:[0,0,0,1] writes the high half and keeps
// the low one (tools/probe/ashr_pk.hip, measured on the box) -- the kept half is why the compiler's
// own use of it had leaked bytes. Two instructions per dword replace four shifts,
// four clamps and three byte permutes.
template <int SH>
__device__ __forceinline__ uint32_t sat4(int32_t v0, int32_t v1, int32_t v2, int32_t v3) {
    uint32_t r;
    asm("v_ashr_pk_u8_i32 %0, %1, %2, %5\n\tv_ashr_pk_u8_i32 %0, %3, %4, %5 op_sel:[0,0,0,1]"
        : "=&v"(r) : "v"(v0), "v"(v1), "v"(v2), "v"(v3), "i"(SH));
    return r;
}
// dtap before its shift and clip: the biased dot (sat4<7> finishes it)
__device__ __forceinline__ int32_t dtap_raw(uint32_t biased, int32_t k) { return dot4_i8(biased, k, 128 * 128 + 64); }

template <bool KH>
__device__ __forceinline__ uint32_t chroma_make(const CPl& c, int r, int M, bool fast, const CRaw& raw) {
    if (!KH) return raw.d0;
    if (fast) {
        const uint64_t w = ((uint64_t)raw.d0 | ((uint64_t)raw.d1 << 32)) ^ 0x8080808080808080ull;
        const uint64_t b = w >> ((M & 1) ? 0 : 16);  // bytes b0..b5 = samples 2M-2 .. 2M+3 (biased)
        const uint32_t w0 = (uint32_t)b, w1 = (uint32_t)(b >> 8), w2 = (uint32_t)(b >> 16);
        // tap4(b3,b2,b1,b0), tap4(b1,b2,b3,b4), tap4(b4,b3,b2,b1), tap4(b2,b3,b4,b5)
        return sat4<7>(dtap_raw(w0, kTapRev), dtap_raw(w1, kTapFwd), dtap_raw(w1, kTapRev), dtap_raw(w2, kTapFwd));
    }
    const uint8_t* row = c.p + (int64_t)r * c.s;
    const int n2 = c.w << 1, s = c.s;
    return pmap([&](int i) {
        const int x = 4 * M + i;
        if (x >= n2) return 0;
        return (int)double_tap(x, c.w, [&](int k) { return (int)row[k]; }, [&](int j) { return (int)row[s - j]; });
    });
}
template <bool KH>
__device__ __forceinline__ uint32_t chroma_row(const CPl& c, int r, int M, bool fast) {
    return chroma_make<KH>(c, r, M, fast, chroma_fetch<KH>(c, r, M, fast));
}

// Vertical doubling at output rows 2k (even) / 2k+1 (odd) from the window w0..w4 = doubled
// rows k-2..k+2 (h >= 4 real rows; the order of the edge cases follows double_tap).
__device__ __forceinline__ uint32_t vtap_even(int k, int h, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
    if (k == 0) return pmap([&](int i) { return tap2(bt(w2, i), bt(w3, i)); });
    if (k == 1) return pmap([&](int i) { return tap3a(bt(w1, i), bt(w2, i), bt(w3, i)); });
    if (k == h - 1) return pmap([&](int i) { return tap3x(bt(w2, i), bt(w1, i), bt(w0, i)); });
    return pmap([&](int i) { return tap4(bt(w3, i), bt(w2, i), bt(w1, i), bt(w0, i)); });
}
__device__ __forceinline__ uint32_t vtap_odd(int k, int h, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t w4) {
    if (k == 0) return pmap([&](int i) { return tap3x(bt(w2, i), bt(w3, i), bt(w4, i)); });
    if (k == h - 2) return pmap([&](int i) { return tap3a(bt(w3, i), bt(w2, i), bt(w1, i)); });
    if (k == h - 1) return pmap([&](int i) { return tap2(bt(w2, i), bt(w1, i)); });
    return pmap([&](int i) { return tap4(bt(w1, i), bt(w2, i), bt(w3, i), bt(w4, i)); });
}

// YCbCr -> RGB of a lane's 4 pixels (jpeg_dec.h:834-853, ycc_to_rgb) as three dwords of packed
// RGB. Each channel is one or two v_dot2 on 16-bit pairs: (Y, cb) and (Y, cr) per pixel, with
// the -128 offsets folded into the constant, e.g. R = 256*Y + 359*cr + (128 - 359*128) =
// (Y << 8) + 359*(cr - 128) + 128; sat4<8> takes clip8(numerator >> 8) of four of them at once.
typedef short icx_short2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ icx_short2 as_s2(uint32_t v) { return __builtin_bit_cast(icx_short2, v); }
__device__ __forceinline__ void ycc4_to_rgb(uint32_t yv, uint32_t cb, uint32_t cr, uint32_t (&w)[3]) {
    // (Y, c) weight pairs as packed int16: (256, 359), (256, -88), (0, -183), (256, 454)
    constexpr uint32_t kR = 256u | (359u << 16), kG1 = 256u | ((uint32_t)(uint16_t)-88 << 16),
                       kG2 = (uint32_t)(uint16_t)-183 << 16, kB = 256u | (454u << 16);
    int32_t R[4], G[4], B[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t sel = (uint32_t)i | (0x0cu << 8) | ((uint32_t)(4 + i) << 16) | (0x0cu << 24);
        const uint32_t yb = __builtin_amdgcn_perm(cb, yv, sel);  // (Y_i, cb_i)
        const uint32_t yr = __builtin_amdgcn_perm(cr, yv, sel);  // (Y_i, cr_i)
        R[i] = dot2_i16(yr, kR, 128 - 359 * 128);
        G[i] = dot2_i16(yr, kG2, dot2_i16(yb, kG1, 128 + (88 + 183) * 128));
        B[i] = dot2_i16(yb, kB, 128 - 454 * 128);
    }
    // [R0 G0 B0 R1] [G1 B1 R2 G2] [B2 R3 G3 B3]
    w[0] = sat4<8>(R[0], G[0], B[0], R[1]);
    w[1] = sat4<8>(G[1], B[1], R[2], G[2]);
    w[2] = sat4<8>(B[2], R[3], G[3], B[3]);
}

struct StreamOut {
    uint8_t* o;
    int W;
    bool vec;  // rows 4-byte aligned
    __device__ __forceinline__ void put3(int y, int x0, const uint32_t (&w)[3], int nb) const {
        // row base (wave-uniform in k_convert_stream: SGPRs) + the lane's 32-bit offset, so the
        // store takes the SGPR-base form instead of a 64-bit multiply-add chain per row
        uint8_t* dst = o + (int64_t)y * W * 3 + (uint32_t)(x0 * 3);
        if (vec && nb == 12) {
            typedef uint32_t u32x3 __attribute__((ext_vector_type(3), aligned(4)));
            const u32x3 v = {w[0], w[1], w[2]};
            __builtin_nontemporal_store(v, reinterpret_cast<u32x3*>(dst));
        } else {
#pragma unroll
            for (int i = 0; i < 12; ++i)
                if (i < nb) dst[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
        }
    }
};

// Data of one row (or row pair): the chroma loads of both components and the luma dwords.
struct Pre {
    CRaw a, e;
    uint32_t y0, y1;
};
// Output rows [Y0, Y1) (Y0 even) of one lane's 4 columns (4M .. 4M+3) with vertical chroma
// doubling (KV layouts, jpeg_dec.h:762-791): a 5-row chroma window slides down in registers;
// luma(y) gives the lane's 4 luma samples of row y, emit(y, luma, cb, cr) converts and stores.
// The sliding chroma window of rows_kv (both components): rows k-2..k+1 of the next row pair
// k, and their biased column dwords (even-output taps).
struct KvWin {
    uint32_t a0, a1, a2, a3, e0, e1, e2, e3;
    uint32_t ca[4], ce[4];
};
__device__ __forceinline__ uint32_t kv_column(uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, int i) {
    const uint32_t sel = 0x0c0c0400u | (uint32_t)(i * 0x0101);  // byte i of the low operand, byte i of the high
    return __builtin_amdgcn_perm(r1, r0, sel) | (__builtin_amdgcn_perm(r3, r2, sel) << 16);
}
// Window for row pair k0: the first four rows, all eight rows' loads issued before any is used.
template <bool KH>
__device__ __forceinline__ void kv_init(KvWin& w, const CPl& c1, const CPl& c2, int M, bool f1, bool f2, int k0) {
    auto cr1 = [&](int r) { return min(max(r, 0), c1.h - 1); };
    auto cr2 = [&](int r) { return min(max(r, 0), c2.h - 1); };
    CRaw ra[4], re[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        ra[i] = chroma_fetch<KH>(c1, cr1(k0 - 2 + i), M, f1);
        re[i] = chroma_fetch<KH>(c2, cr2(k0 - 2 + i), M, f2);
    }
    w.a0 = chroma_make<KH>(c1, cr1(k0 - 2), M, f1, ra[0]);
    w.a1 = chroma_make<KH>(c1, cr1(k0 - 1), M, f1, ra[1]);
    w.a2 = chroma_make<KH>(c1, cr1(k0), M, f1, ra[2]);
    w.a3 = chroma_make<KH>(c1, cr1(k0 + 1), M, f1, ra[3]);
    w.e0 = chroma_make<KH>(c2, cr2(k0 - 2), M, f2, re[0]);
    w.e1 = chroma_make<KH>(c2, cr2(k0 - 1), M, f2, re[1]);
    w.e2 = chroma_make<KH>(c2, cr2(k0), M, f2, re[2]);
    w.e3 = chroma_make<KH>(c2, cr2(k0 + 1), M, f2, re[3]);
    // per output column i, a dword of the 4 window rows' samples (biased)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        w.ca[i] = kv_column(w.a0, w.a1, w.a2, w.a3, i) ^ kBias8;
        w.ce[i] = kv_column(w.e0, w.e1, w.e2, w.e3, i) ^ kBias8;
    }
}
// Output rows [Y0, Y1) (Y0 even) of one lane's 4 columns (4M .. 4M+3) with vertical chroma
// doubling (KV layouts, jpeg_dec.h:762-791), the window w set for row pair Y0 / 2 and left at
// row pair Y1 / 2: luma(y) gives the lane's 4 luma samples of row y, emit(y, luma, cb, cr)
// converts and stores.
template <bool KH, class LumaF, class EmitF>
__device__ __forceinline__ void kv_rows(KvWin& w, const CPl& c1, const CPl& c2, int M, bool f1, bool f2, int Y0, int Y1,
                                        LumaF luma, EmitF emit) {
    const int k0 = Y0 >> 1;
    auto cr1 = [&](int r) { return min(max(r, 0), c1.h - 1); };
    auto cr2 = [&](int r) { return min(max(r, 0), c2.h - 1); };
    // data of row pair k: chroma row k+2, luma rows 2k and 2k+1. Unconditional loads (rows past
    // the strip re-read its last row): a conditional fetch zero-initialised its registers, and
    // that write had to wait for every load in flight (vmcnt(0)).
    auto fetch = [&](int k) {
        Pre p;
        p.a = chroma_fetch<KH>(c1, cr1(k + 2), M, f1);
        p.e = chroma_fetch<KH>(c2, cr2(k + 2), M, f2);
        p.y0 = luma(min(2 * k, Y1 - 1));
        p.y1 = luma(min(2 * k + 1, Y1 - 1));
        return p;
    };
    // E = rows k-2..k+1 (even output 2k: kTapRev), O = rows k-1..k+2 (odd 2k+1: kTapFwd);
    // each row pair shifts one new row into the columns with one v_perm per column.
    auto vsteps = [&](int k, uint32_t (&cc)[4], uint32_t nrow, int h, uint32_t w0, uint32_t w1, uint32_t w2,
                      uint32_t w3, uint32_t& ev, uint32_t& od) {
        const uint32_t nb = nrow ^ kBias8;
        uint32_t oc[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)  // O = (E >> 8) | new row's byte i << 24
            oc[i] = __builtin_amdgcn_perm(nb, cc[i], 0x00030201u | ((uint32_t)(4 + i) << 24));
        if (k >= 2 && k <= h - 3) {  // both outputs interior (wave-uniform)
            ev = sat4<7>(dtap_raw(cc[0], kTapRev), dtap_raw(cc[1], kTapRev), dtap_raw(cc[2], kTapRev), dtap_raw(cc[3], kTapRev));
            od = sat4<7>(dtap_raw(oc[0], kTapFwd), dtap_raw(oc[1], kTapFwd), dtap_raw(oc[2], kTapFwd), dtap_raw(oc[3], kTapFwd));
        } else {
            ev = vtap_even(k, h, w0, w1, w2, w3);
            od = vtap_odd(k, h, w1, w2, w3, nrow);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) cc[i] = oc[i];
    };
    auto step = [&](int k, const Pre& p) {
        const uint32_t a4 = chroma_make<KH>(c1, cr1(k + 2), M, f1, p.a);
        const uint32_t e4 = chroma_make<KH>(c2, cr2(k + 2), M, f2, p.e);
        uint32_t ae, ao, ee, eo;
        vsteps(k, w.ca, a4, c1.h, w.a0, w.a1, w.a2, w.a3, ae, ao);
        vsteps(k, w.ce, e4, c2.h, w.e0, w.e1, w.e2, w.e3, ee, eo);
        emit(2 * k, p.y0, ae, ee);
        if (2 * k + 1 < Y1) emit(2 * k + 1, p.y1, ao, eo);
        w.a0 = w.a1; w.a1 = w.a2; w.a2 = w.a3; w.a3 = a4;
        w.e0 = w.e1; w.e1 = w.e2; w.e2 = w.e3; w.e3 = e4;
    };
    Pre B[kPD + 1];
#pragma unroll
    for (int u = 0; u < kPD; ++u) B[u] = fetch(k0 + u);
    for (int k = k0; 2 * k < Y1; k += kPD + 1) {
#pragma unroll
        for (int u = 0; u <= kPD; ++u) {
            if (2 * (k + u) >= Y1) break;  // wave-uniform
            B[(u + kPD) % (kPD + 1)] = fetch(k + u + kPD);
            step(k + u, B[u]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}
template <bool KH, class LumaF, class EmitF>
__device__ __forceinline__ void rows_kv(const CPl& c1, const CPl& c2, int M, bool f1, bool f2, int Y0, int Y1,
                                        LumaF luma, EmitF emit) {
    KvWin w;
    kv_init<KH>(w, c1, c2, M, f1, f2, Y0 >> 1);
    kv_rows<KH>(w, c1, c2, M, f1, f2, Y0, Y1, luma, emit);
}

// Chroma lanes whose horizontal taps leave the interior formulas (image border, stride-end
// reads): f = the lane's 4 doubled outputs use the interior 4-tap formula and read inside the row.
__device__ __forceinline__ bool interior_taps(const CPl& c, int M) {
    return M >= 1 && 4 * M + 3 <= 2 * c.w - 4 && 2 * M + 5 < c.s;
}
// First lane of the right border (lanes 0 and [edge_from, ceil(W/4)) are border lanes).
__device__ __forceinline__ int edge_from(const CPl& c1, const CPl& c2, int W) {
    auto lim = [](const CPl& c) { return min((2 * c.w - 7) >> 2, (c.s - 6) >> 1) + 1; };  // first M failing
    return max(1, min(min(lim(c1), lim(c2)), (W + 3) >> 2));
}
// One lane's columns 4M .. 4M+3, output rows [Y0, Y1) (Y0 even). The main kernel passes
// f1 = f2 = true (constants: the border taps compile out of its loop); k_convert_edge passes the
// real flags for the border lanes. A lane that is not `live` runs along (with an in-range M) and
// stores nothing, so the wave's loop has no per-lane exit.
template <int K>
__device__ __forceinline__ void lane_strip(const CPl& c1, const CPl& c2, const uint8_t* P0, int s0, int W,
                                           const StreamOut& so, int M, bool f1, bool f2, int Y0, int Y1,
                                           bool live = true) {
    constexpr bool KH = (K & 1) != 0, KV = (K & 2) != 0;
    const int x0 = 4 * M;
    const int nb = live ? min(4, W - x0) * 3 : 0;
    auto emit = [&](int y, uint32_t yv, uint32_t cb, uint32_t cr) {
        uint32_t w[3];
        ycc4_to_rgb(yv, cb, cr, w);
        so.put3(y, x0, w, nb);
    };
    auto luma = [&](int y) { return ld4(P0 + (int64_t)y * s0 + (uint32_t)x0); };
    if (K == 4) {  // gray: stride removal (jpeg_dec.h:854-865)
#pragma unroll 4
        for (int y = Y0; y < Y1; ++y) {
            const uint32_t v = luma(y);
            uint8_t* dst = so.o + (int64_t)y * W + x0;
            if (so.vec && nb == 12) __builtin_nontemporal_store(v, reinterpret_cast<uint32_t*>(dst));
            else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (3 * i < nb) dst[i] = (uint8_t)bt(v, i);
            }
        }
        return;
    }
    // Software pipelining over a ring of kPD + 1 buffers, unrolled so every buffer index is a
    // constant: the loads of the next kPD rows (row pairs) are in flight while the current one
    // is computed; the scheduling barriers keep each buffer's reload after its last use so no
    // in-flight value is copied.
    if (!KV) {
        auto fetch = [&](int y) {  // unconditional (see kv_rows): rows past the strip re-read its last
            Pre p;
            const int yc = min(y, Y1 - 1);
            p.a = chroma_fetch<KH>(c1, yc, M, f1);
            p.e = chroma_fetch<KH>(c2, yc, M, f2);
            p.y0 = luma(yc);
            p.y1 = 0;
            return p;
        };
        auto step = [&](int y, const Pre& p) {
            emit(y, p.y0, chroma_make<KH>(c1, y, M, f1, p.a), chroma_make<KH>(c2, y, M, f2, p.e));
        };
        Pre B[kPD + 1];
#pragma unroll
        for (int u = 0; u < kPD; ++u) B[u] = fetch(Y0 + u);
        for (int y = Y0; y < Y1; y += kPD + 1) {
#pragma unroll
            for (int u = 0; u <= kPD; ++u) {
                if (y + u >= Y1) break;  // wave-uniform
                B[(u + kPD) % (kPD + 1)] = fetch(y + u + kPD);
                step(y + u, B[u]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        return;
    }
    rows_kv<KH>(c1, c2, M, f1, f2, Y0, Y1, luma, emit);
}

struct ConvImg {
    CPl c1, c2;
    const uint8_t* P0;
    int s0;
};
__device__ __forceinline__ ConvImg conv_img(const Desc& d, const uint8_t* pslot, int K) {
    ConvImg ci{};
    ci.P0 = pslot;
    ci.s0 = d.c[0].stride;
    if (K != 4) {
        ci.c1 = CPl{pslot + comp_plane_off(d, 1), d.c[1].w, d.c[1].h, d.c[1].stride};
        ci.c2 = CPl{pslot + comp_plane_off(d, 2), d.c[2].w, d.c[2].h, d.c[2].stride};
    }
    return ci;
}

template <int K>
__device__ __forceinline__ void stream_image(const Desc& d, const uint8_t* pslot, const StreamOut& so) {
    constexpr bool KH = (K & 1) != 0;
    const int W = d.W, H = d.H;
    const ConvImg ci = conv_img(d, pslot, K);
    const int lane = threadIdx.x & 63, wv = wave_index();
    const int nsx = (W + 255) >> 8, nsy = (H + kSH - 1) / kSH, nstrip = nsx * nsy;
    const int nl = (W + 3) >> 2;                      // lanes (4 columns each) of a row
    const int ef = KH ? edge_from(ci.c1, ci.c2, W) : nl;  // border lanes are k_convert_edge's
    const int m0 = KH ? 1 : 0;
    if (ef <= m0) return;  // every lane a border lane
    for (int strip = blockIdx.x * 4 + wv; strip < nstrip; strip += gridDim.x * 4) {  // wave-uniform
        const int sy = strip / nsx, sx = strip - sy * nsx;
        const int M = sx * 64 + lane;
        const bool live = M >= m0 && M < ef;
        lane_strip<K>(ci.c1, ci.c2, ci.P0, ci.s0, W, so, min(max(M, m0), ef - 1), true, true, sy * kSH,
                      min(H, sy * kSH + kSH), live);
    }
}

// The border lanes of the horizontally doubled layouts (4:2:2, 4:2:0): lane 0 and the lanes from
// edge_from on, with the generic taps (double_tap, stride-end reads). One thread per (lane,
// kSH-row strip); a wave's 64 threads all take the generic path, so it runs with full lanes
// instead of as a divergent tail inside k_convert_stream's waves (which cost it 4.2 of 14.6 ms).
#ifndef ICX_SHE
#define ICX_SHE 16
#endif
constexpr int kSHE = ICX_SHE;  // rows per edge item (even): short strips, so the few border lanes fill the chip
template <int K>
__global__ __launch_bounds__(256) void k_convert_edge(const Desc* __restrict__ desc, const uint8_t* __restrict__ planes,
                                                      int64_t plane_cap, uint8_t* __restrict__ out, uint64_t out_stride,
                                                      int fuse) {
    static_assert(K & 1, "horizontally doubled layouts only");
    const int img = blockIdx.y;
    const Desc& d = desc[img];
    if (d.status != kOk || stream_kind(d) != K || (K == 3 && (fuse == 1 || fuse == 3) && fused420(d))) return;
    const uint8_t* pslot = planes + (int64_t)img * plane_cap;
    uint8_t* o = out + (int64_t)img * out_stride;
    const StreamOut so{o, d.W, ((reinterpret_cast<uintptr_t>(o) & 3) == 0) && (d.W & 3) == 0};
    const int W = d.W, H = d.H;
    const ConvImg ci = conv_img(d, pslot, K);
    const int nl = (W + 3) >> 2, ef = edge_from(ci.c1, ci.c2, W);
    const int ne = 1 + max(0, nl - ef);  // lane 0, then lanes ef .. nl-1
    const int nsy = (H + kSHE - 1) / kSHE, items = ne * nsy;
    for (int it = blockIdx.x * blockDim.x + threadIdx.x; it < items; it += gridDim.x * blockDim.x) {
        const int sy = it / ne, e = it - sy * ne;
        const int M = e == 0 ? 0 : ef + e - 1;
        lane_strip<K>(ci.c1, ci.c2, ci.P0, ci.s0, W, so, M, interior_taps(ci.c1, M), interior_taps(ci.c2, M), sy * kSHE,
                      min(H, sy * kSHE + kSHE));
    }
}

// One instantiation per layout (K as in stream_kind), so each gets its own register allocation;
// every instantiation is launched and skips the images of other layouts.
#ifndef ICX_CONV_MINW  // (timing experiments: waves per SIMD k_convert_stream is compiled for)
#define ICX_CONV_MINW 1
#endif
template <int K>
__global__ __launch_bounds__(256, ICX_CONV_MINW) void k_convert_stream(const Desc* __restrict__ desc, const uint8_t* __restrict__ planes,
                                                        int64_t plane_cap, uint8_t* __restrict__ out, uint64_t out_stride,
                                                        int fuse) {
    const int img = blockIdx.y;
    const Desc& d = desc[img];
    if (d.status != kOk || stream_kind(d) != K || (K == 3 && (fuse == 1 || fuse == 3 || fuse == 5) && fused420(d))) return;
    const uint8_t* pslot = planes + (int64_t)img * plane_cap;
    uint8_t* o = out + (int64_t)img * out_stride;
    const StreamOut so{o, d.W, ((reinterpret_cast<uintptr_t>(o) & 3) == 0) && (d.W & 3) == 0};
    stream_image<K>(d, pslot, so);
}

// ---------------------------------------------------- 4:2:0 chroma IDCT + fused luma IDCT/convert
// The common 4:2:0 layout (Y 2x2, Cb and Cr 1x1 per MCU) skips k_idct and k_convert_stream<3>:
// k_idct420c writes the two chroma planes, then k_fused420 transforms each MCU row's luma
// blocks into LDS and converts those 16 rows from there -- the 16.8 MB luma plane per 4096^2
// image never goes through HBM. Both use the lane-pair IDCT; the conversion is rows_kv, the same
// code k_convert_stream runs, with the luma rows read from LDS.
__device__ __forceinline__ bool fused420_shape(const Desc& d) {
    return d.nc == 3 && d.bpm == 6 && d.c[0].hs == 2 && d.c[0].vs == 2 && d.c[1].hs == 1 && d.c[1].vs == 1 &&
           d.c[2].hs == 1 && d.c[2].vs == 1 && stream_kind(d) == 3;
}
__device__ __forceinline__ bool fused420(const Desc& d) { return d.status == kOk && fused420_shape(d); }



// Lane-pair IDCT of one block: c = the block as stored (zig-zag int16), qw = its component's
// dequant table (zig-zag, 4 bytes per register), h = the lane's half; rowd[r] = pixels 4h..4h+3
// of row r. D / n: the int32 DC of a block whose cell 0 holds kDcEscape. Wave-level (the fast
// path is a wave vote): every lane of the wave calls it.
__device__ __forceinline__ void pair_idct(const int4 (&c)[8], const uint32_t (&qw)[16], int h, const int32_t* dcv,
                                          const BlkLoc& loc, uint32_t (&rowd)[8]) {
    auto qt = [&](int z) { return (int32_t)((qw[z >> 2] >> (8 * (z & 3))) & 0xFFu); };
    auto coef = [&](int z) {
        const int4& w = c[z >> 3];
        const int e = z & 7;
        const uint32_t d32 = (uint32_t)(e < 2 ? w.x : e < 4 ? w.y : e < 6 ? w.z : w.w);
        return (int32_t)(int16_t)(d32 >> (16 * (e & 1)));
    };
    // row pass: natural rows 4h + i (the two candidate positions are compile-time; h selects)
    int32_t R[4][8];
    int32_t hi = 0, lo = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int z0 = kZigOfNatC[8 * i + j], z1 = kZigOfNatC[8 * (4 + i) + j];
            const int32_t v0 = m24(coef(z0), qt(z0)), v1 = m24(coef(z1), qt(z1));  // int16 x 8-bit: exact
            R[i][j] = h ? v1 : v0;
            if (i != 0 || j != 0) {
                hi = max(hi, R[i][j]);
                lo = min(lo, R[i][j]);
            }
        }
    }
    // the absolute DC: the pool cell (or its int32 escape) plus the block's offset
    if (h == 0) R[0][0] = wmul(blk_dc((int16_t)c[0].x, dcv, loc), qt(0));
    hi = max(hi, R[0][0]);
    lo = min(lo, R[0][0]);
    const bool fast = __all(hi < (1 << 14) && lo > -(1 << 14));
    if (fast) {
#pragma unroll
        for (int i = 0; i < 4; ++i) idct_row_full(R[i]);
    } else {  // the reference code, shortcuts and 32-bit wrap-around included
#pragma unroll
        for (int i = 0; i < 4; ++i) idct_row<false>(R[i]);
    }
    // quadrant swap: lane h keeps columns 4h..4h+3 of its rows and gets the partner's
    int32_t C[8][4];  // C[r][jj] = natural row r, column 4h + jj
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int32_t keep = h ? R[i][4 + jj] : R[i][jj];
            const int32_t got = pair_swap(h ? R[i][jj] : R[i][4 + jj]);
            C[i][jj] = h ? got : keep;
            C[4 + i][jj] = h ? keep : got;
        }
    }
    if (fast) {  // the four columns' unclipped outputs, then clip and pack a row's four bytes at once
        int32_t o[4][8];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            int32_t col[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) col[r] = C[r][jj];
            idct_col_raw(col, o[jj]);
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) rowd[r] = sat4<14>(o[0][r], o[1][r], o[2][r], o[3][r]);
        return;
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) rowd[r] = 0;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
        int32_t col[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) col[r] = C[r][jj];
        uint8_t o[8];
        idct_col<false>(col, o);
#pragma unroll
        for (int r = 0; r < 8; ++r) rowd[r] |= (uint32_t)o[r] << (8 * jj);
    }
}
// A dequant table (64 bytes of Desc::q, 4-byte aligned) into registers straight from global
// memory: the lane-pair IDCT kernels then use no LDS at all, so they can run beside the other
// pipeline's LDS-bound entropy kernels.
__device__ __forceinline__ void load_qw_g(const uint8_t* q, uint32_t (&qw)[16]) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(q);
#pragma unroll
    for (int k = 0; k < 16; ++k) qw[k] = p[k];
}
__device__ __forceinline__ void load_qw(const uint8_t* qz, uint32_t (&qw)[16]) {  // 64 bytes of LDS, 16-byte aligned
    const uint4* qs = reinterpret_cast<const uint4*>(qz);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint4 w = qs[k];
        qw[4 * k] = w.x; qw[4 * k + 1] = w.y; qw[4 * k + 2] = w.z; qw[4 * k + 3] = w.w;
    }
}
// The block's 16-byte zig-zag chunks that lane h of a pair uses: natural rows 0-3 (h = 0) lie in
// chunks {0,1,2,3,5,6}, rows 4-7 (h = 1) in {1,2,4,5,6,7}. So a lane loads six chunks, and its
// chunk 0 / 3 slots hold chunks 4 / 7 for h = 1 (pair_idct selects between the halves' values,
// and a half never reads the other half's private chunks): 6 loads per lane instead of 8.
__device__ __forceinline__ void load_block(const int16_t* ac, int64_t blk, int h, int4 (&c)[8]) {
    const int4* src = reinterpret_cast<const int4*>(ac + blk * 64);
    c[0] = nt_ld(src + (h ? 4 : 0));
    c[1] = nt_ld(src + 1);
    c[2] = nt_ld(src + 2);
    c[3] = nt_ld(src + (h ? 7 : 3));
    c[5] = nt_ld(src + 5);
    c[6] = nt_ld(src + 6);
    c[4] = c[0];
    c[7] = c[3];
}

// A wave's units wid, wid + nw, ... (wave-uniform loop): unit u's coefficient block is at
// pendf(u) (blk_pend: its pool block and DC offset once resolved), transformed and stored by
// unit(u, c, loc). Software-pipelined: unit u's block is loaded during unit u - nw and its map
// entry during the unit before that, and the loop alternates two register sets, so a wave waits
// only for loads issued one unit earlier -- never for its own stores (unit() must issue the same
// stores on every path, so the compiler can count them) and never for a register copy of a load
// in flight. (Before, the next unit's map entry was waited for right after it was issued,
// together with the unit's own block loads: one full memory latency per unit.)
template <class PendF, class UnitF>
__device__ __forceinline__ void idct_units(const int16_t* ac, const Desc& d, int h, uint32_t wid, uint32_t nw,
                                           uint32_t nunits, PendF pendf, UnitF unit) {
    if (wid >= nunits) return;
    auto at = [&](uint32_t u) { return pendf(min(u, nunits - 1)); };  // (past the end: harmless reloads)
    int4 ca[8], cb[8];
    BlkLoc la = blk_resolve(d, at(wid)), lb;
    load_block(ac, la.blk, h, ca);
    BlkPend pa, pb = at(wid + nw);
    auto step = [&](uint32_t u, const int4 (&D)[8], const BlkLoc& lD, int4 (&Dn)[8], BlkLoc& lDn, const BlkPend& Pn,
                    BlkPend& Pa) {
        lDn = blk_resolve(d, Pn);
        load_block(ac, lDn.blk, h, Dn);
        Pa = at(u + 2 * nw);
        unit(u, D, lD);
    };
    for (uint32_t u = wid;;) {
        step(u, ca, la, cb, lb, pb, pa);
        if ((u += nw) >= nunits) break;
        step(u, cb, lb, ca, la, pa, pb);
        if ((u += nw) >= nunits) break;
    }
}

// Waves per SIMD the 4:2:0 IDCT kernels are compiled for (timing experiments: 5 keeps them at 96
// VGPRs, so a wave fits beside four k_gw_lane waves on a SIMD).
#ifndef ICX_IDCT_Y_MINW
#define ICX_IDCT_Y_MINW 4
#endif
#ifndef ICX_IDCT_C_MINW
#define ICX_IDCT_C_MINW 1
#endif

// Chroma planes of fused420 images: a wave's unit is 16 MCUs of one MCU row; lane pair q < 16
// takes Cb of MCU mx0 + q, q >= 16 Cr of MCU mx0 + q - 16, so each plane row of the unit is
// 128 contiguous bytes written by one store instruction.
__global__ __launch_bounds__(256, ICX_IDCT_C_MINW) void k_idct420c(const Desc* __restrict__ desc, const int16_t* __restrict__ ac,
                                                  const int32_t* __restrict__ dcv, const uint2* __restrict__ map,
                                                  uint8_t* __restrict__ planes, int64_t plane_cap) {
    const int img = blockIdx.y;
    const Desc& d = desc[img];
    if (!fused420(d)) return;
    const int t = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63, q = lane >> 1, h = lane & 1, cc = q >> 4, mq = q & 15;
    uint32_t qw[16], qb[16];
    load_qw_g(d.q[d.c[1].tq], qw);
    load_qw_g(d.q[d.c[2].tq], qb);
#pragma unroll
    for (int k = 0; k < 16; ++k) qw[k] = cc ? qb[k] : qw[k];
    const int mbw = d.mbw, stride = d.c[1].stride;
    // Cb plane base (wave-uniform) and the Cr lanes' 32-bit offset from it (a chroma plane is
    // at most (65535 / 2)^2 bytes)
    uint8_t* Pc = planes + (int64_t)img * plane_cap + comp_plane_off(d, 1);
    const uint32_t ccoff = cc ? (uint32_t)(comp_plane_off(d, 2) - comp_plane_off(d, 1)) : 0u;
    const uint32_t ucols = (uint32_t)((mbw + 15) >> 4), nunits = ucols * (uint32_t)d.mbh;
    const uint32_t chunk0 = (gridDim.x & 7) ? blockIdx.x : (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    const uint32_t wid = chunk0 * 4 + wave, nw = gridDim.x * 4;
    // a lane pair past the row's last MCU transforms that MCU's block again and stores the same
    // bytes at its place (the pair that owns it is in the same unit): every lane stores
    auto pendf = [&](uint32_t u) {
        const uint32_t mby = u / ucols;
        const int mx = (int)((u - mby * ucols) << 4) + mq;
        return blk_pend(d, map, ((int64_t)mby * mbw + min(mx, mbw - 1)) * 6 + 4 + cc);
    };
    auto unit = [&](uint32_t u, const int4 (&c)[8], const BlkLoc& l) {
        const uint32_t mby = u / ucols;
        const int mx = min((int)((u - mby * ucols) << 4) + mq, mbw - 1);
        uint32_t rowd[8];
        pair_idct(c, qw, h, dcv, l, rowd);
        // the unit's row base is wave-uniform (scalar); a lane adds a 32-bit offset per row, so
        // the stores take the SGPR-base + VGPR-offset form with one VALU add each
        uint8_t* const rowp = Pc + (int64_t)mby * 8 * stride;
        const uint32_t lo = ccoff + (uint32_t)(mx * 8 + 4 * h);
#pragma unroll
        for (int r = 0; r < 8; ++r) nt_st(rowd[r], reinterpret_cast<uint32_t*>(rowp + (lo + (uint32_t)(r * stride))));
    };
    idct_units(ac, d, h, wid, nw, nunits, pendf, unit);
}

// Luma planes of fused420 images when the conversion reads them from HBM (ICX_FUSE420 = 2): a
// wave's unit is 8 MCUs of one MCU row; lane pair q takes luma block q & 3 of MCU mx0 + (q >> 2),
// so each store instruction writes two whole 128-byte plane rows (the unit's upper and lower
// block rows).
__global__ __launch_bounds__(256, ICX_IDCT_Y_MINW) void k_idct420y(const Desc* __restrict__ desc, const int16_t* __restrict__ ac,
                                                  const int32_t* __restrict__ dcv, const uint2* __restrict__ map,
                                                  uint8_t* __restrict__ planes, int64_t plane_cap) {
    const int img = blockIdx.y;
    const Desc& d = desc[img];
    if (!fused420(d)) return;
    const int t = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63, q = lane >> 1, h = lane & 1, mq = q >> 2, k = q & 3;
    int sbx, sby;
    (void)mcu_block_comp(d, k, sbx, sby);
    uint32_t qw[16];
    load_qw_g(d.q[d.c[0].tq], qw);
    const int mbw = d.mbw, stride = d.c[0].stride;
    uint8_t* Py = planes + (int64_t)img * plane_cap;  // component 0 is first in the slot
    const uint32_t ucols = (uint32_t)((mbw + 7) >> 3), nunits = ucols * (uint32_t)d.mbh;
    const uint32_t chunk0 = (gridDim.x & 7) ? blockIdx.x : (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    const uint32_t wid = chunk0 * 4 + wave, nw = gridDim.x * 4;
    auto pendf = [&](uint32_t u) {  // (past the row's last MCU: that MCU again, as in k_idct420c)
        const uint32_t mby = u / ucols;
        const int mx = (int)((u - mby * ucols) << 3) + mq;
        return blk_pend(d, map, ((int64_t)mby * mbw + min(mx, mbw - 1)) * 6 + k);
    };
    auto unit = [&](uint32_t u, const int4 (&c)[8], const BlkLoc& l) {
        const uint32_t mby = u / ucols;
        const int mx = min((int)((u - mby * ucols) << 3) + mq, mbw - 1);
        uint32_t rowd[8];
        pair_idct(c, qw, h, dcv, l, rowd);
        uint8_t* const rowp = Py + (int64_t)mby * 16 * stride;  // (as in k_idct420c)
        const uint32_t lo = (uint32_t)(sby * 8 * stride + mx * 16 + sbx * 8 + 4 * h);
#pragma unroll
        for (int r = 0; r < 8; ++r) nt_st(rowd[r], reinterpret_cast<uint32_t*>(rowp + (lo + (uint32_t)(r * stride))));
    };
    idct_units(ac, d, h, wid, nw, nunits, pendf, unit);
}

#ifndef ICX_IDCT1_MINW
#define ICX_IDCT1_MINW 4
#endif
#ifndef ICX_IDCT1_PF
#define ICX_IDCT1_PF 0
#endif
// ---------------------------------------------------- one-lane-per-block 4:2:0 IDCT (mode 4)
// One lane transforms one whole block in registers: no pair hand-off (the lane-pair IDCT spends
// a select per coefficient on which half of the block a lane holds, and a DPP swap plus two
// selects per output of the row pass on the quadrant exchange), every row and column pass
// within the lane. A wave's unit is 64 horizontally adjacent blocks of one block row of a plane
// (512 pixels), so each of the block's 8 row stores is one 8-byte store per lane and the wave
// writes 512 contiguous bytes per instruction. Dequant reads the int16 cell and the 8-bit table
// entry by SDWA into one 24-bit multiply; clip and pack by sat4<14>. NanoJPEG's own row / column
// code (shortcuts and 32-bit wrap-around, jpeg_dec.h:350-442) runs for a block whose dequantized
// coefficients reach 2^14, as in pair_idct (a per-lane branch: valid streams do not take it).
__device__ __forceinline__ void load_block8(const int16_t* ac, int64_t blk, int4 (&c)[8]) {
    const int4* src = reinterpret_cast<const int4*>(ac + blk * 64);
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = nt_ld(src + k);
}
// Dequant of one block into R (natural order, the absolute DC at R[0][0]) and the range of its
// values (the fast-path test of block_transform).
__device__ __forceinline__ void block_dequant(const int4 (&c)[8], const uint32_t (&qw)[16], const int32_t* dcv,
                                              const BlkLoc& loc, int32_t (&R)[8][8], int32_t& hi, int32_t& lo) {
    auto qt = [&](int z) { return (int32_t)((qw[z >> 2] >> (8 * (z & 3))) & 0xFFu); };
    auto coef = [&](int z) {
        const int4& w = c[z >> 3];
        const int e = z & 7;
        const uint32_t d32 = (uint32_t)(e < 2 ? w.x : e < 4 ? w.y : e < 6 ? w.z : w.w);
        return (int32_t)(int16_t)(d32 >> (16 * (e & 1)));
    };
    hi = 0;
    lo = 0;
#pragma unroll
    for (int n = 1; n < 64; ++n) {
        const int z = kZigOfNatC[n];
        R[n >> 3][n & 7] = m24(coef(z), qt(z));  // int16 x 8-bit: exact
        hi = max(hi, R[n >> 3][n & 7]);
        lo = min(lo, R[n >> 3][n & 7]);
    }
    R[0][0] = wmul(blk_dc((int16_t)c[0].x, dcv, loc), qt(0));  // the absolute DC
    hi = max(hi, R[0][0]);
    lo = min(lo, R[0][0]);
}
// rowd[2r], rowd[2r+1] = the 8 pixels of row r
__device__ __forceinline__ void block_transform(int32_t (&R)[8][8], int32_t hi, int32_t lo, uint32_t (&rowd)[16]) {
    if (hi < (1 << 14) && lo > -(1 << 14)) {
#pragma unroll
        for (int i = 0; i < 8; ++i) idct_row_full(R[i]);
#pragma unroll
        for (int half = 0; half < 2; ++half) {  // columns 4 half .. 4 half + 3, then their row dwords
            int32_t o[4][8];  // o[column][row], unclipped
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                int32_t col[8];
#pragma unroll
                for (int r = 0; r < 8; ++r) col[r] = R[r][4 * half + jj];
                idct_col_raw(col, o[jj]);
            }
#pragma unroll
            for (int r = 0; r < 8; ++r) rowd[2 * r + half] = sat4<14>(o[0][r], o[1][r], o[2][r], o[3][r]);
        }
    } else {  // the reference code, shortcuts and 32-bit wrap-around included
#pragma unroll
        for (int i = 0; i < 8; ++i) idct_row<false>(R[i]);
#pragma unroll
        for (int r = 0; r < 16; ++r) rowd[r] = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            int32_t col[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) col[r] = R[r][j];
            uint8_t ob[8];
            idct_col<false>(col, ob);
#pragma unroll
            for (int r = 0; r < 8; ++r) rowd[2 * r + (j >> 2)] |= (uint32_t)ob[r] << (8 * (j & 3));
        }
    }
}
__device__ __forceinline__ void block_idct(const int4 (&c)[8], const uint32_t (&qw)[16], const int32_t* dcv,
                                           const BlkLoc& loc, uint32_t (&rowd)[16]) {
    int32_t R[8][8], hi, lo;
    block_dequant(c, qw, dcv, loc, R, hi, lo);
    block_transform(R, hi, lo, rowd);
}
// Units of one plane: `ucols` units of 64 blocks per block row, `nby` block rows; unit u's lane
// takes block column bx = (u % ucols) * 64 + lane, clamped to the row (a lane past the row's end
// transforms its last block again and stores the same bytes at the same place: every lane
// stores). blkn(bx, by) = the block's index in the image's MCU order. Software-pipelined like
// idct_units: the next unit's block is loaded during this one, its map entry the unit before.
template <class BlkN>
__device__ __forceinline__ void plane_units(const Desc& d, const int16_t* ac, const int32_t* dcv, const uint2* map,
                                            const uint32_t (&qw)[16], uint8_t* P, int stride, uint32_t nbx,
                                            uint32_t nby, uint32_t wid, uint32_t nw, BlkN blkn) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t ucols = (nbx + 63) >> 6, nunits = ucols * nby;
    if (wid >= nunits) return;
    auto pend = [&](uint32_t u) {
        u = min(u, nunits - 1);  // (past the end: harmless reloads)
        const uint32_t by = u / ucols;
        const uint32_t bx = min(((u - by * ucols) << 6) + lane, nbx - 1);
        return blk_pend(d, map, blkn(bx, by));
    };
    auto unit = [&](uint32_t u, const int4 (&c)[8], const BlkLoc& l) {
        const uint32_t by = u / ucols, bx0 = (u - by * ucols) << 6;
        const uint32_t bx = min(bx0 + lane, nbx - 1);
        uint32_t rowd[16];
        block_idct(c, qw, dcv, l, rowd);
        // the unit's row base is wave-uniform; a lane adds its 32-bit column offset
        uint8_t* const rowp = P + (int64_t)by * 8 * stride + (int64_t)bx0 * 8;
        const uint32_t lo = (bx - bx0) * 8;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const uint2 v = make_uint2(rowd[2 * r], rowd[2 * r + 1]);
            nt_st(v, reinterpret_cast<uint2*>(rowp + (lo + (uint32_t)(r * stride))));
        }
    };
#if ICX_IDCT1_PF  // the next unit's block loaded during this one (two register sets)
    int4 ca[8], cb[8];
    BlkLoc la = blk_resolve(d, pend(wid)), lb;
    load_block8(ac, la.blk, ca);
    BlkPend pa, pb = pend(wid + nw);
    auto step = [&](uint32_t u, const int4 (&D)[8], const BlkLoc& lD, int4 (&Dn)[8], BlkLoc& lDn, const BlkPend& Pn,
                    BlkPend& Pa) {
        lDn = blk_resolve(d, Pn);
        load_block8(ac, lDn.blk, Dn);
        Pa = pend(u + 2 * nw);
        unit(u, D, lD);
    };
    for (uint32_t u = wid;;) {
        step(u, ca, la, cb, lb, pb, pa);
        if ((u += nw) >= nunits) break;
        step(u, cb, lb, ca, la, pa, pb);
        if ((u += nw) >= nunits) break;
    }
#else  // only the map entry one unit ahead: the block's loads wait out their latency (other waves run)
    BlkPend p = pend(wid);
    for (uint32_t u = wid; u < nunits; u += nw) {
        const BlkLoc l = blk_resolve(d, p);
        int4 c[8];
        load_block8(ac, l.blk, c);
        p = pend(u + nw);
        unit(u, c, l);
    }
#endif
}
// All three planes of fused420 images: gridDim.x workgroups per image walk the luma units, then
// the Cb and Cr units (one grid-stride sequence over the three planes' units); with luma == 0 only
// the chroma planes (mode 5: k_fused420s transforms the luma).
__global__ __launch_bounds__(256, ICX_IDCT1_MINW) void k_idct420s(const Desc* __restrict__ desc, const int16_t* __restrict__ ac,
                                                                   const int32_t* __restrict__ dcv, const uint2* __restrict__ map,
                                                                   uint8_t* __restrict__ planes, int64_t plane_cap, int luma) {
    const int img = blockIdx.y;
    const Desc& d = desc[img];
    if (!fused420(d)) return;
    const uint32_t wave = (uint32_t)wave_index();
    const uint32_t chunk0 = (gridDim.x & 7) ? blockIdx.x : (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    const uint32_t wid = chunk0 * 4 + wave, nw = gridDim.x * 4;
    const uint32_t mbw = (uint32_t)d.mbw, mbh = (uint32_t)d.mbh;
    uint8_t* const slot = planes + (int64_t)img * plane_cap;
    // luma: 2 x 2 blocks per MCU (k = 2 sby + sbx), block rows 2 mbh
    const uint32_t ynbx = 2 * mbw, yunits = luma ? ((ynbx + 63) >> 6) * (2 * mbh) : 0u;  // (mode 5: chroma only)
    const uint32_t cnbx = mbw, cunits = ((cnbx + 63) >> 6) * mbh;
    // The three planes' units are one sequence (luma, Cb, Cr); a wave takes units wid, wid + nw, ...
    // of it, i.e. in a plane whose units start at `base` the local units first(base), + nw, ...
    auto first = [&](uint32_t base) { return wid >= base ? wid - base : (base - wid + nw - 1) / nw * nw + wid - base; };
    uint32_t qw[16];
    auto uniform_q = [&]() {  // (one table per unit: scalar registers, read by SDWA)
#pragma unroll
        for (int k = 0; k < 16; ++k) qw[k] = __builtin_amdgcn_readfirstlane(qw[k]);
    };
    if (wid < yunits) {  // (wave-uniform)
        load_qw_g(d.q[d.c[0].tq], qw);
        uniform_q();
        plane_units(d, ac, dcv, map, qw, slot, d.c[0].stride, ynbx, 2 * mbh, wid, nw, [&](uint32_t bx, uint32_t by) {
            return (int64_t)(((by >> 1) * mbw + (bx >> 1)) * 6 + ((by & 1) << 1) + (bx & 1));
        });
    }
#pragma unroll
    for (uint32_t cc = 0; cc < 2; ++cc) {
        const uint32_t f = first(yunits + cc * cunits);
        if (f >= cunits) continue;
        load_qw_g(d.q[d.c[1 + cc].tq], qw);
        uniform_q();
        plane_units(d, ac, dcv, map, qw, slot + comp_plane_off(d, 1 + cc), d.c[1 + cc].stride, cnbx, mbh, f, nw,
                    [&](uint32_t bx, uint32_t by) { return (int64_t)((by * mbw + bx) * 6 + 4 + cc); });
    }
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// global stores (__syncthreads would also wait vmcnt(0), i.e. for every RGB store in flight).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Luma IDCT + conversion of fused420 images. Each wave owns a strip of 16 MCUs (256 pixels) by
// kFB MCU rows, like a k_convert_stream strip: per MCU row it transforms the row's 64 luma blocks
// (two rounds of 32 lane pairs) into its own 16 x 256 luma rows in LDS, then converts those 16
// rows with the chroma window carried in registers from the MCU row above (kv_rows: chroma
// from the planes k_idct420c wrote, luma from LDS). No workgroup barriers.
constexpr int kFB = 4;
__global__ __launch_bounds__(256) void k_fused420(const Desc* __restrict__ desc, const int16_t* __restrict__ ac,
                                                  const int32_t* __restrict__ dcv, const uint2* __restrict__ map,
                                                  const uint8_t* __restrict__ planes, int64_t plane_cap, uint8_t* __restrict__ out,
                                                  uint64_t out_stride) {
    const int img = blockIdx.y;
    const Desc& d = desc[img];
    if (!fused420(d)) return;
    __shared__ uint32_t Yl_all[4][16][64];  // per wave: its strip's 16 luma rows of the MCU row
    __shared__ __attribute__((aligned(16))) uint8_t qz[64];
    const int t = threadIdx.x;
    if (t < 64) qz[t] = d.q[d.c[0].tq][t];
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63, h = lane & 1, k = (lane >> 1) & 3;
    uint32_t (*Yl)[64] = Yl_all[wave];
    int sbx, sby;
    (void)mcu_block_comp(d, k, sbx, sby);
    uint32_t qw[16];
    load_qw(qz, qw);
    const int W = d.W, H = d.H, mbw = d.mbw, mbh = d.mbh;
    const uint8_t* pslot = planes + (int64_t)img * plane_cap;
    const CPl c1{pslot + comp_plane_off(d, 1), d.c[1].w, d.c[1].h, d.c[1].stride};
    const CPl c2{pslot + comp_plane_off(d, 2), d.c[2].w, d.c[2].h, d.c[2].stride};
    uint8_t* o = out + (int64_t)img * out_stride;
    const StreamOut so{o, W, ((reinterpret_cast<uintptr_t>(o) & 3) == 0) && (W & 3) == 0};
    const int nsx = (mbw + 15) >> 4, nsy = (mbh + kFB - 1) / kFB, nstrip = nsx * nsy;
    for (int strip = blockIdx.x * 4 + wave; strip < nstrip; strip += gridDim.x * 4) {
        const int sy = strip / nsx, sx = strip - sy * nsx;
        const int mx0 = sx << 4, mb0 = sy * kFB, mb1 = min(mbh, mb0 + kFB);
        const int x0 = 256 * sx + 4 * lane, M = x0 >> 2;
        const bool xl = x0 < W;
        const int nb = min(4, W - x0) * 3;
        const bool f1 = M >= 1 && x0 + 3 <= 2 * c1.w - 4 && 2 * M + 5 < c1.s;
        const bool f2 = M >= 1 && x0 + 3 <= 2 * c2.w - 4 && 2 * M + 5 < c2.s;
        KvWin w;
        kv_init<true>(w, c1, c2, M, f1, f2, 8 * mb0);
        for (int mby = mb0; mby < mb1; ++mby) {
#pragma unroll
            for (int r2 = 0; r2 < 2; ++r2) {  // the MCU row's 16 x 4 luma blocks, 32 per round
                const int mq = (lane >> 3) + 8 * r2, mx = mx0 + mq;
                const bool live = mx < mbw;
                const int64_t n = ((int64_t)mby * mbw + (live ? mx : mbw - 1)) * 6 + k;
                int4 c[8];
                const BlkLoc l = blk_loc(d, map, n);
                load_block(ac, l.blk, h, c);
                uint32_t rowd[8];
                pair_idct(c, qw, h, dcv, l, rowd);
                if (live) {
                    const int lc = mq * 4 + sbx * 2 + h;
#pragma unroll
                    for (int r = 0; r < 8; ++r) Yl[sby * 8 + r][lc] = rowd[r];
                }
            }
            asm volatile("" ::: "memory");  // (a wave's LDS accesses execute in order)
            const int Y0 = 16 * mby, Y1 = min(H, Y0 + 16);
            if (xl) {
                auto luma = [&](int y) { return Yl[y - Y0][lane]; };
                auto emit = [&](int y, uint32_t yv, uint32_t cb, uint32_t cr) {
                    uint32_t w[3];
                    ycc4_to_rgb(yv, cb, cr, w);
                    so.put3(y, x0, w, nb);
                };
                kv_rows<true>(w, c1, c2, M, f1, f2, Y0, Y1, luma, emit);
            }
            asm volatile("" ::: "memory");
        }
    }
}

// Mode 5: the luma IDCT inside the conversion with the one-lane IDCT (k_idct420s transforms only
// the chroma planes). A wave owns a strip of 16 MCUs (256 pixels) by kFB5 MCU rows; per MCU row
// lane l transforms luma block l & 3 of MCU mx0 + (l >> 2) -- the row's 64 blocks, one per lane
// -- into the wave's 16 x 256 luma rows in LDS, then converts those 16 rows as k_fused420 does
// (kv_rows: the chroma window carried in registers from the MCU row above, chroma from the planes,
// luma from LDS). The luma plane (16.8 MB per 4096^2 image, written and read back in mode 4) never
// goes through HBM. The next MCU row's block is loaded before this row's conversion, its map entry
// a row earlier. No workgroup barriers.
#ifndef ICX_FB5
#define ICX_FB5 4
#endif
#ifndef ICX_FUSED5_MINW  // 3: 152 VGPRs, no spills (4 spills; measured slower)
#define ICX_FUSED5_MINW 3
#endif
// (timing variants: ICX_F5_CARRY=0 sets the chroma window up again per MCU row instead of carrying
// it through the IDCT's registers; ICX_F5_PF=0 loads a row's block at the start of its IDCT)
#ifndef ICX_F5_CARRY
#define ICX_F5_CARRY 1
#endif
#ifndef ICX_F5_PF
#define ICX_F5_PF 1
#endif
#ifndef ICX_F5_QV  // 1: the quantisation table in VGPRs (168 VGPRs, no v_readlane): C3 -1.1%
#define ICX_F5_QV 0
#endif
#ifndef ICX_F5_QL  // 1: the table in LDS, into VGPRs per block (short-lived: no v_readlane of spilled SGPRs)
#define ICX_F5_QL 1
#endif
constexpr int kFB5 = ICX_FB5;
__global__ __launch_bounds__(256, ICX_FUSED5_MINW) void k_fused420s(const Desc* __restrict__ desc, const int16_t* __restrict__ ac,
                                                   const int32_t* __restrict__ dcv, const uint2* __restrict__ map,
                                                   const uint8_t* __restrict__ planes, int64_t plane_cap,
                                                   uint8_t* __restrict__ out, uint64_t out_stride) {
    const int img = blockIdx.y;
    const Desc& d = desc[img];
    if (!fused420(d)) return;
    __shared__ __attribute__((aligned(16))) uint32_t Yl_all[4][16][64];  // per wave: 16 luma rows x 256 pixels
    const int wave = wave_index(), lane = threadIdx.x & 63, mq = lane >> 2, k = lane & 3, sbx = k & 1, sby = k >> 1;
    uint32_t (*Yl)[64] = Yl_all[wave];
    uint32_t qw[16];
#if ICX_F5_QL  // the table in LDS, read into VGPRs per block just before the dequantisation
    __shared__ __attribute__((aligned(16))) uint32_t qlds[16];
    if (threadIdx.x < 16) qlds[threadIdx.x] = reinterpret_cast<const uint32_t*>(d.q[d.c[0].tq])[threadIdx.x];
    __syncthreads();
#endif
    load_qw_g(d.q[d.c[0].tq], qw);
#if ICX_F5_QV  // in vector registers, read by SDWA (in scalar registers they were spilled to VGPR lanes: 63 v_readlane per block)
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) asm volatile("" : "+v"(qw[k2]));
#elif ICX_F5_QL
#else
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) qw[k2] = __builtin_amdgcn_readfirstlane(qw[k2]);
#endif
    const int W = d.W, H = d.H, mbw = d.mbw, mbh = d.mbh;
    const uint8_t* pslot = planes + (int64_t)img * plane_cap;
    const CPl c1{pslot + comp_plane_off(d, 1), d.c[1].w, d.c[1].h, d.c[1].stride};
    const CPl c2{pslot + comp_plane_off(d, 2), d.c[2].w, d.c[2].h, d.c[2].stride};
    uint8_t* o = out + (int64_t)img * out_stride;
    const StreamOut so{o, W, ((reinterpret_cast<uintptr_t>(o) & 3) == 0) && (W & 3) == 0};
    const int nsx = (mbw + 15) >> 4, nsy = (mbh + kFB5 - 1) / kFB5, nstrip = nsx * nsy;
    // Border lanes (lane 0 and from edge_from on, as in k_convert_stream) are k_convert_edge's: for
    // their 4 columns this kernel writes the luma plane, which k_convert_edge reads; every other
    // lane converts with the interior taps (compile-time: the generic taps stay out of this kernel).
    uint8_t* const P0 = const_cast<uint8_t*>(pslot);
    const int s0 = d.c[0].stride;
    const int ef = edge_from(c1, c2, W);
    const bool conv = ef > 1;  // (wave-uniform: else every lane is a border lane)
    const uint32_t chunk0 = (gridDim.x & 7) ? blockIdx.x : (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    for (int strip = chunk0 * 4 + wave; strip < nstrip; strip += gridDim.x * 4) {  // wave-uniform
        const int sy = strip / nsx, sx = strip - sy * nsx;
        const int mx0 = sx << 4, mb0 = sy * kFB5, mb1 = min(mbh, mb0 + kFB5);
        const int M = 64 * sx + lane, x0 = 4 * M;
        const bool live = M >= 1 && M < ef;
        const bool border = x0 < W && !live;
        const int Mc = min(max(M, 1), max(ef - 1, 1));
        const int nb = live ? min(4, W - x0) * 3 : 0;
        // block of MCU row mby (a lane past the row's last MCU takes that MCU's block again: a
        // harmless reload, so every load is unconditional)
        const int mxl = min(mx0 + mq, mbw - 1);
        auto nblk = [&](int mby) { return ((int64_t)min(mby, mb1 - 1) * mbw + mxl) * 6 + k; };
        BlkPend p = blk_pend(d, map, nblk(mb0));
#if ICX_F5_CARRY
        KvWin w;
        if (conv) kv_init<true>(w, c1, c2, Mc, true, true, 8 * mb0);
#endif
#if ICX_F5_PF  // the next MCU row's block loaded before this row's conversion
        BlkLoc l = blk_resolve(d, p);
        int4 c[8];
        load_block8(ac, l.blk, c);
        p = blk_pend(d, map, nblk(mb0 + 1));
#endif
        for (int mby = mb0; mby < mb1; ++mby) {
            {
#if !ICX_F5_PF
                const BlkLoc l = blk_resolve(d, p);
                int4 c[8];
                load_block8(ac, l.blk, c);
                p = blk_pend(d, map, nblk(mby + 1));
#endif
                uint32_t rowd[16];
#if ICX_F5_QL
                {
                    asm volatile("" ::: "memory");  // (reloaded per block: not hoisted out of the loop)
                    uint32_t qv[16];
#pragma unroll
                    for (int q4 = 0; q4 < 4; ++q4) {
                        const uint4 t4 = reinterpret_cast<const uint4*>(qlds)[q4];
                        qv[4 * q4] = t4.x;
                        qv[4 * q4 + 1] = t4.y;
                        qv[4 * q4 + 2] = t4.z;
                        qv[4 * q4 + 3] = t4.w;
                    }
                    block_idct(c, qv, dcv, l, rowd);
                }
#else
                block_idct(c, qw, dcv, l, rowd);
#endif
                uint2* dst = reinterpret_cast<uint2*>(&Yl[sby * 8][mq * 4 + sbx * 2]);
#pragma unroll
                for (int r = 0; r < 8; ++r) dst[r * 32] = make_uint2(rowd[2 * r], rowd[2 * r + 1]);
            }
#if ICX_F5_PF
            l = blk_resolve(d, p);
            load_block8(ac, l.blk, c);
            p = blk_pend(d, map, nblk(mby + 2));
#endif
            asm volatile("" ::: "memory");  // (a wave's LDS accesses execute in order)
            const int Y0 = 16 * mby, Y1 = min(H, Y0 + 16);
            if (border) {  // (rare: border strips only)
                for (int y = Y0; y < Y1; ++y)
                    *reinterpret_cast<uint32_t*>(P0 + (int64_t)y * s0 + x0) = Yl[y - Y0][lane];
            }
            if (conv) {
                auto luma = [&](int y) { return Yl[y - Y0][lane]; };
                auto emit = [&](int y, uint32_t yv, uint32_t cb, uint32_t cr) {
                    uint32_t wo[3];
                    ycc4_to_rgb(yv, cb, cr, wo);
                    so.put3(y, 4 * Mc, wo, nb);
                };
#if !ICX_F5_CARRY
                // the chroma window is set up again per MCU row (its rows were just read by this
                // wave, so mostly from L2) rather than carried through the IDCT's registers
                KvWin w;
                kv_init<true>(w, c1, c2, Mc, true, true, Y0 >> 1);
#endif
                kv_rows<true>(w, c1, c2, Mc, true, true, Y0, Y1, luma, emit);
            }
            asm volatile("" ::: "memory");
        }
    }
}

// ------------------------------------------------- 4:2:0 back half in one kernel (mode 3)
// Dequant + IDCT + H/V chroma doubling + YCbCr->RGB of fused420 images without any plane in
// HBM: the coefficient blocks are read once and the RGB written once (the plane round trip was
// half of the back half's bytes). A workgroup owns a strip of kBW MCUs (256 output columns) by
// `seg` MCU rows and walks down it one MCU row per step; the planes of the rows in flight live in
// LDS rings:
//   phase A  IDCT of luma MCU row t+1 and chroma MCU row t+2 (+ the chroma blocks of the MCUs
//            left and right of the strip: the horizontal taps read 2 samples past each side),
//            the lane-pair IDCT of k_idct420y/c into the luma / raw chroma rings; then the
//            horizontal doubling (jpeg_dec.h:736-760, the stride-end quirk included) of chroma
//            row t+1 into the doubled ring
//   barrier
//   phase B  vertical doubling (:762-791) from the doubled rows t-1..t+1 and the conversion
//            (:834-853) of output rows 16t .. 16t+15; 12-byte streaming stores.
// Ring slots are chosen so that phase A of step t+1 never writes what phase B of step t reads
// (one LDS-only barrier per step). The vertical taps read the rows two above and below, so a
// segment also transforms the chroma of the MCU rows above and below it.
#ifndef ICX_BACK_PP  // two register sets for the prefetched blocks (see the loop)
#define ICX_BACK_PP 0
#endif
#ifndef ICX_BACK_MINW  // waves per SIMD k_back420 is compiled for
#define ICX_BACK_MINW 4
#endif
constexpr int kBW = 16;     // strip width in MCUs: 64 lanes x 4 columns
constexpr int kBRaw = 36;   // raw chroma row (dwords): 8 halo + 128 + 8 halo samples
struct BackLds {
    uint32_t y[3][16][64];         // luma rows of MCU rows t-1, t, t+1 (ring of 3)
    uint32_t raw[2][2][8][kBRaw];  // raw Cb / Cr rows of 2 MCU rows, strip + halo columns
    uint32_t dbl[4][2][8][64];     // horizontally doubled Cb / Cr rows of 4 MCU rows
    uint32_t q[3][16];             // dequant tables (zig-zag, bytes) of Y, Cb, Cr
};
__global__ __launch_bounds__(256, ICX_BACK_MINW) void k_back420(const Desc* __restrict__ desc, const int16_t* __restrict__ ac,
                                                 const int32_t* __restrict__ dcv, const uint2* __restrict__ map,
                                                 uint8_t* __restrict__ out, uint64_t out_stride, int seg) {
    const int img = blockIdx.y;
    const Desc& d = desc[img];
    if (!fused420(d)) return;
    __shared__ __attribute__((aligned(16))) BackLds L;
    const int t = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63, p = t >> 1, h = t & 1;
    const int W = d.W, H = d.H, mbw = d.mbw, mbh = d.mbh;
    const int cw = d.c[1].w, chh = d.c[1].h, cs = d.c[1].stride;  // Cb and Cr: same geometry (1x1)
    if (t < 48) L.q[t >> 4][t & 15] = reinterpret_cast<const uint32_t*>(d.q[d.c[t >> 4].tq])[t & 15];
    // pair p's block in an MCU: 0..63 luma block p & 3 of strip MCU p >> 2; 64..95 Cb / Cr of
    // strip MCU p & 15; 96..99 Cb / Cr of the MCU left (96, 97) / right (98, 99) of the strip
    const int kb = p < 64 ? (p & 3) : (p < 96 ? 4 + ((p - 64) >> 4) : 4 + (p & 1));
    const int dmx = p < 64 ? (p >> 2) : (p < 96 ? (p & 15) : (p < 98 ? -1 : kBW));
    int sbx = 0, sby = 0;
    if (kb < 4) (void)mcu_block_comp(d, kb, sbx, sby);
    const uint8_t* qz = reinterpret_cast<const uint8_t*>(L.q[kb < 4 ? 0 : kb - 3]);
    uint8_t* o = out + (int64_t)img * out_stride;
    const StreamOut so{o, W, ((reinterpret_cast<uintptr_t>(o) & 3) == 0) && (W & 3) == 0};
    const int nsx = (mbw + kBW - 1) / kBW, nseg = (mbh + seg - 1) / seg, items = nsx * nseg;
    for (int it = blockIdx.x; it < items; it += gridDim.x) {
        const int sg = it / nsx, sx = it - sg * nsx;
        const int mx0 = sx * kBW, r0 = sg * seg, r1 = min(mbh, r0 + seg);
        const int lo = max(r0 - 1, 0), hi = min(r1, mbh - 1);  // chroma MCU rows the segment needs
        const int M = 64 * sx + lane, x0 = 4 * M;             // the lane's output columns x0 .. x0+3
#ifdef ICX_EXP_BACK_NOSTORE
        uint32_t sink = 0;
#endif
        // step tr transforms luma MCU row tr+1 and chroma MCU row tr+2: whether the pair has a
        // block then, and where it is (clamped into the image where it has none)
        auto live_at = [&](int tr) {
            const int row = kb < 4 ? tr + 1 : tr + 2, mx = mx0 + dmx;
            return (kb < 4 ? row >= r0 && row < r1 : row >= lo && row <= hi) && p < 100 && mx >= 0 && mx < mbw;
        };
        auto pend_at = [&](int tr) {
            const int row = kb < 4 ? tr + 1 : tr + 2;
            const int mxc = min(max(mx0 + dmx, 0), mbw - 1), rowc = min(max(row, 0), mbh - 1);
#ifdef ICX_EXP_BACK_NOMAP  // timing experiment only: blocks as if written in place (wrong pixels)
            return BlkPend{make_uint2(0, 0), d.acbase + ((int64_t)rowc * mbw + mxc) * 6 + kb};
#else
            return blk_pend(d, map, ((int64_t)rowc * mbw + mxc) * 6 + kb);
#endif
        };
        // One step. Software pipeline: D (this step's block) was loaded during the previous step,
        // issued before that step's RGB stores, and its map entry one step before that; this step
        // resolves Pn (the next step's entry), loads the next step's block into Dn and the entry
        // after it into Pa. The loop below alternates two register sets, so no register with a
        // load in flight is ever copied (a copy waits for it: s_waitcnt vmcnt(0)).
        auto step = [&](int tr, const int4 (&D)[8], const BlkLoc& lD, int4 (&Dn)[8], BlkLoc& lDn, const BlkPend& Pn,
                        BlkPend& Pa) {
            // ---- phase A: transforms
            const int ry = tr + 1, rc = tr + 2;
            const bool live = live_at(tr);
            if (__any(live)) {  // wave-uniform
                uint32_t qw[16];
                load_qw(qz, qw);
                uint32_t rowd[8];
                pair_idct(D, qw, h, dcv, lD, rowd);
                if (live) {
                    if (kb < 4) {
                        uint32_t* dst = &L.y[ry % 3][sby * 8][dmx * 4 + sbx * 2 + h];
#pragma unroll
                        for (int r = 0; r < 8; ++r) dst[r * 64] = rowd[r];
                    } else {
                        uint32_t* dst = &L.raw[rc & 1][kb - 4][0][(dmx + 1) * 2 + h];
#pragma unroll
                        for (int r = 0; r < 8; ++r) dst[r * kBRaw] = rowd[r];
                    }
                }
            }
            lDn = blk_resolve(d, Pn);
#ifndef ICX_EXP_BACK_NOLOAD  // timing experiment only: keep transforming the first block (no loads)
            load_block(ac, lDn.blk, h, Dn);  // (past the last step: a harmless reload)
#endif
            Pa = pend_at(tr + 2);
            const int rd = tr + 1;  // horizontal doubling of chroma MCU row rd (written last step)
            if (rd >= lo && rd <= hi) {
                const bool interior = M >= 1 && x0 + 3 <= 2 * cw - 4;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int task = wave * 4 + j, cc = task >> 3, r = task & 7;
                    const uint32_t* rw = L.raw[rd & 1][cc][r];
                    uint32_t v;
                    if (interior) {  // samples 2M-2 .. 2M+3 at raw bytes 2 lane + 6 ..
                        const int b0 = ((2 * lane + 6) >> 2);
                        const uint64_t w = ((uint64_t)rw[b0] | ((uint64_t)rw[b0 + 1] << 32)) ^ 0x8080808080808080ull;
                        const uint64_t b = w >> ((lane & 1) ? 0 : 16);
                        const uint32_t w0 = (uint32_t)b, w1 = (uint32_t)(b >> 8), w2 = (uint32_t)(b >> 16);
                        v = pack4(dtap(w0, kTapRev), dtap(w1, kTapFwd), dtap(w1, kTapRev), dtap(w2, kTapFwd));
                    } else {  // image edges: the generic taps (the right edge reads from the stride end)
                        const uint8_t* rb = reinterpret_cast<const uint8_t*>(rw);
                        const int sh = 8 * mx0 - 8;  // chroma column of raw byte 0
                        auto at = [&](int g) { return (int)rb[min(max(g - sh, 0), 4 * kBRaw - 1)]; };
                        v = pmap([&](int i) {
                            const int x = x0 + i;
                            if (x >= 2 * cw) return 0;
                            return (int)double_tap(x, cw, at, [&](int jj) { return at(cs - jj); });
                        });
                    }
                    L.dbl[rd & 3][cc][r][lane] = v;
                }
            }
#ifndef ICX_EXP_BACK_NOBAR  // timing experiment only: no barrier (wrong pixels)
            lds_barrier();
#endif
            // ---- phase B: vertical doubling + conversion of output rows 16 tr + 4 wave .. + 3
            const int y0 = 16 * tr + 4 * wave;
            if (tr >= r0 && y0 < H) {  // wave-uniform
                const int k0 = y0 >> 1;
                const int nb = x0 < W ? min(4, W - x0) * 3 : 0;
                uint32_t A[2][6];
#pragma unroll
                for (int cc = 0; cc < 2; ++cc)
#pragma unroll
                    for (int i = 0; i < 6; ++i) {
                        const int r = min(max(k0 - 2 + i, 0), chh - 1);
                        A[cc][i] = L.dbl[(r >> 3) & 3][cc][r & 7][lane];
                    }
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int k = k0 + u, y = 2 * k;
                    if (y >= H) break;  // wave-uniform
                    uint32_t ev[2], od[2];
#pragma unroll
                    for (int cc = 0; cc < 2; ++cc) {
                        const uint32_t w0 = A[cc][u], w1 = A[cc][u + 1], w2 = A[cc][u + 2], w3 = A[cc][u + 3],
                                       w4 = A[cc][u + 4];
                        if (k >= 2 && k <= chh - 3) {
                            uint32_t e[4], f[4];
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                e[i] = dtap(kv_column(w0, w1, w2, w3, i) ^ kBias8, kTapRev);
                                f[i] = dtap(kv_column(w1, w2, w3, w4, i) ^ kBias8, kTapFwd);
                            }
                            ev[cc] = pack4(e[0], e[1], e[2], e[3]);
                            od[cc] = pack4(f[0], f[1], f[2], f[3]);
                        } else {
                            ev[cc] = vtap_even(k, chh, w0, w1, w2, w3);
                            od[cc] = vtap_odd(k, chh, w1, w2, w3, w4);
                        }
                    }
                    const uint32_t(*Y)[64] = L.y[tr % 3];
                    uint32_t wv[3];
                    ycc4_to_rgb(Y[y - 16 * tr][lane], ev[0], ev[1], wv);
#ifdef ICX_EXP_BACK_NOSTORE  // timing experiment only: no RGB stores (one per item keeps the work)
                    sink ^= wv[0] ^ wv[1] ^ wv[2];
#else
                    so.put3(y, x0, wv, nb);
#endif
                    if (y + 1 < H) {
                        ycc4_to_rgb(Y[y + 1 - 16 * tr][lane], od[0], od[1], wv);
#ifdef ICX_EXP_BACK_NOSTORE
                        sink ^= wv[0] ^ wv[1] ^ wv[2];
#else
                        so.put3(y + 1, x0, wv, nb);
#endif
                    }
                }
            }
        };
        lds_barrier();  // (the previous item's phase B is done with the rings; the q tables are in)
#if ICX_BACK_PP
        int4 ca[8], cb[8];
        BlkLoc la = blk_resolve(d, pend_at(lo - 2)), lb;
        BlkPend pa, pb = pend_at(lo - 1);
        load_block(ac, la.blk, h, ca);
        for (int tr = lo - 2;;) {
            step(tr, ca, la, cb, lb, pb, pa);
            if (++tr >= r1) break;
            step(tr, cb, lb, ca, la, pa, pb);
            if (++tr >= r1) break;
        }
#else  // one register set (the next step's block overwrites this one's once it is transformed)
        int4 ca[8];
        BlkLoc la = blk_resolve(d, pend_at(lo - 2));
        BlkPend pa = pend_at(lo - 1);
        load_block(ac, la.blk, h, ca);
        for (int tr = lo - 2; tr < r1; ++tr) step(tr, ca, la, ca, la, pa, pa);
#endif
#ifdef ICX_EXP_BACK_NOSTORE
        if (sink == 0x12345678u) o[lane] = 1;
#endif
    }
}

// --------------------------------------------------------------------------- finalize
__global__ void k_finalize(int n, const Desc* __restrict__ desc, int32_t* __restrict__ status,
                           int32_t* __restrict__ dims) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Desc& d = desc[i];
    const int st = d.status == kPending ? kInternalErr : d.status;
    status[i] = st;
    dims[3 * i + 0] = st == kOk ? d.W : 0;
    dims[3 * i + 1] = st == kOk ? d.H : 0;
    dims[3 * i + 2] = st == kOk ? (d.nc == 1 ? 1 : 3) : 0;
}

// ---------------------------------------------------------------------------- launcher
void launch_decode_front(const GroupWs& ws, int n, const uint8_t* d_data, const uint64_t* d_off,
                         const uint64_t* d_size, uint64_t out_stride, hipStream_t st, StageHook* hook, int part) {
    if (n <= 0) return;
    auto B = [&](Stage s) { if (hook) hook->begin(s, st); };
    auto E = [&](Stage s) { if (hook) hook->end(s, st); };
    if (part != kFrontRest) {
        B(kStParse);
        *ws.h_layout = 0;  // (k_parse sets it; the previous group on this workspace was read already)
        hipLaunchKernelGGL(k_parse, dim3(n), dim3(64), 0, st, n, d_data, d_off, d_size, ws.desc, ws.max_w, ws.max_h,
                           out_stride, ws.h_layout);
        E(kStParse);
    }
    launch_spec_entropy(ws, n, d_data, d_off, st, hook, part);
    if (part == kFrontFirst) return;
    B(kStEntropy);
    hipLaunchKernelGGL(k_entropy_seq, dim3(n), dim3(64), 0, st, n, d_data, d_off, ws.desc, ws.ac, ws.dc);
    E(kStEntropy);
}

void launch_decode_back(const GroupWs& ws, int n, uint8_t* d_out, uint64_t out_stride, int32_t* d_status,
                        int32_t* d_dims, hipStream_t st, StageHook* hook, bool known_layout) {
    if (n <= 0) return;
    // the other samplings' kernels, unless the host knows the group has none (k_parse's flag,
    // written before round 0's planning, whose event the host waits for here)
    const bool other = !known_layout || hipEventSynchronize(ws.ev_defer) != hipSuccess || *ws.h_layout != 0;
    auto B = [&](Stage s) { if (hook) hook->begin(s, st); };
    auto E = [&](Stage s) { if (hook) hook->end(s, st); };
    const int tb = 64, nb = (n + tb - 1) / tb;
    B(kStIdct);
    const int64_t maxblk = ws.coef_cap;
    // ~16K workgroups per launch in total; every kernel grid-strides over its image's work. The
    // kernels for the other samplings get kGenericWG in total (ICX_GENERIC_WG overrides): in a
    // 4:2:0 batch they are no-ops, and dispatching 16K empty workgroups each cost ~1% per step.
    static const int gwg = std::getenv("ICX_GENERIC_WG") ? std::max(8, std::atoi(std::getenv("ICX_GENERIC_WG"))) : kGenericWG;
    int gx = (int)std::max<int64_t>(1, std::min<int64_t>((maxblk + 32 * kIdctU - 1) / (32 * kIdctU), gwg / n));
    if (gx >= 8) gx &= ~7;  // XCD-aware chunk order in k_idct needs a multiple of 8
    // 4:2:0 images (fused420), by plane mode (ICX_FUSE420 overrides it: tests, experiments; any
    // other value is the default, since an unknown mode would leave 4:2:0 luma untransformed):
    //   5 (default) k_idct420s transforms the chroma planes, k_fused420s the luma blocks inside
    //     the conversion (no luma plane in HBM); k_convert_edge takes the border lanes
    //   4 k_idct420s (one lane per block) for all three planes, then the stream conversion
    //   3 k_back420, the whole back half without planes
    //   2 the lane-pair IDCT k_idct420y / k_idct420c, then the stream conversion
    //   1 k_idct420c + k_fused420 (round 2's luma IDCT inside the conversion, lane pairs)
    //   0 the generic k_idct
    const int fuse = [] {  // (read per launch: tests switch modes within one process)
        const int v = std::getenv("ICX_FUSE420") ? std::atoi(std::getenv("ICX_FUSE420")) : 5;
        return (v >= 0 && v <= 5) ? v : 5;
    }();
    if (other || fuse == 0) {
        hipLaunchKernelGGL(k_idct, dim3(gx, n), dim3(256), 0, st, ws.desc, ws.ac, ws.dc, ws.map, ws.planes, ws.plane_cap,
                           fuse);
        hipLaunchKernelGGL(k_idct_any, dim3(gx, n), dim3(256), 0, st, ws.desc, ws.ac, ws.dc, ws.map, ws.planes,
                           ws.plane_cap);
    }
    if (fuse == 4 || fuse == 5) {  // 4:2:0: 64 blocks of a block row per wave unit, luma (mode 4) then chroma units
        // (units per wave: ICX_IDCT1_UPW, at least; small images' waves otherwise take one unit
        // each and its dependent map -> block -> store latency alone)
        static const int upw = std::getenv("ICX_IDCT1_UPW") ? std::max(1, std::atoi(std::getenv("ICX_IDCT1_UPW"))) : 1;
        const int64_t units = (maxblk / 6) * (fuse == 4 ? 6 : 2) / 64 + 3;
        const int sgx = (int)std::max<int64_t>(1, std::min<int64_t>((units + 4 * upw - 1) / (4 * upw), 16384 / n)) & ~7;
        hipLaunchKernelGGL(k_idct420s, dim3(std::max(sgx, 8), n), dim3(256), 0, st, ws.desc, ws.ac, ws.dc, ws.map,
                           ws.planes, ws.plane_cap, fuse == 4 ? 1 : 0);
    }
    if (fuse == 1 || fuse == 2) {  // 4:2:0: chroma planes (and, mode 2, luma planes) by the lane-pair IDCT
        const int cgx = (int)std::max<int64_t>(1, std::min<int64_t>((maxblk / 6 / 16 + 31) / 32, 16384 / n)) & ~7;
        hipLaunchKernelGGL(k_idct420c, dim3(std::max(cgx, 8), n), dim3(256), 0, st, ws.desc, ws.ac, ws.dc, ws.map,
                           ws.planes, ws.plane_cap);
        if (fuse == 2) {
            const int ygx = (int)std::max<int64_t>(1, std::min<int64_t>((maxblk / 6 / 8 + 31) / 32, 16384 / n)) & ~7;
            hipLaunchKernelGGL(k_idct420y, dim3(std::max(ygx, 8), n), dim3(256), 0, st, ws.desc, ws.ac, ws.dc, ws.map,
                               ws.planes, ws.plane_cap);
        }
    }
    E(kStIdct);
    // The kernels that read the coefficients inside the conversion (4:2:0 plane modes 1, 3, 5) run
    // before the generic upsample: its ping-pong planes (ws.tmp) live in the coefficient pool
    // (icx_api.cpp ws_alloc_all), which is dead from here on.
    B(kStConvert);
    const int fgx = (int)std::max<int64_t>(1, std::min<int64_t>((((int64_t)(ws.max_w + 255) / 256) *
                                                                  ((ws.max_h + 16 * kFB - 1) / (16 * kFB)) + 3) / 4,
                                                                 16384 / n));
    if (fuse == 3) {  // 4:2:0: the whole back half in k_back420, no planes
        const int seg = std::getenv("ICX_BSEG")  // (read per launch: tests vary it)
             ? std::max(1, std::atoi(std::getenv("ICX_BSEG"))) : 32;
        const int64_t items = (int64_t)((ws.max_w + 16 * kBW - 1) / (16 * kBW)) * (((ws.max_h + 15) / 16 + seg - 1) / seg);
        const int bgx = (int)std::max<int64_t>(1, std::min<int64_t>(items, 16384 / n));
        hipLaunchKernelGGL(k_back420, dim3(bgx, n), dim3(256), 0, st, ws.desc, ws.ac, ws.dc, ws.map, d_out, out_stride,
                           seg);
    }
    if (fuse == 1)
        hipLaunchKernelGGL(k_fused420, dim3(fgx, n), dim3(256), 0, st, ws.desc, ws.ac, ws.dc, ws.map, ws.planes,
                           ws.plane_cap, d_out, out_stride);
    if (fuse == 5) {
        const int64_t fs = ((int64_t)(ws.max_w + 255) / 256) * ((ws.max_h + 16 * kFB5 - 1) / (16 * kFB5));
        static const int spw = std::getenv("ICX_F5_SPW") ? std::max(1, std::atoi(std::getenv("ICX_F5_SPW"))) : 1;
        int f5 = (int)std::max<int64_t>(1, std::min<int64_t>((fs + 4 * spw - 1) / (4 * spw), 16384 / n));
        if (f5 >= 8) f5 &= ~7;  // (XCD-aware strip order needs a multiple of 8)
        hipLaunchKernelGGL(k_fused420s, dim3(f5, n), dim3(256), 0, st, ws.desc, ws.ac, ws.dc, ws.map, ws.planes,
                           ws.plane_cap, d_out, out_stride);
    }
    E(kStConvert);
    B(kStUpsample);
    const int ux = (int)std::max<int64_t>(1, std::min<int64_t>((ws.tmp_cap + 255) / 256, gwg / (3 * n)));
    for (int p = 0; p < 6 && other; ++p)
        hipLaunchKernelGGL(k_upsample, dim3(ux, n * 3), dim3(256), 0, st, ws.desc, ws.planes, ws.tmp, ws.plane_cap,
                           ws.tmp_cap, p);
    E(kStUpsample);
    B(kStConvert);
    const int cx = (int)std::max<int64_t>(1, std::min<int64_t>(((int64_t)ws.max_w * ws.max_h + 255) / 256, gwg / n));
    const int64_t sxw = ((int64_t)(ws.max_w + 255) / 256) * ((ws.max_h + kSH - 1) / kSH) / 4 + 1;
    const int sxg = (int)std::max<int64_t>(1, std::min<int64_t>(sxw, 16384 / n));
    const int sxo = (int)std::max<int64_t>(1, std::min<int64_t>(sxw, gwg / n));  // the other layouts
    hipLaunchKernelGGL(k_convert_stream<3>, dim3(sxg, n), dim3(256), 0, st, ws.desc, ws.planes, ws.plane_cap, d_out,
                       out_stride, fuse);
    if (other) {
        hipLaunchKernelGGL(k_convert_stream<0>, dim3(sxo, n), dim3(256), 0, st, ws.desc, ws.planes, ws.plane_cap, d_out,
                           out_stride, fuse);
        hipLaunchKernelGGL(k_convert_stream<1>, dim3(sxo, n), dim3(256), 0, st, ws.desc, ws.planes, ws.plane_cap, d_out,
                           out_stride, fuse);
        hipLaunchKernelGGL(k_convert_stream<2>, dim3(sxo, n), dim3(256), 0, st, ws.desc, ws.planes, ws.plane_cap, d_out,
                           out_stride, fuse);
        hipLaunchKernelGGL(k_convert_stream<4>, dim3(sxo, n), dim3(256), 0, st, ws.desc, ws.planes, ws.plane_cap, d_out,
                           out_stride, fuse);
    }
    // border lanes of the doubled layouts: ~3 lanes x (H / kSHE) strips per image
    const int64_t egw = (4 * ((ws.max_h + kSHE - 1) / kSHE) + 255) / 256;
    const int egx = (int)std::max<int64_t>(1, std::min<int64_t>(egw, 16384 / n));
    const int ego = (int)std::max<int64_t>(1, std::min<int64_t>(egw, gwg / n));
    hipLaunchKernelGGL(k_convert_edge<3>, dim3(egx, n), dim3(256), 0, st, ws.desc, ws.planes, ws.plane_cap, d_out,
                       out_stride, fuse);
    if (other) {
        hipLaunchKernelGGL(k_convert_edge<1>, dim3(ego, n), dim3(256), 0, st, ws.desc, ws.planes, ws.plane_cap, d_out,
                           out_stride, fuse);
        hipLaunchKernelGGL(k_convert_fused, dim3(cx, n), dim3(256), 0, st, ws.desc, ws.planes, ws.plane_cap, d_out,
                           out_stride);
        hipLaunchKernelGGL(k_convert, dim3(cx, n), dim3(256), 0, st, ws.desc, ws.planes, ws.tmp, ws.plane_cap,
                           ws.tmp_cap, d_out, out_stride);
    }
    hipLaunchKernelGGL(k_finalize, dim3(nb), dim3(tb), 0, st, n, ws.desc, d_status, d_dims);
    E(kStConvert);
}

void launch_decode_group(const GroupWs& ws, int n, const uint8_t* d_data, const uint64_t* d_off,
                         const uint64_t* d_size, uint8_t* d_out, uint64_t out_stride, int32_t* d_status,
                         int32_t* d_dims, hipStream_t st, StageHook* hook) {
    launch_decode_front(ws, n, d_data, d_off, d_size, out_stride, st, hook);
    launch_decode_back(ws, n, d_out, out_stride, d_status, d_dims, st, hook, false);
}

}  // namespace icx
