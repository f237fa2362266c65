// icx_exr.hip -- OpenEXR read on the MI355X: Image::readExr (codecs.cpp:464-493), i.e. tinyexr's
// LoadEXRFromMemory (/root/reference/tinyexr.h:6645-6860) -> RGBA float.
//
// The host parses the header and the offset table and checks every chunk header the way tinyexr
// does (a few hundred bytes of control data); the device does the pixel work:
//   k_exr_unpack   one wave per compressed chunk: the wave inflates (ZIP / ZIPS; wave-uniform, 16 KiB LDS ring) or lane 0 run-decodes
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
// output, as LoadEXRFromMemory does); NONE / RLE / ZIPS / ZIP / PIZ. The multi-part / deep
// version bits are decoded as one part, as LoadEXRFromMemory does (only the tile-offset walk
// differs); PXR24 / B44 / ZFP -> UNSUPPORTED_FORMAT. Pixels no chunk wrote (tinyexr:
// uninitialised memory) are 0.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "icx_exr_plan.h"
#include "icx_internal.h"

namespace icx {

// ------------------------------------------------------------ the wave's inflate (round 6)
// exr_inflate (icx_exr_core.h) with the same decisions, error checks and result, laid out for one
// wave whose decoder state is wave-uniform (SGPRs), without the per-byte memory round trips that
// bounded round 5's version (~860 cycles per output byte: a chunk of 256 KiB took ~90 ms):
//  * input: a 512-byte window in registers (one dword per lane of [wb, wb+256) and of the next
//    256 bytes, loaded 256 bytes ahead); a refill is two v_readlane and a funnel shift, not four
//    dependent byte loads from HBM.
//  * output: bytes go to the W-byte LDS ring only; every 4 KiB completed the wave copies them to
//    the chunk's scratch with 16-byte stores.
//  * matches: the wave copies all bytes of a match at once, lane k byte k (64 per round), from the
//    ring (distance + length <= W) or from the flushed output (farther back); byte k's source is
//    out - dist + (k mod dist), a byte from before the match, so a repeat (dist < length) needs no
//    ordering between lanes.
//  * Adler-32 over the output afterwards, by the wave in parallel (in round 5 four dependent adds
//    and a counter per output byte).
// Input bytes past the chunk read as 0 and are counted (`over`), as BitIn does.
// 32-bit positions (a chunk and its output below 1 GiB; larger ones take exr_inflate).
struct InW {
    const uint8_t* A;    // the chunk's bytes rounded down to 4
    uint32_t n, e;       // bytes; e = n + mis, the end relative to A
    uint32_t wb;         // window start relative to A (multiple of 256)
    uint32_t cur, nxt;   // this lane's dword of [wb, wb + 256) and [wb + 256, wb + 512)
    uint32_t pos;        // next byte (relative to the chunk) into buf
    uint32_t mis;
    uint64_t buf;        // LSB-first bit buffer
    int cnt;
    uint32_t over;
    __device__ __forceinline__ uint32_t ld(uint32_t base) const {  // dword lane of [base, base + 256) (relative to A)
        const uint32_t a = base + 4u * __lane_id();
        if (a + 4u <= e) return *reinterpret_cast<const uint32_t*>(A + a);
        uint32_t v = 0;
        for (uint32_t j = 0; j < 4; ++j)
            if (a + j < e) v |= (uint32_t)A[a + j] << (8 * j);
        return v;
    }
    __device__ __forceinline__ void init(const uint8_t* src, uint32_t nb) {
        mis = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 3u);
        A = src - mis;
        n = nb;
        e = nb + mis;
        wb = 0;
        cur = ld(0);
        nxt = ld(256);
        pos = 0;
        buf = 0;
        cnt = 0;
        over = 0;
    }
    // The window moves in one place only, adv(), which each decode loop calls once per iteration
    // (an iteration consumes at most 16 input bytes, so fill() always finds its 4 bytes in
    // [wb, wb + 512)): with the window's registers written at several inlined sites, the copies
    // the compiler made to merge them waited for every load and store in flight, on every symbol.
    __device__ __forceinline__ void adv() {
        if (pos + mis >= wb + 256u) {  // (wave-uniform) the next window; its successor's load goes out now
            cur = nxt;
            wb += 256u;
            nxt = ld(wb + 256u);
        }
    }
    __device__ __forceinline__ void fill(int k) {  // k <= 32
        if (cnt >= k) return;
        const uint32_t o = pos + mis - wb, i0 = o >> 2, i1 = i0 + 1u;  // (o < 512 - 4)
        const uint32_t v0 = i0 < 64u ? __builtin_amdgcn_readlane(cur, i0) : __builtin_amdgcn_readlane(nxt, i0 - 64u);
        const uint32_t v1 = i1 < 64u ? __builtin_amdgcn_readlane(cur, i1) : __builtin_amdgcn_readlane(nxt, i1 - 64u);
        const uint32_t w = __builtin_amdgcn_alignbyte(v1, v0, o & 3u);
        if (pos + 4u > n) over += 8u * (pos + 4u - max(pos, n));  // (bytes at or past n read as 0: ld does not load them)
        buf |= (uint64_t)w << cnt;
        pos += 4u;
        cnt += 32;
    }
    __device__ __forceinline__ uint32_t bits(int k) {  // k <= 24
        fill(k);
        const uint32_t v = (uint32_t)buf & ((1u << k) - 1u);
        buf >>= k;
        cnt -= k;
        return v;
    }
    __device__ __forceinline__ bool past_end() const { return over > (uint32_t)cnt; }
};
// inf_decode for the wave: a code longer than kInfFast bits is found from the per-length limits
// (the six reads are independent: one LDS round trip, where inf_decode's walk read the counts one
// dependent length at a time). The same symbol or -1 as inf_decode.
__device__ __forceinline__ int inf_decode_w(InW& in, const InfTab& h) {
    in.fill(16);
    const uint32_t e = exr_uni(h.fast[(uint32_t)in.buf & ((1u << kInfFast) - 1u)]);
    if (e) {
        in.buf >>= e & 15u;
        in.cnt -= (int)(e & 15u);
        return (int)(e >> 4);
    }
    // the next 15 stream bits, the first as the most significant (a canonical code's bit order)
    const uint32_t r = __builtin_bitreverse32((uint32_t)in.buf) >> 17;
    uint32_t lim[16];
#pragma unroll
    for (int l = kInfFast + 1; l <= 15; ++l) lim[l] = exr_uni(h.lim[l]);
#pragma unroll
    for (int l = kInfFast + 1; l <= 15; ++l) {
        const uint32_t c = r >> (15 - l);
        if (c < lim[l]) {  // (no shorter code matched: c >= the length's first code)
            in.buf >>= l;
            in.cnt -= l;
            return (int)exr_uni(h.sym[(int)exr_uni((uint32_t)(int32_t)h.off[l]) + (int)c]);
        }
    }
    return -1;
}
static_assert(kInfFast == 9, "inf_decode_w starts the long codes at 10 bits");

// RFC 1951 length / distance bases and extra bits by arithmetic (Deflate's tables, without a
// memory load whose wait would also wait for the flushes' stores)
__device__ __forceinline__ uint32_t len_ext(uint32_t li) { return li < 8u || li == 28u ? 0u : (li - 4u) >> 2; }
__device__ __forceinline__ uint32_t len_base(uint32_t li) {
    return li < 8u ? 3u + li : li == 28u ? 258u : ((4u + ((li - 4u) & 3u)) << len_ext(li)) + 3u;
}
__device__ __forceinline__ uint32_t dist_ext(uint32_t di) { return di < 4u ? 0u : (di - 2u) >> 1; }
__device__ __forceinline__ uint32_t dist_base(uint32_t di) { return di < 4u ? 1u + di : ((2u + (di & 1u)) << dist_ext(di)) + 1u; }

template <int W>
__device__ __forceinline__ bool exr_inflate_wave(const uint8_t* src, int64_t n64, uint8_t* dst, int64_t cap64, int64_t* produced, InfState& st,
                                 uint8_t* ring) {
    static_assert(W >= 1024 && (W & (W - 1)) == 0, "a power-of-two ring of at least 1 KiB");
    *produced = 0;
    if (n64 < 2) return false;
    if (n64 >= (int64_t)1 << 30 || cap64 >= (int64_t)1 << 30) return exr_inflate<W>(src, n64, dst, cap64, produced, st, ring);
    const uint32_t n = (uint32_t)n64, cap = (uint32_t)cap64;
    const uint32_t lane = __lane_id();
    const uint32_t cmf = exr_uni(src[0]), flg = exr_uni(src[1]);
    if ((cmf * 256u + flg) % 31u != 0 || (flg & 32u) || (cmf & 15u) != 8) return false;
    InW in;
    in.init(src, n);
    (void)in.bits(16);  // (the two header bytes)
    uint32_t out = 0, fl = 0;  // bytes out; bytes copied to dst (multiple of 256 until the end)
    // (output past cap fails the chunk; it is found here, before any byte past cap is stored, and at
    // the end -- the same result as exr_inflate's test per byte)
    bool over_cap = false;
    // kFlush bytes from fl, 16 per lane and store (wave-uniform; readfirstlane keeps fl a scalar).
    // Large, so that the input window's loads seldom wait behind flush stores (one vmcnt counts both).
    constexpr uint32_t kFlush = 4096;
    static_assert(W >= 4 * (int)kFlush, "unflushed bytes and the near-match window fit the ring");
    auto flush1 = [&]() {
        over_cap = over_cap || fl + kFlush > cap;
        if (over_cap) return;
#pragma unroll
        for (uint32_t q = 0; q < kFlush / 1024u; ++q) {
            const uint32_t o = fl + 1024u * q + 16u * lane;
            const uint4 v = *reinterpret_cast<const uint4*>(ring + (o & (W - 1)));
            *reinterpret_cast<uint4*>(dst + o) = v;
        }
        fl = exr_uni(fl + kFlush);
    };
    auto flush = [&]() {  // (a literal or a match completes at most one block)
        if (out - fl >= kFlush) flush1();
    };
    auto lit = [&](uint32_t b) {
        if (lane == 0) ring[out & (W - 1)] = (uint8_t)b;
        out = exr_uni(out + 1u);
        if (out - fl >= kFlush) flush1();
    };
    int last = 0;
    while (!last) {
        in.adv();
        last = (int)in.bits(1);
        const uint32_t type = in.bits(2);
        if (type == 0) {  // stored
            in.bits(in.cnt & 7);
            const uint32_t len = in.bits(16), nlen = in.bits(16);
            if (in.past_end() || (len ^ 0xFFFFu) != nlen) return false;
            if (out + len > cap) return false;
            for (uint32_t k = 0; k < len; ++k) {
                in.adv();
                const uint32_t b = in.bits(8);
                if (in.past_end()) return false;
                lit(b);
            }
            continue;
        }
        if (type == 3) return false;
        if (type == 1) {  // fixed codes
            for (int s = 0; s < 288; ++s) st.len[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
            (void)inf_build(st.lit, st.len, 288);
            for (int s = 0; s < 32; ++s) st.len[s] = 5;
            (void)inf_build(st.dist, st.len, 32);
        } else {  // dynamic codes
            const int nlen = (int)in.bits(5) + 257, ndist = (int)in.bits(5) + 1, ncode = (int)in.bits(4) + 4;
            if (nlen > 286 || ndist > 30) return false;
            for (int k = 0; k < 19; ++k) {
                in.adv();
                st.len[Deflate::kClOrder[k]] = k < ncode ? (uint8_t)in.bits(3) : 0;
            }
            if (in.past_end() || !inf_build(st.lit, st.len, 19)) return false;
            int k = 0;
            while (k < nlen + ndist) {
                in.adv();
                const int sym = inf_decode_w(in, st.lit);
                if (sym < 0 || in.past_end()) return false;
                if (sym < 16) {
                    st.len[k++] = (uint8_t)sym;
                    continue;
                }
                uint8_t v = 0;
                int rep;
                if (sym == 16) {
                    if (k == 0) return false;
                    v = (uint8_t)exr_uni(st.len[k - 1]);
                    rep = 3 + (int)in.bits(2);
                } else if (sym == 17) {
                    rep = 3 + (int)in.bits(3);
                } else {
                    rep = 11 + (int)in.bits(7);
                }
                if (k + rep > nlen + ndist) return false;
                while (rep--) st.len[k++] = v;
            }
            if (in.past_end()) return false;
            if (!inf_build(st.lit, st.len, nlen) || !inf_build(st.dist, st.len + nlen, ndist)) return false;
        }
        // (every failure leaves the loop by one break with `bad` set: a single exit besides the
        // block's end, so the compiler does not thread a state variable through every literal)
        bool bad = false;
        for (;;) {
            in.adv();
            // (reading past the input makes past_end() true for good, and every path from there
            // fails: it is tested at the block's end, at each match and before the trailer, not
            // per literal)
            const int sym = inf_decode_w(in, st.lit);
            if ((uint32_t)sym < 256u) {
                if (lane == 0) ring[out & (W - 1)] = (uint8_t)sym;
                out = exr_uni(out + 1u);
                if (out - fl >= kFlush) {
                    flush1();
                    bad = over_cap || in.past_end();  // (also ends a run of literals past the input)
                    if (bad) break;
                }
                continue;
            }
            bad = sym < 0 || in.past_end() || over_cap;
            if (bad || sym == 256) break;
            const uint32_t li = (uint32_t)sym - 257u;
            bad = li >= 29u;
            if (bad) break;
            const uint32_t len = len_base(li) + in.bits((int)len_ext(li));  // (then the distance code)
            const int di = inf_decode_w(in, st.dist);
            bad = di < 0 || di >= 30;
            if (bad) break;
            const uint32_t dist = dist_base((uint32_t)di) + in.bits((int)dist_ext((uint32_t)di));
            bad = in.past_end() || dist > out || out + len > cap;
            if (bad) break;
            // the match, 64 bytes per round: sources from before `out` only (see above); from the
            // ring while none of them can have been overwritten by this match's own bytes, else
            // from dst (dist > W - len >= kFlush + 258: every source byte is flushed)
            const uint32_t q0 = out - dist;
            if (dist + len <= (uint32_t)W) {
                if (dist >= len) {
                    for (uint32_t k = lane; k < len; k += 64u) ring[(out + k) & (W - 1)] = ring[(q0 + k) & (W - 1)];
                } else {
                    for (uint32_t k = lane; k < len; k += 64u) ring[(out + k) & (W - 1)] = ring[(q0 + k % dist) & (W - 1)];
                }
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the flushes' stores)
                for (uint32_t k = lane; k < len; k += 64u) ring[(out + k) & (W - 1)] = dst[q0 + k];
            }
            out = exr_uni(out + len);
            flush();
        }
        if (bad) return false;
    }
    if (over_cap || out > cap) return false;
    // the last bytes (fewer than kFlush): whole dwords, then the tail
    const uint32_t o4 = out & ~3u;
    for (uint32_t k = fl + 4u * lane; k < o4; k += 256u)
        *reinterpret_cast<uint32_t*>(dst + k) = *reinterpret_cast<const uint32_t*>(ring + (k & (W - 1)));
    if (o4 + lane < out) dst[o4 + lane] = ring[(o4 + lane) & (W - 1)];
    in.adv();
    in.bits(in.cnt & 7);  // to a byte boundary
    uint32_t adler = 0;
    for (int k = 0; k < 4; ++k) adler = (adler << 8) | in.bits(8);
    if (in.past_end()) return false;
    // Adler-32 of the output: a = 1 + sum b_i, b = out + sum (out - i) b_i (mod 65521)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint64_t s1 = 0, s2 = 0;
    for (uint32_t i = 4u * lane; i < out; i += 256u) {
        const bool whole = i + 4u <= out;
        const uint32_t v = whole ? *reinterpret_cast<const uint32_t*>(dst + i) : 0u;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t b = whole ? (v >> (8 * j)) & 255u : (i + j < out ? (uint32_t)dst[i + j] : 0u);
            s1 += b;
            s2 += (uint64_t)(out - (i + j)) * b;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s1 += __shfl_xor(s1, o);
        s2 += __shfl_xor(s2, o);
    }
    const uint32_t a1 = (uint32_t)((1 + s1) % 65521u), a2 = (uint32_t)((s2 + (uint64_t)out) % 65521u);
    if (exr_uni(adler) != exr_uni((a2 << 16) | a1)) return false;
    *produced = out;
    return true;
}

// Per compressed chunk (of any image of the call: `file` is the first file's device address, a
// chunk's own at + c.base): decompress (the wave: exr_inflate_wave; RLE: lane 0), then the
// predictor as a workgroup prefix sum. One wave per chunk and a W-byte LDS ring: ~20 KiB of LDS
// with the 16 KiB ring, eight chunks per CU at once.
#ifndef ICX_EXR_WIN
#define ICX_EXR_WIN 16384
#endif
constexpr int kExrWinDev = ICX_EXR_WIN;
constexpr int kUnpackThreads = 64;
__global__ __launch_bounds__(kUnpackThreads) void k_exr_unpack(const uint8_t* __restrict__ file, ExrChunk* __restrict__ ch,
                                                    const int32_t* __restrict__ list, uint8_t* __restrict__ scratch,
                                                    int32_t* __restrict__ fail) {
    __shared__ InfState st;
    __shared__ __attribute__((aligned(16))) uint8_t win[kExrWinDev];  // (dword reads: exr_inflate_wave's flush)
    __shared__ uint32_t part[kUnpackThreads];
    __shared__ int64_t produced;
    ExrChunk& c = ch[list[blockIdx.x]];
    uint8_t* t = scratch + c.scratch;
    const uint8_t* f = file + c.base + c.src;
    bool ok = true;
    int64_t m = 0;
    if (c.mode == 1) {  // (wave-uniform) the whole wave runs the inflate
        ok = exr_inflate_wave<kExrWinDev>(f, c.len, t, c.out_len, &m, st, win);
    } else if (threadIdx.x == 0) {
        ok = exr_unrle(f, c.len, t, c.out_len);
        m = c.out_len;
    }
    if (threadIdx.x == 0) {
        if (!ok) {
            atomicOr(fail + c.img, 1);
            m = 0;
        }
        produced = m;
        c.produced = m;
    }
    __syncthreads();
    m = produced;
    if (m == 0) return;
#ifdef ICX_EXP_NOPRED  // timing experiment only: the inflate alone (output left predicted)
    return;
#endif
    // t'[i] = t[0] + sum_{k=1..i} (t[k] - 128) mod 256: each thread one contiguous segment of whole
    // dwords (t is 16-byte aligned), read and written a dword at a time
    const int64_t seg = ((m + kUnpackThreads - 1) / kUnpackThreads + 3) & ~(int64_t)3;
    const int64_t a = min<int64_t>(m, (int64_t)threadIdx.x * seg), b = min<int64_t>(m, a + seg);
    uint32_t sum = 0;
    int64_t k = a;
    for (; k + 4 <= b; k += 4) sum = __builtin_amdgcn_sad_u8(*reinterpret_cast<const uint32_t*>(t + k), 0u, sum);
    for (; k < b; ++k) sum += t[k];
    sum -= 128u * (uint32_t)(b - a);
    if (a == 0 && b > 0) sum += 128u;  // (t[0] enters as it is)
    part[threadIdx.x] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {  // (64 partial sums: a serial scan is cheap next to the inflate)
        uint32_t run = 0;
        for (int q = 0; q < kUnpackThreads; ++q) {
            const uint32_t v = part[q];
            part[q] = run;
            run += v;
        }
    }
    __syncthreads();
    uint32_t run = part[threadIdx.x];
    for (k = a; k + 4 <= b; k += 4) {
        const uint32_t v = *reinterpret_cast<const uint32_t*>(t + k);
        uint32_t o = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t x = (v >> (8 * j)) & 255u;
            run += k + j == 0 ? x : x - 128u;
            o |= (run & 255u) << (8 * j);
        }
        *reinterpret_cast<uint32_t*>(t + k) = o;
    }
    for (; k < b; ++k) {
        run += k == 0 ? t[0] : (uint32_t)t[k] - 128u;
        t[k] = (uint8_t)run;
    }
}

// A PIZ chunk per workgroup item: the phases of icx_exr_core.h's PIZ section around barriers. The
// Huffman tables live in LDS (code lengths 64 KiB + the 14-bit direct table 64 KiB), then the same
// LDS holds the 64 Ki-entry range LUT; the channel planes are the chunk's scratch. The long-code
// lists (PizWork, 0.9 MB) are not per chunk: the grid is at most kPizSlots workgroups (the LDS
// allows one per CU), each walks the list of chunks with its own slot of a fixed pool, so the
// memory does not grow with the chunk count (a file of many tiny tiles). One thread walks the
// Huffman stream (a serial bit stream), the workgroup does the rest.
constexpr int kPizSlots = 256;
__global__ __launch_bounds__(256) void k_exr_piz(const uint8_t* __restrict__ file, int64_t fsize, ExrChunk* __restrict__ ch,
                                                 const int32_t* __restrict__ list, int nlist, const int32_t* __restrict__ ctype,
                                                 int nch, uint8_t* __restrict__ scratch, PizWork* __restrict__ pool) {
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
    PizWork& w = pool[blockIdx.x];
    for (int item = blockIdx.x; item < nlist; item += gridDim.x) {
        __syncthreads();  // (the previous item is done with the LDS tables and the slot)
        ExrChunk& c = ch[list[item]];
        uint16_t* planes = reinterpret_cast<uint16_t*>(scratch + c.piz_work);
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
}

__global__ __launch_bounds__(256) void k_exr_convert(const uint8_t* __restrict__ file, const uint8_t* __restrict__ scratch,
                                                     const ExrChunk* __restrict__ ch, const int2* __restrict__ map,
                                                     const int32_t* __restrict__ tile_h, const int32_t* __restrict__ ctype,
                                                     const int32_t* __restrict__ coffs, ExrConv cv, float* __restrict__ out) {
    const int64_t npx = (int64_t)cv.w * cv.h;
    for (int64_t px = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; px < npx; px += (int64_t)gridDim.x * blockDim.x)
        reinterpret_cast<uint4*>(out)[px] = exr_pixel(file, scratch, ch, map, tile_h, ctype, coffs, cv, px);
}

// Grow-only device buffers of one context's EXR reads (icx_ctx::exr): one arena carved per call
// into the file copy (host-input reads), scratch, chunk table, maps, work lists, failure flags and
// output, plus pinned failure flags.
struct ExrWs {
    uint8_t* arena = nullptr;
    size_t cap = 0;
    int32_t* h_fail = nullptr;
    size_t h_cap = 0;
    ~ExrWs() {
        if (arena) (void)hipFree(arena);
        if (h_fail) (void)hipHostFree(h_fail);
    }
};
ExrWs* exr_ws_create() { return new ExrWs(); }
void exr_ws_destroy(ExrWs* w) { delete w; }

// n reads in one pass: every file planned on the host (header, offset table, chunk headers), then
// one k_exr_unpack launch over all files' compressed chunks (each workgroup one chunk, so a batch
// keeps thousands in flight where one 2048^2 file has 128), PIZ chunks per file, and a conversion
// per file. d_data[i]: file i on the device (sizes[i] bytes + 16 zero bytes), or nullptr when
// `upload` (then it is copied from data[i] into the arena). d_out[i]: its floats, or nullptr (into
// the arena; *arena_out[i] then says where). codes[i]: tinyexr's code per file. Returns 0, or -100
// with err set (a device failure, or an output buffer too small).
static int exr_batch(hipStream_t st, ExrWs& ws, int n, const uint8_t* const* data, const uint8_t* const* d_data_in,
                     const size_t* sizes, float* const* d_out_in, const size_t* out_floats, int32_t* codes,
                     int32_t* widths, int32_t* heights, float** arena_out, std::string& err) {
    std::vector<ExrPlan> P((size_t)n);
    std::vector<int64_t> cbase((size_t)n, 0), sbase((size_t)n, 0);
    std::vector<ExrChunk> chunks;
    std::vector<int32_t> list;                            // inflate / RLE chunks (global indices)
    std::vector<std::vector<int32_t>> plist((size_t)n);   // PIZ chunks per file (global indices)
    int64_t scr = 0;
    for (int i = 0; i < n; ++i) {
        widths[i] = heights[i] = 0;
        codes[i] = exr_plan(data[i], (int64_t)sizes[i], P[i]);
        if (codes[i] != kExrOk) continue;
        if (d_out_in && d_out_in[i] && (size_t)P[i].w * P[i].h * 4 > out_floats[i]) {
            err = "icx_exr_decode_device: output buffer too small";
            return -100;
        }
        cbase[i] = (int64_t)chunks.size();
        sbase[i] = scr;
        for (size_t k = 0; k < P[i].chunks.size(); ++k) {
            ExrChunk c = P[i].chunks[k];
            c.scratch += scr;
            c.piz_work += scr;
            c.img = i;
            const int32_t g = (int32_t)chunks.size();
            if (c.mode == 3) plist[(size_t)i].push_back(g);
            else if (c.mode != 0) list.push_back(g);
            chunks.push_back(c);
        }
        scr += (P[i].scratch + 255) / 256 * 256;
    }
    // arena layout (256-byte aligned pieces)
    size_t at = 0;
    auto take = [&](size_t bytes) {
        const size_t o = at;
        at += (bytes + 255) & ~(size_t)255;
        return o;
    };
    std::vector<size_t> o_file((size_t)n, 0), o_map((size_t)n), o_th((size_t)n), o_ty((size_t)n), o_of((size_t)n),
        o_plist((size_t)n), o_out((size_t)n, 0);
    std::vector<std::vector<int32_t>> th((size_t)n);
    for (int i = 0; i < n; ++i) {
        if (!d_data_in) o_file[i] = take(sizes[i] + 16);
        if (codes[i] != kExrOk) continue;
        th[i] = P[i].tile_h.empty() ? std::vector<int32_t>(1, 0) : P[i].tile_h;
        o_map[i] = take(sizeof(int2) * std::max<size_t>(1, P[i].map.size()));
        o_th[i] = take(sizeof(int32_t) * th[i].size());
        o_ty[i] = take(sizeof(int32_t) * P[i].nch);
        o_of[i] = take(sizeof(int32_t) * P[i].nch);
        o_plist[i] = take(sizeof(int32_t) * std::max<size_t>(1, plist[i].size()));
        if (!d_out_in || !d_out_in[i]) o_out[i] = take((size_t)P[i].w * P[i].h * 4 * sizeof(float));
    }
    const size_t o_scr = take((size_t)std::max<int64_t>(16, scr));
    size_t npiz = 0;  // PizWork slots: one per k_exr_piz workgroup of the largest launch
    for (int i = 0; i < n; ++i) npiz = std::max(npiz, std::min(plist[i].size(), (size_t)kPizSlots));
    const size_t o_pizw = take(sizeof(PizWork) * std::max<size_t>(1, npiz));
    const size_t o_ch = take(sizeof(ExrChunk) * std::max<size_t>(1, chunks.size()));
    const size_t o_list = take(sizeof(int32_t) * std::max<size_t>(1, list.size()));
    const size_t o_fail = take(sizeof(int32_t) * (size_t)std::max(1, n));
    auto ok = [&](hipError_t e) { return e == hipSuccess; };
    if (at > ws.cap) {
        if (ws.arena) (void)hipFree(ws.arena);
        ws.arena = nullptr;
        ws.cap = 0;
        if (!ok(hipMalloc(&ws.arena, at))) {
            err = "icx_exr_decode: device allocation failed";
            return -100;
        }
        ws.cap = at;
    }
    if ((size_t)std::max(1, n) > ws.h_cap) {
        if (ws.h_fail) (void)hipHostFree(ws.h_fail);
        ws.h_fail = nullptr;
        ws.h_cap = 0;
        if (!ok(hipHostMalloc(&ws.h_fail, sizeof(int32_t) * (size_t)std::max(1, n), hipHostMallocDefault))) {
            ws.h_fail = nullptr;
            err = "icx_exr_decode: pinned allocation failed";
            return -100;
        }
        ws.h_cap = (size_t)std::max(1, n);
    }
    uint8_t* A = ws.arena;
    std::vector<const uint8_t*> dfile((size_t)n);
    for (int i = 0; i < n; ++i) dfile[i] = d_data_in ? d_data_in[i] : A + o_file[i];
    // chunk file bases relative to the first file's device address (k_exr_unpack)
    for (ExrChunk& c : chunks) c.base = (int64_t)(dfile[(size_t)c.img] - dfile[0]);
    uint8_t* d_scr = A + o_scr;
    ExrChunk* d_ch = reinterpret_cast<ExrChunk*>(A + o_ch);
    int32_t* d_list = reinterpret_cast<int32_t*>(A + o_list);
    int32_t* d_fail = reinterpret_cast<int32_t*>(A + o_fail);
    bool good = true;
    // (a file + 16 zero bytes: the PIZ reader loads whole aligned 16-byte words)
    for (int i = 0; i < n && good && !d_data_in; ++i)
        good = ok(hipMemcpyAsync(A + o_file[i], data[i], sizes[i], hipMemcpyHostToDevice, st)) &&
               ok(hipMemsetAsync(A + o_file[i] + sizes[i], 0, 16, st));
    good = good && ok(hipMemcpyAsync(d_ch, chunks.data(), sizeof(ExrChunk) * chunks.size(), hipMemcpyHostToDevice, st)) &&
           ok(hipMemcpyAsync(d_list, list.data(), sizeof(int32_t) * list.size(), hipMemcpyHostToDevice, st)) &&
           ok(hipMemsetAsync(d_fail, 0, sizeof(int32_t) * (size_t)std::max(1, n), st));
    for (int i = 0; i < n && good; ++i) {
        if (codes[i] != kExrOk) continue;
        good = ok(hipMemcpyAsync(A + o_map[i], P[i].map.data(), sizeof(int2) * P[i].map.size(), hipMemcpyHostToDevice, st)) &&
               ok(hipMemcpyAsync(A + o_th[i], th[i].data(), sizeof(int32_t) * th[i].size(), hipMemcpyHostToDevice, st)) &&
               ok(hipMemcpyAsync(A + o_ty[i], P[i].type.data(), sizeof(int32_t) * P[i].nch, hipMemcpyHostToDevice, st)) &&
               ok(hipMemcpyAsync(A + o_of[i], P[i].offs.data(), sizeof(int32_t) * P[i].nch, hipMemcpyHostToDevice, st)) &&
               ok(hipMemcpyAsync(A + o_plist[i], plist[i].data(), sizeof(int32_t) * plist[i].size(), hipMemcpyHostToDevice, st));
    }
    if (!good) {
        err = "icx_exr_decode: device copy failed";
        return -100;
    }
    if (!list.empty() && n > 0)
        hipLaunchKernelGGL(k_exr_unpack, dim3((unsigned)list.size()), dim3(kUnpackThreads), 0, st, dfile[0], d_ch, d_list, d_scr, d_fail);
    for (int i = 0; i < n; ++i) {
        if (codes[i] != kExrOk || plist[i].empty()) continue;
        const unsigned g = (unsigned)std::min(plist[i].size(), (size_t)kPizSlots);
        hipLaunchKernelGGL(k_exr_piz, dim3(g), dim3(256), 0, st, dfile[i], (int64_t)sizes[i], d_ch,
                           reinterpret_cast<const int32_t*>(A + o_plist[i]), (int)plist[i].size(),
                           reinterpret_cast<const int32_t*>(A + o_ty[i]), P[i].nch, d_scr,
                           reinterpret_cast<PizWork*>(A + o_pizw));
    }
    for (int i = 0; i < n; ++i) {
        if (codes[i] != kExrOk) continue;
        const int64_t npx = (int64_t)P[i].w * P[i].h;
        float* out = d_out_in && d_out_in[i] ? d_out_in[i] : reinterpret_cast<float*>(A + o_out[i]);
        if (arena_out) arena_out[i] = out;
        ExrConv cv{};
        cv.w = P[i].w; cv.h = P[i].h; cv.nch = P[i].nch; cv.pds = P[i].pds; cv.tiled = P[i].tiled; cv.tx = P[i].tx;
        cv.ty = P[i].ty; cv.ntx = P[i].ntx; cv.line_order = P[i].line_order;
        for (int k = 0; k < 4; ++k) cv.src[k] = P[i].src[k];
        const unsigned grid = (unsigned)std::min<int64_t>(8192, (npx + 255) / 256);
        hipLaunchKernelGGL(k_exr_convert, dim3(std::max(1u, grid)), dim3(256), 0, st, dfile[i], d_scr, d_ch + cbase[i],
                           reinterpret_cast<const int2*>(A + o_map[i]), reinterpret_cast<const int32_t*>(A + o_th[i]),
                           reinterpret_cast<const int32_t*>(A + o_ty[i]), reinterpret_cast<const int32_t*>(A + o_of[i]), cv,
                           out);
    }
    if (!ok(hipGetLastError()) ||
        !ok(hipMemcpyAsync(ws.h_fail, d_fail, sizeof(int32_t) * (size_t)std::max(1, n), hipMemcpyDeviceToHost, st)) ||
        !ok(hipStreamSynchronize(st))) {
        err = "icx_exr_decode: HIP failure";
        return -100;
    }
    for (int i = 0; i < n; ++i) {
        if (codes[i] != kExrOk) continue;
        if (ws.h_fail[i]) {
            codes[i] = kExrInvalidData;  // "Invalid/Corrupted data found when decoding pixels" (:5512-5524)
        } else {
            widths[i] = P[i].w;
            heights[i] = P[i].h;
        }
    }
    return 0;
}

// One read. Host input (d_file == nullptr): the file is copied to the device, and on success
// *out_rgba = malloc'd w*h*4 floats. Device input: d_file holds the same size bytes plus 16 zero
// bytes, and the floats go to d_out (out_floats of room). Returns a tinyexr code.
int exr_decode(hipStream_t st, ExrWs& ws, const uint8_t* data, size_t size, const uint8_t* d_file, float* d_out,
               size_t out_floats, float** out_rgba, int* width, int* height, std::string& err) {
    int32_t code = 0, w = 0, h = 0;
    float* aout = nullptr;
    float* const outs[1] = {d_out};
    const uint8_t* const ins[1] = {d_file};
    const int rc = exr_batch(st, ws, 1, &data, d_file ? ins : nullptr, &size, d_file ? outs : nullptr, &out_floats, &code,
                             &w, &h, &aout, err);
    if (rc != 0) return rc;
    if (code != kExrOk) return code;
    if (!d_file) {
        const size_t nout = (size_t)w * h * 4 * sizeof(float);
        float* host = (float*)std::malloc(std::max<size_t>(1, nout));
        if (!host || hipMemcpy(host, aout, nout, hipMemcpyDeviceToHost) != hipSuccess) {
            std::free(host);
            err = "icx_exr_decode: host allocation or copy failed";
            return -100;
        }
        *out_rgba = host;
    }
    *width = w;
    *height = h;
    return kExrOk;
}

int exr_decode_batch(hipStream_t st, ExrWs& ws, int n, const uint8_t* const* data, const uint8_t* const* d_data,
                     const size_t* sizes, float* const* d_out, const size_t* out_floats, int32_t* codes, int32_t* widths,
                     int32_t* heights, std::string& err) {
    return exr_batch(st, ws, n, data, d_data, sizes, d_out, out_floats, codes, widths, heights, nullptr, err);
}

int exr_probe(const uint8_t* data, size_t size, int* width, int* height) {
    ExrPlan P;
    const int rc = exr_plan(data, (int64_t)size, P);
    if (width) *width = rc == kExrOk ? P.w : 0;
    if (height) *height = rc == kExrOk ? P.h : 0;
    return rc;
}

}  // namespace icx
