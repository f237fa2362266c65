// icx_exr_core.h -- host/device core of the OpenEXR read (icx_exr.hip): the chunk decompressors
// tinyexr runs inside DecodePixelData (/root/reference/tinyexr.h :3631-4281) and its half -> float
// conversion, as __host__ __device__ code (tests/emu/exr_emu.cpp runs the same functions on the
// CPU against the oracle).
//
// * inflate: RFC 1950 / 1951 as miniz's mz_uncompress accepts it (tinyexr.h:1434-1439 with
//   TINYEXR_USE_MINIZ, codecs.cpp:28): zlib header (method 8, check bits, no preset dictionary;
//   the window size is not checked against a non-wrapping output buffer), stored / fixed /
//   dynamic blocks, Adler-32 trailer; an output past `cap` or input that ends first is a failure.
//   Canonical codes are decoded puff-style (per-length counts; codes of one length are
//   consecutive). Match sources come from a 32 KiB window the caller provides (LDS on the GPU).
// * RLE: rleUncompress (:1589-1619) with DecompressRle's checks (:1696-1719).
// * the predictor + even / odd reorder of both (:1469-1500, :1726-1755) are done by the
//   workgroup (prefix sum) and by the byte addressing of the convert kernel (exr_byte).
#pragma once
#include "icx_jpeg.h"  // ICX_HD

namespace icx {

constexpr int kExrWin = 32768;  // deflate window

struct Deflate {  // RFC 1951 §3.2.5-3.2.7 length / distance bases and extra bits, code-length order
    static constexpr uint16_t kLBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                            35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
    static constexpr uint8_t kLExt[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
    static constexpr uint16_t kDBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385,
                                            513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
    static constexpr uint8_t kDExt[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
    static constexpr uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
};

constexpr int kInfFast = 9;  // bits of the direct decoding table

struct InfTab {  // canonical code: number of codes per length, symbols in code order, and a
                 // direct table of the codes up to kInfFast bits (bit-reversed index: the stream
                 // is LSB first; entry = symbol << 4 | length, 0: a longer code)
    uint16_t count[16];
    uint16_t sym[288];
    uint16_t fast[1 << kInfFast];
};

struct InfState {
    InfTab lit, dist;
    uint8_t len[320];
};

struct BitIn {
    const uint8_t* s;
    int64_t n, pos;     // input bytes, next byte to load
    uint64_t buf;       // LSB-first bit buffer
    int cnt;            // bits in buf (past the end of the input: zero bits)
    int64_t over;       // bits loaded past the end of the input
    ICX_HD void fill(int k) {  // k <= 32: four bytes at a time (independent loads)
        if (cnt >= k) return;
        uint32_t w = 0;
        for (int j = 0; j < 4; ++j) {
            if (pos + j < n) w |= (uint32_t)s[pos + j] << (8 * j);
            else over += 8;
        }
        buf |= (uint64_t)w << cnt;
        pos += 4;
        cnt += 32;
    }
    ICX_HD uint32_t bits(int k) {  // k <= 24
        fill(k);
        const uint32_t v = (uint32_t)(buf & ((1ull << k) - 1ull));
        buf >>= k;
        cnt -= k;
        return v;
    }
    // consumed past the end: a read the input could not serve
    ICX_HD bool past_end() const { return over > (int64_t)cnt; }
};

// Builds the decoding table of n code lengths. miniz's rule (tinfl_decompress: total != 65536 with
// more than one used symbol fails): an over-subscribed code fails, an incomplete one only when
// it has two or more symbols.
ICX_HD bool inf_build(InfTab& h, const uint8_t* len, int n) {
    for (int l = 0; l < 16; ++l) h.count[l] = 0;
    for (int s = 0; s < n; ++s) h.count[len[s]]++;
    const int used = n - h.count[0];
    int left = 1;
    for (int l = 1; l < 16; ++l) {
        left = (left << 1) - h.count[l];
        if (left < 0) return false;
    }
    if (left > 0 && used > 1) return false;
    uint16_t offs[16], next[16];
    offs[1] = 0;
    for (int l = 1; l < 15; ++l) offs[l + 1] = (uint16_t)(offs[l] + h.count[l]);
    next[1] = 0;
    for (int l = 1; l < 15; ++l) next[l + 1] = (uint16_t)((next[l] + h.count[l]) << 1);
    for (int i = 0; i < (1 << kInfFast); ++i) h.fast[i] = 0;
    for (int s = 0; s < n; ++s) {
        const int l = len[s];
        if (!l) continue;
        h.sym[offs[l]++] = (uint16_t)s;
        const uint32_t code = next[l]++;
        if (l > kInfFast) continue;
        uint32_t rev = 0;
        for (int b = 0; b < l; ++b) rev |= ((code >> b) & 1u) << (l - 1 - b);
        for (uint32_t i = rev; i < (1u << kInfFast); i += 1u << l) h.fast[i] = (uint16_t)((s << 4) | l);
    }
    return true;
}

ICX_HD int inf_decode(BitIn& in, const InfTab& h) {
    in.fill(16);
    const uint32_t e = h.fast[in.buf & ((1u << kInfFast) - 1u)];
    if (e) {
        in.buf >>= e & 15u;
        in.cnt -= (int)(e & 15u);
        return (int)(e >> 4);
    }
    uint32_t w = (uint32_t)in.buf;  // a code longer than kInfFast bits (or none): by length
    int code = 0, first = 0, index = 0;
    for (int l = 1; l <= 15; ++l) {
        code |= (int)(w & 1u);
        w >>= 1;
        const int count = h.count[l];
        if (code - count < first) {
            in.buf >>= l;
            in.cnt -= l;
            return h.sym[index + (code - first)];
        }
        index += count;
        first = (first + count) << 1;
        code <<= 1;
    }
    return -1;
}

// mz_uncompress(dst, &cap, src, n): true and *produced = output bytes, or false. `win` is a
// kExrWin-byte window (match sources; written as the output is).
ICX_HD bool exr_inflate(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int64_t* produced, InfState& st,
                        uint8_t* win) {
    *produced = 0;
    if (n < 2) return false;
    const uint32_t cmf = src[0], flg = src[1];
    if ((cmf * 256u + flg) % 31u != 0 || (flg & 32u) || (cmf & 15u) != 8) return false;
    BitIn in{src, n, 2, 0ull, 0, 0};
    int64_t out = 0;
    uint32_t a1 = 1, a2 = 0, nm = 0;  // Adler-32, reduced every 5552 bytes (zlib's NMAX)
    uint32_t acc = 0;                 // output bytes gathered into 32-bit stores (dst 4-byte aligned)
    auto put = [&](uint8_t b) {
        win[out & (kExrWin - 1)] = b;
        acc |= (uint32_t)b << (8 * (out & 3));
        if ((out & 3) == 3) {
            *reinterpret_cast<uint32_t*>(dst + (out & ~(int64_t)3)) = acc;
            acc = 0;
        }
        ++out;
        a1 += b;
        a2 += a1;
        if (++nm == 5552) {
            a1 %= 65521u;
            a2 %= 65521u;
            nm = 0;
        }
    };
    int last = 0;
    while (!last) {
        last = (int)in.bits(1);
        const uint32_t type = in.bits(2);
        if (type == 0) {  // stored
            in.bits(in.cnt & 7);
            const uint32_t len = in.bits(16), nlen = in.bits(16);
            if (in.past_end() || (len ^ 0xFFFFu) != nlen) return false;
            if (out + (int64_t)len > cap) return false;
            for (uint32_t k = 0; k < len; ++k) {
                const uint8_t b = (uint8_t)in.bits(8);
                if (in.past_end()) return false;
                put(b);
            }
            continue;
        }
        if (type == 3) return false;
        if (type == 1) {  // fixed codes
            for (int s = 0; s < 288; ++s) st.len[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
            (void)inf_build(st.lit, st.len, 288);
            for (int s = 0; s < 32; ++s) st.len[s] = 5;  // (32 codes, as miniz: 30 and 31 are invalid distances)
            (void)inf_build(st.dist, st.len, 32);
        } else {  // dynamic codes
            const int nlen = (int)in.bits(5) + 257, ndist = (int)in.bits(5) + 1, ncode = (int)in.bits(4) + 4;
            if (nlen > 286 || ndist > 30) return false;
            for (int k = 0; k < 19; ++k) st.len[Deflate::kClOrder[k]] = k < ncode ? (uint8_t)in.bits(3) : 0;
            if (in.past_end() || !inf_build(st.lit, st.len, 19)) return false;
            int k = 0;
            while (k < nlen + ndist) {
                int sym = inf_decode(in, st.lit);
                if (sym < 0 || in.past_end()) return false;
                if (sym < 16) {
                    st.len[k++] = (uint8_t)sym;
                    continue;
                }
                uint8_t v = 0;
                int rep;
                if (sym == 16) {
                    if (k == 0) return false;
                    v = st.len[k - 1];
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
        for (;;) {
            const int sym = inf_decode(in, st.lit);
            if (sym < 0 || in.past_end()) return false;
            if (sym < 256) {
                if (out >= cap) return false;
                put((uint8_t)sym);
                continue;
            }
            if (sym == 256) break;
            const int li = sym - 257;
            if (li >= 29) return false;
            const int len = Deflate::kLBase[li] + (int)in.bits(Deflate::kLExt[li]);
            const int di = inf_decode(in, st.dist);
            if (di < 0 || di >= 30) return false;
            const int64_t dist = Deflate::kDBase[di] + (int64_t)in.bits(Deflate::kDExt[di]);
            if (in.past_end() || dist > out) return false;
            if (out + len > cap) return false;
            for (int j = 0; j < len; ++j) put(win[(out - dist) & (kExrWin - 1)]);
        }
    }
    if (out & 3) {  // the last partial word (dst holds cap bytes: write only what is ours)
        for (int64_t k = out & ~(int64_t)3; k < out; ++k) dst[k] = (uint8_t)(acc >> (8 * (k & 3)));
    }
    a1 %= 65521u;
    a2 %= 65521u;
    in.bits(in.cnt & 7);  // to a byte boundary
    uint32_t adler = 0;
    for (int k = 0; k < 4; ++k) adler = (adler << 8) | in.bits(8);
    if (in.past_end()) return false;
    if (adler != ((a2 << 16) | a1)) return false;
    *produced = out;
    return true;
}

// DecompressRle's run decode (the byte transform follows): true when exactly `cap` bytes come out.
ICX_HD bool exr_unrle(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap) {
    if (n <= 2) return false;
    int64_t in_len = n, max_len = cap, i = 0, o = 0;
    while (in_len > 0) {
        const int c = (int)(int8_t)src[i++];
        if (c < 0) {
            const int cnt = -c;
            in_len -= cnt + 1;
            max_len -= cnt;
            if (max_len < 0 || in_len < 0) return false;
            for (int k = 0; k < cnt; ++k) dst[o++] = src[i++];
        } else {
            in_len -= 2;
            max_len -= c + 1;
            if (max_len < 0 || in_len < 0) return false;
            const uint8_t b = src[i++];
            for (int k = 0; k <= c; ++k) dst[o++] = b;
        }
    }
    return o == cap;
}

// tinyexr's half_to_float (:966-987), bit for bit.
ICX_HD uint32_t exr_half_bits(uint32_t h) {
    uint32_t o = (h & 0x7fffu) << 13;
    const uint32_t e = 0x0f800000u & o;
    o += (127u - 15u) << 23;
    if (e == 0x0f800000u) {
        o += (128u - 16u) << 23;
    } else if (e == 0) {
        o += 1u << 23;
        const float f = __builtin_bit_cast(float, o) - __builtin_bit_cast(float, 113u << 23);
        o = __builtin_bit_cast(uint32_t, f);
    }
    return o | ((h & 0x8000u) << 16);
}

}  // namespace icx
