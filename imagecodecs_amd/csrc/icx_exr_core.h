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

// Wave-uniform inflate on the GPU: all 64 lanes of k_exr_unpack's wave run one chunk's decode, and
// every value read from memory is made wave-uniform (readfirstlane), so the decoder's state sits in
// SGPRs and its loop runs as scalar instructions (one lane doing it alone ran every step as a
// full-wave VALU op); stores are lane 0's. On the host: the identity, and every store.
ICX_HD uint32_t exr_uni(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_readfirstlane(v);
#else
    return v;
#endif
}
ICX_HD bool exr_lane0() {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == 0u;
#else
    return true;
#endif
}

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
    // per length l: one past the last code (first + count) and the sym index of code c (off + c);
    // the device inflate decodes codes longer than kInfFast bits from these (one round of LDS
    // reads instead of one per length)
    uint16_t lim[16];
    int16_t off[16];
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
        w = exr_uni(w);
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
    h.lim[0] = 0;
    h.off[0] = 0;
    for (int l = 1; l < 16; ++l) {
        h.lim[l] = (uint16_t)(next[l] + h.count[l]);
        h.off[l] = (int16_t)(offs[l] - next[l]);
    }
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

template <class In>  // (BitIn, or k_exr_unpack's register-window reader)
ICX_HD int inf_decode(In& in, const InfTab& h) {
    in.fill(16);
    const uint32_t e = exr_uni(h.fast[in.buf & ((1u << kInfFast) - 1u)]);
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
        const int count = (int)exr_uni(h.count[l]);
        if (code - count < first) {
            in.buf >>= l;
            in.cnt -= l;
            return (int)exr_uni(h.sym[index + (code - first)]);
        }
        index += count;
        first = (first + count) << 1;
        code <<= 1;
    }
    return -1;
}

// mz_uncompress(dst, &cap, src, n): true and *produced = output bytes, or false. `win` is a
// W-byte ring of the latest output (match sources; written as the output is). With W below the
// deflate window (the GPU's 16 KiB LDS ring: twice the decoders per CU), a match from farther back
// reads the bytes from dst, where they were stored at least W bytes of output ago.
template <int W = kExrWin>
ICX_HD bool exr_inflate(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap, int64_t* produced, InfState& st,
                        uint8_t* win) {
    static_assert(W >= 16 && (W & (W - 1)) == 0 && W <= kExrWin, "a power-of-two ring");
    *produced = 0;
    if (n < 2) return false;
    const uint32_t cmf = exr_uni(src[0]), flg = exr_uni(src[1]);
    if ((cmf * 256u + flg) % 31u != 0 || (flg & 32u) || (cmf & 15u) != 8) return false;
    BitIn in{src, n, 2, 0ull, 0, 0};
    int64_t out = 0;
    uint32_t a1 = 1, a2 = 0, nm = 0;  // Adler-32, reduced every 5552 bytes (zlib's NMAX)
    uint32_t acc = 0;                 // output bytes gathered into 32-bit stores (dst 4-byte aligned)
    const bool l0 = exr_lane0();
    auto put = [&](uint8_t b) {
        if (l0) win[out & (W - 1)] = b;
        acc |= (uint32_t)b << (8 * (out & 3));
        if ((out & 3) == 3) {
            if (l0) *reinterpret_cast<uint32_t*>(dst + (out & ~(int64_t)3)) = acc;
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
            if (W == kExrWin || dist <= W) {
                for (int j = 0; j < len; ++j) put((uint8_t)exr_uni(win[(out - dist) & (W - 1)]));
            } else {  // from the output (complete 4-byte words: dist > W >= 16), four loads at a time
                int j = 0;
                for (; j + 4 <= len; j += 4) {
                    const uint8_t* q = dst + (out - dist);
                    const uint8_t b0 = (uint8_t)exr_uni(q[0]), b1 = (uint8_t)exr_uni(q[1]), b2 = (uint8_t)exr_uni(q[2]),
                                  b3 = (uint8_t)exr_uni(q[3]);
                    put(b0);
                    put(b1);
                    put(b2);
                    put(b3);
                }
                for (; j < len; ++j) put((uint8_t)exr_uni(dst[out - dist]));
            }
        }
    }
    if (out & 3) {  // the last partial word (dst holds cap bytes: write only what is ours)
        for (int64_t k = out & ~(int64_t)3; k < out; ++k)
            if (l0) dst[k] = (uint8_t)(acc >> (8 * (k & 3)));
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

// ------------------------------------------------------------------------------------------ PIZ
// DecompressPiz (:3228-3375), with TINYEXR_USE_PIZ 1 (the default, :126-128; codecs.cpp:27-29
// leaves it on). The plan (icx_exr_plan.h) checks the chunk's range header (where DecompressPiz
// returns false); the kernel runs the rest in phases around workgroup barriers:
//   init   (all)  zero the code lengths and the direct table, reset the long-code lists, count
//                 the range bitmap's values (maxValue, :3081-3094)
//   unpack (one)  hufUncompress's header and hufUnpackEncTable (:2979-3016, :2466-2519)
//   count  (all)  code lengths per length (hufCanonicalCodeTable's first loop, :2190-2192)
//   build  (one)  the canonical codes in symbol order and hufBuildDecTable (:2181-2220, :2548-2632)
//   decode (one)  hufDecode (:2804-2920) into the channel planes
//   wavelet(all)  wav2Decode (:1995-2109), one level at a time, its 2x2 groups in parallel
//   lut    (all)  reverseLutFromBitmap + applyLut + the line interleave (:3294-3372)
// tinyexr ignores hufUncompress's result (:3317): a Huffman failure keeps what was decoded and
// leaves the rest of the planes 0, and a failed table unpack leaves its raw code lengths for the
// build (no canonical codes: every code is 0). Reads past the end of the file give 0 (tinyexr
// reads the memory after its buffer; only damaged chunks get there).
constexpr int kHufEncSize = 65537;
constexpr int kHufDecBits = 14;
constexpr int kHufDecSize = 1 << kHufDecBits;
constexpr int kPizLens = 65540;  // code-length bytes (kHufEncSize, rounded to words)

// A PIZ chunk's long-code lists (hufBuildDecTable's HufDec::p, kept in insertion order) in global
// memory: per direct-table entry the first / last symbol, per symbol the next one and its code.
struct PizWork {
    int32_t head[kHufDecSize], tail[kHufDecSize];
    int32_t next[kHufEncSize];
    int32_t pad_;
    uint64_t code[kHufEncSize];  // hcode (length | code << 6) of every listed symbol
};

// The file as the decoder's pointers see it: byte i, 0 past the end. One 16-byte aligned load
// per 16 bytes read in order (the device file buffer holds 16 bytes of slack past the end).
struct PizBytes {
    const uint8_t* f;
    int64_t n;
    int64_t blk = -1;
    uint32_t w[4] = {0, 0, 0, 0};
    ICX_HD uint32_t operator()(int64_t i) {
        if (i < 0 || i >= n) return 0u;
        const int64_t b = i >> 4;
        if (b != blk) {
            const uint4 v = reinterpret_cast<const uint4*>(f)[b];
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
            blk = b;
        }
        return (w[(i >> 2) & 3] >> (8 * (i & 3))) & 0xFFu;
    }
};

struct PizHuf {
    int32_t run;      // 0: hufUncompress returned before hufDecode (the planes stay 0)
    int32_t canon;    // the table unpacked (canonical codes); 0: raw lengths, every code 0
    int32_t im, iM;   // symbol range (iM: the run-length code)
    int32_t nbits;    // hufDecode's input size in bits
    int32_t pad_;
    int64_t ptr;      // file offset of the codes
};

ICX_HD uint32_t piz_u32(PizBytes& F, int64_t p) { return F(p) | F(p + 1) << 8 | F(p + 2) << 16 | F(p + 3) << 24; }

// hufUncompress's header + hufUnpackEncTable (one thread). lens[] must be zero (init phase).
ICX_HD PizHuf piz_unpack(PizBytes& F, int64_t p0, int32_t ncomp, uint8_t* lens) {
    PizHuf r{0, 0, 0, 0, 0, 0, 0};
    if (ncomp == 0) return r;
    const int32_t im = (int32_t)piz_u32(F, p0), iM = (int32_t)piz_u32(F, p0 + 4), nbits = (int32_t)piz_u32(F, p0 + 12);
    if (im < 0 || im >= kHufEncSize || iM < 0 || iM >= kHufEncSize) return r;
    const int64_t pc = p0 + 20;                 // *pcode
    const int64_t ni = (int64_t)ncomp - 20;     // nCompressed - (ptr - compressed)
    int64_t p = pc;
    uint64_t c = 0;
    int lc = 0;
    auto bits = [&](int n) -> uint32_t {
        while (lc < n) {
            c = (c << 8) | F(p++);
            lc += 8;
        }
        lc -= n;
        return (uint32_t)(c >> lc) & ((1u << n) - 1u);
    };
    bool ok = true;
    for (int s = im; s <= iM; ++s) {
        if (p - pc >= ni) { ok = false; break; }
        const uint32_t l = bits(6);
        lens[s] = (uint8_t)l;
        if (l == 63) {  // LONG_ZEROCODE_RUN
            if (p - pc > ni) { ok = false; break; }
            const int zr = (int)bits(8) + 6;  // + SHORTEST_LONG_RUN
            if (s + zr > iM + 1) { ok = false; break; }
            for (int k = 0; k < zr; ++k) lens[s++] = 0;
            --s;
        } else if (l >= 59) {  // SHORT_ZEROCODE_RUN
            const int zr = (int)l - 59 + 2;
            if (s + zr > iM + 1) { ok = false; break; }
            for (int k = 0; k < zr; ++k) lens[s++] = 0;
            --s;
        }
    }
    const int64_t ptr = ok ? p : pc;
    // nBits > 8 * (nCompressed - (ptr - compressed)): a ptrdiff_t (64-bit) product
    if ((int64_t)nbits > 8 * ((int64_t)ncomp - (ptr - p0))) return r;
    r.run = 1;
    r.canon = ok;
    r.im = im;
    r.iM = iM;
    r.nbits = nbits;
    r.ptr = ptr;
    return r;
}

// hufCanonicalCodeTable's first code per length, from the counts n[0..58] (in place).
ICX_HD void piz_first_codes(uint64_t* n) {
    uint64_t c = 0;
    for (int i = 58; i > 0; --i) {
        const uint64_t nc = (c + n[i]) >> 1;
        n[i] = c;
        c = nc;
    }
}

// hufBuildDecTable over the canonical codes (one thread), stopping at its first failure as
// tinyexr does (the failure itself is ignored). dec[] zero and w.head / w.tail -1 on entry;
// nextc[l] = the first code of length l (piz_first_codes).
ICX_HD void piz_build(const PizHuf& H, const uint8_t* lens, uint64_t* nextc, uint32_t* dec, PizWork& w) {
    for (int s = H.im; s <= H.iM; ++s) {
        const uint32_t l = lens[s];
        uint64_t h = l;
        if (H.canon && l > 0) h = (uint64_t)l | (nextc[l]++ << 6);
        const int64_t cc = (int64_t)h >> 6;
        const int ln = (int)(h & 63);
        if ((cc >> ln) != 0) return;  // not an l-bit code
        if (ln > kHufDecBits) {       // long code: a secondary entry
            const int64_t e = cc >> (ln - kHufDecBits);
            if (dec[e] >> 24) return;  // a short code is there
            dec[e] += 1;               // (the list's length)
            w.code[s] = h;
            if (w.tail[e] < 0) w.head[e] = s;
            else w.next[w.tail[e]] = s;
            w.tail[e] = s;
        } else if (ln) {
            const int64_t e0 = cc << (kHufDecBits - ln);
            for (int64_t k = 0; k < ((int64_t)1 << (kHufDecBits - ln)); ++k) {
                if (dec[e0 + k] != 0) return;  // a short or a long code is there
                dec[e0 + k] = (uint32_t)ln << 24 | (uint32_t)s;
            }
        }
    }
}

// hufDecode (one thread) into out[0..no); returns the ushorts written (the rest stays 0).
ICX_HD int64_t piz_decode(PizBytes& F, const PizHuf& H, const uint32_t* dec, const uint8_t* lens, const PizWork& w,
                          uint16_t* out, int64_t no) {
    uint64_t c = 0;
    int lc = 0;
    int64_t in = H.ptr;
    const int64_t ie = H.ptr + ((int64_t)H.nbits + 7) / 8;  // (C division: toward zero)
    const int rlc = H.iM;
    int64_t o = 0;
    uint32_t last = 0;
    auto getcode = [&](int po) -> bool {
        if (po == rlc) {
            if (lc < 8) {
                if (in >= ie) return false;
                c = (c << 8) | F(in++);
                lc += 8;
            }
            lc -= 8;
            const int64_t cs = (int64_t)(((int64_t)c >> lc) & 0xFF);
            if (o + cs > no || o < 1) return false;
            for (int64_t k = 0; k < cs; ++k) out[o++] = (uint16_t)last;
        } else if (o < no) {
            out[o++] = (uint16_t)po;
            last = (uint32_t)po;
        } else {
            return false;
        }
        return true;
    };
    while (in < ie) {
        c = (c << 8) | F(in++);
        lc += 8;
        while (lc >= kHufDecBits) {
            const uint32_t e = dec[((int64_t)c >> (lc - kHufDecBits)) & (kHufDecSize - 1)];
            if (e >> 24) {
                lc -= (int)(e >> 24);
                if (!getcode((int)(e & 0xFFFFFF))) return o;
            } else {
                if (e == 0) return o;  // no code
                int32_t sym = w.head[((int64_t)c >> (lc - kHufDecBits)) & (kHufDecSize - 1)];
                uint32_t j = 0;
                for (; j < e; ++j, sym = w.next[sym]) {
                    const uint64_t h = w.code[sym];
                    const int l = (int)(h & 63);
                    while (lc < l && in < ie) {
                        c = (c << 8) | F(in++);
                        lc += 8;
                    }
                    if (lc >= l && ((int64_t)h >> 6) == (((int64_t)c >> (lc - l)) & (int64_t)((1ull << l) - 1))) {
                        lc -= l;
                        if (!getcode(sym)) return o;
                        break;
                    }
                }
                if (j == e) return o;  // not found
            }
        }
    }
    const int i = (8 - H.nbits) & 7;
    c = (uint64_t)((int64_t)c >> i);
    lc -= i;
    while (lc > 0) {
        const uint32_t e = dec[(c << (kHufDecBits - lc)) & (kHufDecSize - 1)];
        if (!(e >> 24)) return o;
        lc -= (int)(e >> 24);
        if (!getcode((int)(e & 0xFFFFFF))) return o;
    }
    (void)lens;
    return o;
}

// wav2Decode's levels: the largest power of two p2 <= min(nx, ny); then (p, p2) = (p2 / 2, p2),
// halving down to p = 1.
ICX_HD int piz_top_p2(int nx, int ny) {
    const int n = nx < ny ? nx : ny;
    int p = 1;
    while (p <= n) p <<= 1;
    return p >> 1;
}

ICX_HD void piz_wdec(bool w14, uint32_t l, uint32_t h, uint32_t& a, uint32_t& b) {
    if (w14) {  // wdec14 (:1831-1844)
        const int32_t ls = (int16_t)l, hs = (int16_t)h;
        const int32_t ai = ls + (hs & 1) + (hs >> 1);
        a = (uint32_t)ai & 0xFFFFu;
        b = (uint32_t)(ai - hs) & 0xFFFFu;
    } else {  // wdec16 (:1871-1879)
        const int32_t m = (int32_t)l, d = (int32_t)h;
        const int32_t bb = (m - (d >> 1)) & 0xFFFF;
        a = (uint32_t)((d + bb - 32768) & 0xFFFF);
        b = (uint32_t)bb;
    }
}

// Items of one wavelet level: the J x K 2x2 groups, then the odd column's J pairs, then the odd
// line's K pairs (each touches its own samples).
ICX_HD int64_t piz_level_items(int nx, int ny, int p, int p2) {
    const int64_t K = nx / p2, J = ny / p2;
    return J * K + ((nx & p) ? J : 0) + ((ny & p) ? K : 0);
}

ICX_HD void piz_level_item(uint16_t* in, int nx, int ox, int ny, int oy, bool w14, int p, int p2, int64_t it) {
    const int64_t K = nx / p2, J = ny / p2;
    const int64_t ox1 = (int64_t)ox * p, oy1 = (int64_t)oy * p, ox2 = (int64_t)ox * p2, oy2 = (int64_t)oy * p2;
    uint32_t i00, i01, i10, i11, a, b;
    if (it < J * K) {
        uint16_t* px = in + (it / K) * oy2 + (it % K) * ox2;
        uint16_t *p01 = px + ox1, *p10 = px + oy1, *p11 = p10 + ox1;
        piz_wdec(w14, *px, *p10, i00, i10);
        piz_wdec(w14, *p01, *p11, i01, i11);
        piz_wdec(w14, i00, i01, a, b);
        *px = (uint16_t)a;
        *p01 = (uint16_t)b;
        piz_wdec(w14, i10, i11, a, b);
        *p10 = (uint16_t)a;
        *p11 = (uint16_t)b;
        return;
    }
    it -= J * K;
    if ((nx & p) && it < J) {  // odd column
        uint16_t* px = in + it * oy2 + K * ox2;
        piz_wdec(w14, *px, px[oy1], a, b);
        px[oy1] = (uint16_t)b;
        *px = (uint16_t)a;
        return;
    }
    if (nx & p) it -= J;
    uint16_t* px = in + J * oy2 + it * ox2;  // odd line
    piz_wdec(w14, *px, px[ox1], a, b);
    px[ox1] = (uint16_t)b;
    *px = (uint16_t)a;
}

// The workgroup phases (thread t of T; tests/emu runs them with t = 0 .. T-1 in turn).
ICX_HD void piz_inc(uint32_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    atomicAdd(p, 1u);
#else
    ++*p;
#endif
}

// init: code lengths and direct table zero, long-code lists empty, planes zero (tinyexr's
// value-initialised tmpBuffer), per-length counts zero.
ICX_HD void piz_init(int t, int T, uint8_t* lens, uint32_t* dec, PizWork& w, uint16_t* planes, int64_t nus, uint32_t* ncnt) {
    for (int i = t; i < kPizLens / 4; i += T) reinterpret_cast<uint32_t*>(lens)[i] = 0;
    for (int i = t; i < kHufDecSize; i += T) {
        dec[i] = 0;
        w.head[i] = -1;
        w.tail[i] = -1;
    }
    for (int64_t i = t; i < nus; i += T) planes[i] = 0;
    for (int i = t; i < 59; i += T) ncnt[i] = 0;
}

// Bit k of the chunk's range bitmap (bytes minNonZero .. maxNonZero from the file, 0 elsewhere;
// value 0 is always in the LUT: reverseLutFromBitmap's i == 0).
ICX_HD uint32_t piz_bitmap_byte(const uint8_t* file, int64_t bitmap, int32_t mnmx, int b) {
    const int mn = mnmx & 0xFFFF, mx = (mnmx >> 16) & 0xFFFF;
    uint32_t v = (b >= mn && b <= mx) ? file[bitmap + (b - mn)] : 0u;
    return b == 0 ? (v | 1u) : v;
}

// Values of the LUT in thread t's range [256 t, 256 t + 256) (T = 256).
ICX_HD uint32_t piz_lut_count(const uint8_t* file, int64_t bitmap, int32_t mnmx, int t) {
    uint32_t n = 0;
    for (int b = 32 * t; b < 32 * t + 32; ++b) n += (uint32_t)__builtin_popcount(piz_bitmap_byte(file, bitmap, mnmx, b));
    return n;
}

// Thread t's LUT entries from `base` on (its range's values in order), and the zero tail past
// the last value (total = values in the LUT).
ICX_HD void piz_lut_fill(const uint8_t* file, int64_t bitmap, int32_t mnmx, int t, uint32_t base, uint16_t* lut) {
    for (int b = 32 * t; b < 32 * t + 32; ++b) {
        const uint32_t v = piz_bitmap_byte(file, bitmap, mnmx, b);
        for (int k = 0; k < 8; ++k)
            if (v >> k & 1u) lut[base++] = (uint16_t)(8 * b + k);
    }
}
ICX_HD void piz_lut_tail(int t, int T, uint32_t total, uint16_t* lut) {
    for (uint32_t k = total + (uint32_t)t; k < 65536u; k += (uint32_t)T) lut[k] = 0;
}

// count: code lengths per length (lengths 1..58; hufCanonicalCodeTable's counts).
ICX_HD void piz_count(int t, int T, const uint8_t* lens, uint32_t* ncnt) {
    for (int i = t; i < kHufEncSize; i += T) {
        const uint32_t l = lens[i];
        if (l > 0 && l <= 58) piz_inc(&ncnt[l]);
    }
}

// One wavelet level (p, p2) over every channel plane: channel k has ctype[k] (HALF: one ushort
// per sample, else two, each its own plane with stride 2), planes one after the other
// (DecompressPiz's channelData, :3323-3352).
ICX_HD void piz_wavelet_level(int t, int T, uint16_t* planes, const int32_t* ctype, int nch, int nx, int ny, bool w14,
                              int p, int p2) {
    const int64_t per = piz_level_items(nx, ny, p, p2);
    int64_t st = 0;
    for (int k = 0; k < nch; ++k) {
        const int sz = ctype[k] == 1 ? 1 : 2;
        for (int j = 0; j < sz; ++j)
            for (int64_t it = t; it < per; it += T) piz_level_item(planes + st + j, nx, sz, ny, nx * sz, w14, p, p2, it);
        st += (int64_t)nx * ny * sz;
    }
}

// applyLut + the line interleave (:3358-3372): ushort i of the pixel data (line v, channel k,
// sample u of its nx * size) = lut[the plane's ushort].
ICX_HD void piz_interleave(int t, int T, const uint16_t* planes, const uint16_t* lut, const int32_t* ctype, int nch, int nx,
                           int ny, uint16_t* out) {
    int64_t line = 0;
    for (int k = 0; k < nch; ++k) line += (int64_t)nx * (ctype[k] == 1 ? 1 : 2);
    const int64_t n = line * ny;
    for (int64_t i = t; i < n; i += T) {
        const int64_t v = i / line;
        int64_t r = i - v * line, st = 0;
        for (int k = 0; k < nch; ++k) {
            const int64_t m = (int64_t)nx * (ctype[k] == 1 ? 1 : 2);
            if (r < m) {
                out[i] = lut[planes[st + v * m + r]];
                break;
            }
            r -= m;
            st += m * ny;
        }
    }
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
