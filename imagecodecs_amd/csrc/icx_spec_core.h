// icx_spec_core.h -- per-lane logic of the parallel entropy decoder (icx_spec.hip), kept
// __host__ __device__ so the very same code also runs in the CPU emulator used by the
// tests (tests/emu/spec_emu.cpp). No kernels here.
#pragma once
#include "icx_internal.h"

namespace icx {

ICX_HD uint64_t pack_state(int64_t pos, int b, int z) {
    return ((uint64_t)pos << 16) | ((uint64_t)b << 8) | (uint64_t)z;
}
ICX_HD int64_t st_pos(uint64_t s) { return (int64_t)(s >> 16); }
ICX_HD int st_b(uint64_t s) { return (int)((s >> 8) & 0xFF); }
ICX_HD int st_z(uint64_t s) { return (int)(s & 0xFF); }

// Per-lane marker automaton over kChunk raw bytes. Returns kept-byte count before the
// first end event; *end_at = raw offset of the FF that ends the data (or -1), *end_err =
// whether that end is a syntax error (bad marker / FF at EOF) rather than FF D9.
constexpr int kChunk = kTileBytes / 256;

ICX_HD bool carry_after_ff(const uint8_t* R, int64_t a, int32_t* giveup) {
    int k = 0;
    while (a - 1 - k >= 0 && R[a - 1 - k] == 0xFF) {
        if (++k > 4096) { *giveup = 1; break; }  // pathological FF run: image goes sequential
    }
    return k & 1;
}

// Restart markers met by the unstuff automaton (DRI images): counted, and when `pos` is set,
// recorded in stream order as (byte index in U << 3) | marker number.
struct RstSink {
    int32_t n;      // markers seen
    int64_t ubase;  // U index of out[0] (WRITE)
    int64_t* pos;   // destination array (WRITE), indexed by ord
    int32_t ord, cap;
    ICX_HD void hit(int kept, int m) {
        if (pos && ord < cap) pos[ord] = ((ubase + kept) << 3) | (m & 7);
        ++ord;
        ++n;
    }
};

// Bytes R[a-1 .. a+19) as five little-endian words, read with aligned dword loads (the bytes
// before R are the file's headers, a > 0; the bytes after stay inside the scan, a + 24 <= L).
ICX_HD bool ustf_window(const uint8_t* R, int64_t L, int64_t a, uint32_t (&v)[5]) {
    if (a < 1 || a + kChunk + 8 > L) return false;
    const uintptr_t p = reinterpret_cast<uintptr_t>(R + a - 1);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(R + a - 1 - (p & 3));
    const int sh = (int)(p & 3) * 8;
    uint32_t e[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) e[k] = q[k];
#pragma unroll
    for (int k = 0; k < 5; ++k) v[k] = (uint32_t)((((uint64_t)e[k + 1] << 32) | e[k]) >> sh);
    return true;
}
ICX_HD int win_byte(const uint32_t (&v)[5], int i) {  // i = -1 .. 18 -> R[a+i]
    return (int)((v[(i + 1) >> 2] >> (8 * ((i + 1) & 3))) & 0xFF);
}

template <bool WRITE>
ICX_HD int ustf_chunk(const uint8_t* R, int64_t L, int64_t a, int64_t* end_at, int* end_err,
                                          uint8_t* out, int32_t* giveup, RstSink* rs = nullptr) {
    *end_at = -1;
    *end_err = 0;
    if (a >= L) return 0;
    uint32_t v[5];
    if (ustf_window(R, L, a, v)) {
        uint32_t ff = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t w = (v[k] >> 8) | (v[k + 1] << 24);  // R[a+4k .. a+4k+4)
            const uint32_t x = ~w;                               // a zero byte of x is an FF byte of w
            ff |= (x - 0x01010101u) & ~x & 0x80808080u;
        }
        bool after_ff = win_byte(v, -1) == 0xFF && carry_after_ff(R, a, giveup);
        if (!ff && !after_ff) {  // no marker activity: all 16 bytes kept unchanged
            if (WRITE) {
#pragma unroll
                for (int k = 0; k < 16; ++k) out[k] = (uint8_t)win_byte(v, k);
            }
            return kChunk;
        }
        // the automaton below, on the register window (R[a+16] is byte 16 of the window)
        int kept = 0;
#pragma unroll
        for (int k = 0; k < kChunk; ++k) {
            if (after_ff) { after_ff = false; continue; }
            const int c = win_byte(v, k);
            if (c != 0xFF) {
                if (WRITE) out[kept] = (uint8_t)c;
                ++kept;
                continue;
            }
            const int m = win_byte(v, k + 1);
            if (m == 0x00 || m == 0xFF) {
                if (WRITE) out[kept] = 0xFF;
                ++kept;
                after_ff = true;
            } else if ((m & 0xF8) == 0xD0) {
                if (WRITE) { out[kept] = 0xFF; out[kept + 1] = (uint8_t)m; }
                if (rs) rs->hit(kept, m);
                kept += 2;
                after_ff = true;
            } else {
                *end_at = a + k;
                *end_err = m != 0xD9;
                break;
            }
        }
        return kept;
    }
    bool after_ff = carry_after_ff(R, a, giveup);
    int kept = 0;
    const int64_t b = a + kChunk < L ? a + kChunk : L;
    for (int64_t p = a; p < b; ++p) {
        if (after_ff) { after_ff = false; continue; }  // marker byte, consumed with its FF
        const uint8_t c = R[p];
        if (c != 0xFF) {
            if (WRITE) out[kept] = c;
            ++kept;
            continue;
        }
        if (p + 1 >= L) { *end_at = p; *end_err = 1; break; }  // FF ends the file (:477-478)
        const uint8_t m = R[p + 1];
        if (m == 0x00 || m == 0xFF) {  // :465-467
            if (WRITE) out[kept] = 0xFF;
            ++kept;
            after_ff = true;
        } else if ((m & 0xF8) == 0xD0) {  // RSTn: both bytes enter the bit buffer (:472-475)
            if (WRITE) { out[kept] = 0xFF; out[kept + 1] = m; }
            if (rs) rs->hit(kept, m);
            kept += 2;
            after_ff = true;
        } else {  // D9 ends the data (:468); anything else is a syntax error (:470-471)
            *end_at = p;
            *end_err = m != 0xD9;
            break;
        }
    }
    return kept;
}

struct LdsTables {
    Huff huff[4];
    uint8_t nat_of_zig[64];
};

// Per-image MCU layout in registers (wave-uniform): component of MCU block b (2 bits per
// block) and the DC / AC table of block b (4 bits per block: DC in bits 0-1, AC in 2-3), so
// the code-to-code dependency chain holds a single LDS access (the fast Huffman entry).
struct Sel {
    int bpm;
    uint32_t comps;
    uint64_t tabs;
    ICX_HD int comp(int b) const { return (int)((comps >> (2 * b)) & 3u); }
    ICX_HD int tab(int b, bool dc) const { return (int)((tabs >> (4 * b + (dc ? 0 : 2))) & 3u); }
};
ICX_HD Sel make_sel(const Desc& d) {
    Sel s{d.bpm, 0u, 0ull};
    for (int b = 0; b < d.bpm && b < kSpecMaxBpm; ++b) {
        int sbx, sby;
        const int ci = mcu_block_comp(d, b, sbx, sby);
        s.comps |= (uint32_t)ci << (2 * b);
        s.tabs |= (uint64_t)((d.c[ci].dc_tab & 3) | ((d.c[ci].ac_tab & 3) << 2)) << (4 * b);
    }
    return s;
}

// MSB-first reader over U; bytes at or past ulen read as 0xFF (jpeg_dec.h:451-455).
// Latency hiding: U is fetched in 16-byte chunks with one chunk always in flight -- `A` is
// being drained 32 bits at a time into the 64-bit window `buf`; `B` (the next chunk) was
// requested when A was refilled and stays untouched in registers (no byte swap, no tail
// check) until it becomes A, ~24 codes later, so its load latency is hidden. Loads are
// 16-byte aligned and unconditional: the buffer behind U has >= 16 bytes of slack, and a
// chunk at or past ulen is loaded from chunk 0 and replaced by 0xFF when consumed.
struct Reader {
    const uint8_t* u;
    int64_t ulen, ucap;
    uint64_t buf;      // left-aligned window, nb valid bits
    int nb;
    int na;            // 32-bit words left in A
    uint64_t a0, a1;   // chunk A as a 128-bit left-aligned shift register
    uint4 braw;        // chunk B as loaded (prefetched)
    int64_t next;      // index of the chunk B holds + 1
    int64_t base;      // bit position at init
    uint32_t used;     // bits consumed since init (32-bit loop tests in the lane loops)
    ICX_HD uint4 load(int64_t c) const {
        const int64_t o = c * 16;
        return *reinterpret_cast<const uint4*>(u + (o < ulen ? o : 0));
    }
    // chunk c's raw bytes -> big-endian 128-bit (h, l), bytes at or past ulen forced to 0xFF
    ICX_HD void expand(int64_t c, const uint4& v, uint64_t& h, uint64_t& l) const {
        h = ((uint64_t)__builtin_bswap32(v.x) << 32) | __builtin_bswap32(v.y);
        l = ((uint64_t)__builtin_bswap32(v.z) << 32) | __builtin_bswap32(v.w);
        const int64_t valid = ulen - c * 16;
        if (valid < 16) {
            const int kb = valid <= 0 ? 0 : (int)valid * 8;  // bits kept, 0..120
            h = kb >= 64 ? h : (kb == 0 ? ~0ull : h | (~0ull >> kb));
            l = kb <= 64 ? ~0ull : l | (~0ull >> (kb - 64));
        }
    }
    ICX_HD void refill() {
        if (nb <= 32) {
            buf |= (a0 >> 32) << (32 - nb);
            nb += 32;
            a0 = (a0 << 32) | (a1 >> 32);
            a1 <<= 32;
            if (--na == 0) {
                expand(next - 1, braw, a0, a1);
                na = 4;
#if defined(__HIP_DEVICE_COMPILE__)
                // B's old registers must be dead before its next load is issued: if the load
                // is hoisted above the swap, B lands in other registers and the loop-carried
                // copy back waits for the load (s_waitcnt vmcnt(0) on every code).
                __builtin_amdgcn_sched_barrier(0);
#endif
                braw = load(next++);
            }
        }
    }
    ICX_HD void init(const uint8_t* u_, int64_t ulen_, int64_t bitpos) {
        u = u_;
        ulen = ulen_;
        base = bitpos;
        used = 0;
        const int64_t c = bitpos >> 7;
        expand(c, load(c), a0, a1);
        braw = load(c + 1);
        next = c + 2;
        na = 4;
        buf = 0;
        nb = 0;
        int skip = (int)(bitpos & 127);
        refill();
        refill();
        while (skip >= 32) {
            buf <<= 32;
            nb -= 32;
            skip -= 32;
            refill();
        }
        buf <<= skip;
        nb -= skip;
        refill();
    }
    ICX_HD int64_t pos() const { return base + used; }
    ICX_HD uint32_t peek16() const { return (uint32_t)(buf >> 48); }
    ICX_HD uint32_t take(int n) {
        const uint32_t v = n ? (uint32_t)(buf >> (64 - n)) : 0u;
        buf <<= n;
        nb -= n;
        used += (uint32_t)n;
        return v;
    }
};

enum : int { kUnitOk = 0, kUnitErr = 1 };

// One Huffman code + magnitude bits in the state (b, z); z == 0 expects the DC code.
// On return: *coef = coefficient index written (0 = DC, 1..63 AC, -1 none), *val = value.
// Errors (jpeg_dec.h:646, 667, 669) end the block deterministically so speculative lanes
// keep going; on the true path any error makes the image NJ_SYNTAX_ERROR.
ICX_HD int decode_unit(Reader& r, const LdsTables& T, const Sel& S, int& b, int& z, int& coef,
                                           int32_t& val) {
    // One table read, one variable shift for code + magnitude bits, one shift to consume them;
    // the DC / EOB / ZRL / error / end-of-block cases are selects, not branches (the lanes of a
    // wave take different ones on almost every code). Only codes longer than kFastBits branch.
    const bool dc = z == 0;
    const Huff& H = T.huff[S.tab(b, dc)];
    r.refill();
    const uint32_t win = r.peek16();
    uint32_t e = H.fast[win >> (16 - kFastBits)];
    if (e & kSubFlag) e = H.sub[(e & ~kSubFlag) | (win & ((1u << (16 - kFastBits)) - 1))];  // > 10-bit codes
    int len, sym;
    if (e) {
        len = (int)(e >> 8);
        sym = (int)(e & 0xFF);
    } else {
        len = huff_search(H, win, kFastBits + 1, sym);  // invalid codes, oversized tables
    }
    const bool inv = len == 0;               // no such code: consume one bit (jpeg_dec.h:646)
    const int nbx = inv ? 0 : (sym & 15);
    const int tot = inv ? 1 : len + nbx;     // <= 31 bits, refill left >= 33
    const uint32_t m = 1u << nbx;
    const uint32_t raw = (uint32_t)(r.buf >> (64 - tot)) & (m - 1u);
    const int32_t v = (int32_t)(raw < (m >> 1) ? raw - m + 1u : raw);  // njGetVLC sign extension (:653-654)
    r.buf <<= tot;
    r.nb -= tot;
    r.used += (uint32_t)tot;
    const bool eob = !dc && !inv && sym == 0;                              // :667
    const int c = z + (sym >> 4);
    const bool err = inv || (!dc && !eob && ((nbx == 0 && sym != 0xF0) || c > 63));  // :669, :671
    const bool endb = err || eob || (!dc && c == 63);
    const bool keep = !err && !eob;
    coef = dc ? (inv ? -1 : 0) : (keep ? c : -1);
    val = (keep || (dc && !inv)) ? v : 0;
    const int bn = b + 1 == S.bpm ? 0 : b + 1;
    z = endb ? 0 : (dc ? 1 : c + 1);
    b = endb ? bn : b;
    return err ? kUnitErr : kUnitOk;
}

// ------------------------------------------------------------------------ lane logic
// Guess lane: decode [start, end) from the block-start guess (b0, z=0). Records the first
// kRec MCU-start states (b == 0, z == 0) it passes through (rec, *nrec) and its totals tot = {DC codes,
// DC-diff sums per component} over the whole lane. Returns the exit state: the first code
// boundary at or after `end`.
ICX_HD uint64_t lane_guess(const uint8_t* U, int64_t ulen, const LdsTables& T, const Sel& S, int64_t start, int64_t end,
                           int b0, RecState* rec, int32_t* nrec, int32_t* tot) {
    Reader r;
    r.init(U, ulen, start);
    int b = b0, z = 0, coef;
    int32_t val, cnt = 0, ds[3] = {0, 0, 0};
    int nr = 0;
    const uint32_t span = (uint32_t)(end - start);
    while (r.used < span) {
        if (z == 0 && b == 0 && nr < kRec) {  // MCU starts: the true path passes one per MCU
            RecState& e = rec[nr++];
            e.rel = r.used;
            e.b = b;
            e.cnt = cnt;
            e.ds[0] = ds[0];
            e.ds[1] = ds[1];
            e.ds[2] = ds[2];
        }
        const int ci = S.comp(b);
        const bool dc = z == 0;
        decode_unit(r, T, S, b, z, coef, val);
        if (dc) {
            ++cnt;
            ds[ci] = wadd(ds[ci], val);
        }
    }
    *nrec = nr;
    tot[0] = cnt;
    tot[1] = ds[0];
    tot[2] = ds[1];
    tot[3] = ds[2];
    return pack_state(r.pos(), b, z);
}

// Count lane: decode from the (verified) entry state; as soon as a block-start state equals
// one the guess lane recorded, both decodes coincide from there on, so the lane's totals are
// spliced from the guess lane's and its exit is the guess exit (synced = true). Otherwise the
// whole lane is decoded and its own exit returned.
ICX_HD uint64_t lane_count(const uint8_t* U, int64_t ulen, const LdsTables& T, const Sel& S, uint64_t entry, int64_t start,
                           int64_t end, const RecState* rec, int nrec, const int32_t* tot, uint64_t guess_exit,
                           SubRec& out, bool& synced) {
    Reader r;
    r.init(U, ulen, st_pos(entry));
    int b = st_b(entry), z = st_z(entry), coef;
    int32_t val, cnt = 0, ds[3] = {0, 0, 0};
    int m = 0;
    synced = false;
    const uint32_t off = (uint32_t)(st_pos(entry) - start), span = (uint32_t)(end - start);
    while (off + r.used < span) {
        if (z == 0 && b == 0 && m < nrec) {
            const int64_t rel = off + r.used;
            while (m < nrec && (int64_t)rec[m].rel < rel) ++m;
            if (m < nrec && (int64_t)rec[m].rel == rel) {
                out.cnt = cnt + tot[0] - rec[m].cnt;
                out.ds0 = wadd(ds[0], wsub(tot[1], rec[m].ds[0]));
                out.ds1 = wadd(ds[1], wsub(tot[2], rec[m].ds[1]));
                out.ds2 = wadd(ds[2], wsub(tot[3], rec[m].ds[2]));
                out.mism = 0;
                synced = true;
                return guess_exit;
            }
        }
        const int ci = S.comp(b);
        const bool dc = z == 0;
        decode_unit(r, T, S, b, z, coef, val);
        if (dc) {
            ++cnt;
            ds[ci] = wadd(ds[ci], val);
        }
    }
    const uint64_t ex = pack_state(r.pos(), b, z);
    out.cnt = cnt;
    out.ds0 = ds[0];
    out.ds1 = ds[1];
    out.ds2 = ds[2];
    out.mism = ex != guess_exit;
    return ex;
}

// Serial repair of one unsynchronised lane j (its count pass derived the true exit Y[j]):
// adopt it and re-derive the following lanes until one's exit agrees with its guess exit.
// Returns the last lane touched, or -1 if the walk exceeded `max_walk` lanes.
ICX_HD int64_t repair_walk(const uint8_t* U, int64_t ulen, const LdsTables& T, const Sel& S, int64_t j, int64_t nsub,
                           int64_t sub_bits, uint64_t* X, const uint64_t* Y, const RecState* rec, const int32_t* nrec,
                           const int32_t* tot, SubRec* sub, int max_walk) {
    X[j] = Y[j];
    int64_t k = j + 1;
    for (int steps = 0; k < nsub - 1; ++k, ++steps) {
        if (steps >= max_walk) return -1;
        bool synced;
        SubRec out;
        const uint64_t ex = lane_count(U, ulen, T, S, X[k - 1], k * sub_bits, (k + 1) * sub_bits, rec + k * kRec,
                                       nrec[k], tot + 4 * k, X[k], out, synced);
        sub[k] = out;
        if (ex == X[k]) break;
        X[k] = ex;
    }
    return k;
}

}  // namespace icx
