// icx_spec_core.h -- per-lane logic of the parallel entropy decoder (icx_spec.hip), kept
// __host__ __device__ so the very same code also runs in the CPU emulator used by the
// tests (tests/emu/spec_emu.cpp). No kernels here.
#pragma once
#include "icx_internal.h"
#include "icx_step.h"

namespace icx {

ICX_HD uint64_t pack_state(int64_t pos, int b, int z) {
    return ((uint64_t)pos << 16) | ((uint64_t)b << 8) | (uint64_t)z;
}
ICX_HD int64_t st_pos(uint64_t s) { return (int64_t)(s >> 16); }
ICX_HD int st_b(uint64_t s) { return (int)((s >> 8) & 0xFF); }
ICX_HD int st_z(uint64_t s) { return (int)(s & 0xFF); }

// Unstuff helpers (k_ustf_count / k_ustf_write). carry_after_ff: R[a-1] is the end of an FF run;
// whether R[a] is the marker byte of its last FF (odd run: jpeg_dec.h:465-475 pair the bytes up).
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

// ---- coalesced unstuff: 16-byte chunks at 16-byte aligned addresses ----
// A wave's round covers 1 KiB of consecutive aligned chunks, one per lane, so each load is one
// 16-byte access of a contiguous 1 KiB (the 64-byte-per-lane layout of ustf_chunk touched 64
// lines per load instruction). Tiles are cut at aligned addresses: tile t of an image covers
// R-relative bytes [kTileBytes*t - sh, kTileBytes*(t+1) - sh), sh = R's address mod 16, so the
// first chunk of tile 0 starts before the scan (those header bytes are skipped).
ICX_HD int ustf_align(const uint8_t* R) { return (int)(reinterpret_cast<uintptr_t>(R) & 15u); }
ICX_HD int64_t ustf_ntiles(int64_t L, int sh) { return (L + sh + kTileBytes - 1) / kTileBytes; }

struct Ustf16 {
    int kept;        // kept bytes before the chunk's first end event
    int64_t end_at;  // R-relative position of the FF that ends the data (-1: none in the chunk)
    int end_err;     // that end is a syntax error (bad marker / FF at EOF), not FF D9
    uint32_t out[4]; // WRITE: the kept bytes, little-endian, zero-filled
};
ICX_HD bool has_ff(const uint32_t (&D)[4]) {
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t x = ~D[k];  // a zero byte of x is an FF byte of D[k]
        m |= (x - 0x01010101u) & ~x & 0x80808080u;
    }
    return m != 0;
}
// FF bytes ending at R[a-1] among the four bytes before the chunk (pw = R[a-4 .. a) as a
// little-endian dword; a < 1: none): 0..3, or 4 = four or more (the run is walked in memory).
ICX_HD int ff_run4(uint32_t pw, int64_t a) {
    if (a < 1) return 0;
    int k = 0;
    while (k < 4 && ((pw >> (24 - 8 * k)) & 0xFFu) == 0xFFu) ++k;
    return k;
}
// Chunk R[a .. a+16), given as four little-endian dwords D (a may be < 0: bytes before the scan
// are not part of it; bytes at or past L are ignored). nx = R[a+16] when a+16 < L; prun =
// ff_run4 of the bytes before it. NanoJPEG's marker rules (jpeg_dec.h:447-482).
template <bool WRITE>
ICX_HD Ustf16 ustf16(const uint8_t* R, int64_t L, int64_t a, const uint32_t (&D)[4], int nx, int prun,
                     int32_t* giveup, RstSink* rs) {
    Ustf16 o;
    o.end_at = -1;
    o.end_err = 0;
    const bool prev_ff = prun > 0;
    if (a >= 0 && a + 16 < L && prun <= 1) {
        // The common case, stuffing only: every FF of the chunk is followed by 00 (byte 15's by the
        // next chunk's byte 0), and a single FF before the chunk by byte 0 = 00. Then each FF drops
        // the byte after it (the chunk's own bytes: FFs at 0..14; byte 0 for the FF before it), and
        // nothing ends the data. Per dword: FF bytes by a carry-free add, the byte after each by a
        // funnel shift, one AND-OR against the FF bytes' masks, one bit count -- no byte-position
        // masks unless bytes are dropped and written (ustf16's mask tier below computed 00 and FF
        // position masks for every chunk).
        uint32_t bad = prun ? (D[0] & 0xFFu) : 0u, nff = 0u, f[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t w = D[k];
            f[k] = ((w & 0x7F7F7F7Fu) + 0x01010101u) & w & 0x80808080u;  // bit 7 of each FF byte
            const uint32_t nw = k < 3 ? D[k + 1] : (uint32_t)nx;
            const uint32_t after = (uint32_t)((((uint64_t)nw << 32) | w) >> 8);  // byte i: the byte after byte i
            bad |= after & ((f[k] << 1) - (f[k] >> 7));                          // FF bytes' masks
            nff += (uint32_t)__builtin_popcount(k < 3 ? f[k] : f[k] & 0x7FFFFFFFu);
        }
        if (bad == 0u) {
            o.kept = 16 - (int)nff - prun;
            if (WRITE) {
                uint64_t q0 = (uint64_t)D[0] | ((uint64_t)D[1] << 32), q1 = (uint64_t)D[2] | ((uint64_t)D[3] << 32);
                if (nff | (uint32_t)prun) {
                    uint32_t ffm = 0;
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        ffm |= (((f[k] >> 7) & 1u) | ((f[k] >> 14) & 2u) | ((f[k] >> 21) & 4u) | ((f[k] >> 28) & 8u)) << (4 * k);
                    for (uint32_t m = ((ffm << 1) | (uint32_t)prun) & 0xFFFFu; m;) {  // highest dropped byte first
                        const int p = 31 - __builtin_clz(m);
                        m &= ~(1u << p);
                        const int b = 8 * (p & 7);
                        const uint64_t keep = b ? (1ull << b) - 1ull : 0ull;  // bytes below p
                        if (p >= 8) {
                            q1 = (q1 & keep) | ((q1 >> 8) & ~keep);
                        } else {
                            q0 = (q0 & keep) | ((q0 >> 8) & ~keep) | (q1 << 56);
                            q1 >>= 8;
                        }
                    }
                }
                o.out[0] = (uint32_t)q0;
                o.out[1] = (uint32_t)(q0 >> 32);
                o.out[2] = (uint32_t)q1;
                o.out[3] = (uint32_t)(q1 >> 32);
            }
            return o;
        }
    }
    // byte 0 is the marker byte of an FF before the chunk (an odd FF run ends at a-1)
    const bool carry = prev_ff && (prun < 4 ? (prun & 1) != 0 : carry_after_ff(R, a, giveup));
    if (a >= 0 && a + 16 < L) {
        // Stuffing only (every FF is followed by 00 -- all an encoder writes between markers):
        // the bytes after the FFs are dropped, bit masks instead of the byte automaton.
        uint32_t ffm = 0, zm = (nx & 0xFF) == 0 ? 1u << 16 : 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t w = D[k];
            const uint32_t f = ((w & 0x7F7F7F7Fu) + 0x01010101u) & w & 0x80808080u;     // byte == FF
            const uint32_t z = ~(((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w) & 0x80808080u;  // byte == 00
            ffm |= (((f >> 7) & 1u) | ((f >> 14) & 2u) | ((f >> 21) & 4u) | ((f >> 28) & 8u)) << (4 * k);
            zm |= (((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u)) << (4 * k);
        }
        // a carried byte 0 is no FF of its own; 00 / FF there are dropped (an RSTn byte is kept;
        // anything else ended the data in the previous chunk, and this chunk is not counted)
        uint32_t drop0 = 0;
        if (carry) {
            ffm &= ~1u;
            const uint32_t c0 = D[0] & 0xFFu;
            drop0 = (c0 == 0u || c0 == 0xFFu) ? 1u : 0u;
        }
        const uint32_t drop = (ffm << 1) | drop0;  // bit 16: the next chunk's byte 0 (it drops it itself)
        if (((ffm << 1) & ~zm) == 0u) {
            o.kept = 16 - __builtin_popcount(drop & 0xFFFFu);
            if (WRITE) {
                uint64_t q0 = (uint64_t)D[0] | ((uint64_t)D[1] << 32), q1 = (uint64_t)D[2] | ((uint64_t)D[3] << 32);
                for (uint32_t m = drop & 0xFFFFu; m;) {  // highest dropped byte first
                    const int p = 31 - __builtin_clz(m);
                    m &= ~(1u << p);
                    const int b = 8 * (p & 7);
                    const uint64_t keep = b ? (1ull << b) - 1ull : 0ull;  // bytes below p
                    if (p >= 8) {
                        q1 = (q1 & keep) | ((q1 >> 8) & ~keep);
                    } else {
                        q0 = (q0 & keep) | ((q0 >> 8) & ~keep) | (q1 << 56);
                        q1 >>= 8;
                    }
                }
                o.out[0] = (uint32_t)q0;
                o.out[1] = (uint32_t)(q0 >> 32);
                o.out[2] = (uint32_t)q1;
                o.out[3] = (uint32_t)(q1 >> 32);
            }
            return o;
        }
    }
    const int lo = a < 0 ? (int)-a : 0;
    const int hi = a + 16 <= L ? 16 : (int)(L - a);
    uint64_t w0 = 0, w1 = 0;
    int kept = 0;
    auto keep = [&](uint32_t c) {
        if (WRITE) {
            if (kept < 8) w0 |= (uint64_t)c << (8 * kept);
            else w1 |= (uint64_t)c << (8 * (kept - 8));
        }
        ++kept;
    };
    // Byte 0 follows an odd FF run (the previous chunk's last FF reads it as its marker byte):
    // 00 / FF are dropped; an RSTn byte is kept HERE (the previous chunk kept only the FF, so a
    // chunk never keeps more than 16 bytes); anything else ended the data in the previous chunk.
    bool skip = false;  // this byte is the marker byte of the FF before it
    if (lo == 0 && hi > 0 && carry) {
        const uint32_t c0 = D[0] & 0xFFu;
        if ((c0 & 0xF8u) == 0xD0u) keep(c0);
        skip = true;
    }
    bool done = false;
    // bytes by 64-bit shifts of two registers (an indexed D[k >> 2] would go to scratch)
    const uint64_t q0 = (uint64_t)D[0] | ((uint64_t)D[1] << 32), q1 = (uint64_t)D[2] | ((uint64_t)D[3] << 32);
    auto byte = [&](int k) { return (uint32_t)((k < 8 ? q0 >> (8 * k) : q1 >> (8 * (k - 8))) & 0xFFu); };
    for (int k = lo; k < hi && !done; ++k) {
        if (skip) { skip = false; continue; }  // marker byte, consumed with its FF
        const uint32_t c = byte(k);
        if (c != 0xFFu) { keep(c); continue; }
        if (a + k + 1 >= L) { o.end_at = a + k; o.end_err = 1; done = true; continue; }  // FF ends the file (:477-478)
        const uint32_t m = k < 15 ? byte(k + 1) : (uint32_t)nx;
        if (m == 0x00u || m == 0xFFu) {  // :465-467
            keep(0xFFu);
            skip = true;
        } else if ((m & 0xF8u) == 0xD0u) {  // RSTn: both bytes enter the bit buffer (:472-475)
            if (rs) rs->hit(kept, (int)m);
            keep(0xFFu);
            if (k < 15) keep(m);  // (at k = 15 the next chunk keeps the marker byte)
            skip = true;
        } else {  // D9 ends the data (:468); anything else is a syntax error (:470-471)
            o.end_at = a + k;
            o.end_err = m != 0xD9u;
            done = true;
        }
    }
    o.kept = kept;
    if (WRITE) {
        o.out[0] = (uint32_t)w0;
        o.out[1] = (uint32_t)(w0 >> 32);
        o.out[2] = (uint32_t)w1;
        o.out[3] = (uint32_t)(w1 >> 32);
    }
    return o;
}

// Per-image MCU layout in registers (wave-uniform): component of MCU block b (2 bits per
// block) and the DC / AC table of block b (4 bits per block: DC in bits 0-1, AC in 2-3).
struct Sel {
    int bpm;
    uint32_t comps;
    uint64_t tabs;
    ICX_HD int comp(int b) const { return (int)((comps >> (2 * b)) & 3u); }
    // bit b: block (b + 1) mod bpm belongs to another component than block b
    ICX_HD uint32_t chg_mask() const {
        uint32_t m = 0;
        for (int b = 0; b < bpm && b < 16; ++b) m |= (uint32_t)(comp(b) != comp(b + 1 == bpm ? 0 : b + 1)) << b;
        return m;
    }
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

// U as the lane readers see it: the unstuffed data, then 0xFF from ulen up to (ulen/16 + 2)*16
// (written by k_ustf_scan), so chunk u_pad_chunk(ulen) and every chunk before it are readable
// and every byte at or past ulen reads 0xFF (jpeg_dec.h:451-455). Chunks past that index are
// read as that all-0xFF chunk.
ICX_HD uint32_t u_pad_chunk(int64_t ulen) { return (uint32_t)(ulen >> 4) + 1u; }
ICX_HD int64_t u_pad_end(int64_t ulen) { return ((ulen >> 4) + 2) << 4; }

// Restart intervals (DRI): how interval j ends for NanoJPEG, when it started where lane j did and
// its R MCUs decoded without error ending at byte `endbyte` (bits consumed, rounded up: the
// njByteAlign). It then reads 16 bits there and wants FF D0+(j&7) (jpeg_dec.h:707-715): bytes
// past ulen read 0xFF, and a read that fetches the error byte (errpos) is a syntax error whatever
// it returns. Exact: marker j (rs = its record, pos << 3 | number, or -1) is at endbyte, so lane
// j+1 starts where NanoJPEG continues. Error: anything but FF D0+(j&7) -- NanoJPEG stops with a
// syntax error. Elsewhere: FF D0+(j&7) that is not marker j's position (data bytes that look like
// it, or another marker of that number) -- NanoJPEG continues where no lane started.
enum : int { kDriExact = 0, kDriError = 1, kDriElsewhere = 2 };
ICX_HD int dri_end_kind(const uint8_t* U, int64_t ulen, int64_t errpos, int64_t endbyte, int64_t j, int64_t rs) {
    if (errpos <= endbyte + 1) return kDriError;
    const int b0 = endbyte < ulen ? U[endbyte] : 0xFF;
    const int b1 = endbyte + 1 < ulen ? U[endbyte + 1] : 0xFF;
    if (b0 != 0xFF || b1 != (0xD0 | (int)(j & 7))) return kDriError;
    return rs >= 0 && (rs >> 3) == endbyte ? kDriExact : kDriElsewhere;
}

// Wave-wide helpers that are the identity on the host (the CPU emulator runs one lane).
// (__builtin_amdgcn_ballot_w64 on the bool itself: the lane mask a compare leaves in an SGPR pair is
// used as it is; HIP's __any(int) / __ballot(int) first turn the bool into a 0 / 1 VGPR and compare it
// again, two VALU per vote.)
ICX_HD bool wave_any(bool p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_ballot_w64(p) != 0;
#else
    return p;
#endif
}
ICX_HD uint64_t wave_ballot(bool p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_ballot_w64(p);
#else
    return p ? 1u : 0u;
#endif
}
// The lane's bit of a wave-uniform mask as a lane condition: the mask's SGPR pair is the condition
// (no VALU). Lane masks kept as ballots and combined with scalar ANDs stay in SGPRs; a ballot of an
// AND of lane bools is lowered through a VGPR (two VALU).
ICX_HD bool lane_in(uint64_t m) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_inverse_ballot_w64(m);
#else
    return m != 0;
#endif
}

#ifndef ICX_RD_SUBB
#define ICX_RD_SUBB 1
#endif
// MSB-first reader over U (padded as above).
// Latency hiding at the WAVE level: a wave's vmcnt counts every lane's loads in issue order, so a
// lane cannot wait for "its own" older load while a neighbour's newer one is in flight. Loads
// are therefore issued only at slots -- every 4th refill, a point all lanes of a wave reach
// together when they call decode_unit in lockstep -- and their data is first used at the NEXT
// slot, 4 codes later. Between slots a lane draws on registers only: the 64-bit window `buf`,
// chunk A (128 bits, drained 32 bits per refill) and chunk B (expanded at the slot, taken when A
// runs out). A refill takes at most one word and a code at most 31 bits, so 4 refills use at
// most 4 words: with B full after every slot, A never runs dry before the next slot.
struct Reader {
    const uint8_t* u;
    uint32_t cmax;     // chunks past cmax read as chunk cmax (all 0xFF)
    uint32_t next;     // chunk to load at the next slot that finds B taken
    uint64_t buf;      // left-aligned window, nb valid bits
    int nb;
    int na;            // 32-bit words left in A
    uint64_t a0, a1;   // chunk A as a 128-bit left-aligned shift register
    uint64_t b0, b1;   // chunk B, byte-swapped (valid when hb)
    uint4 lraw;        // chunk L, the load in flight (chunk next - 1)
    bool hb;
    uint32_t tick;     // refills since the last slot phase reset
    int64_t base;      // bit position at init
    uint32_t used;     // bits consumed since init (32-bit loop tests in the lane loops)
    ICX_HD uint4 load(uint32_t c) const {
        return gload16(u + (size_t)(c < cmax ? c : cmax) * 16);
    }
    ICX_HD static void expand(const uint4& v, uint64_t& h, uint64_t& l) {
        h = ((uint64_t)__builtin_bswap32(v.x) << 32) | __builtin_bswap32(v.y);
        l = ((uint64_t)__builtin_bswap32(v.z) << 32) | __builtin_bswap32(v.w);
    }
    ICX_HD void slot() {
        if (!hb) {  // B was taken since the last slot: L (issued >= 4 refills ago) becomes B
            expand(lraw, b0, b1);
            hb = true;
            lraw = load(next);
            next = next < cmax ? next + 1 : cmax;
        }
    }
    // Branch-free except for the slot: one word from A into buf when buf runs low, B into A when
    // A runs out.
    ICX_HD void refill() {
        if ((tick++ & 3u) == 0) slot();
        const bool need = nb <= 32;
        const uint64_t w = (a0 >> 32) << ((32 - nb) & 63);
        buf |= need ? w : 0ull;
        nb += need ? 32 : 0;
#if defined(__HIP_DEVICE_COMPILE__) && ICX_RD_SUBB
        {  // na -= need: the compare's lane mask as the borrow (one VALU, not a select and a subtract)
            int32_t r;
            uint64_t c;
            asm("v_subb_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(c) : "v"(na), "s"(wave_ballot(need)));
            na = r;
        }
#else
        na -= need ? 1 : 0;
#endif
        const bool take = na == 0;
        const uint64_t s0 = (a0 << 32) | (a1 >> 32), s1 = a1 << 32;
        a0 = take ? b0 : (need ? s0 : a0);
        a1 = take ? b1 : (need ? s1 : a1);
        na = take ? 4 : na;
        hb = hb && !take;
    }
    // Call where every lane of the wave is about to decode in lockstep: the next refill is a slot.
    ICX_HD void phase() { tick = 0; }
    ICX_HD void init(const uint8_t* u_, int64_t ulen, int64_t bitpos) {
        u = u_;
        cmax = u_pad_chunk(ulen);
        base = bitpos;
        used = 0;
        const int64_t c64 = bitpos >> 7;
        const uint32_t c = c64 < (int64_t)cmax ? (uint32_t)c64 : cmax;
        expand(load(c), a0, a1);
        expand(load(c + 1), b0, b1);
        hb = true;
        lraw = load(c + 2);
        next = c + 3 < cmax ? c + 3 : cmax;
        na = 4;
        buf = 0;
        nb = 0;
        tick = 1;  // no slot during init
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
        tick = 0;
    }
    ICX_HD int64_t pos() const { return base + used; }
    ICX_HD void consume(uint32_t n) {
        buf <<= n;
        nb -= (int)n;
        used += n;
    }
    ICX_HD uint32_t peek16() const { return (uint32_t)(buf >> 48); }
    ICX_HD uint32_t take(int n) {
        const uint32_t v = n ? (uint32_t)(buf >> (64 - n)) : 0u;
        buf <<= n;
        nb -= n;
        used += (uint32_t)n;
        return v;
    }
};

ICX_HD uint32_t ubfe(uint32_t x, uint32_t off, uint32_t w) {  // bits [off, off + w) of x
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_ubfe(x, off, w);
#else
    return w ? (x >> off) & ((1u << w) - 1u) : 0u;
#endif
}
// njGetVLC's sign extension (jpeg_dec.h:653-654) of an nbx-bit magnitude (nbx = 0: 0).
ICX_HD int32_t extend_mag(uint32_t raw, uint32_t nbx) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t mask;  // (1 << nbx) - 1 in one instruction (the compiler emits a shift and a not)
    asm("v_bfm_b32 %0, %1, 0" : "=v"(mask) : "v"(nbx));
#else
    const uint32_t mask = (1u << nbx) - 1u;
#endif
    return (int32_t)(raw <= (mask >> 1) ? raw - mask : raw);
}

// One step-table lookup (icx_step.h) for block b's DC (dc) or AC code: refill, peek, entry
// (table chosen by T.bsel[b]); long codes behind wave-uniform branches whose bodies are selects
// (a wave where no lane needs one skips it): the pool, and the canonical walk for windows the
// pool does not hold (pathological tables only).
template <class Tab>
ICX_HD uint32_t step_lookup(Reader& r, const Tab& T, const Huff* H, const Sel& S, int b, bool dc, uint32_t& x) {
    r.refill();
    x = (uint32_t)(r.buf >> 32);
    uint32_t e = T.look_b(b, dc, x);
    if (wave_any((e & kStSlow) != 0u)) {
        const uint32_t ep = T.pool_b(b, dc, x);
        if (wave_any((e & kStSearch) != 0u)) {
            const uint32_t es = T.resolve(S.tab(b, dc), x, e & kStSearch ? e : kStSub, H);
            e = (e & kStSearch) ? es : e;
        }
        e = (e & kStSub) ? ep : e;
    }
    return e;
}
static_assert(sizeof(ScanTab::bsel) / sizeof(ScanTab::bsel[0]) == kSpecMaxBpm, "bsel covers every block of an MCU");
template <class Tab>
ICX_HD void set_block_sel(Tab& T, const Huff* H, const Sel& S) {
    for (int b = 0; b < kSpecMaxBpm; ++b) {
        const int bb = b < S.bpm ? b : 0;
        T.set_bsel(H, b, S.tab(bb, true), S.tab(bb, false));
    }
}

// SCAN step (guess / count / repair): one lookup -- a run of symbols of the current block, or
// the DC code -- in the state (b, z); z == 0 expects the DC code. *dcv = the DC value when
// the lookup was a DC code (0 for an invalid one). Returns true on a decode error (jpeg_dec.h
// :646, :669, :671), which ends the block deterministically so speculative lanes keep going;
// on the true path an error makes the image NJ_SYNTAX_ERROR.
template <class ScanT>
ICX_HD bool scan_step(Reader& r, const ScanT& T, const Huff* H, const Sel& S, int& b, int& z, int32_t& dcv) {
    const bool dc = z == 0;
    uint32_t x;
    const uint32_t e = step_lookup(r, T, H, S, b, dc, x);
    const uint32_t zm = (e >> 21) & 127u;
    const bool usem = (uint32_t)z + zm <= 64u;
    const uint32_t tot = usem ? (e >> 16) & 31u : st_tot1(e);
    const uint32_t zad = usem ? zm : st_zad1(e);
    const bool eob = usem ? ((e >> 28) & 1u) != 0 : st_eob1(e) != 0;
    const bool e1 = !usem && st_err1(e);
    const uint32_t nbx = st_nbx1(e);
    dcv = extend_mag(ubfe(x, 32u - st_tot1(e), nbx), nbx);
    r.consume(tot);
    const int zn = z + (int)zad;
    const bool err = e1 || (zn > 64 && !eob);
    const bool endb = eob || zn >= 64 || err;
    const int bn = b + 1 == S.bpm ? 0 : b + 1;
    b = endb ? bn : b;
    z = endb ? 0 : zn;
    return err;
}

// WRITE step: one lookup, one symbol or a pair, with their coefficient positions (zig-zag
// order) and values. The DC code's value is the DC diff (v1, c1 = 0). `near_err`: a second
// symbol whose 16-bit peek (:644) would fetch the error byte is not paired, so the error is
// flagged exactly where NanoJPEG's sequential reader meets it.
struct WriteOut {
    int32_t v1, v2;
    int c1, c2;
    bool w1, w2;  // write v1 at c1 / v2 at c2
    bool err;
    // Slot cells for a block assembled in place (k_gw_lane, k_spec_write): v1 goes to n1, then
    // (v2 if w2, else 0) to n2, n2 written first. n1 = c1 when w1, else the unreached cursor z;
    // n2 = c2 when w2, else n1 (the 0 lands where the n1 write then overwrites it). n1 is taken
    // mod 64 where c1 would pass 63, which only a decode error does (the block is then garbage:
    // a discarded speculative one, or a failing image).
    int n1, n2;
};
template <class Tab>
ICX_HD WriteOut write_step(Reader& r, const Tab& T, const Huff* H, const Sel& S, int& b, int& z, bool near_err) {
    const bool dc = z == 0;
    uint32_t x;
    const uint32_t e = step_lookup(r, T, H, S, b, dc, x);
    const uint32_t tot1 = st_tot1(e), nbx1 = st_nbx1(e), zad1 = st_zad1(e);
    const uint32_t tot2 = (e >> 16) & 15u, nbx2 = (e >> 20) & 15u, zad2 = (e >> 24) & 31u, eob2 = (e >> 29) & 1u;
    const bool pair = tot2 != 0u && (uint32_t)z + zad1 + zad2 + eob2 <= 64u && !near_err;
    WriteOut o;
    o.v1 = extend_mag(ubfe(x, 32u - tot1, nbx1), nbx1);
    o.v2 = extend_mag(ubfe(x, 32u - tot1 - tot2, nbx2), nbx2);
    r.consume(tot1 + (pair ? tot2 : 0u));
    o.c1 = z + (int)zad1 - 1;
    o.c2 = o.c1 + (int)zad2;
    o.w1 = !st_eob1(e) && !st_err1(e);
    o.w2 = pair && !eob2;
    {  // (zad1 = 0 exactly for EOB / invalid codes, and a pair's second symbol has zad2 >= 1)
        const int zn1 = z + (int)zad1;
        const int n1 = zn1 - (zad1 != 0u ? 1 : 0);
        o.n1 = n1 & 63;                                  // (past 63 only on a decode error: kept in the slot)
        o.n2 = o.w2 ? zn1 + (int)zad2 - 1 : o.n1;        // (a pair's cell is <= 63 by the pair test)
    }
    const bool eob = pair ? eob2 != 0 : st_eob1(e) != 0;
    const int zn = z + (int)zad1 + (pair ? (int)zad2 : 0);
    o.err = st_err1(e) || (zn > 64 && !eob);
    const bool endb = eob || zn >= 64 || o.err;
    const int bn = b + 1 == S.bpm ? 0 : b + 1;
    b = endb ? bn : b;
    z = endb ? 0 : zn;
    return o;
}

// ------------------------------------------------------------------------ lane logic
// Guess lane: decode [start - lead, end) from the block-start guess (b0, z=0) at start - lead
// (clamped to 0). Records the first kRec MCU-start states (b == 0, z == 0) it passes through at
// or after `start` (rec, *nrec; rel = bits past `start`) and its totals tot = {DC codes, DC-diff
// sums per component} over everything it decoded. Returns the exit state: the first lookup
// boundary at or after `end`. The lead lets the lane resynchronise before `start`, so its first
// recorded state is (almost always) on the true path and the count lane splices at once; only
// differences of the totals are ever used (tot - rec[m]), so the extra prefix cancels.
// Per-component DC sums kept rotated with the current block's component (d0 is block b's, d1 / d2
// the next two in MCU order: NanoJPEG has 1 or 3 components, in order in the MCU), so a DC code
// updates d0 alone and a block end whose next block has another component rotates by one (the
// k_gw_lane scheme; a 3-way select per DC code and per update otherwise). At an MCU start (b = 0)
// they are in component order.
struct DcRot {
    int32_t d0 = 0, d1 = 0, d2 = 0;
    ICX_HD void rotate_if(bool r) {
        const int32_t t = d0;
        d0 = r ? d1 : d0;
        d1 = r ? d2 : d1;
        d2 = r ? t : d2;
    }
    ICX_HD void out(int c, int32_t* s) const {  // component order, the rotation at component c
        s[c] = d0;
        s[c == 2 ? 0 : c + 1] = d1;
        s[c == 0 ? 2 : c - 1] = d2;
    }
};

ICX_HD uint64_t lane_guess(const uint8_t* U, int64_t ulen, const ScanTab& T, const Huff* H, const Sel& S, int64_t start,
                           int64_t end, int b0, RecState* rec, int32_t* nrec, int32_t* tot, int64_t lead = 0) {
    const int64_t s0 = start - lead > 0 ? start - lead : 0;
    Reader r;
    r.init(U, ulen, s0);
    int b = b0, z = 0;
    int32_t val, cnt = 0;
    DcRot ds;
    const uint32_t chgm = S.chg_mask();
    int nr = 0;
    const uint32_t pre = (uint32_t)(start - s0), span = (uint32_t)(end - s0);
    while (r.used < span) {
        if (z == 0 && b == 0 && nr < kRec && r.used >= pre) {  // MCU starts: the true path passes one per MCU
            RecState& e = rec[nr++];
            e.rel = r.used - pre;
            e.b = b;
            e.cnt = cnt;
            e.ds[0] = ds.d0;  // (b = 0: the rotation is at component 0)
            e.ds[1] = ds.d1;
            e.ds[2] = ds.d2;
        }
        const bool dc = z == 0;
        const int bcur = b;
        scan_step(r, T, H, S, b, z, val);
        cnt += dc ? 1 : 0;
        ds.d0 = dc ? wadd(ds.d0, val) : ds.d0;
        ds.rotate_if(z == 0 && ubfe(chgm, (uint32_t)bcur, 1u) != 0u);  // (z = 0: block bcur ended)
    }
    *nrec = nr;
    tot[0] = cnt;
    ds.out(S.comp(b), tot + 1);
    return pack_state(r.pos(), b, z);
}

// Count lane: decode from the (verified) entry state; as soon as a block-start state equals
// one the guess lane recorded, both decodes coincide from there on, so the lane's totals are
// spliced from the guess lane's and its exit is the guess exit (synced = true). Otherwise the
// whole lane is decoded and its own exit returned.
ICX_HD uint64_t lane_count(const uint8_t* U, int64_t ulen, const ScanTab& T, const Huff* H, const Sel& S,
                           uint64_t entry, int64_t start, int64_t end, const RecState* rec, int nrec, const int32_t* tot,
                           uint64_t guess_exit, SubRec& out, bool& synced, uint32_t* bits = nullptr) {
    Reader r;
    r.init(U, ulen, st_pos(entry));
    int b = st_b(entry), z = st_z(entry);
    int32_t val, cnt = 0;
    DcRot ds;  // (all 0: the rotation starts at block b's component)
    const uint32_t chgm = S.chg_mask();
    int m = 0;
    synced = false;
    const uint32_t off = (uint32_t)(st_pos(entry) - start), span = (uint32_t)(end - start);
    while (off + r.used < span) {
        if (z == 0 && b == 0 && m < nrec) {
            const int64_t rel = off + r.used;
            while (m < nrec && (int64_t)rec[m].rel < rel) ++m;
            if (m < nrec && (int64_t)rec[m].rel == rel) {
                int32_t d[3];
                ds.out(0, d);  // (b = 0)
                out.cnt = cnt + tot[0] - rec[m].cnt;
                out.ds0 = wadd(d[0], wsub(tot[1], rec[m].ds[0]));
                out.ds1 = wadd(d[1], wsub(tot[2], rec[m].ds[1]));
                out.ds2 = wadd(d[2], wsub(tot[3], rec[m].ds[2]));
                out.mism = 0;
                synced = true;
                if (bits) *bits = r.used;
                return guess_exit;
            }
        }
        const bool dc = z == 0;
        const int bcur = b;
        scan_step(r, T, H, S, b, z, val);
        cnt += dc ? 1 : 0;
        ds.d0 = dc ? wadd(ds.d0, val) : ds.d0;
        ds.rotate_if(z == 0 && ubfe(chgm, (uint32_t)bcur, 1u) != 0u);
    }
    const uint64_t ex = pack_state(r.pos(), b, z);
    if (bits) *bits = r.used;
    int32_t d[3];
    ds.out(S.comp(b), d);
    out.cnt = cnt;
    out.ds0 = d[0];
    out.ds1 = d[1];
    out.ds2 = d[2];
    out.mism = ex != guess_exit;
    return ex;
}

// Serial repair of one unsynchronised lane j (its count pass derived the true exit Y[j]):
// adopt it and re-derive the following lanes until one's exit agrees with its guess exit.
// Returns the last lane touched, or -1 if the walk exceeded `max_walk` lanes.
ICX_HD int64_t repair_walk(const uint8_t* U, int64_t ulen, const ScanTab& T, const Huff* H, const Sel& S, int64_t j,
                           int64_t nsub, int64_t sub_bits, uint64_t* X, const uint64_t* Y, const RecState* rec,
                           const int32_t* nrec, const int32_t* tot, SubRec* sub, int max_walk) {
    X[j] = Y[j];
    int64_t k = j + 1;
    for (int steps = 0; k < nsub - 1; ++k, ++steps) {
        if (steps >= max_walk) return -1;
        bool synced;
        SubRec out;
        const uint64_t ex = lane_count(U, ulen, T, H, S, X[k - 1], k * sub_bits, (k + 1) * sub_bits, rec + k * kRec,
                                       nrec[k], tot + 4 * k, X[k], out, synced);
        sub[k] = out;
        if (ex == X[k]) break;
        X[k] = ex;
    }
    return k;
}

// ------------------------------------------------------------------ guess-write path
// (icx_spec.hip k_gw*; tests/emu/spec_emu.cpp emu_gw_decode runs the same functions lane by lane)

// Error-byte bounds of a lane reading from bit `e0`, as k_spec_write tests them: NanoJPEG fetches
// bytes to cover a 16-bit peek before each code (jpeg_dec.h:644), so a lookup starting past
// err_peek fails, a second symbol is only paired while its own peek stays clear (err_pair), and
// a lookup ending past err_rel fails. Relative to e0, clamped to 2^30 (no error byte).
struct ErrBounds {
    uint32_t err_rel;
    int32_t err_peek, err_pair;
    ICX_HD void set(int64_t errbits, int64_t e0) {
        const uint32_t kFar = 1u << 30;
        const int64_t rel = errbits == INT64_MAX ? (int64_t)kFar : errbits - e0;
        err_rel = (uint32_t)(rel < 0 ? 0 : (rel > (int64_t)kFar ? (int64_t)kFar : rel));
        err_peek = (int32_t)err_rel - 16;
        err_pair = err_peek - WriteTab::kAcBits;
    }
    ICX_HD bool near(uint32_t u0) const { return (int32_t)u0 > err_pair; }
    ICX_HD bool fail(uint32_t u0, bool step_err, uint32_t u1) const {
        return (int32_t)u0 > err_peek || step_err || u1 > err_rel;
    }
};

// The fewest bits any MCU of the frame can take on a valid stream: per block the shortest DC code
// plus its magnitude bits, plus the AC table's EOB code (a block without EOB holds 63 AC symbols).
// Restart intervals go to the guess-write path only when this is at least 8 (lane_span's exit rule).
ICX_HD int huff_count(const Huff& t, int L) { return (int)((t.bound[L] - t.bound[L - 1]) >> (16 - L)); }
ICX_HD int min_mcu_bits(const Desc& d) {
    // (per Huffman table once: the shortest DC code + its category's bits, the EOB code's length)
    int tmin[8], done = 0, bits = 0;
    for (int b = 0; b < d.bpm && b < kSpecMaxBpm; ++b) {
        int sbx, sby;
        const int ci = mcu_block_comp(d, b, sbx, sby);
        const int td = d.c[ci].dc_tab & 3, ta = 4 + (d.c[ci].ac_tab & 3);
        for (int t : {td, ta}) {
            if (done >> t & 1) continue;
            const Huff& h = d.huff[t & 3];
            int m = 64;
            for (int L = 1; L <= 16 && L < m; ++L) {
                const int n = huff_count(h, L);
                for (int q = 0; q < n; ++q) {
                    const int sym = h.sym[h.first[L] + q];
                    const int v = t < 4 ? L + (sym & 15) : (sym == 0 ? L : 64);
                    m = v < m ? v : m;
                }
            }
            tmin[t] = m;
            done |= 1 << t;
        }
        bits += tmin[td] + tmin[ta];
    }
    return bits;
}

// Lane j's range in U bits and how it ends.
//  * kint == 0 (no restart markers): lanes of sub_bytes, the last to the end of the data; a lane
//    exits at its first block start at or after `end`.
//  * kint > 0 (guess-write over restart intervals): interval m = j / kint runs from the byte after
//    marker m-1 (RS[m-1] >> 3, plus its 2 bytes; byte 0 for m = 0) to marker m (RS[m] >> 3; the last
//    interval to ulen), cut into kint lanes. The interval's first lane starts where NanoJPEG does
//    after the marker (byte-aligned, b = 0, DC predictors 0: synchronised by construction); the
//    others' lead stops at that point (`floor`). NanoJPEG's R MCUs end in the byte before the marker
//    (jpeg_dec.h:707-715 byte-aligns there), and an MCU takes at least 8 bits (k_spec_plan only sends
//    such images here), so the true path's first MCU start at or past bit 8 em - 7 is the
//    interval's end: the interval's last lane exits at the first block start at or after `end`
//    whose block-in-MCU is at most `bmax` (0: an MCU start). Missing markers give degenerate but
//    bounded ranges; k_gw_scan then sends the image to the interval lanes (mode 3).
struct LaneSpan {
    int64_t start, end;  // bits
    int64_t floor;       // a lead starts no earlier
    int bmax;            // the exit's block-in-MCU is at most this
    bool first;          // starts in a known state (b = 0, predictors 0)
};
ICX_HD LaneSpan lane_span(int64_t j, int64_t nsub, int64_t sub_bytes, int64_t ulen, int kint, int64_t nint,
                          const int64_t* RS, int64_t nrst) {
    LaneSpan L;
    if (kint <= 0) {
        L.start = j * sub_bytes * 8;
        L.end = j == nsub - 1 ? ulen * 8 : (j + 1) * sub_bytes * 8;
        L.floor = 0;
        L.bmax = 255;
        L.first = j == 0;
        return L;
    }
    const int64_t m = j / kint, ii = j - m * kint;
    auto at = [&](int64_t k) { return k < nrst ? (RS[k] >> 3) : ulen; };  // marker k's byte (missing: the end)
    const int64_t sm = m == 0 ? 0 : (at(m - 1) + 2 < ulen ? at(m - 1) + 2 : ulen);
    const int64_t em = m + 1 < nint ? (at(m) > sm ? at(m) : sm) : ulen;
    const int64_t len = em - sm, sub = (len + kint - 1) / kint > 0 ? (len + kint - 1) / kint : 1;
    const int64_t st = sm + ii * sub < em ? sm + ii * sub : em;
    L.start = st * 8;
    L.floor = sm * 8;
    L.first = ii == 0;
    if (ii == kint - 1 && m + 1 < nint) {
        L.end = em * 8 - 7 > L.start ? em * 8 - 7 : L.start;
        L.bmax = 0;
    } else {
        L.end = (ii == kint - 1 ? em : (sm + (ii + 1) * sub < em ? sm + (ii + 1) * sub : em)) * 8;
        L.bmax = 255;
    }
    return L;
}

// Count lane (write tables): from the true entry (a block start), store every block through
// `sink` until the first MCU start the guess lane recorded (*m = its index: from there on the guess
// lane's blocks are the true ones) or -- no such state -- the first block start at or after `end`
// whose block-in-MCU is at most bmax (lane_span; *m = -1, *exit = that state). sink.begin(t) readies block t (false: no pool left, the walk
// stops with *m = -3), sink.cell(t, zz, v) stores a coefficient, sink.dc(t, v) the block's
// lane-local DC, cumulative from the entry. Returns the blocks stored, *cds their DC sums, *err
// the first block whose decode failed (INT32_MAX: none; error semantics as k_spec_write's).
template <class Sink>
ICX_HD int32_t gc_walk(const uint8_t* U, int64_t ulen, const WriteTab& TW, const Huff* H, const Sel& S, uint64_t entry,
                       int64_t start, int64_t end, const RecState* rec, int nrec, int64_t errbits, Sink& sink,
                       int32_t* cds, int* m, uint64_t* exit, int32_t* err, int bmax = 255) {
    Reader r;
    r.init(U, ulen, st_pos(entry));
    ErrBounds eb;
    eb.set(errbits, st_pos(entry));
    int b = st_b(entry), z = 0, ci = 0, mi = 0;
    int32_t t = 0;
    cds[0] = cds[1] = cds[2] = 0;
    *err = INT32_MAX;
    for (;;) {
        const bool dc = z == 0;
        if (dc) {
            const int64_t p = r.pos();
            if (b == 0 && mi < nrec) {
                while (mi < nrec && (int64_t)rec[mi].rel < p - start) ++mi;
                if (mi < nrec && (int64_t)rec[mi].rel == p - start) { *m = mi; return t; }
            }
            if (p >= end && b <= bmax) { *m = -1; *exit = pack_state(p, b, 0); return t; }
            ci = S.comp(b);
            if (!sink.begin(t)) { *m = -3; return t; }
        }
        const uint32_t u0 = r.used;
        const WriteOut o = write_step(r, TW, H, S, b, z, eb.near(u0));
        if (eb.fail(u0, o.err, r.used) && *err == INT32_MAX) *err = t;
        if (dc) {
            cds[ci] = wadd(cds[ci], o.v1);
            sink.dc(t, cds[ci]);
        } else if (o.w1) {
            sink.cell(t, o.c1 & 63, o.v1);
        }
        if (o.w2) sink.cell(t, o.c2 & 63, o.v2);
        if (z == 0) ++t;
    }
}

// The image's last blocks when the lanes' blocks end before the frame's (the data stops early,
// no error decided the status): NanoJPEG reads on into the 0xFF padding (jpeg_dec.h:451-455), and
// so does this walk, from the last lane's exit, `need` blocks or up to the first failure. Blocks
// go through `sink` as in gc_walk; *ds their DC sums from the entry; returns the blocks stored and
// *err the first failed one (INT32_MAX: none).
template <class Sink>
ICX_HD int32_t gw_tail(const uint8_t* U, int64_t ulen, const WriteTab& TW, const Huff* H, const Sel& S, uint64_t entry,
                       int64_t need, int64_t errbits, Sink& sink, int32_t* ds, int32_t* err) {
    Reader r;
    r.init(U, ulen, st_pos(entry));
    ErrBounds eb;
    eb.set(errbits, st_pos(entry));
    int b = st_b(entry), z = 0, ci = 0;
    int32_t t = 0;
    ds[0] = ds[1] = ds[2] = 0;
    *err = INT32_MAX;
    while (t < need && *err == INT32_MAX) {
        const bool dc = z == 0;
        if (dc) {
            ci = S.comp(b);
            if (!sink.begin(t)) return -1;
        }
        const uint32_t u0 = r.used;
        const WriteOut o = write_step(r, TW, H, S, b, z, eb.near(u0));
        if (eb.fail(u0, o.err, r.used)) *err = t;
        if (dc) {
            ds[ci] = wadd(ds[ci], o.v1);
            sink.dc(t, ds[ci]);
        } else if (o.w1) {
            sink.cell(t, o.c1 & 63, o.v1);
        }
        if (o.w2) sink.cell(t, o.c2 & 63, o.v2);
        if (z == 0) ++t;
    }
    return t;
}

// A lane's true totals (blocks it owns, DC sums) from its guess and count records.
ICX_HD int32_t gw_lane_total(const GwOut& g, const GcRec& c, const RecState* rec, int32_t* ds) {
    if (c.m == -2) {
        ds[0] = g.ds[0]; ds[1] = g.ds[1]; ds[2] = g.ds[2];
        return g.k;
    }
    if (c.m < 0) {
        ds[0] = c.cds[0]; ds[1] = c.cds[1]; ds[2] = c.cds[2];
        return c.c;
    }
    const RecState& e = rec[c.m];
    for (int q = 0; q < 3; ++q) ds[q] = wadd(c.cds[q], wsub(g.ds[q], e.ds[q]));
    return c.c + g.k - e.cnt;
}
// Block index (lane-relative) of the first true-path decode failure, INT32_MAX if none: the
// count lane's blocks, then the guess lane's after the splice (its blocks before are not on the
// true path).
ICX_HD int32_t gw_lane_err(const GwOut& g, const GcRec& c, const RecState* rec) {
    if (c.m == -2) return g.err;
    if (c.err != INT32_MAX) return c.err;
    if (c.m < 0 || g.err == INT32_MAX) return INT32_MAX;
    const int32_t m0 = rec[c.m].cnt;
    return g.err >= m0 ? c.c + (g.err - m0) : INT32_MAX;
}
// Pool block of guess slot s of a lane: the static region, then the chained overflow chunks.
struct GwSlots {
    int64_t sbase;      // pool block of slot 0
    int32_t S;          // static slots
    int32_t chunk;      // current chunk while walking (-1 before the first)
    int32_t chunk_idx;  // its index in the lane's chain
    ICX_HD int64_t addr(int32_t s, int32_t chunk0, const int32_t* chunk_next) {
        if (s < S) return sbase + s;
        const int32_t q = (s - S) / kGwChunk;
        if (chunk < 0 || q < chunk_idx) { chunk = chunk0; chunk_idx = 0; }
        while (chunk_idx < q && chunk >= 0) { chunk = chunk_next[chunk]; ++chunk_idx; }
        return (int64_t)chunk * kGwChunk + (s - S) % kGwChunk;
    }
};

}  // namespace icx
