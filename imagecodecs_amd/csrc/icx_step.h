// icx_step.h -- "step tables" for the parallel entropy decoder: one 32-bit entry per
// lookahead window that already says what a lane does next, so one LDS lookup replaces the
// Huffman decode plus NanoJPEG's block-state logic (jpeg_dec.h:643-676) for one or more
// symbols.
//
// A lane peeks x = its next 32 stream bits (MSB first); entry = T.dc[t][x >> (32 - DB)] for a
// DC code (table t = 0, 1) or T.ac[t - 2][x >> (32 - AB)] for an AC code (t = 2, 3). Every
// entry's low half describes the FIRST symbol (the "single" fields):
//   [0:5)   tot1  bits it takes: code + magnitude (no such code: 1, as jpeg_dec.h:646 leaves it)
//   [5:9)   nbx1  magnitude bits (the value is bits [tot1 - nbx1, tot1) of x, MSB first)
//   [9:14)  zad1  coefficient advance: DC 1, AC run + 1 (ZRL 16), EOB and errors 0
//   [14]    eob1  AC symbol 0x00 (:667)
//   [15]    err1  no such code, or an AC symbol of size 0 other than EOB / ZRL (:669)
// The high half depends on the pass (SCAN: guess / count, where only positions and DC values
// matter; WRITE: the write pass, which needs every value):
//   SCAN  [16:21) totm  bits of the longest run of complete symbols that starts with the first
//                       and whose codes lie inside the window (the last one's magnitude bits
//                       may reach past it), ending at the first EOB
//         [21:28) zadm  the run's coefficient advance + eobm; 127 = run unusable
//         [28]    eobm  the run ends with EOB
//         A lane at coefficient cursor z takes the run iff z + zadm <= 64, i.e. the block does
//         not reach coefficient 63 before the run's last symbol (NanoJPEG stops at 63, :671).
//   WRITE [16:20) tot2, [20:24) nbx2, [24:29) zad2, [29] eob2: an optional second symbol
//         (tot2 = 0: none), taken iff z + zad1 + zad2 + eob2 <= 64.
// Flags: [31] SUB -- the first code is longer than the window: the exact single-symbol entry is
// pool[soff[t] + (x >> 16) - sbase[t]]; [30] SEARCH -- beyond what the pool holds (pathological
// tables only): the canonical walk over the image's Huff table (global memory) decides.
#pragma once
#include "icx_jpeg.h"

namespace icx {

constexpr uint32_t kStSub = 1u << 31, kStSearch = 1u << 30, kStSlow = kStSub | kStSearch;

ICX_HD uint32_t st_tot1(uint32_t e) { return e & 31u; }
ICX_HD uint32_t st_nbx1(uint32_t e) { return (e >> 5) & 15u; }
ICX_HD uint32_t st_zad1(uint32_t e) { return (e >> 9) & 31u; }
ICX_HD uint32_t st_eob1(uint32_t e) { return (e >> 14) & 1u; }
ICX_HD uint32_t st_err1(uint32_t e) { return (e >> 15) & 1u; }

// Single-symbol fields of code length L (0: no such code) and symbol s.
ICX_HD uint32_t st_single(int L, int s, bool dc) {
    if (L == 0) return 1u | (1u << 15);
    uint32_t nbx = 0, zad = 0, eob = 0, err = 0;
    if (dc) {
        nbx = (uint32_t)(s & 15);
        zad = 1;
    } else if (s == 0) {
        eob = 1;
    } else if ((s & 15) == 0 && s != 0xF0) {
        err = 1;
    } else {
        nbx = (uint32_t)(s & 15);
        zad = (uint32_t)(s >> 4) + 1;
    }
    const uint32_t tot = (uint32_t)L + nbx;
    return tot | (nbx << 5) | (zad << 9) | (eob << 14) | (err << 15);
}

// SCAN high half of a lone symbol (DC, long codes, errors): the run is the symbol itself.
ICX_HD uint32_t st_scan_lone(uint32_t lo) {
    const uint32_t tot = st_tot1(lo), eob = st_eob1(lo);
    const uint32_t zadm = st_err1(lo) ? 127u : st_zad1(lo) + eob;
    return lo | (tot << 16) | (zadm << 21) | (eob << 28);
}

// Code at the top of a window whose bits past `avail` are unknown (zero here): its length if
// the known bits determine it (canonical codes: L <= avail), else 0; *invalid = the known bits
// already lie past every code.
ICX_HD int st_code_known(const Huff& t, uint32_t win16, int avail, int& s, bool& invalid) {
    const int L = huff_search(t, win16, 1, s);
    invalid = L == 0;
    return (L != 0 && L <= avail) ? L : 0;
}

// Long-code windows of table h for a B-bit first level: [bound[B], end) with `end` rounded up
// to whole B-bit prefixes (a prefix holding both codes and the invalid tail goes to the pool).
ICX_HD uint32_t st_sub_need(const Huff& h, int B) {
    const uint32_t g = 1u << (16 - B);
    const uint32_t end = (h.bound[16] + g - 1) / g * g;
    return end > h.bound[B] ? end - h.bound[B] : 0u;
}

template <int DB, int AB, int POOL, bool SCAN>
struct StepTab {
    static constexpr int kDcBits = DB, kAcBits = AB, kPool = POOL;
    static constexpr bool kScan = SCAN;
    uint32_t dc[2][1 << DB];
    uint32_t ac[2][1 << AB];
    uint32_t pool[POOL];
    uint32_t sbase[4], soff[4], sn[4];  // per table: first pool window, pool offset, pool entries
    uint32_t pad_[4];                   // (16-byte multiple: staged into LDS with 16-byte copies)
    // Per block-in-MCU b (set_bsel): byte offsets in this struct of b's DC and AC first-level
    // tables, and their pool deltas soff[t] - sbase[t]. One LDS read of bsel[b] replaces the
    // table selection arithmetic of every lookup (a 64-bit selector shift and ~12 VALU).
    uint32_t bsel[16][4];  // 16 = kSpecMaxBpm (checked in icx_spec_core.h)

    static ICX_HD int bits(int t) { return t < 2 ? DB : AB; }
    // pool layout: tables in order, each gets what it needs while the pool lasts
    static ICX_HD void layout(const Huff* h, uint32_t (&off)[4], uint32_t (&n)[4]) {
        uint32_t o = 0;
        for (int t = 0; t < 4; ++t) {
            const uint32_t need = st_sub_need(h[t], bits(t));
            n[t] = need <= (uint32_t)POOL - o ? need : 0u;
            off[t] = o;
            o += n[t];
        }
    }
    // first-level entry p of table t
    static ICX_HD uint32_t first(const Huff* h, int t, uint32_t p, const uint32_t (&n)[4]) {
        const int B = bits(t);
        const bool dc = t < 2;
        const Huff& hh = h[t];
        int s = 0;
        bool inv = false;
        const int L = st_code_known(hh, p << (16 - B), B, s, inv);
        if (inv) return SCAN ? st_scan_lone(st_single(0, 0, dc)) : st_single(0, 0, dc);
        if (L == 0) {  // longer than the window: the pool, if it holds this whole prefix
            const uint32_t g = 1u << (16 - B);
            return ((p + 1) * g - hh.bound[B] <= n[t]) ? kStSub : kStSearch;
        }
        const uint32_t lo = st_single(L, s, dc);
        if (dc || st_err1(lo)) return SCAN ? st_scan_lone(lo) : lo;
        if (SCAN) {  // extend the run while the next code lies inside the window
            uint32_t used = st_tot1(lo), zadm = st_zad1(lo), eobm = st_eob1(lo);
            while (!eobm && used < (uint32_t)B) {
                const uint32_t rest = (p << used) & ((1u << B) - 1u);
                int s2 = 0;
                bool inv2 = false;
                const int L2 = st_code_known(hh, rest << (16 - B), B - (int)used, s2, inv2);
                if (L2 == 0) break;
                const uint32_t e2 = st_single(L2, s2, false);
                if (st_err1(e2) || used + st_tot1(e2) > 31u) break;
                used += st_tot1(e2);
                zadm += st_zad1(e2);
                eobm = st_eob1(e2);
            }
            if (used > 31u) return st_scan_lone(lo);
            return lo | (used << 16) | ((zadm + eobm) << 21) | (eobm << 28);
        }
        // WRITE: a second symbol when the first is a coefficient that leaves room in the window
        if (st_eob1(lo) || st_tot1(lo) + 2 > (uint32_t)B) return lo;
        const uint32_t used = st_tot1(lo);
        const uint32_t rest = (p << used) & ((1u << B) - 1u);
        int s2 = 0;
        bool inv2 = false;
        const int L2 = st_code_known(hh, rest << (16 - B), B - (int)used, s2, inv2);
        if (L2 == 0) return lo;
        const uint32_t e2 = st_single(L2, s2, false);
        if (st_err1(e2) || st_tot1(e2) > 15u) return lo;
        return lo | (st_tot1(e2) << 16) | (st_nbx1(e2) << 20) | (st_zad1(e2) << 24) | (st_eob1(e2) << 29);
    }
    // exact single entry of 16-bit window w of table t (pool entries, SEARCH resolution)
    static ICX_HD uint32_t exact(const Huff& hh, int t, uint32_t w) {
        int s = 0;
        const int L = w < 65536u ? huff_search(hh, w, 1, s) : 0;
        const uint32_t lo = st_single(L, s, t < 2);
        return SCAN ? st_scan_lone(lo) : lo;
    }
    // Cooperative build: a workgroup calls fill(h, k) for k = 0 .. entries()-1.
    static ICX_HD int entries() { return 2 * (1 << DB) + 2 * (1 << AB) + POOL + 12; }
    ICX_HD void fill(const Huff* h, int k) {
        uint32_t off[4], n[4];
        layout(h, off, n);
        if (k < 2 * (1 << DB)) { dc[k >> DB][k & ((1 << DB) - 1)] = first(h, k >> DB, (uint32_t)(k & ((1 << DB) - 1)), n); return; }
        k -= 2 * (1 << DB);
        if (k < 2 * (1 << AB)) { ac[k >> AB][k & ((1 << AB) - 1)] = first(h, 2 + (k >> AB), (uint32_t)(k & ((1 << AB) - 1)), n); return; }
        k -= 2 * (1 << AB);
        if (k < POOL) {
            uint32_t e = 0;
            for (int t = 0; t < 4; ++t)
                if ((uint32_t)k >= off[t] && (uint32_t)k < off[t] + n[t]) e = exact(h[t], t, h[t].bound[bits(t)] + (uint32_t)k - off[t]);
            pool[k] = e;
            return;
        }
        k -= POOL;
        if (k < 4) sbase[k] = h[k].bound[bits(k)];
        else if (k < 8) soff[k - 4] = off[k - 4];
        else if (k < 12) sn[k - 8] = n[k - 8];
    }
    // bsel[b] for a block whose DC table is tdc (0, 1) and AC table tac (2, 3); tables come
    // from fill(), so this only needs h (for the pool layout) and the table numbers.
    ICX_HD void set_bsel(const Huff* h, int b, int tdc, int tac) {
        uint32_t off[4], n[4];
        layout(h, off, n);
        const char* base = reinterpret_cast<const char*>(this);
        bsel[b][0] = (uint32_t)(reinterpret_cast<const char*>(&dc[tdc & 1][0]) - base);
        bsel[b][1] = (uint32_t)(reinterpret_cast<const char*>(&ac[(tac - 2) & 1][0]) - base);
        bsel[b][2] = off[tdc & 3] - h[tdc & 3].bound[bits(tdc & 3)];
        bsel[b][3] = off[tac & 3] - h[tac & 3].bound[bits(tac & 3)];
    }
    // First-level entry for block b's DC (dc) or AC code at peek x.
    ICX_HD uint32_t look_b(int b, bool dc, uint32_t x) const {
        const uint32_t off = dc ? bsel[b][0] : bsel[b][1];
        const uint32_t idx = dc ? x >> (32 - DB) : x >> (32 - AB);
        return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(this) + off + 4u * idx);
    }
    // The long-code pool entry of that window (meaningful when the first-level entry is SUB;
    // clamped for lanes that only ride along).
    ICX_HD uint32_t pool_b(int b, bool dc, uint32_t x) const {
        const uint32_t i = (x >> 16) + (dc ? bsel[b][2] : bsel[b][3]);
        return pool[i < (uint32_t)POOL ? i : POOL - 1];
    }
    // Entry of table t for the peek x (32 bits); SUB / SEARCH entries resolved (the caller
    // decides whether to look: a wave-uniform branch on the GPU).
    ICX_HD uint32_t look(int t, uint32_t x) const {
        return t < 2 ? dc[t][x >> (32 - DB)] : ac[t - 2][x >> (32 - AB)];
    }
    ICX_HD uint32_t resolve(int t, uint32_t x, uint32_t e, const Huff* h) const {
        const uint32_t w = x >> 16;
        if (e & kStSub) {
            const uint32_t i = soff[t] + (w - sbase[t]);
            return pool[i < (uint32_t)POOL ? i : POOL - 1];  // (clamped for lanes that only ride along)
        }
        const uint32_t r = exact(h[t], t, w);
#if defined(__HIP_DEVICE_COMPILE__)
        // The walk's global loads complete here (vmcnt(0); lgkmcnt / expcnt untouched): without
        // it the compiler's wait tracking keeps them "in flight" past the join of this rare path
        // and puts an s_waitcnt vmcnt(0) -- for every prefetch and store -- into every lookup.
        __builtin_amdgcn_s_waitcnt(0x0F70);
#endif
        return r;
    }
};

// Guess / count: multi-symbol runs in a 12-bit AC window. Write pass: pairs in a 10-bit AC
// window -- its LDS also holds 512 lanes x 128-byte coefficient slots, so the tables must stay
// under 15.5 KB for two workgroups per CU.
using ScanTab = StepTab<9, 12, 1280, true>;
using WriteTab = StepTab<8, 10, 1280, false>;
#ifdef ICX_EXP_GW8  // timing experiment only: an 11-bit scan table for k_gw_lane's lead
using ScanTab11 = StepTab<9, 11, 1280, true>;
#endif

// One image's step tables in global memory (built by k_step_tabs from Desc::huff).
struct StepSet {
    ScanTab scan;
    WriteTab write;
#ifdef ICX_EXP_GW8
    ScanTab11 scan11;
#endif
};

}  // namespace icx
