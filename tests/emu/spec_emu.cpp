// spec_emu.cpp -- TEST-ONLY CPU emulator of the parallel entropy decoder (icx_spec.hip).
// It runs the kernels' per-lane logic (imagecodecs_amd/csrc/icx_spec_core.h, the same
// __host__ __device__ code the GPU executes) lane by lane on the host, mirroring each
// kernel's bookkeeping, so the algorithm can be checked on a machine without a GPU.
// Never linked into libicx.so.
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "../../imagecodecs_amd/csrc/icx_spec_core.h"

using namespace icx;

// The unstuff pass as k_ustf_count / k_ustf_scan / k_ustf_write compute it, with tiles cut at
// alignment `sh` (the GPU uses R's address mod 16): per tile, four rounds of 64 lanes x 16-byte
// chunks, each round's kept bytes before its first end event. Returns ulen; U gets the data plus
// the 0xFF reader padding; rst (optional) gets the restart-marker records in stream order.
static int64_t emu_unstuff(const uint8_t* R, int64_t L, int sh, std::vector<uint8_t>& U, int64_t& errpos,
                           int32_t& giveup, std::vector<int64_t>* rst) {
    const int64_t ntiles = ustf_ntiles(L, sh);
    struct Lane { Ustf16 u; int n; int64_t a; uint32_t D[4]; int nx; int pf; };
    auto round = [&](int64_t t0, int r, Lane* ln) {
        for (int l = 0; l < 64; ++l) {
            Lane& x = ln[l];
            x.a = t0 + r * 1024 + l * 16;
            for (int k = 0; k < 4; ++k) {
                x.D[k] = 0;
                for (int b = 0; b < 4; ++b) {
                    const int64_t p = x.a + 4 * k + b;
                    if (p >= 0 && p < L) x.D[k] |= (uint32_t)R[p] << (8 * b);
                }
            }
            x.nx = x.a + 16 < L && x.a + 16 >= 0 ? R[x.a + 16] : 0;
            uint32_t pw = 0;  // R[a-4 .. a) (bytes before the scan: not FF here, unused by ff_run4)
            for (int b = 0; b < 4; ++b) {
                const int64_t p = x.a - 4 + b;
                if (p >= 0 && p < L) pw |= (uint32_t)R[p] << (8 * b);
            }
            x.pf = ff_run4(pw, x.a);
            RstSink rs{0, 0, nullptr, 0, 0};
            x.u = ustf16<true>(R, L, x.a, x.D, x.nx, x.pf, &giveup, &rs);
            x.n = rs.n;
        }
        int64_t e = INT64_MAX;
        for (int l = 0; l < 64; ++l) if (ln[l].u.end_at >= 0 && ln[l].u.end_at < e) e = ln[l].u.end_at;
        return e;
    };
    auto before = [](const Lane& x, int64_t e) { return x.u.end_at >= 0 ? x.u.end_at <= e : x.a < e; };
    std::vector<TileRec> tiles(ntiles);
    Lane ln[64];
    for (int64_t t = 0; t < ntiles; ++t) {
        const int64_t t0 = t * kTileBytes - sh;
        int kept = 0, nrst = 0, err = 0;
        int64_t tend = -1;
        for (int r = 0; r < kTileBytes / 1024 && t0 + r * 1024 < L; ++r) {
            const int64_t e = round(t0, r, ln);
            for (int l = 0; l < 64; ++l)
                if (before(ln[l], e)) { kept += ln[l].u.kept; nrst += ln[l].n; }
            if (e != INT64_MAX) {
                for (int l = 0; l < 64; ++l) if (ln[l].u.end_at == e) err = ln[l].u.end_err;
                tend = e;
                break;
            }
        }
        tiles[t] = TileRec{kept, err, tend, nrst, 0};
    }
    int64_t fe = -1;
    for (int64_t t = 0; t < ntiles; ++t)
        if (tiles[t].end_at >= 0) { fe = t; break; }
    int64_t ulen = 0;
    for (int64_t t = 0; t < ntiles; ++t)
        if (fe < 0 || t <= fe) ulen += tiles[t].kept;
    errpos = (fe >= 0 && tiles[fe].end_err) ? ulen : INT64_MAX;
    U.assign((size_t)u_pad_end(ulen) + 64, 0xFF);  // reader padding (icx_spec_core.h u_pad_end)
    int64_t o = 0;
    for (int64_t t = 0; t < ntiles && o < ulen; ++t) {
        const int64_t t0 = t * kTileBytes - sh;
        for (int r = 0; r < kTileBytes / 1024 && t0 + r * 1024 < L; ++r) {
            const int64_t e = round(t0, r, ln);
            for (int l = 0; l < 64; ++l) {
                if (!before(ln[l], e)) continue;
                if (rst && ln[l].n) {
                    std::vector<int64_t> tmp(8);
                    RstSink rs{0, o, tmp.data(), 0, 8};
                    (void)ustf16<false>(R, L, ln[l].a, ln[l].D, ln[l].nx, ln[l].pf, &giveup, &rs);
                    for (int k = 0; k < rs.n && k < 8; ++k) rst->push_back(tmp[k]);
                }
                for (int k = 0; k < ln[l].u.kept; ++k)
                    if (o + k < ulen) U[o + k] = (uint8_t)(ln[l].u.out[k >> 2] >> (8 * (k & 3)));
                o += ln[l].u.kept;
            }
            if (e != INT64_MAX) break;
        }
    }
    return ulen;
}

// guess-lane lead in bits: k_spec_guess's kGuessLead, or ICX_GUESS_LEAD as for libicx.so
static int64_t g_lead = std::getenv("ICX_GUESS_LEAD") ? std::atoll(std::getenv("ICX_GUESS_LEAD")) : kGuessLead;
static std::vector<uint32_t>* g_count_bits = nullptr;  // emu_count_study: bits each count lane decoded

extern "C" {

void emu_set_lead(int64_t lead) { g_lead = lead; }

// Returns: 0 parallel path finished (status in *status), 1 image would fall back to the
// sequential kernel, 2 not eligible for the parallel path (status = header result).
// coef: nblocks*64 int16 natural order; dc: nblocks int32 absolute. *nblocks = total blocks.
int emu_spec_decode(const uint8_t* file, int64_t size, int sub_bytes, int16_t* coef, int32_t* dc,
                    int64_t cap_blocks, int64_t* nblocks, int32_t* status, int64_t* stats /*[4]*/) {
    auto dp = std::make_unique<Desc>();
    Desc& d = *dp;
    *status = parse_headers(file, size, d);
    *nblocks = 0;
    const int64_t scan_len = d.size - d.scan_off;
    if (!(d.status == kPending && d.restart == 0 && d.nc >= 1 && d.bpm <= kSpecMaxBpm && scan_len > 0)) return 2;
    const int64_t total = (int64_t)d.mbw * d.mbh * d.bpm;
    *nblocks = total;
    if (total > cap_blocks) return 2;
    const uint8_t* R = file + d.scan_off;
    // ---- unstuff (k_ustf_count / k_ustf_scan / k_ustf_write)
    std::vector<uint8_t> U;
    int64_t errpos;
    int32_t giveup = 0;
    const int64_t ulen = emu_unstuff(R, scan_len, ustf_align(R), U, errpos, giveup, nullptr);
    if (giveup) { stats[1]++; return 1; }
    // ---- tables (k_step_tabs)
    auto SSp = std::make_unique<StepSet>();
    StepSet& SS = *SSp;
    for (int k = 0; k < ScanTab::entries(); ++k) SS.scan.fill(d.huff, k);
    for (int k = 0; k < WriteTab::entries(); ++k) SS.write.fill(d.huff, k);
    set_block_sel(SS.scan, d.huff, make_sel(d));
    set_block_sel(SS.write, d.huff, make_sel(d));
    const ScanTab& T = SS.scan;
    const WriteTab& TW = SS.write;
    const Huff* H = d.huff;
    const int64_t S = sub_bytes;
    const int64_t nsub = ulen > 0 ? (ulen + S - 1) / S : 1;
    const Sel SL = make_sel(d);
    // ---- guess (k_spec_guess)
    const int64_t sb = S * 8;
    std::vector<uint64_t> X(nsub, 0), Y(nsub, 0);
    std::vector<RecState> rec(nsub * kRec);
    std::vector<int32_t> nrec(nsub, 0), tot(nsub * 4, 0);
    for (int64_t j = 0; j + 1 < nsub; ++j)
        X[j] = lane_guess(U.data(), ulen, T, H, SL, j * sb, (j + 1) * sb, 0, rec.data() + j * kRec, &nrec[j], &tot[4 * j],
                          g_lead);
    // ---- count (k_spec_count)
    std::vector<SubRec> sub(nsub, SubRec{0, 0, 0, 0, 0});
    std::vector<int32_t> queue;
    int64_t synced_lanes = 0;
    for (int64_t j = 0; j + 1 < nsub; ++j) {
        const uint64_t entry = j == 0 ? pack_state(0, 0, 0) : X[j - 1];
        bool synced;
        uint32_t cbits = 0;
        Y[j] = lane_count(U.data(), ulen, T, H, SL, entry, j * sb, (j + 1) * sb, rec.data() + j * kRec, nrec[j],
                          &tot[4 * j], X[j], sub[j], synced, &cbits);
        if (g_count_bits) g_count_bits->push_back(cbits);
        synced_lanes += synced;
        if (sub[j].mism) queue.push_back((int32_t)j);
    }
    stats[2] += (int64_t)queue.size();
    stats[3] += synced_lanes;
    // ---- repair (k_spec_repair)
    if ((int)queue.size() > kMaxRepair) { stats[1]++; return 1; }
    int64_t done = -1;
    for (int32_t j : queue) {
        if (j <= done) continue;
        done = repair_walk(U.data(), ulen, T, H, SL, j, nsub, sb, X.data(), Y.data(), rec.data(), nrec.data(), tot.data(),
                           sub.data(), 64);
        if (done < 0) { stats[1]++; return 1; }
    }
    // ---- scan (k_spec_scan)
    std::vector<LaneEntry> ent(nsub);
    int64_t G = 0;
    int32_t P[3] = {0, 0, 0};
    for (int64_t j = 0; j < nsub; ++j) {
        ent[j] = LaneEntry{G, P[0], P[1], P[2], 0};
        if (j + 1 < nsub) {
            G += sub[j].cnt;
            P[0] = wadd(P[0], sub[j].ds0);
            P[1] = wadd(P[1], sub[j].ds1);
            P[2] = wadd(P[2], sub[j].ds2);
        }
    }
    // ---- write (k_spec_write)
    bool anybad = false;
    std::memset(coef, 0, sizeof(int16_t) * 64 * total);
    for (int64_t j = 0; j < nsub; ++j) {
        const uint64_t entry = j == 0 ? pack_state(0, 0, 0) : X[j - 1];
        const bool last = j == nsub - 1;
        const int64_t limit = last ? INT64_MAX : st_pos(X[j]);
        Reader r;
        r.init(U.data(), ulen, st_pos(entry));
        int b = st_b(entry), z = st_z(entry);
        while (z != 0) (void)write_step(r, TW, H, SL, b, z, false);
        int32_t pred[3] = {ent[j].p0, ent[j].p1, ent[j].p2};
        const int64_t errbits = errpos == INT64_MAX ? INT64_MAX : errpos * 8;
        bool bad = false;
        int64_t bi = ent[j].G;
        int ci = 0;
        while (bi < total) {  // k_spec_write's flat loop
            const bool dcl = z == 0;
            if (dcl) {
                if (r.pos() >= limit) break;
                ci = SL.comp(b);
            }
            const int64_t p0 = r.pos();
            if (p0 + 16 > errbits) bad = true;
            const WriteOut o = write_step(r, TW, H, SL, b, z, p0 + 16 + WriteTab::kAcBits > errbits);
            if (o.err || r.pos() > errbits) bad = true;
            if (bad) break;
            if (dcl) { pred[ci] = wadd(pred[ci], o.v1); dc[bi] = pred[ci]; }
            else if (o.w1) coef[bi * 64 + nat_of_zig(o.c1 & 63)] = (int16_t)o.v1;
            if (o.w2) coef[bi * 64 + nat_of_zig(o.c2 & 63)] = (int16_t)o.v2;
            if (z == 0) ++bi;
        }
        anybad |= bad;
    }
    *status = anybad ? kSyntaxError : kOk;
    stats[0]++;
    return 0;
}

// Restart-interval streams (k_spec_write mode 3 + k_spec_finish): lane j decodes interval j from
// the byte after the (j-1)-th restart marker in U, R MCUs with zero DC predictors; the first
// interval that does not end at its own marker (dri_end_kind) decides the image. Returns 0
// parallel result (status in *status; coef / dc as emu_spec_decode), 1 the image would go to the
// sequential kernel, 2 not eligible. *first = SpecImg::dri_first.
int emu_dri_decode(const uint8_t* file, int64_t size, int16_t* coef, int32_t* dc, int64_t cap_blocks, int64_t* nblocks,
                   int32_t* status, int32_t* first) {
    auto dp = std::make_unique<Desc>();
    Desc& d = *dp;
    *status = parse_headers(file, size, d);
    *nblocks = 0;
    *first = INT32_MAX;
    const int64_t scan_len = d.size - d.scan_off;
    if (!(d.status == kPending && d.restart > 0 && d.nc >= 1 && d.bpm <= kSpecMaxBpm && scan_len > 0)) return 2;
    const int64_t total = (int64_t)d.mbw * d.mbh * d.bpm;
    *nblocks = total;
    if (total > cap_blocks) return 2;
    const uint8_t* R = file + d.scan_off;
    std::vector<uint8_t> U;
    std::vector<int64_t> rst;
    int64_t errpos;
    int32_t giveup = 0;
    const int64_t ulen = emu_unstuff(R, scan_len, ustf_align(R), U, errpos, giveup, &rst);
    if (giveup) return 1;
    auto SSp = std::make_unique<StepSet>();
    for (int k = 0; k < WriteTab::entries(); ++k) SSp->write.fill(d.huff, k);
    set_block_sel(SSp->write, d.huff, make_sel(d));
    const WriteTab& TW = SSp->write;
    const Sel SL = make_sel(d);
    const int64_t nint = ((int64_t)d.mbw * d.mbh + d.restart - 1) / d.restart;
    const int64_t iblocks = (int64_t)d.restart * d.bpm;
    const int64_t errbits = errpos == INT64_MAX ? INT64_MAX : errpos * 8;
    std::memset(coef, 0, sizeof(int16_t) * 64 * total);
    int32_t key = INT32_MAX;
    for (int64_t j = 0; j < nint; ++j) {
        int64_t start_byte = 0;
        if (j > 0) {
            if (j - 1 >= (int64_t)rst.size()) continue;  // marker missing: an earlier interval decides
            start_byte = (rst[j - 1] >> 3) + 2;
        }
        Reader r;
        r.init(U.data(), ulen, start_byte * 8);
        int b = 0, z = 0, ci = 0;
        int32_t pred[3] = {0, 0, 0};
        int64_t bi = j * iblocks, used_end = start_byte * 8;
        const int64_t bend = std::min(total, bi + iblocks);
        bool bad = false;
        while (bi < bend) {  // k_spec_write's loop, one lane
            const bool dcl = z == 0;
            if (dcl) ci = SL.comp(b);
            const int64_t p0 = r.pos();
            if (p0 + 16 > errbits) bad = true;
            const WriteOut o = write_step(r, TW, d.huff, SL, b, z, p0 + 16 + WriteTab::kAcBits > errbits);
            if (o.err || r.pos() > errbits) bad = true;
            if (bad) break;
            if (dcl) { pred[ci] = wadd(pred[ci], o.v1); dc[bi] = pred[ci]; }
            else if (o.w1) coef[bi * 64 + nat_of_zig(o.c1 & 63)] = (int16_t)o.v1;
            if (o.w2) coef[bi * 64 + nat_of_zig(o.c2 & 63)] = (int16_t)o.v2;
            if (z == 0) { ++bi; used_end = r.pos(); }
        }
        int kind = bad ? kDriError : kDriExact;
        if (!bad && j + 1 < nint)
            kind = dri_end_kind(U.data(), ulen, errpos, (used_end + 7) >> 3, j, j < (int64_t)rst.size() ? rst[j] : -1);
        if (kind != kDriExact) key = std::min(key, (int32_t)(2 * j + (kind == kDriElsewhere)));
    }
    *first = key;
    if (key != INT32_MAX && (key & 1)) return 1;
    *status = key == INT32_MAX ? kOk : kSyntaxError;
    return 0;
}
}

// ---- guess-write path (k_gw_lane / k_gw_check / k_gw_count / k_gw_repair / k_gw_scan / k_gw_map) ----
// The group's coefficient pool as the kernels address it: zig-zag int16 blocks, int32 DC escapes,
// overflow chunks chained through chunk_next, taken from `next` upwards.
struct EmuPool {
    std::vector<int16_t> coef;
    std::vector<int32_t> dc;
    std::vector<int32_t> chunk_next;
    int64_t next = 0, cap = 0;
    void init(int64_t blocks, int64_t static_end) {
        cap = blocks;
        coef.assign((size_t)blocks * 64, 0x5A5A);  // garbage: every stored block must be written whole
        dc.assign((size_t)blocks, 0);
        chunk_next.assign((size_t)(blocks / kGwChunk + 1), -1);
        next = (static_end + kGwChunk - 1) / kGwChunk * kGwChunk;
    }
    int64_t take(int64_t n) {  // the kernels' atomicAdd on the pool counter; -1 when exhausted
        if (next + n > cap) return -1;
        const int64_t b = next;
        next += n;
        return b;
    }
};
// Count lanes' blocks: a chain of pool chunks taken as the walk goes (k_gw_count's ChainSink).
struct EmuSink {
    EmuPool* P;
    int32_t chunk0 = -1, chunk = -1;
    int64_t cur = 0;  // pool block of the block in progress
    bool begin(int32_t t) {
        if (t % kGwChunk == 0) {
            const int64_t nb = P->take(kGwChunk);
            if (nb < 0) return false;
            const int32_t c = (int32_t)(nb / kGwChunk);
            if (chunk < 0) chunk0 = c;
            else P->chunk_next[chunk] = c;
            chunk = c;
        }
        cur = (int64_t)chunk * kGwChunk + t % kGwChunk;
        std::memset(&P->coef[(size_t)cur * 64], 0, 128);
        return true;
    }
    void cell(int32_t, int zz, int32_t v) { P->coef[(size_t)cur * 64 + zz] = (int16_t)v; }
    void dc(int32_t, int32_t v) {
        const int16_t c = dc_cell(v);
        P->coef[(size_t)cur * 64] = c;
        if (c == kDcEscape) P->dc[(size_t)cur] = v;
    }
};

// One guess-write lane (k_gw_lane's per-lane logic, scalar): decode [start - lead, end) from a
// guessed block start; from the first block start at or after `start` (g0) store every block
// started before the first block start at or after `end` (the exit), recording MCU starts.
static uint64_t emu_gw_lane(const uint8_t* U, int64_t ulen, const WriteTab& TW, const Huff* H, const Sel& S, int64_t start,
                            int64_t end, int64_t lead, int64_t errbits, int64_t sbase, int32_t Sst, EmuPool& P,
                            RecState* rec, GwOut& out) {
    const int64_t s0 = start - lead > 0 ? start - lead : 0;
    Reader r;
    r.init(U, ulen, s0);
    ErrBounds eb;
    eb.set(errbits, s0);
    const uint32_t pre = (uint32_t)(start - s0), span = (uint32_t)(end - s0);
    int b = 0, z = 0, ci = 0, phase = 0;
    out.k = 0;
    out.ds[0] = out.ds[1] = out.ds[2] = 0;
    out.err = INT32_MAX;
    out.chunk0 = -1;
    out.nrec = 0;
    out.over = 0;
    int32_t chunk = -1;  // current overflow chunk
    int64_t addr = 0;    // pool block of the block in progress
    for (;;) {
        if (z == 0) {
            const uint32_t u = r.used;
            if (phase == 0 && u >= pre) {
                phase = 1;
                out.g0 = pack_state(s0 + u, b, 0);
            }
            if (phase == 1 && u >= span) return pack_state(s0 + u, b, 0);
            if (phase == 1 && b == 0 && out.nrec < kRecGw) {
                RecState& e = rec[out.nrec++];
                e.rel = u - pre;
                e.b = 0;
                e.cnt = out.k;
                e.ds[0] = out.ds[0]; e.ds[1] = out.ds[1]; e.ds[2] = out.ds[2];
            }
            ci = S.comp(b);
            if (phase == 1) {  // the block's pool slot
                const int32_t k = out.k;
                if (k < Sst) {
                    addr = sbase + k;
                } else {
                    if ((k - Sst) % kGwChunk == 0) {
                        const int64_t nb = P.take(kGwChunk);
                        if (nb < 0) { out.over = 1; addr = P.cap - 1; }  // (the kernels write a scratch block)
                        else {
                            const int32_t c = (int32_t)(nb / kGwChunk);
                            if (chunk < 0) out.chunk0 = c;
                            else P.chunk_next[chunk] = c;
                            chunk = c;
                        }
                    }
                    if (!out.over) addr = (int64_t)chunk * kGwChunk + (k - Sst) % kGwChunk;
                }
                std::memset(&P.coef[(size_t)addr * 64], 0, 128);
            }
        }
        const bool dc = z == 0;
        const uint32_t u0 = r.used;
        const WriteOut o = write_step(r, TW, H, S, b, z, eb.near(u0));
        if (phase == 1) {
            if (eb.fail(u0, o.err, r.used) && out.err == INT32_MAX) out.err = out.k;
            int16_t* blk = &P.coef[(size_t)addr * 64];
            if (dc) {
                out.ds[ci] = wadd(out.ds[ci], o.v1);
                blk[0] = dc_cell(out.ds[ci]);
                if (blk[0] == kDcEscape) P.dc[(size_t)addr] = out.ds[ci];
            } else if (o.w1) {
                blk[o.c1 & 63] = (int16_t)o.v1;
            }
            if (o.w2) blk[o.c2 & 63] = (int16_t)o.v2;
            if (z == 0) ++out.k;
        }
    }
}

static int64_t g_gw_stats[8];  // lanes, synced at start, count lanes, spliced, repaired, overflow chunks, pool used
// count lanes by the guess record they spliced at (m = 0 .. kRec-1); [kRec]: never spliced, whole
// lane decoded (m = -1); [kRec + 1]: other (accumulated over calls; emu_gw_splice_hist reads it)
static int64_t g_gw_splice_hist[kRec + 2];

extern "C" {

void emu_gw_splice_hist(int64_t* out /*[kRec + 2]*/, int reset) {
    for (int k = 0; k < kRec + 2; ++k) {
        out[k] = g_gw_splice_hist[k];
        if (reset) g_gw_splice_hist[k] = 0;
    }
}

// The guess-write path end to end on the CPU. Returns like emu_spec_decode; static_frac scales
// the static slots per lane (k_spec_plan's kGwStaticSlack; small values force overflow chunks).
int emu_gw_decode(const uint8_t* file, int64_t size, int sub_bytes, int64_t lead, double static_frac, int16_t* coef,
                  int32_t* dcout, int64_t cap_blocks, int64_t* nblocks, int32_t* status, int64_t* stats /*[8]*/) {
    auto dp = std::make_unique<Desc>();
    Desc& d = *dp;
    *status = parse_headers(file, size, d);
    *nblocks = 0;
    const int64_t scan_len = d.size - d.scan_off;
    if (!(d.status == kPending && d.restart == 0 && d.nc >= 1 && d.bpm <= kSpecMaxBpm && scan_len > 0)) return 2;
    const int64_t total = (int64_t)d.mbw * d.mbh * d.bpm;
    *nblocks = total;
    if (total > cap_blocks) return 2;
    const uint8_t* R = file + d.scan_off;
    std::vector<uint8_t> U;
    int64_t errpos;
    int32_t giveup = 0;
    const int64_t ulen = emu_unstuff(R, scan_len, ustf_align(R), U, errpos, giveup, nullptr);
    if (giveup) return 1;
    const int64_t errbits = errpos == INT64_MAX ? INT64_MAX : errpos * 8;
    auto SSp = std::make_unique<StepSet>();
    StepSet& SS = *SSp;
    for (int k = 0; k < ScanTab::entries(); ++k) SS.scan.fill(d.huff, k);
    for (int k = 0; k < WriteTab::entries(); ++k) SS.write.fill(d.huff, k);
    const Sel SL = make_sel(d);
    set_block_sel(SS.scan, d.huff, SL);
    set_block_sel(SS.write, d.huff, SL);
    const Huff* H = d.huff;
    const int64_t sb = (int64_t)sub_bytes * 8;
    const int64_t nsub = ulen > 0 ? (ulen + sub_bytes - 1) / sub_bytes : 1;
    auto lane_end = [&](int64_t j) { return j == nsub - 1 ? ulen * 8 : (j + 1) * sb; };
    const int32_t Sst = (int32_t)std::max<double>(1.0, static_frac * (double)total / (double)nsub + 1.0);
    EmuPool P;
    P.init(nsub * Sst + 4 * total + 64 * nsub + 1024, nsub * Sst);
    // ---- k_gw_lane
    std::vector<uint64_t> X(nsub);
    std::vector<GwOut> g(nsub);
    std::vector<RecState> rec(nsub * kRec);
    for (int64_t j = 0; j < nsub; ++j) {
        X[j] = emu_gw_lane(U.data(), ulen, SS.write, H, SL, j * sb, lane_end(j), j ? lead : 0, errbits, j * Sst, Sst, P,
                           &rec[j * kRec], g[j]);
        if (g[j].over) return 1;
    }
    // ---- k_gw_check + k_gw_count: lanes not synchronised at their start
    std::vector<GcRec> c(nsub);
    std::vector<uint64_t> Y(nsub, 0);
    std::vector<int64_t> queue;
    auto count_lane = [&](int64_t j, uint64_t entry) -> bool {  // false: pool exhausted
        GcRec& q = c[j];
        uint64_t ex = 0;
        EmuSink sk{&P};
        q.c = gc_walk(U.data(), ulen, SS.write, H, SL, entry, j * sb, lane_end(j), &rec[j * kRec], g[j].nrec, errbits, sk,
                      q.cds, &q.m, &ex, &q.err);
        q.chunk0 = sk.chunk0;
        Y[j] = ex;
        return q.m != -3;
    };
    int64_t counted = 0, spliced = 0;
    for (int64_t j = 0; j < nsub; ++j) {
        const uint64_t entry = j == 0 ? pack_state(0, 0, 0) : X[j - 1];
        c[j] = GcRec{-1, 0, 0, -2, {0, 0, 0}, INT32_MAX};
        if (g[j].g0 == entry) continue;
        ++counted;
        if (!count_lane(j, entry)) return 1;
        spliced += c[j].m >= 0;
        ++g_gw_splice_hist[c[j].m >= 0 ? std::min<int>(c[j].m, kRec - 1) : kRec + (c[j].m == -1 ? 0 : 1)];
        if (c[j].m < 0 && j + 1 < nsub && Y[j] != X[j]) queue.push_back(j);
    }
    // ---- k_gw_repair: an unspliced count lane whose exit differs re-derives the next lanes
    int64_t repaired = 0, done = -1;
    for (int64_t j : queue) {
        if (j <= done) continue;
        X[j] = Y[j];
        int64_t k = j + 1, steps = 0;
        for (; k < nsub; ++k, ++steps) {
            if (steps >= kGwMaxWalk) return 1;
            ++repaired;
            if (g[k].g0 == X[k - 1]) { c[k] = GcRec{-1, 0, 0, -2, {0, 0, 0}, INT32_MAX}; break; }
            if (!count_lane(k, X[k - 1])) return 1;
            if (c[k].m >= 0 || k + 1 == nsub || Y[k] == X[k]) break;
            X[k] = Y[k];
        }
        done = k;
    }
    // ---- k_gw_scan: lane totals -> first block index and DC predictors; true-path errors
    std::vector<int64_t> G(nsub + 1, 0);
    std::vector<int32_t> Pd(3 * nsub, 0);
    int32_t Pc[3] = {0, 0, 0};
    bool bad = false;
    for (int64_t j = 0; j < nsub; ++j) {
        int32_t ds[3];
        const int32_t n = gw_lane_total(g[j], c[j], &rec[j * kRec], ds);
        for (int q = 0; q < 3; ++q) { Pd[3 * j + q] = Pc[q]; Pc[q] = wadd(Pc[q], ds[q]); }
        const int32_t e = gw_lane_err(g[j], c[j], &rec[j * kRec]);
        if (e != INT32_MAX && G[j] + e < total) bad = true;
        G[j + 1] = G[j] + n;
    }
    // ---- k_gw_tail: the blocks run past the data (no error decided the status): read on into
    // the 0xFF padding from the last lane's exit, as NanoJPEG does
    std::vector<int64_t> maddr(total, 0);
    std::vector<int32_t> moff(total, 0);
    if (G[nsub] < total && !bad) {
        const uint64_t entry = c[nsub - 1].m == -1 ? Y[nsub - 1] : X[nsub - 1];
        EmuSink sk{&P};
        int32_t tds[3], terr;
        const int32_t got = gw_tail(U.data(), ulen, SS.write, H, SL, entry, total - G[nsub], errbits, sk, tds, &terr);
        if (got < 0) return 1;
        if (terr != INT32_MAX) bad = true;
        GwSlots ts{0, 0, -1, 0};
        for (int32_t t = 0; t < got && !bad; ++t) {
            const int64_t n = G[nsub] + t;
            maddr[n] = ts.addr(t, sk.chunk0, P.chunk_next.data());
            moff[n] = Pc[SL.comp((int)(n % d.bpm))];
        }
        stats[7] += 1;
    }
    for (int64_t j = 0; j < nsub && !bad; ++j) {
        GwSlots sl{j * Sst, Sst, -1, 0};
        const int32_t m0 = c[j].m >= 0 ? rec[j * kRec + c[j].m].cnt : 0;
        for (int64_t n = G[j]; n < G[j + 1] && n < total; ++n) {
            const int32_t t = (int32_t)(n - G[j]);
            const int ci = SL.comp((int)(n % d.bpm));
            if (t < c[j].c && c[j].m != -2) {
                GwSlots cs{0, 0, -1, 0};
                maddr[n] = cs.addr(t, c[j].chunk0, P.chunk_next.data());
                moff[n] = Pd[3 * j + ci];
            } else {
                maddr[n] = sl.addr(t - (c[j].m == -2 ? 0 : c[j].c) + m0, g[j].chunk0, P.chunk_next.data());
                moff[n] = c[j].m >= 0 ? wadd(Pd[3 * j + ci], wsub(c[j].cds[ci], rec[j * kRec + c[j].m].ds[ci]))
                                      : Pd[3 * j + ci];
            }
        }
    }
    std::memset(coef, 0, sizeof(int16_t) * 64 * total);
    for (int64_t n = 0; n < total && !bad; ++n) {
        const int16_t* blk = &P.coef[(size_t)maddr[n] * 64];
        const int32_t dl = blk[0] == kDcEscape ? P.dc[(size_t)maddr[n]] : blk[0];
        dcout[n] = wadd(dl, moff[n]);
        for (int zz = 1; zz < 64; ++zz) coef[n * 64 + nat_of_zig(zz)] = blk[zz];
    }
    *status = bad ? kSyntaxError : kOk;
    int64_t synced = 0;
    for (int64_t j = 0; j < nsub; ++j) synced += c[j].m == -2;
    stats[0] += nsub; stats[1] += synced; stats[2] += counted; stats[3] += spliced; stats[4] += repaired;
    stats[5] += (P.next - (nsub * Sst + kGwChunk - 1) / kGwChunk * kGwChunk) / kGwChunk;
    stats[6] += P.next;
    return 0;
}
}

#include <unordered_map>
extern "C" {
// Count-pass study (tuning aid): run emu_spec_decode with guess lead `lead` and report the bits
// each count lane decoded before it spliced (or its whole lane); returns the number of lanes
// (at most cap written to out).
int64_t emu_count_study(const uint8_t* file, int64_t size, int64_t lead, int16_t* coef, int32_t* dc, int64_t cap_blocks,
                        uint32_t* out, int64_t cap) {
    std::vector<uint32_t> bits;
    g_count_bits = &bits;
    const int64_t old = g_lead;
    g_lead = lead;
    int64_t nb = 0, st[4] = {0, 0, 0, 0};
    int32_t status = 0;
    emu_spec_decode(file, size, kSubBytes, coef, dc, cap_blocks, &nb, &status, st);
    g_lead = old;
    g_count_bits = nullptr;
    for (int64_t k = 0; k < (int64_t)bits.size() && k < cap; ++k) out[k] = bits[k];
    return (int64_t)bits.size();
}

// Sync-distance study: for `nstarts` evenly spaced start bits, decode from a guessed state
// (b = guess_b, z = 0) and report the bits consumed until the lane's state equals the true
// decoder's state at the same position (-1 if not within `maxbits`).
int emu_sync_study(const uint8_t* file, int64_t size, int nstarts, int guess_b, int64_t maxbits, int64_t* out) {
    auto dp = std::make_unique<Desc>();
    Desc& d = *dp;
    if (parse_headers(file, size, d) != kPending || d.restart || d.bpm > kSpecMaxBpm) return -1;
    const uint8_t* R = file + d.scan_off;
    const int64_t L = d.size - d.scan_off;
    std::vector<uint8_t> U;
    int64_t errpos; int32_t gu = 0;
    const int64_t ulen = emu_unstuff(R, L, ustf_align(R), U, errpos, gu, nullptr);
    auto SSp = std::make_unique<StepSet>();
    for (int k = 0; k < ScanTab::entries(); ++k) SSp->scan.fill(d.huff, k);
    set_block_sel(SSp->scan, d.huff, make_sel(d));
    const ScanTab& T = SSp->scan;
    const Huff* H = d.huff;
    std::unordered_map<int64_t, int> truth;  // pos -> (b<<8|z)
    {
        Reader r; r.init(U.data(), ulen, 0);
        int b = 0, z = 0; int32_t v;
        const int64_t total = (int64_t)d.mbw * d.mbh * d.bpm;
        int64_t blocks = 0;
        truth[0] = 0;
        while (blocks < total) { bool dc = z == 0; scan_step(r, T, H, make_sel(d), b, z, v); if (dc) ++blocks; truth[r.pos()] = (b << 8) | z; }
    }
    for (int s = 0; s < nstarts; ++s) {
        const int64_t start = (ulen * 8) * s / nstarts;
        Reader r; r.init(U.data(), ulen, start);
        int b = guess_b, z = 0; int32_t v;
        out[s] = -1;
        while (r.pos() - start < maxbits) {
            scan_step(r, T, H, make_sel(d), b, z, v);
            auto it = truth.find(r.pos());
            if (it != truth.end() && it->second == ((b << 8) | z)) { out[s] = r.pos() - start; break; }
        }
    }
    return 0;
}
}

// ---- two-level Huffman lookup self-check (tests/test_spec_emu.py) ----
// Builds a table from counts[1..16] and symbols, fills fast + subtables, and returns how many of
// the 65536 windows huff_lookup decodes differently from the canonical walk; *nsub_out = number
// of subtables the table needed.
extern "C" int emu_huff_selftest(const uint8_t* counts17, const uint8_t* syms, int nsyms, int* nsub_out) {
    auto Tp = std::make_unique<Huff>();
    Huff& t = *Tp;
    std::memset(&t, 0, sizeof t);
    for (int i = 0; i < nsyms && i < 256; ++i) t.sym[i] = syms[i];
    huff_finalize(t, counts17);
    huff_fill_fast(t, 0, 1);
    *nsub_out = (int)(((t.bound[16] + 63) >> 6) - (t.bound[kFastBits] >> 6));
    int bad = 0;
    for (uint32_t w = 0; w < 65536; ++w) {
        int s1 = -1, s2 = -1;
        const int l1 = huff_lookup(t, w, s1), l2 = huff_search(t, w, 1, s2);
        if (l1 != l2 || (l1 && s1 != s2)) ++bad;
    }
    return bad;
}

// ---- step-table self-check (tests/test_spec_emu.py) ----
// One DC table (index 0) and one AC table (index 2) from counts/symbols; `nblocks` blocks of a
// random bit stream (seed) are decoded three ways from the same start: symbol by symbol with the
// canonical walk and NanoJPEG's block rules (the reference semantics), with scan_step and with
// write_step. Returns the number of disagreements: block-start positions, DC values, error
// flags, and every coefficient the write steps place.
static uint64_t emu_rng(uint64_t& s) { s += 0x9E3779B97F4A7C15ull; uint64_t z = s; z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; return z ^ (z >> 31); }
extern "C" int emu_step_selftest(const uint8_t* dcc17, const uint8_t* dcs, int ndc, const uint8_t* acc17, const uint8_t* acs,
                                 int nac, uint64_t seed, int nblocks, int64_t* stats /*[4]: blocks, symbols, lookups scan, lookups write*/) {
    auto Hp = std::make_unique<Huff[]>(4);
    Huff* H = Hp.get();
    std::memset(H, 0, sizeof(Huff) * 4);
    for (int i = 0; i < ndc && i < 256; ++i) H[0].sym[i] = dcs[i];
    for (int i = 0; i < nac && i < 256; ++i) H[2].sym[i] = acs[i];
    huff_finalize(H[0], dcc17);
    huff_finalize(H[2], acc17);
    uint8_t zero17[17] = {0};
    huff_finalize(H[1], zero17);
    huff_finalize(H[3], zero17);
    auto SSp = std::make_unique<StepSet>();
    for (int k = 0; k < ScanTab::entries(); ++k) SSp->scan.fill(H, k);
    for (int k = 0; k < WriteTab::entries(); ++k) SSp->write.fill(H, k);
    // random stream: mostly well-formed blocks would need an encoder; random bits exercise every
    // entry kind (errors included) and the decoders must agree on all of them
    const int64_t nbytes = (int64_t)nblocks * 64 + 64;
    std::vector<uint8_t> U(nbytes + 64, 0xFF);
    for (int64_t i = 0; i < nbytes; ++i) U[i] = (uint8_t)emu_rng(seed);
    Desc d;
    std::memset(&d, 0, sizeof d);
    d.bpm = 1;
    d.nc = 1;
    d.c[0].nblk = 1; d.c[0].hs = 1; d.c[0].vs = 1; d.c[0].dc_tab = 0; d.c[0].ac_tab = 2;
    const Sel SL = make_sel(d);
    set_block_sel(SSp->scan, H, SL);
    set_block_sel(SSp->write, H, SL);
    const int64_t ulen = nbytes;
    int bad = 0;
    // reference: symbol by symbol
    std::vector<int64_t> starts;
    std::vector<int32_t> dcs_ref;
    std::vector<int> errs;
    std::vector<int16_t> coefs;
    {
        int64_t pos = 0;
        auto win = [&](int64_t p) { uint32_t v = 0; for (int i = 0; i < 4; ++i) v = (v << 8) | U[(p >> 3) + i]; return (uint32_t)(((uint64_t)v << (p & 7)) >> 8) >> 8; };
        for (int blk = 0; blk < nblocks; ++blk) {
            starts.push_back(pos);
            std::vector<int16_t> c(64, 0);
            int s = 0, err = 0;
            int L = huff_search(H[0], win(pos) & 0xFFFF, 1, s);
            int32_t v = 0;
            if (!L) { err = 1; pos += 1; }
            else { pos += L; int nb = s & 15; if (nb) { v = extend((int32_t)((win(pos) & 0xFFFF) >> (16 - nb)), nb); pos += nb; } stats[1]++; }
            dcs_ref.push_back(v);
            int k = 0;
            while (!err) {
                L = huff_search(H[2], win(pos) & 0xFFFF, 1, s);
                if (!L) { err = 1; pos += 1; break; }
                pos += L; stats[1]++;
                if (!s) break;
                if (!(s & 15) && s != 0xF0) { err = 1; break; }
                int nb = s & 15; v = 0;
                if (nb) { v = extend((int32_t)((win(pos) & 0xFFFF) >> (16 - nb)), nb); pos += nb; }
                k += (s >> 4) + 1;
                if (k > 63) { err = 1; break; }
                c[k] = (int16_t)v;
                if (k == 63) break;
            }
            errs.push_back(err);
            coefs.insert(coefs.end(), c.begin(), c.end());
        }
        starts.push_back(pos);
    }
    // scan_step
    {
        Reader r; r.init(U.data(), ulen, 0);
        int b = 0, z = 0;
        for (int blk = 0; blk < nblocks; ++blk) {
            if (r.pos() != starts[blk]) { ++bad; break; }
            int err = 0;
            int32_t dv = 0, v;
            bool first = true;
            do {
                const bool dc = z == 0;
                err |= scan_step(r, SSp->scan, H, SL, b, z, v);
                if (dc && first) dv = v;
                first = false;
                stats[2]++;
            } while (z != 0);
            if (err != errs[blk]) ++bad;
            if (!errs[blk] && dv != dcs_ref[blk]) ++bad;
        }
        if (r.pos() != starts[nblocks]) ++bad;
    }
    // write_step
    {
        Reader r; r.init(U.data(), ulen, 0);
        int b = 0, z = 0;
        for (int blk = 0; blk < nblocks; ++blk) {
            if (r.pos() != starts[blk]) { ++bad; break; }
            std::vector<int16_t> c(64, 0);
            int err = 0;
            int32_t dv = 0;
            do {
                const bool dc = z == 0;
                const WriteOut o = write_step(r, SSp->write, H, SL, b, z, false);
                err |= o.err;
                if (dc) dv = o.v1;
                else if (o.w1 && o.c1 < 64) c[o.c1] = (int16_t)o.v1;
                if (o.w2 && o.c2 < 64) c[o.c2] = (int16_t)o.v2;
                stats[3]++;
            } while (z != 0);
            if (err != errs[blk]) ++bad;
            if (!errs[blk]) {
                if (dv != dcs_ref[blk]) ++bad;
                for (int k = 1; k < 64; ++k) bad += c[k] != coefs[(size_t)blk * 64 + k];
            }
        }
        if (r.pos() != starts[nblocks]) ++bad;
    }
    stats[0] += nblocks;
    return bad;
}

// ---- unstuff at a forced tile alignment (tests/test_spec_emu.py) ----
// The scan of `file` unstuffed with tiles cut at alignment sh (0..15); returns ulen (-1: no scan
// or buffer too small), *errpos as the GPU's SpecImg::errpos, *giveup, and the restart records.
extern "C" int64_t emu_unstuff_sh(const uint8_t* file, int64_t size, int sh, uint8_t* out, int64_t cap, int64_t* errpos,
                                  int32_t* giveup, int64_t* rst, int64_t rst_cap, int64_t* nrst, int64_t* scan_off) {
    auto dp = std::make_unique<Desc>();
    Desc& d = *dp;
    if (parse_headers(file, size, d) != kPending) return -1;
    *scan_off = d.scan_off;
    const int64_t L = d.size - d.scan_off;
    if (L <= 0) return -1;
    std::vector<uint8_t> U;
    std::vector<int64_t> rs;
    int32_t gu = 0;
    const int64_t ulen = emu_unstuff(file + d.scan_off, L, sh, U, *errpos, gu, &rs);
    *giveup = gu;
    *nrst = (int64_t)rs.size();
    for (int64_t k = 0; k < (int64_t)rs.size() && k < rst_cap; ++k) rst[k] = rs[k];
    if (ulen > cap) return -1;
    std::memcpy(out, U.data(), (size_t)ulen);
    return ulen;
}

extern "C" {
// Write-pass study (tuning aid): decode the whole scan with write_step and report, for a wave of
// 64 lanes that each take 1/64 of the lookups in lockstep, out[0] lookups, out[1] lookups that
// needed the long-code pool (SUB), out[2] wave iterations, out[3] iterations where some lane
// needed the pool, out[4] iterations where some lane completed a block, out[5] blocks.
int emu_write_study(const uint8_t* file, int64_t size, int64_t* out) {
    auto dp = std::make_unique<Desc>();
    Desc& d = *dp;
    if (parse_headers(file, size, d) != kPending || d.restart || d.bpm > kSpecMaxBpm) return -1;
    const uint8_t* R = file + d.scan_off;
    std::vector<uint8_t> U;
    int64_t errpos; int32_t gu = 0;
    const int64_t ulen = emu_unstuff(R, d.size - d.scan_off, ustf_align(R), U, errpos, gu, nullptr);
    auto SSp = std::make_unique<StepSet>();
    for (int k = 0; k < WriteTab::entries(); ++k) SSp->write.fill(d.huff, k);
    const Sel SL = make_sel(d);
    set_block_sel(SSp->write, d.huff, SL);
    const WriteTab& TW = SSp->write;
    std::vector<uint8_t> ev;  // per lookup: bit0 SUB, bit1 block completed
    Reader r; r.init(U.data(), ulen, 0);
    int b = 0, z = 0;
    const int64_t total = (int64_t)d.mbw * d.mbh * d.bpm;
    int64_t blocks = 0;
    while (blocks < total) {
        const bool dc = z == 0;
        r.refill();  // (write_step refills again: harmless for the peek below)
        const uint32_t e = TW.look_b(b, dc, (uint32_t)(r.buf >> 32));
        (void)write_step(r, TW, d.huff, SL, b, z, false);
        const bool done = z == 0;
        blocks += done;
        ev.push_back((uint8_t)(((e & kStSlow) ? 1 : 0) | (done ? 2 : 0)));
    }
    const int64_t n = (int64_t)ev.size(), per = (n + 63) / 64;
    int64_t nsub = 0, it_sub = 0, it_done = 0;
    for (uint8_t v : ev) nsub += v & 1;
    for (int64_t i = 0; i < per; ++i) {
        int any_s = 0, any_d = 0;
        for (int l = 0; l < 64; ++l) {
            const int64_t k = l * per + i;
            if (k < n) { any_s |= ev[k] & 1; any_d |= (ev[k] >> 1) & 1; }
        }
        it_sub += any_s;
        it_done += any_d;
    }
    out[0] = n; out[1] = nsub; out[2] = per; out[3] = it_sub; out[4] = it_done; out[5] = blocks;
    return 0;
}
}

// Write-table width study (tuning aid): lookups per block of a sequential write_step decode with
// AC windows of 10 / 11 / 12 bits (pairs fit more often in wider windows). out[k] = lookups
// with AC window 10 + k, out[3] = blocks.
template <int AB>
static int64_t write_lookups(const Desc& d, const std::vector<uint8_t>& U, int64_t ulen, int64_t total) {
    using Tab = StepTab<8, AB, 1280, false>;
    auto T = std::make_unique<Tab>();
    for (int k = 0; k < Tab::entries(); ++k) T->fill(d.huff, k);
    const Sel SL = make_sel(d);
    set_block_sel(*T, d.huff, SL);
    Reader r; r.init(U.data(), ulen, 0);
    int b = 0, z = 0;
    int64_t blocks = 0, n = 0;
    while (blocks < total) {
        (void)write_step(r, *T, d.huff, SL, b, z, false);
        ++n;
        blocks += z == 0;
    }
    return n;
}
extern "C" int emu_write_width_study(const uint8_t* file, int64_t size, int64_t* out) {
    auto dp = std::make_unique<Desc>();
    Desc& d = *dp;
    if (parse_headers(file, size, d) != kPending || d.restart || d.bpm > kSpecMaxBpm) return -1;
    const uint8_t* R = file + d.scan_off;
    std::vector<uint8_t> U;
    int64_t errpos; int32_t gu = 0;
    const int64_t ulen = emu_unstuff(R, d.size - d.scan_off, ustf_align(R), U, errpos, gu, nullptr);
    const int64_t total = (int64_t)d.mbw * d.mbh * d.bpm;
    out[0] = write_lookups<10>(d, U, ulen, total);
    out[1] = write_lookups<11>(d, U, ulen, total);
    out[2] = write_lookups<12>(d, U, ulen, total);
    out[3] = total;
    return 0;
}
