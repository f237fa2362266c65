// icx_spec.hip -- massively parallel, bit-exact Huffman decode of baseline JPEG on gfx950.
//
// NanoJPEG decodes the entropy-coded segment with one serial bit reader
// (njDecodeScan, jpeg_dec.h:678-718). Here every image is cut into subsequences of
// kSubBytes unstuffed bytes, one lane each, and decoded speculatively; JPEG's Huffman
// codes self-synchronise, so a lane that starts at a guessed state soon lands on the
// true symbol/block boundaries. Correctness never depends on that luck: every lane's
// exit state is re-derived from its predecessor's and compared, and an image with an
// unresolved disagreement falls back to the sequential kernel (k_entropy_seq).
//
//   k_spec_plan     which images take this path; flat tile / lane-group numbering
//   k_ustf_count    NanoJPEG's marker rules (jpeg_dec.h:447-482) per 4 KiB tile:
//   k_ustf_scan       FF00/FFFF -> FF, FFDn kept, FFD9 / bad marker ends the data;
//   k_ustf_write      writes the unstuffed stream U (reads past its end give 0xFF)
//   k_spec_guess    lane j decodes subsequence j from a guessed state -> exit state X[j]
//   k_spec_count    lane j re-decodes from X[j-1]: blocks started, DC-diff sums, and
//                   whether its exit state reproduces X[j]
//   k_spec_scan     per image: block index + DC predictor at every lane entry;
//                   picks the fallback for images whose chain does not verify
//   k_spec_write    lane j decodes the blocks that START in its range (whole blocks),
//                   writes quantized coefficients; true-path errors flag the image
// A lane's state is (bit position in U, block-in-MCU b, coefficient cursor z).
#include <hip/hip_runtime.h>
#include <rocprim/warp/warp_scan.hpp>

#include "icx_spec_core.h"

namespace icx {

// ------------------------------------------------------------------------------- plan
__device__ int block_exclusive_scan(int v, int* sh) {  // blockDim.x <= 1024, returns exclusive
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int o = 1; o < (int)blockDim.x; o <<= 1) {
        const int x = t >= o ? sh[t - o] : 0;
        __syncthreads();
        sh[t] += x;
        __syncthreads();
    }
    const int incl = sh[t];
    __syncthreads();
    return incl - v;
}

__global__ __launch_bounds__(1024) void k_spec_plan(int n, Desc* __restrict__ desc, SpecImg* __restrict__ spec,
                                                    int32_t* __restrict__ tilepre, int32_t* __restrict__ wgpre,
                                                    int32_t* __restrict__ wg2pre, int32_t* __restrict__ totals,
                                                    int64_t ucap) {
    __shared__ int sh[1024];
    int carry_t = 0, carry_w = 0, carry_w2 = 0;
    for (int i0 = 0; i0 < n; i0 += blockDim.x) {
        const int i = i0 + threadIdx.x;
        int nt = 0, nw = 0, nw2 = 0;
        if (i < n) {
            const Desc& d = desc[i];
            SpecImg& s = spec[i];
            s.mode = 0;
            s.err = 0;
            s.nrepair = 0;
            s.nrst = 0;
            const int64_t scan_len = d.size - d.scan_off;
            // (U also holds the reader padding: u_pad_end(ulen) <= ulen + 32, ulen <= scan_len)
            const bool ok = d.status == kPending && d.nc >= 1 && d.bpm <= kSpecMaxBpm && scan_len > 0 &&
                            scan_len + 64 <= ucap;
            if (ok) {
                s.mode = d.restart == 0 ? 1 : 3;
                s.scan_len = scan_len;
                s.total_blocks = (int64_t)d.mbw * d.mbh * d.bpm;
                nt = (int)((scan_len + kTileBytes - 1) / kTileBytes);
                // lanes: 2 KiB subsequences, or (DRI) one per restart interval
                const int64_t nmcu = (int64_t)d.mbw * d.mbh;
                const int64_t nsub = s.mode == 1 ? (scan_len + kSubBytes - 1) / kSubBytes
                                                 : (nmcu + d.restart - 1) / d.restart;
                s.nint = s.mode == 3 ? (int32_t)nsub : 0;
                nw = (int)((nsub + kLanes - 1) / kLanes);
                nw2 = (int)((nsub + kWriteLanesBig - 1) / kWriteLanesBig);
            }
            s.ntiles = nt;
            s.nwg = nw;
        }
        const int et = block_exclusive_scan(nt, sh);
        const int ew = block_exclusive_scan(nw, sh);
        const int ew2 = block_exclusive_scan(nw2, sh);
        if (i < n) {
            tilepre[i] = carry_t + et;
            wgpre[i] = carry_w + ew;
            wg2pre[i] = carry_w2 + ew2;
            spec[i].tile_base = carry_t + et;
            spec[i].wg_base = carry_w + ew;
        }
        __shared__ int last_t, last_w, last_w2;
        if (threadIdx.x == blockDim.x - 1) { last_t = et + nt; last_w = ew + nw; last_w2 = ew2 + nw2; }
        __syncthreads();
        carry_t += last_t;
        carry_w += last_w;
        carry_w2 += last_w2;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        tilepre[n] = carry_t;
        wgpre[n] = carry_w;
        wg2pre[n] = carry_w2;
        totals[0] = carry_t;
        totals[1] = carry_w;
        totals[2] = carry_w2;
    }
}

// image owning flat item x, given exclusive prefix pre[0..n] (pre[n] = total)
__device__ __forceinline__ int find_image(const int32_t* pre, int n, int x) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= x) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// ---------------------------------------------------------------------------- unstuff
// Unstuff tiles: one wave per 4 KiB raw tile, 64 raw bytes (four 16-byte chunks) per lane; wave
// shuffles for the prefix / min, no block barriers. Each wave walks a contiguous range of the
// flat tile list, so the owning image only ever advances (no per-tile search).
constexpr int kLaneRaw = kTileBytes / 64;

__device__ __forceinline__ int wave_incl_scan(int v) {  // rocprim's DPP cross-lane scan
    using WScan = rocprim::warp_scan<int, 64>;
    typename WScan::storage_type st;  // empty for the cross-lane implementation
    int r;
    WScan().inclusive_scan(v, r, st);
    return r;
}
__device__ __forceinline__ long long wave_min_ll(long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}

// One lane's 64 raw bytes: kept bytes before the lane's first end event (written to `out` when
// WRITE), that event's raw offset (-1: none) and whether it is an error.
template <bool WRITE>
__device__ __forceinline__ int ustf_lane(const uint8_t* R, int64_t L, int64_t a, int64_t& end_at, int& end_err,
                                         uint8_t* out, int32_t& giveup, RstSink& rs) {
    int kept = 0;
    end_at = -1;
    end_err = 0;
    const int64_t ub = rs.ubase;
#pragma unroll
    for (int c = 0; c < kLaneRaw / kChunk; ++c) {
        int64_t e;
        int er;
        rs.ubase = ub + kept;
        kept += ustf_chunk<WRITE>(R, L, a + c * kChunk, &e, &er, WRITE ? out + kept : nullptr, &giveup, &rs);
        if (e >= 0) {
            end_at = e;
            end_err = er;
            break;
        }
    }
    return kept;
}

struct TileRange {
    int t, t1, i;
};
__device__ __forceinline__ TileRange wave_tiles(const int32_t* tilepre, int n, int total) {
    const int nw = gridDim.x * (blockDim.x >> 6), w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int per = (total + nw - 1) / nw;
    TileRange r;
    r.t = min(total, w * per);
    r.t1 = min(total, r.t + per);
    r.i = r.t < r.t1 ? find_image(tilepre, n, r.t) : 0;
    return r;
}

__global__ __launch_bounds__(256) void k_ustf_count(int n, const uint8_t* __restrict__ data,
                                                    const uint64_t* __restrict__ off, const Desc* __restrict__ desc,
                                                    SpecImg* __restrict__ spec, const int32_t* __restrict__ tilepre,
                                                    const int32_t* __restrict__ totals, TileRec* __restrict__ tiles) {
    const int lane = threadIdx.x & 63;
    TileRange tr = wave_tiles(tilepre, n, totals[0]);
    for (int t = tr.t; t < tr.t1; ++t) {
        while (t >= tilepre[tr.i + 1]) ++tr.i;
        const int i = tr.i;
        const uint8_t* R = data + off[i] + desc[i].scan_off;
        const int64_t L = spec[i].scan_len;
        const int64_t a = (int64_t)(t - tilepre[i]) * kTileBytes + (int64_t)lane * kLaneRaw;
        int64_t end_at;
        int end_err;
        int32_t giveup = 0;
        RstSink rs{0, 0, nullptr, 0, 0};
        const int kept = ustf_lane<false>(R, L, a, end_at, end_err, nullptr, giveup, rs);
        if (giveup) atomicOr(&spec[i].err, kSpecGiveUp);
        const long long tend = wave_min_ll(end_at >= 0 ? (long long)end_at : LLONG_MAX);
        // kept bytes (and restart markers) before the tile's first end event
        const bool before = end_at >= 0 ? end_at <= tend : a < tend;
        const int incl = wave_incl_scan(before ? kept : 0);
        const int rincl = wave_incl_scan(before ? rs.n : 0);
        const uint64_t owner = __ballot(end_at >= 0 && end_at == tend);  // the unique lane owning that FF
        const int err = __shfl(end_err, owner ? __ffsll((long long)owner) - 1 : 0);
        if (lane == 63) {
            TileRec r;
            r.kept = incl;
            r.end_at = tend == LLONG_MAX ? -1 : tend;
            r.end_err = owner ? err : 0;
            r.nrst = rincl;
            r.pad_ = 0;
            tiles[t] = r;
        }
    }
}

// Per image: exclusive prefix of kept bytes over tiles, data length, error position.
__global__ __launch_bounds__(256) void k_ustf_scan(int n, SpecImg* __restrict__ spec, TileRec* __restrict__ tiles,
                                                   int32_t* __restrict__ tile_obase, int32_t* __restrict__ tile_rbase,
                                                   uint8_t* __restrict__ U, int64_t ucap) {
    __shared__ int sh[256];
    __shared__ int s_first_end;
    const int i = blockIdx.x;
    if (i >= n) return;
    SpecImg& s = spec[i];
    if (s.mode != 1 && s.mode != 3) return;
    if (threadIdx.x == 0) s_first_end = INT32_MAX;
    __syncthreads();
    for (int t = threadIdx.x; t < s.ntiles; t += blockDim.x)
        if (tiles[s.tile_base + t].end_at >= 0) atomicMin(&s_first_end, t);
    __syncthreads();
    const int fe = s_first_end;
    int64_t carry = 0;
    int32_t rcarry = 0;
    for (int t0 = 0; t0 < s.ntiles; t0 += blockDim.x) {
        const int t = t0 + threadIdx.x;
        const bool in = t < s.ntiles && t <= fe;
        const int k = in ? tiles[s.tile_base + t].kept : 0;
        const int nr = in ? tiles[s.tile_base + t].nrst : 0;
        const int ex = block_exclusive_scan(k, sh);
        const int rex = block_exclusive_scan(nr, sh);
        if (t < s.ntiles) {
            tile_obase[s.tile_base + t] = (int32_t)(carry + ex);
            tile_rbase[s.tile_base + t] = rcarry + rex;
        }
        __shared__ int s_sum, s_rsum;
        if (threadIdx.x == blockDim.x - 1) { s_sum = ex + k; s_rsum = rex + nr; }
        __syncthreads();
        carry += s_sum;
        rcarry += s_rsum;
        __syncthreads();
    }
    {  // 0xFF padding behind the data for the lane readers (icx_spec_core.h, u_pad_end)
        uint8_t* u = U + (int64_t)i * ucap;
        for (int64_t p = carry + threadIdx.x; p < u_pad_end(carry); p += blockDim.x) u[p] = 0xFF;
    }
    if (threadIdx.x == 0) {
        s.ulen = carry;
        s.nrst = rcarry;
        s.errpos = (fe != INT32_MAX && tiles[s.tile_base + fe].end_err) ? carry : INT64_MAX;
        const int64_t nsub = carry > 0 ? (carry + kSubBytes - 1) / kSubBytes : 1;
        s.nsub = s.mode == 3 ? s.nint : (int32_t)nsub;
    }
}

__global__ __launch_bounds__(256) void k_ustf_write(int n, const uint8_t* __restrict__ data,
                                                    const uint64_t* __restrict__ off, const Desc* __restrict__ desc,
                                                    const SpecImg* __restrict__ spec, const int32_t* __restrict__ tilepre,
                                                    const int32_t* __restrict__ totals, const TileRec* __restrict__ tiles,
                                                    const int32_t* __restrict__ tile_obase,
                                                    const int32_t* __restrict__ tile_rbase, uint8_t* __restrict__ U,
                                                    int64_t ucap, int64_t* __restrict__ rst, int64_t rst_cap) {
    __shared__ uint32_t sbuf_all[4][kTileBytes / 4 + 8];  // per wave: the tile's kept bytes
    const int lane = threadIdx.x & 63;
    uint32_t* sbuf = sbuf_all[threadIdx.x >> 6];
    uint8_t* sb = reinterpret_cast<uint8_t*>(sbuf);
    TileRange tr = wave_tiles(tilepre, n, totals[0]);
    for (int t = tr.t; t < tr.t1; ++t) {
        while (t >= tilepre[tr.i + 1]) ++tr.i;
        const int i = tr.i;
        const SpecImg& s = spec[i];
        const int64_t obase = tile_obase[t];  // == ulen for every tile past the first end event
        if (obase >= s.ulen) continue;        // wave-uniform
        const int64_t tend = tiles[t].end_at;
        const uint8_t* R = data + off[i] + desc[i].scan_off;
        const int64_t a = (int64_t)(t - tilepre[i]) * kTileBytes + (int64_t)lane * kLaneRaw;
        int64_t end_at;
        int end_err;
        int32_t giveup = 0;
        RstSink rs0{0, 0, nullptr, 0, 0};
        const int kept = ustf_lane<false>(R, s.scan_len, a, end_at, end_err, nullptr, giveup, rs0);
        const bool before = end_at >= 0 ? (tend < 0 || end_at <= tend) : (tend < 0 || a < tend);
        const int k = before ? kept : 0;
        const int incl = wave_incl_scan(k);
        const int nr = before ? rs0.n : 0;
        const int rincl = wave_incl_scan(nr);
        if (k) {
            // restart markers go to the image's list in stream order (ordinal = markers before)
            RstSink rs{0, obase + (incl - k), nr ? rst + (int64_t)i * rst_cap : nullptr,
                       tile_rbase[t] + rincl - nr, (int32_t)min<int64_t>(rst_cap, INT32_MAX)};
            ustf_lane<true>(R, s.scan_len, a, end_at, end_err, sb + (incl - k), giveup, rs);
        }
        const int tile_kept = __shfl(incl, 63);
        __builtin_amdgcn_wave_barrier();
        // copy out: bytes up to the first 16-byte boundary and after the last one byte-wise
        // (they may share a 16-byte unit with the neighbouring tiles), the rest as 16-byte units
        const int64_t nout = min<int64_t>(tile_kept, s.ulen - obase);
        uint8_t* dst = U + (int64_t)i * ucap + obase;  // U + i*ucap is 4 KiB aligned
        const int head = (int)min<int64_t>(nout, (16 - (obase & 15)) & 15);
        const int nunit = (int)((nout - head) >> 4);
        const int tail0 = head + nunit * 16;
        if (lane < head) dst[lane] = sb[lane];
        if (lane < nout - tail0) dst[tail0 + lane] = sb[tail0 + lane];
        for (int u = lane; u < nunit; u += 64) {
            const int b0 = head + 16 * u, shb = (b0 & 3) * 8;
            const uint32_t* q = sbuf + (b0 >> 2);
            uint32_t v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (uint32_t)((((uint64_t)q[j + 1] << 32) | q[j]) >> shb);
            *reinterpret_cast<uint4*>(dst + b0) = make_uint4(v[0], v[1], v[2], v[3]);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// -------------------------------------------------------------------- entropy lanes
// Step tables (icx_step.h), one set per image, built once per group from the parsed Huffman
// tables; each workgroup below stages the format it decodes with into LDS.
__global__ __launch_bounds__(256) void k_step_tabs(int n, const Desc* __restrict__ desc, StepSet* __restrict__ steps) {
    __shared__ Huff h[4];
    const int i = blockIdx.x;
    if (i >= n || desc[i].status != kPending) return;
    {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(&desc[i].huff[0]);
        uint32_t* dst = reinterpret_cast<uint32_t*>(&h[0]);
        for (int k = threadIdx.x; k < (int)(sizeof(h) / 4); k += blockDim.x) dst[k] = src[k];
    }
    __syncthreads();
    StepSet& S = steps[i];
    for (int k = threadIdx.x; k < ScanTab::entries(); k += blockDim.x) S.scan.fill(h, k);
    for (int k = threadIdx.x; k < WriteTab::entries(); k += blockDim.x) S.write.fill(h, k);
}

template <class Tab>
__device__ __forceinline__ void stage_tab(Tab& T, const Tab& src) {
    static_assert(sizeof(Tab) % 16 == 0, "16-byte copies");
    const uint4* s = reinterpret_cast<const uint4*>(&src);
    uint4* d = reinterpret_cast<uint4*>(&T);
    for (int k = threadIdx.x; k < (int)(sizeof(Tab) / 16); k += blockDim.x) d[k] = s[k];
}
__device__ __forceinline__ const ScanTab& set_part(const StepSet& S, const ScanTab*) { return S.scan; }
__device__ __forceinline__ const WriteTab& set_part(const StepSet& S, const WriteTab*) { return S.write; }

// Workgroup wg of a flat numbering (prefix pre over images): the image, with its tables staged.
template <class Tab>
__device__ __forceinline__ int wg_image_setup(const int32_t* pre, int n, int wg, int& cur, Tab& T,
                                              const StepSet* steps) {
    const int i = find_image(pre, n, wg);
    if (i != cur) {
        __syncthreads();
        stage_tab(T, set_part(steps[i], (const Tab*)nullptr));
        __syncthreads();
        cur = i;
    }
    return i;
}

// NL lanes per workgroup; `wpre` numbers each image's lanes in NL-lane groups (totals[tsel]).
template <int NL>
__global__ __launch_bounds__(NL) void k_spec_guess(int n, const Desc* __restrict__ desc, const SpecImg* __restrict__ spec,
                                                   const int32_t* __restrict__ wpre, const int32_t* __restrict__ totals,
                                                   int tsel, const StepSet* __restrict__ steps,
                                                   const uint8_t* __restrict__ U, int64_t ucap, uint64_t* __restrict__ X,
                                                   RecState* __restrict__ rec, int32_t* __restrict__ nrec,
                                                   int32_t* __restrict__ gtot) {
    __shared__ ScanTab T;
    int cur = -1;
    const int total = totals[tsel];
    for (int wg = blockIdx.x; wg < total; wg += gridDim.x) {
        const int i = wg_image_setup(wpre, n, wg, cur, T, steps);
        const SpecImg& s = spec[i];
        if (s.mode != 1) continue;  // uniform per workgroup
        const int64_t j = (int64_t)(wg - wpre[i]) * NL + threadIdx.x;
        if (j >= s.nsub - 1) continue;  // the last lane's exit is never needed
        const int64_t f = (int64_t)s.wg_base * kLanes + j;
        const int64_t sb = (int64_t)kSubBytes * 8;
        X[f] = lane_guess(U + (int64_t)i * ucap, s.ulen, T, desc[i].huff, make_sel(desc[i]), j * sb, (j + 1) * sb, 0,
                          rec + f * kRec, nrec + f, gtot + 4 * f);
    }
}

template <int NL>
__global__ __launch_bounds__(NL) void k_spec_count(int n, const Desc* __restrict__ desc, SpecImg* __restrict__ spec,
                                                   const int32_t* __restrict__ wpre, const int32_t* __restrict__ totals,
                                                   int tsel, const StepSet* __restrict__ steps,
                                                   const uint8_t* __restrict__ U, int64_t ucap,
                                                   const uint64_t* __restrict__ X, uint64_t* __restrict__ Y,
                                                   const RecState* __restrict__ rec, const int32_t* __restrict__ nrec,
                                                   const int32_t* __restrict__ gtot, SubRec* __restrict__ sub,
                                                   int32_t* __restrict__ repair) {
    __shared__ ScanTab T;
    int cur = -1;
    const int total = totals[tsel];
    for (int wg = blockIdx.x; wg < total; wg += gridDim.x) {
        const int i = wg_image_setup(wpre, n, wg, cur, T, steps);
        SpecImg& s = spec[i];
        if (s.mode != 1) continue;  // uniform per workgroup
        const int64_t j = (int64_t)(wg - wpre[i]) * NL + threadIdx.x;
        if (j >= s.nsub - 1) continue;
        const int64_t base = (int64_t)s.wg_base * kLanes, f = base + j;
        const int64_t sb = (int64_t)kSubBytes * 8;
        const uint64_t entry = j == 0 ? pack_state(0, 0, 0) : X[f - 1];
        SubRec out;
        bool synced;
        Y[f] = lane_count(U + (int64_t)i * ucap, s.ulen, T, desc[i].huff, make_sel(desc[i]), entry, j * sb, (j + 1) * sb,
                          rec + f * kRec, nrec[f], gtot + 4 * f, X[f], out, synced);
        sub[f] = out;
        if (out.mism) {  // queue for the serial repair walk
            const int q = atomicAdd(&s.nrepair, 1);
            if (q < kMaxRepair) repair[(int64_t)i * kMaxRepair + q] = (int32_t)j;
        }
    }
}

// One workgroup per image with queued lanes; lane 0 walks them in order (they are rare:
// a guess lane that never resynchronised inside its 2 KiB).
__global__ __launch_bounds__(64) void k_spec_repair(int n, const Desc* __restrict__ desc, SpecImg* __restrict__ spec,
                                                    const StepSet* __restrict__ steps,
                                                    const uint8_t* __restrict__ U, int64_t ucap, uint64_t* __restrict__ X,
                                                    const uint64_t* __restrict__ Y, const RecState* __restrict__ rec,
                                                    const int32_t* __restrict__ nrec, const int32_t* __restrict__ gtot,
                                                    SubRec* __restrict__ sub, int32_t* __restrict__ repair) {
    __shared__ ScanTab T;
    const int i = blockIdx.x;
    SpecImg& s = spec[i];
    if (s.mode != 1 || s.nrepair == 0) return;
    stage_tab(T, steps[i].scan);
    __syncthreads();
    if (threadIdx.x != 0) return;
    if (s.nrepair > kMaxRepair) { s.mode = 2; return; }
    int32_t* q = repair + (int64_t)i * kMaxRepair;
    const int nq = s.nrepair;
    for (int a = 1; a < nq; ++a) {  // insertion sort (short list)
        const int32_t v = q[a];
        int c = a - 1;
        while (c >= 0 && q[c] > v) { q[c + 1] = q[c]; --c; }
        q[c + 1] = v;
    }
    const int64_t base = (int64_t)s.wg_base * kLanes;
    int64_t done = -1;
    for (int a = 0; a < nq; ++a) {
        const int64_t j = q[a];
        if (j <= done) continue;  // re-derived by an earlier walk
        done = repair_walk(U + (int64_t)i * ucap, s.ulen, T, desc[i].huff, make_sel(desc[i]), j, s.nsub, (int64_t)kSubBytes * 8, X + base,
                           Y + base, rec + base * kRec, nrec + base, gtot + 4 * base, sub + base, 64);
        if (done < 0) { s.mode = 2; return; }  // pathological stream: sequential decode
    }
}

// Per image: block index and DC predictors at every lane entry (after repair all lane
// chains agree, so these are the true values).
__global__ __launch_bounds__(256) void k_spec_scan(int n, SpecImg* __restrict__ spec, SubRec* __restrict__ sub,
                                                   LaneEntry* __restrict__ ent) {
    __shared__ int sh[256];
    __shared__ int s_cnt, s_d0, s_d1, s_d2;
    const int i = blockIdx.x;
    if (i >= n) return;
    SpecImg& s = spec[i];
    if (s.mode != 1) return;
    if (s.err & kSpecGiveUp) { if (threadIdx.x == 0) s.mode = 2; return; }
    const int64_t base = (int64_t)s.wg_base * kLanes;
    int64_t G = 0;
    int32_t P0 = 0, P1 = 0, P2 = 0;
    for (int64_t j0 = 0; j0 < s.nsub; j0 += blockDim.x) {
        const int64_t j = j0 + threadIdx.x;
        const bool live = j < s.nsub - 1;
        const SubRec rec = live ? sub[base + j] : SubRec{0, 0, 0, 0, 0};
        // int32 prefix sums (wrap-around adds commute, matching dcpred += diff)
        const int e = block_exclusive_scan(rec.cnt, sh);
        const int e0 = block_exclusive_scan(rec.ds0, sh);
        const int e1 = block_exclusive_scan(rec.ds1, sh);
        const int e2 = block_exclusive_scan(rec.ds2, sh);
        if (j < s.nsub) {
            LaneEntry le;
            le.G = G + e;
            le.p0 = wadd(P0, e0);
            le.p1 = wadd(P1, e1);
            le.p2 = wadd(P2, e2);
            ent[base + j] = le;
        }
        if (threadIdx.x == blockDim.x - 1) {
            s_cnt = e + rec.cnt;
            s_d0 = wadd(e0, rec.ds0);
            s_d1 = wadd(e1, rec.ds1);
            s_d2 = wadd(e2, rec.ds2);
        }
        __syncthreads();
        G += s_cnt;
        P0 = wadd(P0, s_d0);
        P1 = wadd(P1, s_d1);
        P2 = wadd(P2, s_d2);
        __syncthreads();
    }
}

// One flat loop over lookups per lane (lanes of a wave never wait for each other at block
// boundaries); each block is assembled in the lane's LDS slot and leaves as eight 16-byte
// stores when it ends (scattered 2-byte global stores amplified HBM writes ~10x).
// 128-byte lane slot; 16-byte chunk q of lane t lives at chunk q ^ (t & 7), so the b128 reads
// of a 16-lane group hit distinct banks.
__device__ __forceinline__ int slot_elem(int t, int n) { return (((n >> 3) ^ (t & 7)) << 3) | (n & 7); }

// NL lanes per workgroup; `wpre` numbers the image's lanes in NL-lane groups (wgpre for 256,
// wg2pre for kWriteLanesBig), `total` = totals[1] or totals[2].
template <int NL>
__global__ __launch_bounds__(NL) void k_spec_write(int want, int n, const Desc* __restrict__ desc, SpecImg* __restrict__ spec,
                                                    const int32_t* __restrict__ wpre, const int32_t* __restrict__ totals,
                                                    const StepSet* __restrict__ steps,
                                                    const uint8_t* __restrict__ U, int64_t ucap,
                                                    const uint64_t* __restrict__ X, const LaneEntry* __restrict__ ent,
                                                    int16_t* __restrict__ ac, int32_t* __restrict__ dcv,
                                                    int64_t coef_cap, const int64_t* __restrict__ rst, int64_t rst_cap) {
    __shared__ WriteTab T;
    __shared__ int4 slots[NL][8];
    __shared__ uint8_t done_lane[NL / 64][64];  // per wave: lanes that completed a block, by rank
    int cur = -1;
    const int total = totals[NL == kLanes ? 1 : 2];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int4* slot = &slots[threadIdx.x][0];
    int16_t* sv = reinterpret_cast<int16_t*>(slot);
#pragma unroll
    for (int q = 0; q < 8; ++q) slot[q] = make_int4(0, 0, 0, 0);
    for (int wg = blockIdx.x; wg < total; wg += gridDim.x) {
        const int i = wg_image_setup(wpre, n, wg, cur, T, steps);
        SpecImg& s = spec[i];
        // uniform per workgroup; `want` (1 or 3) limits a launch to one mode
        if ((s.mode != 1 && s.mode != 3) || (want && s.mode != want)) continue;
        const bool dri = s.mode == 3;
        const int64_t j = (int64_t)(wg - wpre[i]) * NL + threadIdx.x;
        const Sel S = make_sel(desc[i]);
        const Huff* H = desc[i].huff;
        // DRI: lane j = restart interval j, from the byte after marker j-1, exactly R MCUs, DC 0
        const int64_t* RS = rst + (int64_t)i * rst_cap;
        const int64_t iblocks = (int64_t)desc[i].restart * desc[i].bpm;
        bool lane_ok = true;
        int64_t start_byte = 0;
        if (dri && j < s.nsub && j > 0) {
            if (j - 1 < s.nrst && j - 1 < rst_cap) start_byte = (RS[j - 1] >> 3) + 2;
            else lane_ok = false;  // marker missing: the sequential decoder decides
        }
        const int64_t base = (int64_t)s.wg_base * kLanes;
        const int64_t errbits = s.errpos == INT64_MAX ? INT64_MAX : s.errpos * 8;
        int4* A = reinterpret_cast<int4*>(ac + (int64_t)i * coef_cap * 64);
        int32_t* D = dcv + (int64_t)i * coef_cap;
        const int64_t total_blocks = s.total_blocks;
        bool act = j < s.nsub && lane_ok;
        // every lane runs a reader (lanes past the image's last lane idle at position 0)
        const uint64_t entry = dri ? pack_state(start_byte * 8, 0, 0)
                                   : ((!act || j == 0) ? pack_state(0, 0, 0) : X[base + j - 1]);
        Reader r;
        r.init(U + (int64_t)i * ucap, s.ulen, st_pos(entry));
        int b = st_b(entry), z = st_z(entry), ci = 0;
        int32_t pred[3] = {0, 0, 0};
        int64_t bi = 0, limit = 0;
        bool bad = false;
        // the block in progress at entry belongs to the previous lane
        while (z != 0) (void)write_step(r, T, H, S, b, z, false);
        // lane-relative 32-bit bounds: territory end and the first fetch that is a syntax error
        const int64_t e0 = st_pos(entry);
        const uint32_t kFar = 1u << 30;
        const uint32_t err_rel = errbits == INT64_MAX ? kFar : (uint32_t)min<int64_t>(kFar, max<int64_t>(0, errbits - e0));
        uint32_t lim_rel = kFar;
        int64_t bend = total_blocks;  // block index the lane stops at
        uint32_t used_end = 0;        // bits consumed when the lane's last block completed
        if (act && dri) {
            bi = j * iblocks;
            bend = min(total_blocks, bi + iblocks);
            act = bi < bend;
        } else if (act) {
            limit = j == s.nsub - 1 ? INT64_MAX : st_pos(X[base + j]);
            if (limit != INT64_MAX) lim_rel = (uint32_t)min<int64_t>(kFar, max<int64_t>(0, limit - e0));
            const LaneEntry le = ent[base + j];
            pred[0] = le.p0;
            pred[1] = le.p1;
            pred[2] = le.p2;
            bi = le.G;
            act = bi < total_blocks;
        }
        // The predictors come from a load issued before the loop: without this the compiler
        // waits for them at their first use inside the loop with vmcnt(0) -- i.e. for every
        // coefficient store and prefetch in flight -- on every DC code.
        asm volatile("" : "+v"(pred[0]), "+v"(pred[1]), "+v"(pred[2]));
        r.phase();  // the prelude above ran a lane-dependent number of lookups
        // Wave-uniform loop: one lookup (one symbol or a pair) per active lane per iteration,
        // then the wave flushes the blocks its lanes completed together -- eight 128-byte blocks
        // per round, each lane moving one 16-byte chunk LDS -> HBM and zeroing it (coalesced
        // full-line stores, no divergent per-lane flush).
        while (__any(act)) {
            // The reader advances on every lane, active or not (an idle lane decodes harmless
            // garbage; its loads are clamped to U): keeping Reader updates out of divergent
            // branches stops the compiler from routing the in-flight chunk through loop-header
            // copies, which made every iteration wait for the newest load and all stores.
            const bool dc = z == 0;
            if (dc) {  // a block starts: stop at the next lane's territory
                if (r.used >= lim_rel) act = false;
                ci = S.comp(b);
            }
            // NanoJPEG fetches bytes to cover a 16-bit peek before each code (:644); a second
            // symbol is only paired when its own peek stays clear of the error byte
            const uint32_t u0 = r.used;
            const bool peek_bad = u0 + 16 > err_rel;
            const WriteOut o = write_step(r, T, H, S, b, z, u0 + 16 + WriteTab::kAcBits > err_rel);
            bool done = false;
            int64_t bdone = 0;
            if (act) {
                if (peek_bad || o.err || r.used > err_rel) {
                    bad = true;
                    act = false;
                } else {
                    int32_t v1 = o.v1;
                    if (dc) {
                        pred[ci] = wadd(pred[ci], v1);
                        v1 = dc_cell(pred[ci]);
                        if (v1 == kDcEscape) D[bi] = pred[ci];
                    }
                    // zig-zag order (k_idct reorders); an error ends the lane before its slot
                    // could be misused, so the positions are only masked into the slot
                    if (o.w1) sv[slot_elem(threadIdx.x, o.c1 & 63)] = (int16_t)v1;
                    if (o.w2) sv[slot_elem(threadIdx.x, o.c2 & 63)] = (int16_t)o.v2;
                    if (z == 0) {
                        done = true;
                        bdone = bi++;
                        act = bi < bend;
                        used_end = r.used;  // (the reader keeps moving once the lane is idle)
                    }
                }
            }
            const uint64_t m = __ballot(done);
            if (m) {  // wave-uniform; every lane takes part
                if (done) {
                    const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    done_lane[wave][rank] = (uint8_t)lane;
                }
                __builtin_amdgcn_wave_barrier();
                const int cnt = __popcll(m);
                for (int k0 = 0; k0 < cnt; k0 += 8) {
                    const int e = k0 + (lane >> 3), q = lane & 7;
                    const int src = done_lane[wave][min(e, cnt - 1)];
                    const int bsrc = __shfl((int)bdone, src);  // block index of that lane's block
                    if (e < cnt) {
                        const int sl = (wave << 6) | src;
                        int4* sp = &slots[sl][0];
                        const int sq = q ^ (sl & 7);
#ifndef ICX_EXP_NOSTORE  // timing experiment only: drop the coefficient stores
                        A[(int64_t)bsrc * 8 + q] = sp[sq];
#endif
                        sp[sq] = make_int4(0, 0, 0, 0);
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
        if (bad) {
            atomicOr(&s.err, kSpecSyntax);
#pragma unroll
            for (int q = 0; q < 8; ++q) slot[q] = make_int4(0, 0, 0, 0);
        }
        if (dri && j < s.nsub) {
            // NanoJPEG after R MCUs: byte-align, read 16 bits = FF D0+(j&7) (jpeg_dec.h:707-715).
            // The parallel result stands only if that is exactly marker j at the aligned end of
            // the interval and no error byte was in the data; else the sequential decoder runs.
            bool exact = lane_ok && s.errpos == INT64_MAX;
            if (exact && !bad && j + 1 < s.nsub) {
                const int64_t endbyte = (start_byte * 8 + used_end + 7) >> 3;
                exact = j < s.nrst && j < rst_cap && (RS[j] >> 3) == endbyte && (int)(RS[j] & 7) == (int)(j & 7);
            }
            if (!exact) atomicOr(&s.err, kSpecGiveUp);
        }
    }
}

__global__ void k_spec_finish(int n, Desc* __restrict__ desc, SpecImg* __restrict__ spec,
                              int32_t* __restrict__ stats) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SpecImg& s = spec[i];
    if (s.mode == 3 && (s.err & kSpecGiveUp)) s.mode = 2;  // DRI markers not where NanoJPEG reads them
    if (s.mode == 1 || s.mode == 3) desc[i].status = (s.err & kSpecSyntax) ? kSyntaxError : kOk;
    // path statistics: [0] parallel path (incl. DRI intervals), [1] parallel -> sequential
    // fallback, [2] sequential only
    if (s.mode == 1 || s.mode == 3) atomicAdd(&stats[0], 1);
    else if (s.mode == 2) atomicAdd(&stats[1], 1);
    else if (desc[i].status == kPending) atomicAdd(&stats[2], 1);
}

void launch_spec_entropy(const GroupWs& ws, int n, const uint8_t* d_data, const uint64_t* d_off, hipStream_t st,
                         StageHook* hook) {
    auto B = [&](Stage s) { if (hook) hook->begin(s, st); };
    auto E = [&](Stage s) { if (hook) hook->end(s, st); };
    const int g = 2048;  // grid-stride launches: >> 256 CUs
    B(kStUnstuff);
    hipLaunchKernelGGL(k_spec_plan, dim3(1), dim3(1024), 0, st, n, ws.desc, ws.spec, ws.tilepre, ws.wgpre, ws.wg2pre,
                       ws.totals, ws.ucap);
    hipLaunchKernelGGL(k_step_tabs, dim3(n), dim3(256), 0, st, n, ws.desc, ws.steps);
    hipLaunchKernelGGL(k_ustf_count, dim3(g), dim3(256), 0, st, n, d_data, d_off, ws.desc, ws.spec, ws.tilepre,
                       ws.totals, ws.tiles);
    hipLaunchKernelGGL(k_ustf_scan, dim3(n), dim3(256), 0, st, n, ws.spec, ws.tiles, ws.tile_obase, ws.tile_rbase,
                       ws.U, ws.ucap);
    hipLaunchKernelGGL(k_ustf_write, dim3(g), dim3(256), 0, st, n, d_data, d_off, ws.desc, ws.spec, ws.tilepre,
                       ws.totals, ws.tiles, ws.tile_obase, ws.tile_rbase, ws.U, ws.ucap, ws.rst, ws.rst_cap);
    E(kStUnstuff);
    B(kStEntropy);
    // guess / count: 512-lane workgroups (the 41 KB scan tables amortised over more lanes)
    hipLaunchKernelGGL(k_spec_guess<kWriteLanesBig>, dim3(g), dim3(kWriteLanesBig), 0, st, n, ws.desc, ws.spec, ws.wg2pre,
                       ws.totals, 2, ws.steps, ws.U, ws.ucap, ws.X, ws.rec, ws.nrec, ws.guess_cnt);
    hipLaunchKernelGGL(k_spec_count<kWriteLanesBig>, dim3(g), dim3(kWriteLanesBig), 0, st, n, ws.desc, ws.spec, ws.wg2pre,
                       ws.totals, 2, ws.steps, ws.U, ws.ucap, ws.X, ws.Y, ws.rec, ws.nrec, ws.guess_cnt, ws.sub, ws.repair);
    hipLaunchKernelGGL(k_spec_repair, dim3(n), dim3(64), 0, st, n, ws.desc, ws.spec, ws.steps, ws.U, ws.ucap, ws.X, ws.Y,
                       ws.rec, ws.nrec, ws.guess_cnt, ws.sub, ws.repair);
    hipLaunchKernelGGL(k_spec_scan, dim3(n), dim3(256), 0, st, n, ws.spec, ws.sub, ws.ent);
    E(kStEntropy);
    B(kStWrite);
    if ((int64_t)ws.max_w * ws.max_h >= (int64_t)2048 * 2048) {  // >= 1 MB of entropy data per image
        // 2 KiB subsequences: 512-lane workgroups (tables amortised); restart intervals (DRI,
        // typically one per MCU row, so a few hundred long lanes per image): 256-lane workgroups,
        // which a 512-lane numbering would leave half idle
        hipLaunchKernelGGL(k_spec_write<kWriteLanesBig>, dim3(g), dim3(kWriteLanesBig), 0, st, 1, n, ws.desc, ws.spec,
                           ws.wg2pre, ws.totals, ws.steps, ws.U, ws.ucap, ws.X, ws.ent, ws.ac, ws.dc, ws.coef_cap, ws.rst, ws.rst_cap);
        hipLaunchKernelGGL(k_spec_write<kLanes>, dim3(g), dim3(kLanes), 0, st, 3, n, ws.desc, ws.spec, ws.wgpre,
                           ws.totals, ws.steps, ws.U, ws.ucap, ws.X, ws.ent, ws.ac, ws.dc, ws.coef_cap, ws.rst, ws.rst_cap);
    } else {
        hipLaunchKernelGGL(k_spec_write<kLanes>, dim3(g), dim3(kLanes), 0, st, 0, n, ws.desc, ws.spec, ws.wgpre,
                           ws.totals, ws.steps, ws.U, ws.ucap, ws.X, ws.ent, ws.ac, ws.dc, ws.coef_cap, ws.rst, ws.rst_cap);
    }
    E(kStWrite);
    hipLaunchKernelGGL(k_spec_finish, dim3((n + 63) / 64), dim3(64), 0, st, n, ws.desc, ws.spec, ws.stats);
}

}  // namespace icx
