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

#include <algorithm>
#include <cstdlib>
#include <type_traits>

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

__global__ __launch_bounds__(1024) void k_spec_plan(int n, const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
                                                    Desc* __restrict__ desc, SpecImg* __restrict__ spec,
                                                    int32_t* __restrict__ tilepre, int32_t* __restrict__ wgpre,
                                                    int32_t* __restrict__ wg2pre, int32_t* __restrict__ totals,
                                                    int64_t upool, int64_t lanes_cap, int sub_bytes, int64_t pool_cap,
                                                    unsigned long long* __restrict__ pool_next, int gw, int round,
                                                    int last_round, int32_t* __restrict__ defer_out, int dri_min) {
    __shared__ int sh[1024];
    __shared__ int last[7];
    if (round > 0) {  // a later round with nothing deferred plans nothing, at once
        int any = 0;
        for (int i = threadIdx.x; i < n; i += blockDim.x) any |= spec[i].mode == 4;
        if (!__syncthreads_or(any)) {
            if (threadIdx.x == 0) {
                totals[0] = totals[1] = totals[2] = 0;
                tilepre[n] = wgpre[n] = wg2pre[n] = 0;
                if (defer_out) defer_out[0] = defer_out[1] = defer_out[2] = 0;
            }
            return;
        }
    }
    int carry_t = 0, carry_w = 0, carry_w2 = 0, carry_u = 0, carry_c = 0, carry_r = 0, carry_a = 0, carry_d = 0, carry_i = 0, carry_k = 0;
    const int64_t pool_units = upool >> 12, wg_cap = lanes_cap / kLanes;
    for (int i0 = 0; i0 < n; i0 += blockDim.x) {
        const int i = i0 + threadIdx.x;
        // Candidates, with the work they would take: U pool units (whole 4 KiB, + the reader
        // padding: u_pad_end(ulen) <= ulen + 32, ulen <= scan_len), tiles and lanes.
        // Rounds (launch_spec_entropy): round 0 plans every image; a candidate that does not fit
        // the U pool / lane records is deferred (mode 4) and planned again in the next round, over
        // the pools the earlier round's images no longer need; in the last round it goes to the
        // sequential kernel. Images planned in an earlier round are left alone (mode 5).
        const int64_t scan_len = i < n ? desc[i].size - desc[i].scan_off : 0;
        const bool mine = i < n && (round == 0 || spec[i].mode == 4);
        const bool cand = mine && desc[i].status == kPending && desc[i].nc >= 1 && desc[i].bpm <= kSpecMaxBpm &&
                          scan_len > 0 && scan_len < ((int64_t)1 << 40);
        int nt = 0, nw = 0, nw2 = 0, nu = 0, kint = 0;
        int64_t sb = kSubBytes, nsub = 0, nlanes = 0;
        if (cand) {
            const Desc& d = desc[i];
            nu = (int)min<int64_t>((scan_len + 64 + 4095) >> 12, INT32_MAX / 4);
            nt = (int)ustf_ntiles(scan_len, ustf_align(data + off[i] + d.scan_off));
            // lanes: subsequences of kSubBytesSmall .. kSubBytes unstuffed bytes, sized so the
            // image's lanes fill whole 512-lane workgroups (a 1024^2 q90 image: 512 lanes of
            // 768 B, not 194 lanes of 2 KiB in a workgroup 62% idle); or (DRI) one per
            // restart interval. sub_bytes > 0 (ICX_SUB_BYTES) fixes the size.
            const int64_t nmcu = (int64_t)d.mbw * d.mbh;
            sb = sub_bytes;
            if (sb <= 0) {  // (sub_bytes < 0: experiments with another longest lane, -sub_bytes)
                const int64_t smax = sub_bytes < 0 ? -(int64_t)sub_bytes : kSubBytes;
                const int64_t full = (int64_t)kWriteLanesBig * smax;
                const int64_t nwg = (scan_len + full - 1) / full;
                sb = (scan_len + nwg * kWriteLanesBig - 1) / (nwg * kWriteLanesBig);
                sb = min<int64_t>(smax, max<int64_t>(kSubBytesSmall, (sb + 15) & ~15));
            }
            nsub = d.restart == 0 ? (scan_len + sb - 1) / sb : (nmcu + d.restart - 1) / d.restart;
            // restart intervals on the guess-write path: long intervals, every MCU >= 8 bits
            // (lane_span), cut into kint lanes of at most kSubBytes
            if (d.restart != 0 && gw && dri_min > 0 && scan_len / nsub >= dri_min && min_mcu_bits(d) >= 8) {
                const int64_t avg = scan_len / nsub;
                kint = (int)min<int64_t>(64, max<int64_t>(2, (avg + kSubBytes - 1) / kSubBytes));
                sb = (avg + kint - 1) / kint;
            }
            nlanes = kint ? nsub * kint : nsub;
            nw = (int)min<int64_t>((nlanes + kLanes - 1) / kLanes, INT32_MAX / 4);
            nw2 = (int)((nlanes + kWriteLanesBig - 1) / kWriteLanesBig);
        }
        // Capacity: an image whose U units or lane records would pass the workspace's goes to
        // the sequential kernel. Only subsequence lanes have records (X, rec, sub, ent: a DRI
        // interval lane needs none), numbered apart from the workgroups. The prefixes count
        // every candidate, so they bound what the images taken below use.
        const int nwc = cand && (desc[i].restart == 0 || kint) ? nw : 0;
        const int eu = block_exclusive_scan(nu, sh);
        const int ec = block_exclusive_scan(nwc, sh);
        const bool ok = cand && (int64_t)carry_u + eu + nu <= pool_units && (int64_t)carry_c + ec + nwc <= wg_cap;
        if (threadIdx.x == blockDim.x - 1) { last[3] = eu + nu; last[4] = ec + nwc; }
        if (!ok) nt = nw = nw2 = 0;
        const int nwr = ok ? nwc : 0;
        const int er = block_exclusive_scan(nwr, sh);
        if (threadIdx.x == blockDim.x - 1) last[5] = er + nwr;
        // Coefficient pool region, whole kGwChunk units: a guess-write image gets nsub lanes x
        // gw_S static slots (1.1 x its blocks, so a sequential fallback fits too), every other
        // decodable image its blocks (written in place: k_entropy_seq, the DRI lanes).
        // (round 0 reserves every image's region, a deferred candidate's as for the guess-write
        // path, so the image keeps it in a later round)
        const int64_t tb = i < n && desc[i].status == kPending ? (int64_t)desc[i].mbw * desc[i].mbh * desc[i].bpm : 0;
        const bool gwr = gw && cand && (desc[i].restart == 0 || kint), gwi = gwr && ok;
        const int32_t gS = gwr ? (int32_t)((tb * 11 / 10 + nlanes - 1) / nlanes + 1) : 0;
        const int64_t region = gwr ? nlanes * gS : tb;
        const int na = round ? 0 : (int)min<int64_t>((region + kGwChunk - 1) / kGwChunk, INT32_MAX / 4);
        const int ea = block_exclusive_scan(na, sh);
        if (threadIdx.x == blockDim.x - 1) last[6] = ea + na;
        if (mine) {
            const Desc& d = desc[i];
            SpecImg& s = spec[i];
            s.mode = ok ? (d.restart == 0 || kint ? 1 : 3) : (cand && !last_round ? 4 : 0);
            s.err = 0;
            s.nrepair = 0;
            s.ncount = 0;
            s.dri_first = INT32_MAX;
            s.nrst = 0;
            s.sub_bytes = ok ? (int32_t)sb : kSubBytes;
            s.uoff = ((int64_t)carry_u + eu) << 12;
            s.ulen = 0;
            s.scan_len = ok ? scan_len : 0;
            s.total_blocks = ok ? (int64_t)d.mbw * d.mbh * d.bpm : 0;
            s.nint = ok && (s.mode == 3 || kint) ? (int32_t)nsub : 0;
            s.kint = ok ? kint : 0;
            s.ntiles = nt;
            s.nwg = nw;
            s.gw_S = gS;
            Desc& dd = desc[i];
            if (round == 0) dd.acbase = ((int64_t)carry_a + ea) * kGwChunk;
            dd.mapped = gwi;
            // (cannot happen with the workspace's pool of 2.5 x coef_cap per slot: reported, not written)
            if (round == 0 && dd.acbase + region > pool_cap && dd.status == kPending) {
                dd.status = kOutOfMem;
                s.mode = 0;
                dd.mapped = 0;
            }
        }
        carry_d += __syncthreads_count(mine && !ok && cand && !last_round);  // deferred to the next round
        carry_i += __syncthreads_count(ok && desc[i].restart != 0 && !kint);  // restart-interval lanes (mode 3)
        carry_k += __syncthreads_count(ok && kint);                         // interval-aligned guess-write lanes
        const int et = block_exclusive_scan(nt, sh);
        const int ew = block_exclusive_scan(nw, sh);
        const int ew2 = block_exclusive_scan(nw2, sh);
        if (i < n) {
            tilepre[i] = carry_t + et;
            wgpre[i] = carry_w + ew;
            wg2pre[i] = carry_w2 + ew2;
            spec[i].tile_base = carry_t + et;
            spec[i].wg_base = carry_r + er;  // lane records, in 256-lane units
        }
        if (threadIdx.x == blockDim.x - 1) { last[0] = et + nt; last[1] = ew + nw; last[2] = ew2 + nw2; }
        __syncthreads();
        carry_t += last[0];
        carry_w += last[1];
        carry_w2 += last[2];
        carry_u = min(carry_u + last[3], INT32_MAX / 4);
        carry_c = min(carry_c + last[4], INT32_MAX / 4);
        carry_r += last[5];
        carry_a = min(carry_a + last[6], INT32_MAX / 4);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        tilepre[n] = carry_t;
        wgpre[n] = carry_w;
        wg2pre[n] = carry_w2;
        totals[0] = carry_t;
        totals[1] = carry_w;
        totals[2] = carry_w2;
        // overflow chunks and count blocks from here (a later round goes on from where it is: the
        // earlier rounds' chunks hold their images' blocks)
        if (round == 0) *pool_next = (unsigned long long)carry_a * kGwChunk;
        // images deferred to the next round, for the host (pinned memory: icx_jpeg_batch_decode
        // launches a next round only while there are any)
        if (defer_out) {
            defer_out[0] = carry_d;
            defer_out[1] = carry_i;
            defer_out[2] = carry_k;
        }
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
// Unstuff tiles: one wave per 4 KiB raw tile cut at 16-byte aligned addresses (icx_spec_core.h
// ustf16), four rounds of 64 consecutive aligned 16-byte chunks, one per lane: every load is a
// contiguous 1 KiB per wave instruction. Neighbouring bytes come from the adjacent lanes. Wave
// shuffles give the prefix / min, no block barriers. Each wave walks a contiguous range of the
// flat tile list, so the owning image only ever advances (no per-tile search).
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

struct TileRange {
    int t, t1, i;
};
__device__ __forceinline__ TileRange wave_tiles(const int32_t* tilepre, int n, int total) {
    // w as a wave-uniform value (readfirstlane): derived from threadIdx.x, the compiler would
    // treat the tile loops as divergent (exec-masked loads, vmcnt(0) at every join)
    const int nw = gridDim.x * (blockDim.x >> 6),
              w = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)));
    const int per = (total + nw - 1) / nw;
    TileRange r;
    r.t = min(total, w * per);
    r.t1 = min(total, r.t + per);
    r.i = r.t < r.t1 ? find_image(tilepre, n, r.t) : 0;
    return r;
}

// A tile's four rounds of chunks, loaded up front (4 KiB per wave in flight): lane l of round r
// holds R-relative chunk a = t0 + 1024 r + 16 l (an aligned address). Neighbour bytes of a
// round come from the adjacent lanes, and across rounds from lane 0 / lane 63 of the next /
// previous round; only the tile's first prev dword and last next dword are extra loads.
struct ChunkIn {
    uint32_t D[4];
    int nx;    // R[a+16]
    int prun;  // ff_run4: FF bytes ending at R[a-1]
};
struct TileChunks {
    uint4 V0, V1, V2, V3;  // rounds r, r+1, r+2, r+3 (shifted down after each round)
    uint32_t pw, nx3;      // lane 0: R[a-4 .. a) of the current round; lane 63: R[a+16 ..) of round 3
    int r;
    __device__ __forceinline__ void load(const uint8_t* R, int64_t L, int64_t t0, int lane) {
        static_assert(kTileBytes == 4096, "four 1 KiB rounds");
        // Unconditional loads from clamped addresses (the last aligned chunk holding scan bytes),
        // zero-selected past the data: a load inside a branch gets its own vmcnt(0) at the join.
        const int64_t alast = ((int64_t)(ustf_align(R) + L - 1) & ~(int64_t)15) - ustf_align(R);
        auto ld = [&](int64_t a) {
            const uint4 v = gload16(R + (a < L ? a : alast));
            return a < L ? v : make_uint4(0u, 0u, 0u, 0u);
        };
        const int64_t a0 = t0 + lane * 16;
        V0 = ld(a0); V1 = ld(a0 + 1024); V2 = ld(a0 + 2048); V3 = ld(a0 + 3072);
        // R[t0-4 .. t0) (headers before the scan when t0 < 1: inside the file, unused), and the
        // dword after the tile
        const uint32_t p = gload4(R + t0 - 4);
        pw = t0 >= 1 ? p : 0u;
        const int64_t an = t0 + kTileBytes;
        const uint32_t q = gload4(R + (an < L ? an : alast));
        nx3 = an < L ? q : 0u;
        r = 0;
    }
    // the current round's chunk, then advance (wave-level: every lane calls it)
    __device__ __forceinline__ ChunkIn next(int64_t a, int lane) {
        ChunkIn c;
        c.D[0] = V0.x; c.D[1] = V0.y; c.D[2] = V0.z; c.D[3] = V0.w;
        uint32_t p = __shfl_up(V0.w, 1);
        if (lane == 0) p = pw;
        uint32_t nw = __shfl_down(V0.x, 1);
        const uint32_t q = __shfl(V1.x, 0);  // the next round's first dword
        if (lane == 63) nw = r == 3 ? nx3 : q;
        pw = __shfl(V0.w, 63);
        V0 = V1; V1 = V2; V2 = V3;
        ++r;
        c.nx = (int)(nw & 0xFFu);
        c.prun = ff_run4(p, a);
        return c;
    }
};
__device__ __forceinline__ int wave_sum(int v) { return __shfl(wave_incl_scan(v), 63); }

// The image owning the wave's current tile, with its scan parameters kept in registers (reloaded
// only when the tile walk crosses into the next image; per-tile reloads were four dependent
// global loads per 4 KiB tile).
struct TileImg {
    int i, t_first, t_end;  // image, its first flat tile, one past its last
    const uint8_t* R;
    int64_t L;
    __device__ __forceinline__ void set(int img, const uint8_t* data, const uint64_t* off, const Desc* desc,
                                        const SpecImg* spec, const int32_t* tilepre) {
        i = __builtin_amdgcn_readfirstlane(img);
        t_first = __builtin_amdgcn_readfirstlane(tilepre[i]);
        t_end = __builtin_amdgcn_readfirstlane(tilepre[i + 1]);
        R = data + off[i] + desc[i].scan_off;
        L = spec[i].scan_len;
    }
    __device__ __forceinline__ int64_t t0(int t) const {  // R-relative start of flat tile t
        return (int64_t)(t - t_first) * kTileBytes - ustf_align(R);
    }
};

__global__ __launch_bounds__(256) void k_ustf_count(int n, const uint8_t* __restrict__ data,
                                                    const uint64_t* __restrict__ off, const Desc* __restrict__ desc,
                                                    SpecImg* __restrict__ spec, const int32_t* __restrict__ tilepre,
                                                    const int32_t* __restrict__ totals, TileRec* __restrict__ tiles) {
    const int lane = threadIdx.x & 63;
    const TileRange tr = wave_tiles(tilepre, n, totals[0]);
    // Software pipelined over the wave's tiles: tile t + 1 is loaded while tile t is scanned.
    TileImg im, imn;
    TileChunks tc, tn;
    if (tr.t < tr.t1) {
        im.set(tr.i, data, off, desc, spec, tilepre);
        tc.load(im.R, im.L, im.t0(tr.t), lane);
    }
    imn = im;
    for (int t = tr.t; t < tr.t1; ++t) {
        if (t + 1 < tr.t1) {  // wave-uniform
            while (t + 1 >= imn.t_end) imn.set(imn.i + 1, data, off, desc, spec, tilepre);
            tn.load(imn.R, imn.L, imn.t0(t + 1), lane);
        }
        const int i = im.i;
        const uint8_t* R = im.R;
        const int64_t L = im.L;
        const int64_t t0 = im.t0(t);
        int32_t giveup = 0;
        int kept = 0, nrst = 0, err = 0;  // per lane until the end of the tile
        long long tend = LLONG_MAX;
        for (int r = 0; r < kTileBytes / 1024 && t0 + r * 1024 < L; ++r) {
            const int64_t a = t0 + r * 1024 + lane * 16;
            RstSink rs{0, 0, nullptr, 0, 0};
            const ChunkIn c = tc.next(a, lane);
            const Ustf16 u = ustf16<false>(R, L, a, c.D, c.nx, c.prun, &giveup, &rs);
            if (__any(u.end_at >= 0)) {  // the tile's data ends in this round (wave-uniform, rare)
                const long long e = wave_min_ll(u.end_at >= 0 ? (long long)u.end_at : LLONG_MAX);
                // kept bytes (and restart markers) before the first end event
                const bool before = u.end_at >= 0 ? u.end_at <= e : a < e;
                kept += before ? u.kept : 0;
                nrst += before ? rs.n : 0;
                const uint64_t owner = __ballot(u.end_at >= 0 && u.end_at == e);
                err = __shfl(u.end_err, __ffsll((long long)owner) - 1);
                tend = e;
                break;
            }
            kept += u.kept;
            nrst += rs.n;
        }
        kept = wave_sum(kept);
        nrst = __any(nrst) ? wave_sum(nrst) : 0;
        if (__any(giveup) && lane == 0) atomicOr(&spec[i].err, kSpecGiveUp);
        if (lane == 0) {
            TileRec rec;
            rec.kept = kept;
            rec.end_at = tend == LLONG_MAX ? -1 : tend;
            rec.end_err = tend == LLONG_MAX ? 0 : err;
            rec.nrst = nrst;
            rec.pad_ = 0;
            tiles[t] = rec;
        }
        tc = tn;
        im = imn;
    }
}

// Per image: exclusive prefix of kept bytes over tiles, data length, error position.
__global__ __launch_bounds__(256) void k_ustf_scan(int n, SpecImg* __restrict__ spec, TileRec* __restrict__ tiles,
                                                   int32_t* __restrict__ tile_obase, int32_t* __restrict__ tile_rbase,
                                                   uint8_t* __restrict__ U) {
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
        uint8_t* u = U + s.uoff;
        for (int64_t p = carry + threadIdx.x; p < u_pad_end(carry); p += blockDim.x) u[p] = 0xFF;
    }
    if (threadIdx.x == 0) {
        s.ulen = carry;
        s.nrst = rcarry;
        s.errpos = (fe != INT32_MAX && tiles[s.tile_base + fe].end_err) ? carry : INT64_MAX;
        const int64_t nsub = carry > 0 ? (carry + s.sub_bytes - 1) / s.sub_bytes : 1;
        s.nsub = s.mode == 3 ? s.nint : (s.kint > 0 ? s.nint * s.kint : (int32_t)nsub);
    }
}

__global__ __launch_bounds__(256) void k_ustf_write(int n, const uint8_t* __restrict__ data,
                                                    const uint64_t* __restrict__ off, const Desc* __restrict__ desc,
                                                    const SpecImg* __restrict__ spec, const int32_t* __restrict__ tilepre,
                                                    const int32_t* __restrict__ totals, const TileRec* __restrict__ tiles,
                                                    const int32_t* __restrict__ tile_obase,
                                                    const int32_t* __restrict__ tile_rbase, uint8_t* __restrict__ U,
                                                    int64_t* __restrict__ rst, int64_t rst_cap) {
    constexpr int kBufW = kTileBytes / 4 + 8;           // per wave: the tile's kept bytes (+ slack)
    __shared__ uint32_t sbuf_all[4][kBufW];
    const int lane = threadIdx.x & 63;
    uint32_t* sbuf = sbuf_all[threadIdx.x >> 6];
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(sbuf);
    const TileRange tr = wave_tiles(tilepre, n, totals[0]);
    // Software pipelined like k_ustf_count: tile t + 1 is loaded while tile t is written.
    TileImg im, imn;
    TileChunks tc, tn;
    int64_t ulen = 0;
    int32_t obv = 0;  // lane k: tile_obase[tb + k] for the current block of 64 tiles
    if (tr.t < tr.t1) {
        im.set(tr.i, data, off, desc, spec, tilepre);
        tc.load(im.R, im.L, im.t0(tr.t), lane);
    }
    imn = im;
    for (int t = tr.t; t < tr.t1; ++t) {
        if (t + 1 < tr.t1) {  // wave-uniform
            while (t + 1 >= imn.t_end) imn.set(imn.i + 1, data, off, desc, spec, tilepre);
            tn.load(imn.R, imn.L, imn.t0(t + 1), lane);
        }
        ulen = spec[im.i].ulen;  // (0 for an image the plan took off the path: its tiles write nothing)
        if (spec[im.i].mode != 1 && spec[im.i].mode != 3) ulen = 0;
        if (t == tr.t || ((t - tr.t) & 63) == 0) obv = tr.t + ((t - tr.t) & ~63) + lane < tr.t1 ? tile_obase[t + lane] : 0;
        const int i = im.i;
        const int64_t obase = __shfl(obv, (t - tr.t) & 63);  // == ulen for every tile past the first end event
        if (obase >= 0 && obase < ulen) {                    // wave-uniform
        const uint8_t* R = im.R;
        const int64_t L = im.L;
        const int64_t t0 = im.t0(t);
        for (int k = lane; k < kBufW / 4; k += 64) reinterpret_cast<uint4*>(sbuf)[k] = make_uint4(0u, 0u, 0u, 0u);
        __builtin_amdgcn_wave_barrier();
        int32_t giveup = 0;
        int kept = 0, nrst = 0;
        for (int r = 0; r < kTileBytes / 1024 && t0 + r * 1024 < L; ++r) {
            const int64_t a = t0 + r * 1024 + lane * 16;
            RstSink rs0{0, 0, nullptr, 0, 0};
            const ChunkIn c = tc.next(a, lane);
            const Ustf16 u = ustf16<true>(R, L, a, c.D, c.nx, c.prun, &giveup, &rs0);
            // (the data's end is rare: the 64-bit wave minimum only runs in a round that has it)
            const long long e = __any(u.end_at >= 0) ? wave_min_ll(u.end_at >= 0 ? (long long)u.end_at : LLONG_MAX)
                                                     : LLONG_MAX;
            const bool before = u.end_at >= 0 ? u.end_at <= e : a < e;
            const int k = before ? u.kept : 0;
            const int incl = wave_incl_scan(k);
            const int nr = before ? rs0.n : 0;
            if (__any(nr)) {  // restart markers go to the image's list in stream order (DRI images)
                const int rincl = wave_incl_scan(nr);
                if (nr) {
                    RstSink rs{0, obase + kept + (incl - k), rst + (int64_t)i * rst_cap, tile_rbase[t] + nrst + rincl - nr,
                               (int32_t)min<int64_t>(rst_cap, INT32_MAX)};
                    (void)ustf16<false>(R, L, a, c.D, c.nx, c.prun, &giveup, &rs);
                }
                nrst += __shfl(rincl, 63);
            }
            if (k) {  // the kept bytes at byte offset ob of the tile buffer (ORed into zeroed dwords)
                const int ob = kept + incl - k, q = ob >> 2, sft = ob & 3;
                const uint32_t* d = u.out;
                if (k == 16 && (ob & 15) == 0) {  // the common case: a whole aligned 16-byte unit of its own
                    reinterpret_cast<uint4*>(sbuf)[q >> 2] = make_uint4(d[0], d[1], d[2], d[3]);
                } else if (sft == 0) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) atomicOr(&sbuf[q + j], d[j]);
                } else {
                    atomicOr(&sbuf[q], d[0] << (8 * sft));
#pragma unroll
                    for (int j = 1; j < 4; ++j) atomicOr(&sbuf[q + j], __builtin_amdgcn_alignbyte(d[j], d[j - 1], 4 - sft));
                    atomicOr(&sbuf[q + 4], d[3] >> (32 - 8 * sft));
                }
            }
            kept += __shfl(incl, 63);
            if (e != LLONG_MAX) break;  // wave-uniform: the data ends in this round
        }
        __builtin_amdgcn_wave_barrier();
        // copy out: bytes up to the first 16-byte boundary and after the last one byte-wise
        // (they may share a 16-byte unit with the neighbouring tiles), the rest as 16-byte units
        const int64_t nout = min<int64_t>(kept, ulen - obase);
        uint8_t* dst = U + spec[i].uoff + obase;  // (uoff is 4 KiB aligned)
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
        tc = tn;
        im = imn;
    }
}

// ---- one-pass unstuff (k_ustf_one: count, scan and write in one launch) ----
// A wave takes tiles in ticket order (an atomic counter), so every tile with a smaller ticket is
// held by a wave that is running or done, and takes its next ticket once its tile's aggregate is
// out. It compacts its tile's kept bytes into LDS, publishes
// the tile's aggregate (kept bytes, restart markers, whether the data ends in it), then looks back
// over the image's earlier tiles -- 64 at a time, one per lane, nearest first -- until it meets an
// inclusive prefix (or the image's first tile), publishes its own inclusive prefix and writes its
// bytes at that offset. The tile that ends the data (or the image's last tile) sets the image's
// length, markers, error position and lane count and writes the reader padding (k_ustf_scan's
// work). A state word is 2 flag bits (1 aggregate, 2 inclusive), an end bit, 21 bits of restart
// markers and 40 bits of kept bytes (scan_len < 2^40); the array is zeroed before each launch.
constexpr uint64_t kTsAgg = 1, kTsInc = 2;
constexpr int kTsRstBits = 21;
__device__ __forceinline__ uint64_t ts_pack(uint64_t flag, bool end, int64_t nrst, int64_t kept) {
    return flag << 62 | (uint64_t)end << 61 | (uint64_t)nrst << 40 | (uint64_t)kept;
}
__device__ __forceinline__ int64_t ts_kept(uint64_t v) { return (int64_t)(v & (((uint64_t)1 << 40) - 1)); }
__device__ __forceinline__ int64_t ts_rst(uint64_t v) { return (int64_t)((v >> 40) & ((1u << kTsRstBits) - 1)); }
__device__ __forceinline__ bool ts_end(uint64_t v) { return (v >> 61) & 1; }
__device__ __forceinline__ long long wave_sum_ll(long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
// The image owning flat tile t: the largest i with pre[i] <= t (pre non-decreasing, pre[0] <= t),
// two rounds of one load per lane for n <= 4096 images.
__device__ __forceinline__ int find_image_wave(const int32_t* pre, int n, int t, int lane) {
    if (n > 4096) return find_image(pre, n, t);
    const int step = (n + 63) >> 6;
    const int k = lane * step;
    const uint64_t m = __ballot(k < n && pre[min(k, n - 1)] <= t);
    const int base = (63 - __clzll((long long)m)) * step;
    const int k2 = base + lane;
    const uint64_t m2 = __ballot(lane < step && k2 < n && pre[min(k2, n - 1)] <= t);
    return base + 63 - __clzll((long long)m2);
}
constexpr int kTsSpinMax = 1 << 22;  // a predecessor that never publishes: the image gives up

__global__ __launch_bounds__(256) void k_ustf_one(int n, const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
                                                  const Desc* __restrict__ desc, SpecImg* __restrict__ spec,
                                                  const int32_t* __restrict__ tilepre, const int32_t* __restrict__ totals,
                                                  uint64_t* __restrict__ tstate, uint8_t* __restrict__ U,
                                                  int64_t* __restrict__ rst, int64_t rst_cap) {
    constexpr int kBufW = kTileBytes / 4 + 8;
    __shared__ uint32_t sbuf_all[4][kBufW];
    const int lane = threadIdx.x & 63;
    uint32_t* sbuf = sbuf_all[threadIdx.x >> 6];
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(sbuf);
    const int total = totals[0];
    unsigned int* ticket = reinterpret_cast<unsigned int*>(tstate + total);  // (one word past the tiles)
    auto take = [&]() {
        int v = 0;
        if (lane == 0) v = (int)atomicAdd(ticket, 1u);
        return __builtin_amdgcn_readfirstlane(__shfl(v, 0));
    };
    // Relaxed (monotonic) agent-scope accesses: a state word carries everything a reader uses, so
    // no ordering with other data is needed -- and an acquire / release at agent scope invalidates /
    // writes back the whole L2 of the XCD on gfx950 (40x slower at C3: every spin iteration
    // emptied the cache under the other waves' tiles).
    auto ts_load = [&](int q) { return __hip_atomic_load(tstate + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    auto ts_store = [&](int q, uint64_t v) {
        if (lane == 0) __hip_atomic_store(tstate + q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    TileImg im, imn;
    TileChunks tc, tn;
    int t = take();
    if (t < total) {
        im.set(find_image_wave(tilepre, n, t, lane), data, off, desc, spec, tilepre);
        tc.load(im.R, im.L, im.t0(t), lane);
    }
    while (t < total) {  // wave-uniform
        const int i = im.i;
        SpecImg& s = spec[i];
        const bool on = s.mode == 1 || s.mode == 3;
        const uint8_t* R = im.R;
        const int64_t L = im.L;
        const int64_t t0 = im.t0(t);
        for (int k = lane; k < kBufW / 4; k += 64) reinterpret_cast<uint4*>(sbuf)[k] = make_uint4(0u, 0u, 0u, 0u);
        __builtin_amdgcn_wave_barrier();
        int32_t giveup = 0;
        int kept = 0, nrst = 0, end_err = 0;
        bool own_end = false;
        for (int r = 0; on && r < kTileBytes / 1024 && t0 + r * 1024 < L; ++r) {
            const int64_t a = t0 + r * 1024 + lane * 16;
            RstSink rs0{0, 0, nullptr, 0, 0};
            const ChunkIn c = tc.next(a, lane);
            const Ustf16 u = ustf16<true>(R, L, a, c.D, c.nx, c.prun, &giveup, &rs0);
            const long long e = __any(u.end_at >= 0) ? wave_min_ll(u.end_at >= 0 ? (long long)u.end_at : LLONG_MAX)
                                                     : LLONG_MAX;
            const bool before = u.end_at >= 0 ? u.end_at <= e : a < e;
            const int k = before ? u.kept : 0;
            const int incl = wave_incl_scan(k);
            nrst += before ? rs0.n : 0;
            if (k) {  // (as k_ustf_write)
                const int ob = kept + incl - k, q = ob >> 2, sft = ob & 3;
                const uint32_t* d = u.out;
                if (k == 16 && (ob & 15) == 0) {
                    reinterpret_cast<uint4*>(sbuf)[q >> 2] = make_uint4(d[0], d[1], d[2], d[3]);
                } else if (sft == 0) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) atomicOr(&sbuf[q + j], d[j]);
                } else {
                    atomicOr(&sbuf[q], d[0] << (8 * sft));
#pragma unroll
                    for (int j = 1; j < 4; ++j) atomicOr(&sbuf[q + j], __builtin_amdgcn_alignbyte(d[j], d[j - 1], 4 - sft));
                    atomicOr(&sbuf[q + 4], d[3] >> (32 - 8 * sft));
                }
            }
            kept += __shfl(incl, 63);
            if (e != LLONG_MAX) {  // wave-uniform: the data ends in this round
                const uint64_t owner = __ballot(u.end_at >= 0 && u.end_at == e);
                end_err = __shfl(u.end_err, __ffsll((long long)owner) - 1);
                own_end = true;
                break;
            }
        }
        nrst = __any(nrst) ? wave_sum(nrst) : 0;
        if (__any(giveup) && lane == 0) atomicOr(&s.err, kSpecGiveUp);
        ts_store(t, ts_pack(kTsAgg, own_end, min(nrst, (1 << kTsRstBits) - 1), kept));
        // The next ticket only now: a wave holding a ticket it has not scanned would make every
        // look-back that reaches that tile wait for this wave's whole current tile (and so on
        // down the tickets: a serial chain). Its image and chunks load during the look-back.
        const int tnx = take();
        if (tnx < total) {
            imn.set(find_image_wave(tilepre, n, tnx, lane), data, off, desc, spec, tilepre);
            tn.load(imn.R, imn.L, imn.t0(tnx), lane);
        }
        // look back: the prefix before this tile (pk bytes, pr markers) and whether the data ended
        // before it (pe)
        int64_t pk = 0, pr = 0, ak = 0, ar = 0;
        bool pe = false, ae = false, stuck = false;
        for (int p = t - 1;; p -= 64) {  // wave-uniform
            const int q = p - lane;
            uint64_t v = ts_pack(kTsInc, false, 0, 0);  // before the image's first tile: prefix 0
            if (q >= im.t_first) {
                int spins = 0;
                for (v = ts_load(q); (v >> 62) == 0 && spins < kTsSpinMax; ++spins) {
                    __builtin_amdgcn_s_sleep(1);
                    v = ts_load(q);
                }
                if ((v >> 62) == 0) {
                    stuck = true;
                    v = ts_pack(kTsInc, false, 0, 0);
                }
            }
            const uint64_t mi = __ballot((v >> 62) == kTsInc);
            const int m = mi ? __ffsll((long long)mi) - 1 : 64;  // nearest inclusive prefix
            const uint64_t vm = __shfl(v, m & 63);
            if (m < 64 && ts_end(vm)) {  // the data ended at or before it: its prefix is final
                pk = ts_kept(vm);
                pr = ts_rst(vm);
                pe = true;
                break;
            }
            // the farthest (earliest) tile below m whose data ends: the tiles nearer than it
            // follow the end and count for nothing, nor does what nearer windows summed
            const uint64_t me = __ballot(lane < m && ts_end(v));
            const int e = me ? 63 - __clzll((long long)me) : -1;
            const bool in = lane < m && lane >= (e < 0 ? 0 : e);
            const int64_t wk = wave_sum_ll(in ? ts_kept(v) : 0), wr = wave_sum_ll(in ? ts_rst(v) : 0);
            if (e >= 0) { ak = wk; ar = wr; ae = true; }
            else { ak += wk; ar += wr; }
            if (m < 64) {
                pk = ts_kept(vm) + ak;
                pr = ts_rst(vm) + ar;
                pe = ae;
                break;
            }
        }
        if (__any(stuck) && lane == 0) atomicOr(&s.err, kSpecGiveUp);
        const int64_t ik = pe ? pk : pk + kept, ir = pe ? pr : pr + nrst;
        if (ir >= (1 << kTsRstBits) && lane == 0) atomicOr(&s.err, kSpecGiveUp);
        ts_store(t, ts_pack(kTsInc, pe || own_end, min<int64_t>(ir, (1 << kTsRstBits) - 1), ik));
        __builtin_amdgcn_wave_barrier();
        if (on && !pe) {
            const int64_t obase = pk;
            if (nrst) {  // restart markers to the image's list in stream order (DRI images): a second
                         // walk of the tile (now in L2), placing them at the known prefix
                TileChunks t2;
                t2.load(R, L, t0, lane);
                int kk = 0, nr_done = 0;
                int32_t gdummy = 0;
                for (int r = 0; r < kTileBytes / 1024 && t0 + r * 1024 < L; ++r) {
                    const int64_t a = t0 + r * 1024 + lane * 16;
                    RstSink rs0{0, 0, nullptr, 0, 0};
                    const ChunkIn c = t2.next(a, lane);
                    const Ustf16 u = ustf16<false>(R, L, a, c.D, c.nx, c.prun, &gdummy, &rs0);
                    const long long e = __any(u.end_at >= 0) ? wave_min_ll(u.end_at >= 0 ? (long long)u.end_at : LLONG_MAX)
                                                             : LLONG_MAX;
                    const bool before = u.end_at >= 0 ? u.end_at <= e : a < e;
                    const int k = before ? u.kept : 0;
                    const int incl = wave_incl_scan(k);
                    const int nr = before ? rs0.n : 0;
                    if (__any(nr)) {
                        const int rincl = wave_incl_scan(nr);
                        if (nr) {
                            RstSink rs{0, obase + kk + (incl - k), rst + (int64_t)i * rst_cap, (int32_t)(pr + nr_done + rincl - nr),
                                       (int32_t)min<int64_t>(rst_cap, INT32_MAX)};
                            (void)ustf16<false>(R, L, a, c.D, c.nx, c.prun, &gdummy, &rs);
                        }
                        nr_done += __shfl(rincl, 63);
                    }
                    kk += __shfl(incl, 63);
                    if (e != LLONG_MAX) break;
                }
            }
            // copy out (as k_ustf_write)
            const int64_t nout = kept;
            uint8_t* dst = U + s.uoff + obase;
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
            if (own_end || t == im.t_end - 1) {  // the data's end: the image's stream is complete
                const int64_t ulen = obase + kept;
                uint8_t* u = U + s.uoff;
                for (int64_t p = ulen + lane; p < u_pad_end(ulen); p += 64) u[p] = 0xFF;
                if (lane == 0) {
                    s.ulen = ulen;
                    s.nrst = (int32_t)ir;
                    s.errpos = own_end && end_err ? ulen : INT64_MAX;
                    const int64_t nsub = ulen > 0 ? (ulen + s.sub_bytes - 1) / s.sub_bytes : 1;
                    s.nsub = s.mode == 3 ? s.nint : (s.kint > 0 ? s.nint * s.kint : (int32_t)nsub);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        t = tnx;
        tc = tn;
        im = imn;
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
#ifdef ICX_EXP_GW8
    for (int k = threadIdx.x; k < ScanTab11::entries(); k += blockDim.x) S.scan11.fill(h, k);
#endif
    if (threadIdx.x == 0) {
        const Sel sel = make_sel(desc[i]);
        set_block_sel(S.scan, h, sel);
        set_block_sel(S.write, h, sel);
#ifdef ICX_EXP_GW8
        set_block_sel(S.scan11, h, sel);
#endif
    }
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
                                                   const uint8_t* __restrict__ U, uint64_t* __restrict__ X,
                                                   RecState* __restrict__ rec, int32_t* __restrict__ nrec,
                                                   int32_t* __restrict__ gtot, int lead) {
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
        const int64_t sb = (int64_t)s.sub_bytes * 8;
        X[f] = lane_guess(U + s.uoff, s.ulen, T, desc[i].huff, make_sel(desc[i]), j * sb, (j + 1) * sb, 0,
                          rec + f * kRec, nrec + f, gtot + 4 * f,
                          // a quarter of the lane, at most 2048 bits (C2's 768-byte lanes, one box,
                          // two rounds each: 1536 bits 160.2-160.7 GP/s, 1024 158.4-158.6, 768 154)
                          lead >= 0 ? lead : min(2048, s.sub_bytes * 2));
    }
}

template <int NL>
__global__ __launch_bounds__(NL) void k_spec_count(int n, const Desc* __restrict__ desc, SpecImg* __restrict__ spec,
                                                   const int32_t* __restrict__ wpre, const int32_t* __restrict__ totals,
                                                   int tsel, const StepSet* __restrict__ steps,
                                                   const uint8_t* __restrict__ U,
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
        const int64_t sb = (int64_t)s.sub_bytes * 8;
        const uint64_t entry = j == 0 ? pack_state(0, 0, 0) : X[f - 1];
        SubRec out;
        bool synced;
        Y[f] = lane_count(U + s.uoff, s.ulen, T, desc[i].huff, make_sel(desc[i]), entry, j * sb, (j + 1) * sb,
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
                                                    const uint8_t* __restrict__ U, uint64_t* __restrict__ X,
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
        done = repair_walk(U + s.uoff, s.ulen, T, desc[i].huff, make_sel(desc[i]), j, s.nsub, (int64_t)s.sub_bytes * 8, X + base,
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

// A pointer every lane of the wave holds, as the compiler's uniform (SGPR) value.
__device__ __forceinline__ const uint8_t* uniform_ptr(const uint8_t* p) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return reinterpret_cast<const uint8_t*>(((uint64_t)hi << 32) | lo);
}
// x + (this lane's bit of the mask m): one v_addc with the mask as its carry-in (a select of 0 / 1
// and an add otherwise).
__device__ __forceinline__ int32_t add_lane_bit(int32_t x, uint64_t m) {
    int32_t r;
    uint64_t c;
    asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(c) : "v"(x), "s"(m));
    return r;
}

__device__ __forceinline__ int32_t sub_lane_bit(int32_t x, uint64_t m) {  // x - (this lane's bit of m)
    int32_t r;
    uint64_t c;
    asm("v_subb_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(c) : "v"(x), "s"(m));
    return r;
}

// One flat loop over lookups per lane (lanes of a wave never wait for each other at block
// boundaries); each block is assembled in the lane's LDS slot and leaves as eight 16-byte
// stores when it ends (scattered 2-byte global stores amplified HBM writes ~10x).
// 128-byte lane slot; 16-byte chunk q of lane t lives at chunk q ^ (t & 7), so the b128 reads
// of a 16-lane group hit distinct banks.
__device__ __forceinline__ int slot_elem(int t, int n) { return n ^ ((t & 7) << 3); }  // = (n/8 ^ t%8)*8 + n%8

// NL lanes per workgroup; `wpre` numbers the image's lanes in NL-lane groups (wgpre for 256,
// wg2pre for kWriteLanesBig), `total` = totals[1] or totals[2].
template <int NL>
__global__ __launch_bounds__(NL) void k_spec_write(int want, int n, const Desc* __restrict__ desc, SpecImg* __restrict__ spec,
                                                    const int32_t* __restrict__ wpre, const int32_t* __restrict__ totals,
                                                    const StepSet* __restrict__ steps,
                                                    const uint8_t* __restrict__ U,
                                                    const uint64_t* __restrict__ X, const LaneEntry* __restrict__ ent,
                                                    int16_t* __restrict__ ac, int32_t* __restrict__ dcv,
                                                    const int64_t* __restrict__ rst, int64_t rst_cap) {
    __shared__ WriteTab T;
    __shared__ int4 slots[NL][8];
    __shared__ uint8_t done_lane[NL / 64][64];  // per wave: lanes that completed a block, by rank
    int cur = -1;
    const int total = totals[NL == kLanes ? 1 : 2];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    int4* slot = &slots[threadIdx.x][0];
    int16_t* sv = reinterpret_cast<int16_t*>(slot);
#pragma unroll
    for (int q = 0; q < 8; ++q) slot[q] = make_int4(0, 0, 0, 0);
    for (int wg = blockIdx.x; wg < total; wg += gridDim.x) {
        {  // uniform per workgroup; `want` (1 or 3) limits a launch to one mode. Tested before the
           // tables are staged: the guess-write path's DRI launch spans every image's workgroups.
            const int m = spec[find_image(wpre, n, wg)].mode;
            if ((m != 1 && m != 3) || (want && m != want)) continue;
        }
        const int i = wg_image_setup(wpre, n, wg, cur, T, steps);
        SpecImg& s = spec[i];
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
        int4* A = reinterpret_cast<int4*>(ac + desc[i].acbase * 64);  // (in place: the image's pool region)
        int32_t* D = dcv + desc[i].acbase;
        const int32_t total_blocks = (int32_t)s.total_blocks;  // (an image's blocks fit 31 bits: <= 65535^2 / 64 x 6)
        bool act = j < s.nsub && lane_ok;
        // every lane runs a reader (lanes past the image's last lane idle at position 0)
        const uint64_t entry = dri ? pack_state(start_byte * 8, 0, 0)
                                   : ((!act || j == 0) ? pack_state(0, 0, 0) : X[base + j - 1]);
        Reader r;
        r.init(U + s.uoff, s.ulen, st_pos(entry));
        r.u = uniform_ptr(r.u);  // (one image per workgroup: the stream base and end chunk stay in SGPRs)
        r.cmax = __builtin_amdgcn_readfirstlane(r.cmax);
        int b = st_b(entry), z = st_z(entry);
        int32_t pred[3] = {0, 0, 0};
        int32_t bi = 0;
        int64_t limit = 0;
        bool bad = false;
        // the block in progress at entry belongs to the previous lane
        while (z != 0) (void)write_step(r, T, H, S, b, z, false);
        // lane-relative 32-bit bounds: territory end and the first fetch that is a syntax error
        const int64_t e0 = st_pos(entry);
        const uint32_t kFar = 1u << 30;
        const uint32_t err_rel = errbits == INT64_MAX ? kFar : (uint32_t)min<int64_t>(kFar, max<int64_t>(0, errbits - e0));
        uint32_t lim_rel = kFar;
        // the loop's error-byte tests as one compare each: u0 + 16 > err_rel, u0 + 16 + kAcBits > err_rel
        const int32_t err_peek = (int32_t)err_rel - 16, err_pair = err_peek - WriteTab::kAcBits;
        int32_t bend = total_blocks;  // block index the lane stops at
        uint32_t used_end = 0;        // bits consumed when the lane's last block completed
        if (act && dri) {
            const int64_t b0 = j * iblocks;
            act = b0 < total_blocks;
            bi = act ? (int32_t)b0 : 0;
            bend = (int32_t)min<int64_t>(total_blocks, b0 + iblocks);
        } else if (act) {
            limit = j == s.nsub - 1 ? INT64_MAX : st_pos(X[base + j]);
            if (limit != INT64_MAX) lim_rel = (uint32_t)min<int64_t>(kFar, max<int64_t>(0, limit - e0));
            const LaneEntry le = ent[base + j];
            pred[0] = le.p0;
            pred[1] = le.p1;
            pred[2] = le.p2;
            act = le.G < total_blocks;
            bi = act ? (int32_t)le.G : 0;
        }
        // DC predictors rotated with the current block's component (as in k_gw_lane): dc0 is the
        // predictor of block b's component, dc1 / dc2 those of the next two in MCU order (NanoJPEG
        // has 1 or 3 components, in order in the MCU); a block end whose next block has another
        // component rotates them by one, and a DC code reads and updates dc0 alone.
        const int c0 = S.comp(b);
        int32_t dc0 = c0 == 0 ? pred[0] : (c0 == 1 ? pred[1] : pred[2]);
        int32_t dc1 = c0 == 0 ? pred[1] : (c0 == 1 ? pred[2] : pred[0]);
        int32_t dc2 = c0 == 0 ? pred[2] : (c0 == 1 ? pred[0] : pred[1]);
        const uint32_t chgm = S.chg_mask();
        // The predictors come from a load issued before the loop: without this the compiler
        // waits for them at their first use inside the loop with vmcnt(0) -- i.e. for every
        // coefficient store and prefetch in flight -- on every DC code.
        asm volatile("" : "+v"(dc0), "+v"(dc1), "+v"(dc2));
        r.phase();  // the prelude above ran a lane-dependent number of lookups
#ifdef ICX_EXP_CYC  // timing experiment only: per-wave loop cycles and iterations (printf)
        const uint64_t cyc0 = clock64();
        int it_w = 0;
#endif
        // Wave-uniform loop: one lookup (one symbol or a pair) per active lane per iteration,
        // then the wave flushes the blocks its lanes completed together -- eight 128-byte blocks
        // per round, each lane moving one 16-byte chunk LDS -> HBM and zeroing it (coalesced
        // full-line stores, no divergent per-lane flush).
        // Active lanes as a wave mask (as in k_gw_lane): the loop test and the block counter's
        // carry are scalar ANDs of single-compare ballots.
        uint64_t am = wave_ballot(act);
        while (am) {
#ifdef ICX_EXP_CYC
            ++it_w;
#endif
            // The reader advances on every lane, active or not (an idle lane decodes harmless
            // garbage; its loads are clamped to U): keeping Reader updates out of divergent
            // branches stops the compiler from routing the in-flight chunk through loop-header
            // copies, which made every iteration wait for the newest load and all stores.
            const bool dc = z == 0;
            // a block starts: stop at the next lane's territory
            am &= ~(wave_ballot(dc) & wave_ballot(r.used >= lim_rel));
            const bool act = lane_in(am);
            // NanoJPEG fetches bytes to cover a 16-bit peek before each code (:644); a second
            // symbol is only paired when its own peek stays clear of the error byte
            const uint32_t u0 = r.used;
            const int bcur = b;
            const WriteOut o = write_step(r, T, H, S, b, z, (int32_t)u0 > err_pair);
            // Bookkeeping by selects, not per-lane branches (each divergent `if` cost its exec-mask
            // save / restore and a branch in every iteration).
            const bool fail = (int32_t)u0 > err_peek || o.err || r.used > err_rel;
            bad = bad || (act && fail);
            const uint64_t okm = am & ~wave_ballot(fail);
            const bool ok = lane_in(okm);
            const bool okdc = ok && dc;
            const int32_t pc = wadd(dc0, o.v1);
            dc0 = okdc ? pc : dc0;
            const bool dc_in = (uint32_t)pc + 32767u < 65535u;  // dc_cell's range test, reused for the escape
            const int32_t cell = dc_in ? pc : kDcEscape;
            if (okdc && !dc_in) D[bi] = pc;  // DC outside int16 (corrupt streams only)
            // Both slot writes always issue (zig-zag order; k_idct reorders). A symbol that writes
            // nothing stores 0 at a coefficient the block has not reached: the cursor (EOB), or
            // the one after the first symbol (no pair) -- which is that symbol's own cell when it
            // was coefficient 63, so the pair's cell is written first and the first symbol's
            // value lands last. A lane that stopped scribbles in its own slot, which is zeroed
            // before its next use.
            // (v1 is 0 for EOB and invalid codes; an invalid DC code fails the lane, so its cell
            // is never stored)
            sv[slot_elem(threadIdx.x, o.n2)] = (int16_t)(o.w2 ? o.v2 : 0);
            sv[slot_elem(threadIdx.x, o.n1)] = (int16_t)(dc ? cell : o.v1);
            const uint64_t m = wave_ballot(z == 0) & okm;
            const bool done = lane_in(m);
            const int32_t bdone = bi;
            bi = add_lane_bit(bi, m);  // bi += done
            am = okm & ~(m & ~wave_ballot(bi < bend));  // act = ok && (!done || bi < bend)
            used_end = done ? r.used : used_end;  // (the reader keeps moving once the lane is idle)
            {  // the block ended: the next block's component (frozen once the lane stopped)
                const bool rot = done && ubfe(chgm, (uint32_t)bcur, 1u) != 0u;
                const int32_t t0 = dc0;
                dc0 = rot ? dc1 : dc0;
                dc1 = rot ? dc2 : dc1;
                dc2 = rot ? t0 : dc2;
            }
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
                    const int bsrc = __shfl(bdone, src);  // block index of that lane's block
                    if (e < cnt) {
                        const int sl = (wave << 6) | src;
                        int4* sp = &slots[sl][0];
                        const int sq = q ^ (sl & 7);
#ifndef ICX_EXP_NOSTORE  // timing experiment only: drop the coefficient stores
                        {  // streaming (evict-first) stores: the lanes' U lines stay in L2 (fetch 6.3x -> 2.2x U)
                            typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
                            const int4 v = sp[sq];
                            const i32x4 vv = {v.x, v.y, v.z, v.w};
                            __builtin_nontemporal_store(vv, reinterpret_cast<i32x4*>(A) + (int64_t)bsrc * 8 + q);
                        }
#endif
                        sp[sq] = make_int4(0, 0, 0, 0);
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
#ifdef ICX_EXP_CYC
        if (lane == 0 && blockIdx.x % 64 == 0 && wg == (int)blockIdx.x && wave < 2)
            printf("CYC wg %d wave %d iters %d per_iter %llu\n", wg, wave, it_w,
                   (unsigned long long)((clock64() - cyc0) / max(1, it_w)));
#endif
        if (bad) atomicOr(&s.err, kSpecSyntax);
        // stopped lanes scribbled in their slots: zero them for the next workgroup item
#pragma unroll
        for (int q = 0; q < 8; ++q) slot[q] = make_int4(0, 0, 0, 0);
        if (dri && j < s.nsub && lane_ok) {
            // NanoJPEG after R MCUs: byte-align, read 16 bits = FF D0+(j&7) (jpeg_dec.h:707-715).
            // The first interval that does not end at its own marker decides the image
            // (k_spec_finish): a decode error or a wrong marker there is NanoJPEG's syntax error
            // (no sequential decode needed); FF D0+(j&7) read somewhere else than marker j
            // (data bytes that look like it) resumes NanoJPEG where no lane started: sequential.
            // (A lane whose start marker is missing always follows such an interval.)
            int kind = bad ? kDriError : kDriExact;
            if (!bad && j + 1 < s.nsub) {
                const int64_t endbyte = (start_byte * 8 + used_end + 7) >> 3;
                const int64_t rsj = j < s.nrst && j < rst_cap ? RS[j] : -1;
                kind = dri_end_kind(U + s.uoff, s.ulen, s.errpos, endbyte, j, rsj);
            }
            if (kind != kDriExact) atomicMin(&s.dri_first, (int32_t)(2 * j + (kind == kDriElsewhere)));
        }
    }
}

// ======================================================================= guess-write path
// The default for images without restart markers (ICX_GW=0 selects the guess / count / write
// passes above). Each lane decodes once, with the write tables, from `lead` bits before its range
// and stores the blocks that start in its range itself (k_gw_lane); a lane whose first block start
// is not its predecessor's exit (not synchronised at its start) is decoded again from that exit
// up to the first MCU start it shares with the guess (k_gw_check / k_gw_count), and only those
// blocks are stored twice. The blocks land in the group's coefficient pool in lane order; a map
// gives the IDCT each block's pool block and DC offset (k_gw_scan, k_gw_map). The per-lane logic
// is icx_spec_core.h's gw_* / gc_*, which tests/emu/spec_emu.cpp runs lane by lane on the CPU.


// NL lanes per workgroup (the wg2pre numbering: kWriteLanesBig). Two loops per lane:
//  1. the lead: from `lead` bits before the lane's start to its first block start at or after
//     the start (g0), with the scan tables (runs of symbols per lookup; nothing is stored). The
//     scan tables sit in the LDS the slots use later, so they cost no occupancy.
//  2. k_spec_write's loop from g0 -- one lookup per lane per iteration, completed blocks
//     assembled in LDS slots and flushed by the whole wave -- storing every block until the
//     first block start at or after the lane's end (the exit), recording MCU starts for the
//     count lanes' splice.
#ifndef ICX_GW_MINW  // (timing experiments: waves per SIMD k_gw_lane is compiled for)
#define ICX_GW_MINW 1
#endif
// CHK: the instance for images whose data ends in a syntax error (SpecImg::errpos set): every
// lookup tests NanoJPEG's error-byte bounds (ErrBounds). A stream that ends in FF D9 -- every valid
// one -- takes the instance without them (round 6: -4 VALU a lookup). Both are launched; each
// skips the other's images before staging any table. (One kernel with both loops behind a
// uniform branch took 117 VGPRs instead of 95 / 98, and in the two-pipeline step the back half's
// kernels then no longer fit beside it on a SIMD.)
template <int NL, bool CHK>
__global__ __launch_bounds__(NL, ICX_GW_MINW) void k_gw_lane(int n, const Desc* __restrict__ desc, SpecImg* __restrict__ spec,
                                                const int32_t* __restrict__ wpre, const int32_t* __restrict__ totals,
                                                const StepSet* __restrict__ steps, const uint8_t* __restrict__ U,
                                                int16_t* __restrict__ ac, int32_t* __restrict__ dcv,
                                                int32_t* __restrict__ chunk_next, unsigned long long* __restrict__ pool_next,
                                                int64_t pool_cap, uint64_t* __restrict__ X, GwOut* __restrict__ gwo,
                                                RecState* __restrict__ rec, int lead, const int64_t* __restrict__ rst,
                                                int64_t rst_cap) {
    __shared__ WriteTab T;
#ifdef ICX_EXP_GW8  // timing experiment only: 64-byte int8 slots (values truncated), 11-bit lead tables
    constexpr int kSQ = 4;  // 16-byte quarters per slot
    using LeadTab = ScanTab11;
    typedef int8_t Cell;
#else
    constexpr int kSQ = 8;
    using LeadTab = ScanTab;
    typedef int16_t Cell;
#endif
    union SlotsOrScan {  // the lead loop's scan tables, then the write loop's slots
        LeadTab st;
        int4 slots[NL][kSQ];
    };
    static_assert(sizeof(LeadTab) <= sizeof(int4) * NL * kSQ, "scan tables fit the slots' LDS");
    __shared__ SlotsOrScan L;
    __shared__ uint8_t done_lane[NL / 64][64];  // per wave: lanes that completed a block, by rank
    int cur = -1;
    const int total = totals[2];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    int4* slot = &L.slots[threadIdx.x][0];
    Cell* sv = reinterpret_cast<Cell*>(slot);
#ifdef ICX_EXP_GW8
    auto slot_cell = [](int t, int n) { return n ^ ((t & 3) << 4); };
#else
    auto slot_cell = [](int t, int n) { return slot_elem(t, n); };
#endif
    int4* A = reinterpret_cast<int4*>(ac);
    const int32_t scratch = (int32_t)pool_cap;  // (a lane the pool could not hold writes here)
    for (int wg = blockIdx.x; wg < total; wg += gridDim.x) {
        {  // uniform per workgroup; tested before the tables are staged
            const SpecImg& s0 = spec[find_image(wpre, n, wg)];
            if (s0.mode != 1 || (s0.errpos != INT64_MAX) != CHK) continue;
        }
        const int i = wg_image_setup(wpre, n, wg, cur, T, steps);
        SpecImg& s = spec[i];
        __syncthreads();  // (the previous item's slots are done with)
#ifdef ICX_EXP_GW8
        stage_tab(L.st, steps[i].scan11);
#else
        stage_tab(L.st, steps[i].scan);
#endif
        __syncthreads();
        const int64_t j = (int64_t)(wg - wpre[i]) * NL + threadIdx.x;
        const Sel S = make_sel(desc[i]);
        const Huff* H = desc[i].huff;
        const bool act = j < s.nsub;
        const int64_t f = (int64_t)s.wg_base * kLanes + (act ? j : 0);
        // (restart intervals: lane_span cuts each interval into s.kint lanes)
        const LaneSpan ls = lane_span(act ? j : 0, s.nsub, s.sub_bytes, s.ulen, s.kint, s.nint, rst + (int64_t)i * rst_cap,
                                      min<int64_t>(s.nrst, rst_cap));
        const int64_t start = ls.start, end = ls.end;
        const int64_t ld = ls.first ? 0 : (lead >= 0 ? lead : min(kGuessLead, s.sub_bytes * 2));
        const int64_t s0 = act ? max(start - ld, ls.floor) : 0;
        const int bmax = ls.bmax;  // (255, or 0 for an interval's last lane: it exits at an MCU start)
        const uint32_t kFar = 1u << 30;
        const uint32_t pre = act ? (uint32_t)(start - s0) : 0u, span = act ? (uint32_t)(end - s0) : 0u;
        Reader r;
        r.init(U + s.uoff, s.ulen, s0);
        r.u = uniform_ptr(r.u);  // (one image per workgroup: the stream base and end chunk stay in SGPRs)
        r.cmax = __builtin_amdgcn_readfirstlane(r.cmax);
        int b = 0, z = 0;
        {  // 1. the lead
            int32_t v;
            while (!(z == 0 && r.used >= pre)) scan_step(r, L.st, H, S, b, z, v);
        }
        const uint64_t g0 = pack_state(s0 + r.used, b, 0);
        __syncthreads();  // every wave is done with the scan tables: the slots take their LDS
#pragma unroll
        for (int q = 0; q < kSQ; ++q) slot[q] = make_int4(0, 0, 0, 0);
        __builtin_amdgcn_wave_barrier();
        r.phase();  // the lead ran a lane-dependent number of lookups
        ErrBounds eb;
        eb.set(s.errpos == INT64_MAX ? INT64_MAX : s.errpos * 8, s0);
        const int32_t Sst = s.gw_S;
        const int32_t sbase = (int32_t)(desc[i].acbase + j * Sst);
        RecState* R = rec + f * kRec;
        int nrec = 0;
        // Lanes still storing (false from the exit on, and for lanes past the image's last), as a
        // wave mask: every lane condition below is a ballot of one compare ANDed with lane masks
        // in SGPRs, and a lane reads its bit by lane_in (round 6: 6 VALU per lookup fewer than
        // per-lane bools, whose ballots and opaque selects cost two each).
        uint64_t lm = wave_ballot(act);
        int32_t k = 0, err = INT32_MAX, chunk = -1, chunk0 = -1, over = 0, addr = 0;
        // Lane-local DC sums rotated with the current block's component: dc0 is the sum of block
        // b's component, dc1 / dc2 those of the next two in MCU order. An MCU runs through the
        // components in order (0 .. 0, 1 .. 1, 2 .. 2, then block 0 again), so a block end whose
        // next block has another component rotates them by one, and a DC code reads and updates
        // dc0 alone (round 6: 2 compares, 2 selects and 3 predicated updates per lookup became 1
        // bit test and 4 selects). At an MCU start (b == 0, component 0) they are ds[0..2].
        int32_t dc0 = 0, dc1 = 0, dc2 = 0;
        const uint32_t chgm = S.chg_mask();
        uint32_t ul = 0;  // exit: bits read and block-in-MCU there
        int bl = 0;
        int32_t left = Sst, nxt = sbase;  // slots left in the current run (static, then chunks), the next one
        bool rec_on = true;  // some live lane of the wave still records MCU starts (wave-uniform)
        bool any_over = false;  // some lane's pool ran out: its nxt stays at the scratch block (wave-uniform)
        (void)kFar;
        uint32_t span_o = span;
        asm volatile("" : "+v"(span_o));  // (else `u >= span` is folded with `act` into an OR, whose ballot takes a VGPR)
        // 2. store every block from g0 on
        if (lm) do {
            const bool bs = z == 0;
            const uint64_t bsm = wave_ballot(bs);
            const uint32_t u = r.used;
            const uint64_t lvm = bsm & wave_ballot(u >= span_o) & wave_ballot(b <= bmax) & lm;
            if (lvm) {  // (wave-uniform: a lane leaves once, so the exit state's selects run rarely)
                const bool leave = lane_in(lvm);
                ul = leave ? u : ul;
                bl = leave ? b : bl;
            }
            lm &= ~lvm;
            const uint64_t om = bsm & lm;  // live && bs: its lanes own a block start
            const bool own_bs = lane_in(om);
            if (rec_on) {  // (wave-uniform: skipped once every lane has its kRecGw records)
                const uint64_t rcm = om & wave_ballot(b == 0) & wave_ballot(nrec < kRecGw);
                if (rcm) {  // MCU start: a splice point for the count lane
                    if (lane_in(rcm)) {
                        RecState e;
                        e.rel = u - pre;
                        e.b = 0;
                        e.cnt = k;
                        e.ds[0] = dc0;  // (b == 0: the rotation is at component 0)
                        e.ds[1] = dc1;
                        e.ds[2] = dc2;
                        R[nrec] = e;
                        ++nrec;
                    }
                    rec_on = (lm & wave_ballot(nrec < kRecGw)) != 0;
                }
            }
            const uint64_t nm = om & wave_ballot(left == 0);
            if (nm) {  // an overflow chunk from the pool's tail (flat regions)
                if (lane_in(nm)) {
                    const unsigned long long nb = atomicAdd(pool_next, (unsigned long long)kGwChunk);
                    if (nb + kGwChunk <= (unsigned long long)pool_cap) {
                        const int32_t c = (int32_t)(nb / kGwChunk);
                        if (chunk < 0) chunk0 = c;
                        else chunk_next[chunk] = c;
                        chunk = c;
                        nxt = c * kGwChunk;
                    } else {
                        over = 1;
                        nxt = scratch;
                    }
                    left = over ? INT32_MAX : kGwChunk;
                }
                any_over = any_over || wave_any(over != 0);
            }
            addr = own_bs ? nxt : addr;
            nxt = add_lane_bit(nxt, any_over ? om & ~wave_ballot(over != 0) : om);  // nxt += own_bs && !over
            left = sub_lane_bit(left, om);                                           // left -= own_bs
            // one lookup (every lane: the reader moves on idle lanes too, see k_spec_write)
            const uint32_t u0 = r.used;
            const int bcur = b;
            const WriteOut o = write_step(r, T, H, S, b, z, CHK ? eb.near(u0) : false);
            const bool fail = CHK ? eb.fail(u0, o.err, r.used) : o.err;
            err = lane_in(lm) && fail && err == INT32_MAX ? k : err;
            const bool owndc = own_bs;
            const int32_t pc = wadd(dc0, o.v1);
            dc0 = owndc ? pc : dc0;
            const bool dc_in = (uint32_t)pc + 32767u < 65535u;  // dc_cell's range test, reused for the escape
            const int32_t cell = dc_in ? pc : kDcEscape;
            if (owndc && !dc_in) dcv[addr] = pc;  // lane-local DC outside int16 (rare)
            // (v1 is 0 for EOB and invalid codes; an invalid DC code is a decode error, so that
            // block is a discarded speculative one or the image fails)
            sv[slot_cell(threadIdx.x, o.n2)] = (Cell)(o.w2 ? o.v2 : 0);
            sv[slot_cell(threadIdx.x, o.n1)] = (Cell)(bs ? cell : o.v1);
            const uint64_t m = wave_ballot(z == 0) & lm;
            const bool done = lane_in(m);
            k = add_lane_bit(k, m);  // k += done
            {  // the block ended: the next block's component (frozen once the lane left)
                const bool rot = done && ubfe(chgm, (uint32_t)bcur, 1u) != 0u;
                const int32_t t0 = dc0;
                dc0 = rot ? dc1 : dc0;
                dc1 = rot ? dc2 : dc1;
                dc2 = rot ? t0 : dc2;
            }
            if (m) {  // wave-uniform: flush the completed blocks, 8 per round
                if (done) {
                    const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    done_lane[wave][rank] = (uint8_t)lane;
                }
                __builtin_amdgcn_wave_barrier();
                const int cnt = __popcll(m);
                constexpr int kPer = 64 / kSQ;  // blocks per flush round
                for (int k0 = 0; k0 < cnt; k0 += kPer) {
                    const int e = k0 + lane / kSQ, q = lane % kSQ;
                    const int src = done_lane[wave][min(e, cnt - 1)];
                    const int bsrc = __shfl(addr, src);
                    if (e < cnt) {
                        const int sl = (wave << 6) | src;
                        int4* sp = &L.slots[sl][0];
                        const int sq = q ^ (sl & (kSQ - 1));
#ifndef ICX_EXP_NOSTORE  // timing experiment only: drop the coefficient stores
                        typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
                        const int4 v = sp[sq];
                        const i32x4 vv = {v.x, v.y, v.z, v.w};
                        __builtin_nontemporal_store(vv, reinterpret_cast<i32x4*>(A) + (int64_t)bsrc * kSQ + q);
#endif
                        sp[sq] = make_int4(0, 0, 0, 0);
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
        } while (lm);
        if (act) {
            X[f] = pack_state(s0 + ul, bl, 0);
            GwOut g;
            g.g0 = g0;
            g.k = k;
            {  // un-rotate: at the exit the rotation is at block bl's component
                const int c = S.comp(bl);
                g.ds[c] = dc0;
                g.ds[c == 2 ? 0 : c + 1] = dc1;
                g.ds[c == 0 ? 2 : c - 1] = dc2;
            }
            g.err = err;
            g.chunk0 = chunk0;
            g.nrec = nrec;
            g.over = over;
            gwo[f] = g;
            if (over) atomicOr(&s.err, kSpecGiveUp);
        }
    }
}

// Lanes whose first block start is not their predecessor's exit: queued for the count decode
// (one entry per lane, any image); the others are synchronised at their start.
__global__ __launch_bounds__(256) void k_gw_check(int n, SpecImg* __restrict__ spec, const int32_t* __restrict__ wpre,
                                                  const int32_t* __restrict__ totals, const uint64_t* __restrict__ X,
                                                  const GwOut* __restrict__ gwo, GcRec* __restrict__ crec,
                                                  int2* __restrict__ clist, const int64_t* __restrict__ rst, int64_t rst_cap) {
    const int total = totals[1];
    for (int wg = blockIdx.x; wg < total; wg += gridDim.x) {
        const int i = find_image(wpre, n, wg);
        const SpecImg& s = spec[i];
        if (s.mode != 1) continue;
        const int64_t j = (int64_t)(wg - wpre[i]) * kLanes + threadIdx.x;
        if (j >= s.nsub) continue;
        const int64_t f = (int64_t)s.wg_base * kLanes + j;
        // (an image's first lane, and a restart interval's: NanoJPEG's state is known there)
        const LaneSpan ls = lane_span(j, s.nsub, s.sub_bytes, s.ulen, s.kint, s.nint, rst + (int64_t)i * rst_cap,
                                      min<int64_t>(s.nrst, rst_cap));
        const uint64_t entry = ls.first ? pack_state(ls.start, 0, 0) : X[f - 1];
        GcRec c;
        c.chunk0 = -1;
        c.pad_ = 0;
        c.c = 0;
        c.m = -2;
        c.cds[0] = c.cds[1] = c.cds[2] = 0;
        c.err = INT32_MAX;
        crec[f] = c;
        if (gwo[f].g0 != entry) {  // the image's list, in its own lane-record range
            const int q = atomicAdd(&spec[i].ncount, 1);
            clist[(int64_t)s.wg_base * kLanes + q] = make_int2(i, (int)j);
        }
    }
}

// Global-memory block sink of a count lane (gc_walk): a chain of pool chunks taken by atomic add
// as the walk goes; whole 128-byte blocks zeroed, then the decoded cells.
struct ChainSink {
    int16_t* ac;
    int32_t* dcv;
    int32_t* chunk_next;
    unsigned long long* pool_next;
    int64_t pool_cap;
    int32_t chunk0, chunk;
    int64_t cur;
    __device__ bool begin(int32_t t) {
        if (t % kGwChunk == 0) {
            const unsigned long long nb = atomicAdd(pool_next, (unsigned long long)kGwChunk);
            if (nb + kGwChunk > (unsigned long long)pool_cap) return false;
            const int32_t c = (int32_t)(nb / kGwChunk);
            if (chunk < 0) chunk0 = c;
            else chunk_next[chunk] = c;
            chunk = c;
        }
        cur = (int64_t)chunk * kGwChunk + t % kGwChunk;
        int4* p = reinterpret_cast<int4*>(ac + cur * 64);
#pragma unroll
        for (int q = 0; q < 8; ++q) p[q] = make_int4(0, 0, 0, 0);
        return true;
    }
    __device__ void cell(int32_t, int zz, int32_t v) { ac[cur * 64 + zz] = (int16_t)v; }
    __device__ void dc(int32_t, int32_t v) {
        const int16_t c = dc_cell(v);
        ac[cur * 64] = c;
        if (c == kDcEscape) dcv[cur] = v;
    }
};

// A restart-interval image on the guess-write path that its lanes cannot decide exactly (k_gw_scan,
// k_gw_repair): the interval lanes (mode 3) decide it, in place (k_spec_finish clears Desc::mapped).
__device__ __forceinline__ void dri_gw_fallback(SpecImg& s) {
    s.mode = 3;
    s.nsub = s.nint;
    s.err = 0;
    s.dri_first = INT32_MAX;
    s.tail_n = 0;
}

// One count lane (k_gw_count, k_gw_repair): from the true entry to the splice with the guess lane
// (or its whole range), storing those blocks; *exit = its own exit when it did not splice.
__device__ void gw_count_lane(const Desc& d, const SpecImg& s, const StepSet& SS, const uint8_t* U, int64_t j, int64_t f,
                              uint64_t entry, const GwOut& g, const RecState* rec, int16_t* ac, int32_t* dcv,
                              int32_t* chunk_next, unsigned long long* pool_next, int64_t pool_cap, GcRec* crec,
                              uint64_t* exit, int32_t* give_up, const int64_t* RS, int64_t nrst) {
    const Sel S = make_sel(d);
    const LaneSpan ls = lane_span(j, s.nsub, s.sub_bytes, s.ulen, s.kint, s.nint, RS, nrst);
    ChainSink sink{ac, dcv, chunk_next, pool_next, pool_cap, -1, -1, 0};
    GcRec c;
    c.pad_ = 0;
    c.c = gc_walk(U + s.uoff, s.ulen, SS.write, d.huff, S, entry, ls.start, ls.end, rec, g.nrec,
                  s.errpos == INT64_MAX ? INT64_MAX : s.errpos * 8, sink, c.cds, &c.m, exit, &c.err, ls.bmax);
    c.chunk0 = sink.chunk0;
    if (c.m == -3) *give_up = 1;  // the pool ran out
    crec[f] = c;
}

// One workgroup per image: its queued lanes (a few percent of all), one per thread, with the
// image's scan and write tables staged in LDS.
__global__ __launch_bounds__(512) void k_gw_count(int n, const Desc* __restrict__ desc, SpecImg* __restrict__ spec,
                                                  const StepSet* __restrict__ steps, const uint8_t* __restrict__ U,
                                                  const uint64_t* __restrict__ X, const GwOut* __restrict__ gwo,
                                                  const RecState* __restrict__ rec, int16_t* __restrict__ ac,
                                                  int32_t* __restrict__ dcv, int32_t* __restrict__ chunk_next,
                                                  unsigned long long* __restrict__ pool_next, int64_t pool_cap,
                                                  GcRec* __restrict__ crec, uint64_t* __restrict__ Y,
                                                  const int2* __restrict__ clist, int32_t* __restrict__ repair,
                                                  const int64_t* __restrict__ rst, int64_t rst_cap) {
    __shared__ StepSet SS;
    const int i = blockIdx.x;
    if (i >= n) return;
    SpecImg& s = spec[i];
    if (s.mode != 1 || s.ncount == 0) return;
    stage_tab(SS.scan, steps[i].scan);
    stage_tab(SS.write, steps[i].write);
    __syncthreads();
    const int64_t base = (int64_t)s.wg_base * kLanes;
    for (int q = threadIdx.x; q < s.ncount; q += blockDim.x) {
        const int64_t j = clist[base + q].y;
        const int64_t f = base + j;
        uint64_t ex = 0;
        int32_t give_up = 0;
        gw_count_lane(desc[i], s, SS, U, j, f, X[f - 1], gwo[f], rec + f * kRec, ac, dcv, chunk_next, pool_next, pool_cap,
                      crec, &ex, &give_up, rst + (int64_t)i * rst_cap, min<int64_t>(s.nrst, rst_cap));
        if (give_up) atomicOr(&s.err, kSpecGiveUp);
        Y[f] = ex;
        // no splice, another exit: repair walk (not into the next restart interval: its first lane
        // starts in a known state)
        if (crec[f].m < 0 && j + 1 < s.nsub && ex != X[f] && !(s.kint > 0 && (j + 1) % s.kint == 0)) {
            const int r = atomicAdd(&s.nrepair, 1);
            if (r < kMaxRepair) repair[(int64_t)i * kMaxRepair + r] = (int32_t)j;
        }
    }
}

// Serial repair walks (one thread per image with queued lanes): adopt the count lane's exit and
// re-derive the following lanes until one is synchronised at its start or splices.
__global__ __launch_bounds__(64) void k_gw_repair(int n, const Desc* __restrict__ desc, SpecImg* __restrict__ spec,
                                                  const StepSet* __restrict__ steps, const uint8_t* __restrict__ U,
                                                  uint64_t* __restrict__ X, const uint64_t* __restrict__ Y,
                                                  const GwOut* __restrict__ gwo, const RecState* __restrict__ rec,
                                                  int16_t* __restrict__ ac, int32_t* __restrict__ dcv,
                                                  int32_t* __restrict__ chunk_next, unsigned long long* __restrict__ pool_next,
                                                  int64_t pool_cap, GcRec* __restrict__ crec, int32_t* __restrict__ repair,
                                                  const int64_t* __restrict__ rst, int64_t rst_cap) {
    const int i = blockIdx.x;
    if (i >= n || threadIdx.x != 0) return;
    SpecImg& s = spec[i];
    if (s.mode != 1 || s.nrepair == 0) return;
    const int64_t* RS = rst + (int64_t)i * rst_cap;
    const int64_t nrst = min<int64_t>(s.nrst, rst_cap);
    // (too long a walk: the sequential kernel; with restart intervals, their lanes -- mode 3)
    auto give_up_walk = [&] {
        if (s.kint > 0) dri_gw_fallback(s);
        else s.mode = 2;
    };
    if (s.nrepair > kMaxRepair) { give_up_walk(); return; }
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
        if (j <= done) continue;
        X[base + j] = Y[base + j];
        int64_t k = j + 1;
        for (int steps_ = 0; k < s.nsub; ++k, ++steps_) {
            if (s.kint > 0 && k % s.kint == 0) break;  // a restart interval's first lane: synchronised
            if (steps_ >= kGwMaxWalk) { give_up_walk(); return; }
            const int64_t f = base + k;
            if (gwo[f].g0 == X[f - 1]) {
                GcRec c;
                c.chunk0 = -1; c.pad_ = 0; c.c = 0; c.m = -2; c.cds[0] = c.cds[1] = c.cds[2] = 0; c.err = INT32_MAX;
                crec[f] = c;
                break;
            }
            uint64_t ex = 0;
            int32_t give_up = 0;
            gw_count_lane(desc[i], s, steps[i], U, k, f, X[f - 1], gwo[f], rec + f * kRec, ac, dcv, chunk_next, pool_next,
                          pool_cap, crec, &ex, &give_up, RS, nrst);
            if (give_up) { give_up_walk(); return; }
            if (crec[f].m >= 0 || k + 1 == s.nsub || ex == X[f]) break;
            X[f] = ex;
        }
        done = k;
    }
}

// Per image: each lane's first block index and DC predictors (exclusive scans of the lane
// totals), and the status: a decode failure on the true path before the image's last block is
// NanoJPEG's syntax error; blocks that run out before the last one (data ends early) or an
// exhausted pool send the image to the sequential kernel.
__global__ __launch_bounds__(256) void k_gw_scan(int n, Desc* __restrict__ desc, SpecImg* __restrict__ spec,
                                                 const GwOut* __restrict__ gwo, const GcRec* __restrict__ crec,
                                                 const RecState* __restrict__ rec, LaneEntry* __restrict__ ent,
                                                 const uint64_t* __restrict__ X, const uint64_t* __restrict__ Y,
                                                 const uint8_t* __restrict__ U, const int64_t* __restrict__ rst,
                                                 int64_t rst_cap) {
    __shared__ int sh[256];
    __shared__ int s_cnt, s_d0, s_d1, s_d2;
    __shared__ int s_bad;
    const int i = blockIdx.x;
    if (i >= n) return;
    SpecImg& s = spec[i];
    if (s.mode != 1) return;
    if (s.kint > 0) {
        // Restart intervals (round 6): no scan across intervals -- interval m's first block is
        // m R bpm and its DC predictors start at 0 -- one thread per interval chains its kint
        // lanes. The result is NanoJPEG's exactly when every interval holds R MCUs ending at an MCU
        // start in the byte before marker m, which is the expected FF D0+(m&7) at its recorded
        // place (dri_end_kind: exact), with no decode error on the true path, and the last interval
        // reaches the frame's last block. Anything else (corrupt or truncated data, missing
        // markers, an exhausted pool) goes to the interval lanes (mode 3), which decide it.
        const int64_t K = s.kint, nint = s.nint, base = (int64_t)s.wg_base * kLanes;
        const int64_t iblk = (int64_t)desc[i].restart * desc[i].bpm;
        const int64_t* RS = rst + (int64_t)i * rst_cap;
        const int64_t nrst = min<int64_t>(s.nrst, rst_cap);
        if (threadIdx.x == 0) s_bad = (s.err & kSpecGiveUp) != 0 || nrst < nint - 1;
        __syncthreads();
        const bool give_up = s_bad != 0;
        for (int64_t m = threadIdx.x; m < nint && !give_up; m += blockDim.x) {
            const int64_t G0 = m * iblk;
            int32_t cnt = 0, p0 = 0, p1 = 0, p2 = 0;
            bool bad = false;
            for (int64_t ii = 0; ii < K; ++ii) {
                const int64_t f = base + m * K + ii;
                const GwOut g = gwo[f];
                const GcRec c = crec[f];
                int32_t d[3];
                const int32_t nb = gw_lane_total(g, c, rec + f * kRec, d);
                const int32_t e = gw_lane_err(g, c, rec + f * kRec);
                LaneEntry le;
                le.G = G0 + cnt;
                le.p0 = p0;
                le.p1 = p1;
                le.p2 = p2;
                le.pad = nb;
                ent[f] = le;
                if (e != INT32_MAX && le.G + e < s.total_blocks) bad = true;
                cnt += nb;
                p0 = wadd(p0, d[0]);
                p1 = wadd(p1, d[1]);
                p2 = wadd(p2, d[2]);
                if (ii == K - 1 && m + 1 < nint) {  // the interval's end, where NanoJPEG reads marker m
                    const uint64_t ex = c.m == -1 ? Y[f] : X[f];
                    const int64_t em = RS[m] >> 3, p = st_pos(ex);
                    if (st_b(ex) != 0 || p < em * 8 - 7 || p > em * 8) bad = true;
                    if (dri_end_kind(U + s.uoff, s.ulen, s.errpos, em, m, RS[m]) != kDriExact) bad = true;
                }
            }
            if (m + 1 < nint ? cnt != iblk : cnt < s.total_blocks - G0) bad = true;
            if (bad) atomicOr(&s_bad, 1);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            s.tail_n = 0;
            if (s_bad) dri_gw_fallback(s);
        }
        return;
    }
    if (s.err & kSpecGiveUp) {
        if (threadIdx.x == 0) { s.mode = 2; desc[i].mapped = 0; }
        return;
    }
    if (threadIdx.x == 0) s_bad = 0;
    __syncthreads();
    const int64_t base = (int64_t)s.wg_base * kLanes;
    int64_t G = 0;
    int32_t P0 = 0, P1 = 0, P2 = 0;
    for (int64_t j0 = 0; j0 < s.nsub; j0 += blockDim.x) {
        const int64_t j = j0 + threadIdx.x;
        const bool live = j < s.nsub;
        int32_t cnt = 0, d[3] = {0, 0, 0}, e = INT32_MAX;
        if (live) {
            const GwOut g = gwo[base + j];
            const GcRec c = crec[base + j];
            cnt = gw_lane_total(g, c, rec + (base + j) * kRec, d);
            e = gw_lane_err(g, c, rec + (base + j) * kRec);
        }
        // int32 prefix sums (wrap-around adds commute, matching dcpred += diff)
        const int ec = block_exclusive_scan(cnt, sh);
        const int e0 = block_exclusive_scan(d[0], sh);
        const int e1 = block_exclusive_scan(d[1], sh);
        const int e2 = block_exclusive_scan(d[2], sh);
        if (live) {
            LaneEntry le;
            le.G = G + ec;
            le.p0 = wadd(P0, e0);
            le.p1 = wadd(P1, e1);
            le.p2 = wadd(P2, e2);
            le.pad = cnt;
            ent[base + j] = le;
            if (e != INT32_MAX && le.G + e < s.total_blocks) atomicOr(&s_bad, 1);
        }
        if (threadIdx.x == blockDim.x - 1) {
            s_cnt = ec + cnt;
            s_d0 = wadd(e0, d[0]);
            s_d1 = wadd(e1, d[1]);
            s_d2 = wadd(e2, d[2]);
        }
        __syncthreads();
        G += s_cnt;
        P0 = wadd(P0, s_d0);
        P1 = wadd(P1, s_d1);
        P2 = wadd(P2, s_d2);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        s.tail_n = 0;
        if (s_bad) {
            s.err |= kSpecSyntax;
        } else if (G < s.total_blocks) {  // the data ends early: NanoJPEG reads on into the padding (k_gw_tail)
            s.tail_G = G;
            s.tail_n = s.total_blocks - G;
            s.tail_p[0] = P0;
            s.tail_p[1] = P1;
            s.tail_p[2] = P2;
        }
    }
}

// The blocks past the lanes' when the data ends before the frame's last MCU (rare; one thread per
// such image): gw_tail from the last lane's exit, stored in a chunk chain, mapped here.
__global__ __launch_bounds__(64) void k_gw_tail(int n, Desc* __restrict__ desc, SpecImg* __restrict__ spec,
                                                const StepSet* __restrict__ steps, const uint8_t* __restrict__ U,
                                                const uint64_t* __restrict__ X, const uint64_t* __restrict__ Y,
                                                const GcRec* __restrict__ crec, int16_t* __restrict__ ac,
                                                int32_t* __restrict__ dcv, int32_t* __restrict__ chunk_next,
                                                unsigned long long* __restrict__ pool_next, int64_t pool_cap,
                                                uint2* __restrict__ map) {
    const int i = blockIdx.x;
    if (i >= n || threadIdx.x != 0) return;
    SpecImg& s = spec[i];
    if (s.mode != 1 || s.tail_n == 0 || (s.err & kSpecSyntax)) return;
    Desc& d = desc[i];
    const int64_t last = (int64_t)s.wg_base * kLanes + s.nsub - 1;
    const uint64_t entry = crec[last].m == -1 ? Y[last] : X[last];
    const Sel S = make_sel(d);
    ChainSink sink{ac, dcv, chunk_next, pool_next, pool_cap, -1, -1, 0};
    int32_t ds[3], err;
    const int32_t got = gw_tail(U + s.uoff, s.ulen, steps[i].write, d.huff, S, entry, s.tail_n,
                                s.errpos == INT64_MAX ? INT64_MAX : s.errpos * 8, sink, ds, &err);
    if (got < 0) { s.mode = 2; d.mapped = 0; return; }  // the pool ran out: the sequential kernel
    if (err != INT32_MAX) { s.err |= kSpecSyntax; return; }
    GwSlots ts{0, 0, -1, 0};
    for (int32_t t = 0; t < got; ++t) {
        const int64_t nb = s.tail_G + t;
        const int ci = S.comp((int)(nb % d.bpm));
        map[d.acbase + nb] = make_uint2((uint32_t)ts.addr(t, sink.chunk0, chunk_next), (uint32_t)s.tail_p[ci]);
    }
}

// The map entries {pool block, DC offset} of every lane's blocks. A wave takes 64 consecutive lanes:
// each thread loads one lane's records, then the wave writes the lanes' entries one lane after
// the other, one entry per thread per round (512 contiguous bytes per store instruction). Blocks
// in overflow chunks find their chunk by walking the lane's chain (short: flat regions only).
__global__ __launch_bounds__(256) void k_gw_map(int n, const Desc* __restrict__ desc, const SpecImg* __restrict__ spec,
                                                const int32_t* __restrict__ wpre, const int32_t* __restrict__ totals,
                                                const GwOut* __restrict__ gwo, const GcRec* __restrict__ crec,
                                                const RecState* __restrict__ rec, const LaneEntry* __restrict__ ent,
                                                const int32_t* __restrict__ chunk_next, uint2* __restrict__ map) {
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t nchunks = (int64_t)totals[1] * (kLanes / 64);
    for (int64_t C = (int64_t)blockIdx.x * 4 + wave; C < nchunks; C += (int64_t)gridDim.x * 4) {
        const int grp = (int)(C / (kLanes / 64));
        const int i = find_image(wpre, n, grp);
        const SpecImg& s = spec[i];
        if (s.mode != 1 || (s.err & kSpecSyntax)) continue;  // (wave-uniform)
        const int64_t j0 = (int64_t)(grp - wpre[i]) * kLanes + (C % (kLanes / 64)) * 64;
        if (j0 >= s.nsub) continue;
        const Desc& d = desc[i];
        const Sel S = make_sel(d);
        const int32_t Sst = s.gw_S;
        // this thread's lane: its first block, count, offsets and block sources
        const int64_t j = j0 + lane;
        const bool live = j < s.nsub;
        const int64_t f = (int64_t)s.wg_base * kLanes + (live ? j : j0);
        const GwOut g = gwo[f];
        const GcRec c = crec[f];
        const LaneEntry le = ent[f];
        int32_t P0 = le.p0, P1 = le.p1, P2 = le.p2, Q0 = P0, Q1 = P1, Q2 = P2, m0 = 0;
        if (c.m >= 0) {
            const RecState e = rec[f * kRec + c.m];
            m0 = e.cnt;
            Q0 = wadd(P0, wsub(c.cds[0], e.ds[0]));
            Q1 = wadd(P1, wsub(c.cds[1], e.ds[1]));
            Q2 = wadd(P2, wsub(c.cds[2], e.ds[2]));
        }
        const int32_t cc = c.m != -2 ? c.c : 0;
        const int64_t nb = live ? min<int64_t>(le.pad, s.total_blocks - le.G) : 0;
        const int nl = (int)min<int64_t>(64, s.nsub - j0);
        for (int q = 0; q < nl; ++q) {  // wave-uniform: lane q's entries
            const int64_t G = __shfl(le.G, q), nbq = __shfl(nb, q);
            const int32_t ccq = __shfl(cc, q), m0q = __shfl(m0, q), c0q = __shfl(c.chunk0, q), g0q = __shfl(g.chunk0, q);
            const int32_t p0 = __shfl(P0, q), p1 = __shfl(P1, q), p2 = __shfl(P2, q);
            const int32_t q0 = __shfl(Q0, q), q1 = __shfl(Q1, q), q2 = __shfl(Q2, q);
            const int64_t sbase = d.acbase + (j0 + q) * Sst;
            GwSlots gs{sbase, Sst, -1, 0}, cs{0, 0, -1, 0};
            for (int64_t t = lane; t < nbq; t += 64) {
                const int ci = S.comp((int)((G + t) % d.bpm));
                uint2 e;
                if (t < ccq) {
                    e.x = (uint32_t)cs.addr((int32_t)t, c0q, chunk_next);
                    e.y = (uint32_t)(ci == 0 ? p0 : (ci == 1 ? p1 : p2));
                } else {
                    e.x = (uint32_t)gs.addr((int32_t)(t - ccq + m0q), g0q, chunk_next);
                    e.y = (uint32_t)(ci == 0 ? q0 : (ci == 1 ? q1 : q2));
                }
                map[d.acbase + G + t] = e;
            }
        }
    }
}

__global__ void k_spec_finish(int n, Desc* __restrict__ desc, SpecImg* __restrict__ spec,
                              int32_t* __restrict__ stats) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SpecImg& s = spec[i];
    if (s.mode == 4 || s.mode == 5) return;  // deferred to the next round / finished in an earlier one
    if (s.mode == 3 && s.dri_first != INT32_MAX)  // the first interval not ending at its marker
        s.err |= (s.dri_first & 1) ? kSpecGiveUp : kSpecSyntax;
    if (s.mode == 3 && (s.err & kSpecGiveUp)) s.mode = 2;  // NanoJPEG resumes where no lane started
    if (s.mode != 1) desc[i].mapped = 0;  // the sequential kernel writes in place
    if (s.mode == 1 || s.mode == 3) desc[i].status = (s.err & kSpecSyntax) ? kSyntaxError : kOk;
    // path statistics: [0] parallel path (incl. DRI intervals), [1] parallel -> sequential
    // fallback, [2] sequential only
    if (s.mode == 1 || s.mode == 3) atomicAdd(&stats[0], 1);
    else if (s.mode == 2) atomicAdd(&stats[1], 1);
    else if (desc[i].status == kPending) atomicAdd(&stats[2], 1);
    s.mode = 5;
}

void launch_spec_entropy(const GroupWs& ws, int n, const uint8_t* d_data, const uint64_t* d_off, hipStream_t st,
                         StageHook* hook, int part) {
    // Rounds over the group (k_spec_plan): an image that does not fit the U pool / lane records
    // left by the images before it is deferred to the next round instead of the sequential
    // kernel (a batch of 4:4:4 q100 photos at 1.3 B/px overflows a pool sized for 1 B/px). A round
    // with no deferred image costs only its launches (every kernel finds no work).
    // Up to kMaxRounds rounds (ICX_ROUNDS: 1..8). Each round after the first finds the U pool
    // empty, so it plans at least (pool - largest scan) bytes of the deferred images: with the
    // pool at 2 B/px per slot (ws_per_slot) eight rounds hold a group averaging up to ~14 B/px of
    // entropy data (a 4:4:4 q100 photo is 1.3-2.5), and only what is past that, or a scan larger
    // than the whole pool, is left to the sequential kernel. A round with nothing deferred is a
    // handful of empty launches (k_spec_plan finds no deferred image and returns, every other
    // kernel then finds no work) with 1/32 of the grid-stride workgroups; each costs ~0.3% of a
    // C3 step (measured: eight rounds 216.6-216.9 GP/s against 220.9-221.2 with one). So the batch
    // entry launches round 0 alone (part kFrontFirst) and later (part kFrontRest) each next round
    // only while the previous round's k_spec_plan deferred an image (its count in pinned memory,
    // ws.h_defer, read once ws.ev_defer has completed): rounds until nothing is deferred, at most
    // ICX_ROUNDS. kFrontAll (the single-call paths) launches every round unconditionally.
    const int rounds = [] {  // (read per launch: tests vary it)
        const char* e = std::getenv("ICX_ROUNDS");
        return e ? std::max(1, std::min(8, std::atoi(e))) : kMaxRounds;
    }();
    if (part == kFrontFirst) {  // round 0 up to its restart-interval write (kFrontRest finishes it)
        launch_spec_round(ws, n, d_data, d_off, st, hook, 0, rounds == 1, kRoundHead);
        return;
    }
    if (part == kFrontRest) {  // round 0's tail: the restart-interval write only if its plan gave DRI lanes
        const bool known = hipEventSynchronize(ws.ev_defer) == hipSuccess;
        launch_spec_round(ws, n, d_data, d_off, st, hook, 0, rounds == 1,
                          !known || ws.h_defer[1] != 0 ? kRoundTail : ws.h_defer[2] != 0 ? kRoundTailGw : kRoundTailNoDri);
        if (!known) return;
    }
    for (int r = part == kFrontRest ? 1 : 0; r < rounds; ++r) {
        if (part == kFrontRest) {  // the previous round's k_spec_plan: anything deferred?
            if (hipEventSynchronize(ws.ev_defer) != hipSuccess || ws.h_defer[0] == 0) break;
        }
        launch_spec_round(ws, n, d_data, d_off, st, hook, r, r + 1 == rounds, kRoundAll);
    }
}

void launch_spec_round(const GroupWs& ws, int n, const uint8_t* d_data, const uint64_t* d_off, hipStream_t st,
                       StageHook* hook, int round, int last, int piece) {
    auto B = [&](Stage s) { if (hook) hook->begin(s, st); };
    auto E = [&](Stage s) { if (hook) hook->end(s, st); };
    static const int g0 = std::getenv("ICX_EGRID") ? std::max(1, std::atoi(std::getenv("ICX_EGRID"))) : 2048;  // grid-stride launches: >> 256 CUs
    const int g = round == 0 ? g0 : std::max(32, g0 / 32);
    // Guess lanes start kGuessLead bits before their range (ICX_GUESS_LEAD overrides), so they are
    // resynchronised when they reach it and the count lanes splice at their first MCU start.
    // (per image: at most a quarter of a short lane, the lead is extra work on every lane)
    static const int lead = std::getenv("ICX_GUESS_LEAD") ? std::max(0, std::atoi(std::getenv("ICX_GUESS_LEAD"))) : -1;
    // (at least kSubBytesSmall: the lane records are sized for lanes of that length, ws_per_slot)
    static const int sub_env = std::getenv("ICX_SUB_BYTES") ? std::max(kSubBytesSmall, std::atoi(std::getenv("ICX_SUB_BYTES"))) & ~15
                               : std::getenv("ICX_SUB_MAX") ? -(std::max(kSubBytesSmall, std::atoi(std::getenv("ICX_SUB_MAX"))) & ~15) : 0;
    // Guess-write for large images; the three-pass path where lanes are short: a workspace for
    // images of up to kGwMinPixels pixels has them (a 1024^2 q90 image: 512 lanes of 768 B, where
    // the lead and splice records weigh more: C2 159 vs 142-150 GP/s; 2048^2, 1.5 KB lanes: 153
    // vs 148; 4096^2, 2.5 KB lanes: 207 vs 220).
    // ICX_GW=0 / 1 forces one (read per launch: tests run both paths in one process).
    const char* gw_env = std::getenv("ICX_GW");
    const int gw = gw_env ? (std::atoi(gw_env) != 0) : ((int64_t)ws.max_w * ws.max_h > kGwMinPixels ? 1 : 0);
    const bool big = !gw && (std::getenv("ICX_BIG_WG") ? std::atoi(std::getenv("ICX_BIG_WG")) != 0 : true);
    // restart intervals on the guess-write path (ICX_DRI_GW: 0 never, 1 from kSubBytesSmall bytes per
    // interval; read per launch: tests run both paths)
    const char* dri_env = std::getenv("ICX_DRI_GW");
    const int dri_min = dri_env ? (std::atoi(dri_env) != 0 ? kSubBytesSmall : 0) : kDriGwMin;
    if (piece == kRoundAll || piece == kRoundHead) {
        B(kStUnstuff);
        hipLaunchKernelGGL(k_spec_plan, dim3(1), dim3(1024), 0, st, n, d_data, d_off, ws.desc, ws.spec, ws.tilepre, ws.wgpre, ws.wg2pre,
                           ws.totals, ws.upool, ws.lanes_cap, sub_env, ws.pool_cap, ws.pool_next, gw, round, last, ws.h_defer,
                           dri_min);
        (void)hipEventRecord(ws.ev_defer, st);
        if (round == 0)  // (an image's tables serve every round)
            hipLaunchKernelGGL(k_step_tabs, dim3(n), dim3(256), 0, st, n, ws.desc, ws.steps);
        // ICX_USTF1=1: the one-pass unstuff (k_ustf_one, its tile states in the tile records' memory:
        // 8 bytes per tile plus the ticket, of 24 per tile); otherwise count, scan, write
        const char* one_env = std::getenv("ICX_USTF1");
        if (one_env && std::atoi(one_env) != 0) {
            uint64_t* ts = reinterpret_cast<uint64_t*>(ws.tiles);
            (void)hipMemsetAsync(ts, 0, sizeof(uint64_t) * (size_t)(ws.tiles_cap + 2), st);
            hipLaunchKernelGGL(k_ustf_one, dim3(g), dim3(256), 0, st, n, d_data, d_off, ws.desc, ws.spec, ws.tilepre, ws.totals,
                               ts, ws.U, ws.rst, ws.rst_cap);
        } else {
            hipLaunchKernelGGL(k_ustf_count, dim3(g), dim3(256), 0, st, n, d_data, d_off, ws.desc, ws.spec, ws.tilepre,
                               ws.totals, ws.tiles);
            hipLaunchKernelGGL(k_ustf_scan, dim3(n), dim3(256), 0, st, n, ws.spec, ws.tiles, ws.tile_obase, ws.tile_rbase,
                               ws.U);
            hipLaunchKernelGGL(k_ustf_write, dim3(g), dim3(256), 0, st, n, d_data, d_off, ws.desc, ws.spec, ws.tilepre,
                               ws.totals, ws.tiles, ws.tile_obase, ws.tile_rbase, ws.U, ws.rst, ws.rst_cap);
        }
        E(kStUnstuff);
        // Guess-write path (default; ICX_GW=0: guess, count, write)
        if (gw) {
            B(kStWrite);
            hipLaunchKernelGGL((k_gw_lane<kWriteLanesBig, false>), dim3(g), dim3(kWriteLanesBig), 0, st, n, ws.desc, ws.spec,
                               ws.wg2pre, ws.totals, ws.steps, ws.U, ws.ac, ws.dc, ws.chunk_next, ws.pool_next, ws.pool_cap,
                               ws.X, ws.gw, ws.rec, lead, ws.rst, ws.rst_cap);
            // (the CHK instance on a small grid: it usually finds no image of its own, and 2048
            // empty workgroups of 80 KB of LDS each waited ~0.5 ms for LDS beside the other pipeline)
            hipLaunchKernelGGL((k_gw_lane<kWriteLanesBig, true>), dim3(std::min(g, 128)), dim3(kWriteLanesBig), 0, st, n,
                               ws.desc, ws.spec,
                               ws.wg2pre, ws.totals, ws.steps, ws.U, ws.ac, ws.dc, ws.chunk_next, ws.pool_next, ws.pool_cap,
                               ws.X, ws.gw, ws.rec, lead, ws.rst, ws.rst_cap);
            E(kStWrite);
            B(kStEntropy);
            hipLaunchKernelGGL(k_gw_check, dim3(g), dim3(kLanes), 0, st, n, ws.spec, ws.wgpre, ws.totals, ws.X, ws.gw, ws.crec,
                               ws.clist, ws.rst, ws.rst_cap);
            hipLaunchKernelGGL(k_gw_count, dim3(n), dim3(512), 0, st, n, ws.desc, ws.spec, ws.steps, ws.U, ws.X, ws.gw, ws.rec,
                               ws.ac, ws.dc, ws.chunk_next, ws.pool_next, ws.pool_cap, ws.crec, ws.Y, ws.clist, ws.repair,
                               ws.rst, ws.rst_cap);
            hipLaunchKernelGGL(k_gw_repair, dim3(n), dim3(64), 0, st, n, ws.desc, ws.spec, ws.steps, ws.U, ws.X, ws.Y, ws.gw,
                               ws.rec, ws.ac, ws.dc, ws.chunk_next, ws.pool_next, ws.pool_cap, ws.crec, ws.repair, ws.rst,
                               ws.rst_cap);
            hipLaunchKernelGGL(k_gw_scan, dim3(n), dim3(256), 0, st, n, ws.desc, ws.spec, ws.gw, ws.crec, ws.rec, ws.ent, ws.X,
                               ws.Y, ws.U, ws.rst, ws.rst_cap);
            hipLaunchKernelGGL(k_gw_tail, dim3(n), dim3(64), 0, st, n, ws.desc, ws.spec, ws.steps, ws.U, ws.X, ws.Y, ws.crec,
                               ws.ac, ws.dc, ws.chunk_next, ws.pool_next, ws.pool_cap, ws.map);
            hipLaunchKernelGGL(k_gw_map, dim3(g), dim3(kLanes), 0, st, n, ws.desc, ws.spec, ws.wgpre, ws.totals, ws.gw, ws.crec,
                               ws.rec, ws.ent, ws.chunk_next, ws.map);
            E(kStEntropy);
        } else {
        B(kStEntropy);
        // guess / count / write: 512-lane workgroups (tables amortised over more lanes), which each
        // image's lanes fill (k_spec_plan); ICX_BIG_WG=0 selects 256-lane ones (experiments)
        if (big) {
            hipLaunchKernelGGL(k_spec_guess<kWriteLanesBig>, dim3(g), dim3(kWriteLanesBig), 0, st, n, ws.desc, ws.spec, ws.wg2pre,
                               ws.totals, 2, ws.steps, ws.U, ws.X, ws.rec, ws.nrec, ws.guess_cnt, lead);
            hipLaunchKernelGGL(k_spec_count<kWriteLanesBig>, dim3(g), dim3(kWriteLanesBig), 0, st, n, ws.desc, ws.spec, ws.wg2pre,
                               ws.totals, 2, ws.steps, ws.U, ws.X, ws.Y, ws.rec, ws.nrec, ws.guess_cnt, ws.sub, ws.repair);
        } else {
            hipLaunchKernelGGL(k_spec_guess<kLanes>, dim3(g), dim3(kLanes), 0, st, n, ws.desc, ws.spec, ws.wgpre,
                               ws.totals, 1, ws.steps, ws.U, ws.X, ws.rec, ws.nrec, ws.guess_cnt, lead);
            hipLaunchKernelGGL(k_spec_count<kLanes>, dim3(g), dim3(kLanes), 0, st, n, ws.desc, ws.spec, ws.wgpre,
                               ws.totals, 1, ws.steps, ws.U, ws.X, ws.Y, ws.rec, ws.nrec, ws.guess_cnt, ws.sub, ws.repair);
        }
        hipLaunchKernelGGL(k_spec_repair, dim3(n), dim3(64), 0, st, n, ws.desc, ws.spec, ws.steps, ws.U, ws.X, ws.Y,
                           ws.rec, ws.nrec, ws.guess_cnt, ws.sub, ws.repair);
        hipLaunchKernelGGL(k_spec_scan, dim3(n), dim3(256), 0, st, n, ws.spec, ws.sub, ws.ent);
        E(kStEntropy);
        B(kStWrite);
        if (big) {
            // subsequences: 512-lane workgroups; restart intervals (DRI, typically one per MCU row, so
            // a few hundred long lanes per image): 256-lane workgroups, which a 512-lane numbering
            // would leave half idle
            hipLaunchKernelGGL(k_spec_write<kWriteLanesBig>, dim3(g), dim3(kWriteLanesBig), 0, st, 1, n, ws.desc, ws.spec,
                               ws.wg2pre, ws.totals, ws.steps, ws.U, ws.X, ws.ent, ws.ac, ws.dc, ws.rst, ws.rst_cap);
        } else {
            hipLaunchKernelGGL(k_spec_write<kLanes>, dim3(g), dim3(kLanes), 0, st, 0, n, ws.desc, ws.spec, ws.wgpre,
                               ws.totals, ws.steps, ws.U, ws.X, ws.ent, ws.ac, ws.dc, ws.rst, ws.rst_cap);
        }
        E(kStWrite);
        }
    }
    if (piece == kRoundHead) return;
    // the round's tail: restart intervals (DRI) -- one write lane per interval, 256-lane workgroups
    // (the non-big three-pass launch above took them) -- and the round's end
    if ((gw || big) && piece != kRoundTailNoDri) {
        B(kStWrite);  // (the write stage's second bracket: restart-interval lanes)
        // (kRoundTailGw: only fallbacks of guess-write DRI images, rare; 2048 empty workgroups of
        // 48 KB of LDS would cost as much as the CHK instance's did)
        hipLaunchKernelGGL(k_spec_write<kLanes>, dim3(piece == kRoundTailGw ? std::min(g, 128) : g), dim3(kLanes), 0, st, 3,
                           n, ws.desc, ws.spec, ws.wgpre,
                           ws.totals, ws.steps, ws.U, ws.X, ws.ent, ws.ac, ws.dc, ws.rst, ws.rst_cap);
        E(kStWrite);
    }
    hipLaunchKernelGGL(k_spec_finish, dim3((n + 63) / 64), dim3(64), 0, st, n, ws.desc, ws.spec, ws.stats);
}

}  // namespace icx
