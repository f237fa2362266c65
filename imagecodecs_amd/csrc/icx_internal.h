// icx_internal.h -- declarations shared by the host API (icx_api.cpp) and the kernel
// launchers (icx_decode.hip). Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "icx_jpeg.h"

namespace icx {

// ---- speculative parallel entropy decode (icx_spec.hip) ----
constexpr int kTileBytes = 4096;   // raw bytes per unstuff tile (256 lanes x 16 B)
constexpr int kSubBytes = 2560;      // longest decode lane (unstuffed bytes per subsequence)
constexpr int kMaxRounds = 8;        // entropy rounds per group at most (launch_spec_entropy; ICX_ROUNDS 1..8)
constexpr int kPoolPerSlotX4 = 10;   // coefficient pool: 2.5 x an image's blocks per workspace slot (icx_api.cpp)
constexpr int kSubBytesSmall = 512;  // shortest: k_spec_plan sizes each image's lanes in between so
                                     // they fill whole 512-lane workgroups (icx_spec.hip)
constexpr int kRec = 16;           // block-start states a guess lane records for resync
constexpr int kGenericWG = 4096;    // workgroups per launch of the other-sampling back-half kernels
constexpr int kGuessLead = 4096;     // bits a guess lane decodes before its range (k_gw_lane, k_spec_guess):
                                     // at most a quarter of the lane (min(kGuessLead, 2 x lane bytes))
constexpr int kMaxRepair = 1024;   // unsynchronised lanes repaired per image before giving up
constexpr int kLanes = 256;        // lanes per decode workgroup (lane records are numbered in these)
constexpr int kWriteLanesBig = 512;  // write-pass workgroup for large images: tables amortised
                                     // over 512 lanes -> 2 workgroups / CU = 4 waves per SIMD
constexpr int kSpecMaxBpm = 16;    // blocks per MCU handled by the parallel path
enum : int32_t { kSpecSyntax = 1, kSpecGiveUp = 2 };

struct SpecImg {
    int32_t mode;          // 0 not on this path, 1 active, 2 fall back to the sequential kernel,
                           // 3 restart intervals (DRI): one write lane per interval, 4 deferred to the
                           // next round (the pools were full), 5 finished in an earlier round
    int32_t err;           // kSpecSyntax | kSpecGiveUp (atomicOr)
    int32_t ntiles, tile_base;
    int32_t nwg, wg_base;  // 256-lane decode groups; the image's first lane record / 256 (subsequence
                           // images only: a flat numbering over the batch group's lane records)
    int32_t nsub, nrepair;   // lanes; unsynchronised lanes queued for repair
    int32_t nint, nrst;      // DRI (modes 3, and 1 with kint): restart intervals; restart markers found in U
    int32_t sub_bytes;       // unstuffed bytes per decode lane (mode 1)
    int32_t gw_S;            // guess-write static pool slots per lane (mode 1)
    int64_t scan_len;      // raw entropy-coded bytes (file end - scan start)
    int64_t ulen;          // unstuffed data bytes before FF D9 / end of file / bad marker
    int64_t errpos;        // unstuffed index whose fetch is a syntax error (INT64_MAX: none)
    int64_t total_blocks;
    int64_t uoff;          // byte offset of the image's unstuffed stream in GroupWs::U (4 KiB aligned)
    int32_t ncount;        // guess-write lanes queued for the count decode (k_gw_check)
    int32_t dri_first;     // DRI: 2 j + (kind == kDriElsewhere) of the first interval j not ending
                           // at its marker (dri_end_kind; atomicMin, INT32_MAX: none)
    int64_t tail_G, tail_n;  // guess-write: the lanes' blocks end at block tail_G, tail_n before the
    int32_t tail_p[3];       // frame's last (k_gw_tail reads on into the padding; DC predictors there)
    int32_t kint;            // guess-write over restart intervals (mode 1, DRI): lanes per interval
                             // (lane j in interval j / kint, icx_spec_core.h lane_span); 0 otherwise
};
struct TileRec { int32_t kept, end_err; int64_t end_at; int32_t nrst, pad_; };
struct SubRec { int32_t cnt, ds0, ds1, ds2; int32_t mism; };
// A block-start state seen by a guess lane: bit offset from the lane start, block-in-MCU,
// DC codes decoded before it, and the per-component DC-diff sums before it.
struct RecState { uint32_t rel; int32_t b, cnt; int32_t ds[3]; };
struct LaneEntry { int64_t G; int32_t p0, p1, p2, pad; };

// ---- guess-write path (icx_spec.hip k_gw_*; icx_spec_core.h gw_*) ----
// A guess lane decodes with the write tables and stores the blocks that start in its range
// itself; only lanes not synchronised at their start are decoded again (from the true entry, up
// to the first state they share with the guess). Blocks go to the group's coefficient pool:
// kGwStaticSlack x the image's average blocks per lane in a static region per lane, then chunks
// of kGwChunk blocks taken from the pool's tail by atomic add (flat areas hold thousands of
// blocks per lane), chained through GroupWs::chunk_next.
constexpr int kGwChunk = 32;
constexpr int kRecGw = kRec;    // MCU starts a guess-write lane records (the count lanes splice at the first
                                // they reach; a lane that cannot splice is count-decoded whole). (8 was
                                // tried in round 6: k_gw_lane -1%, but k_gw_count 0.64 -> 1.65 ms per 256
                                // images -- a few lanes of the C3 pool splice past record 7)
constexpr int64_t kGwMinPixels = 2048 * 2048;  // workspaces for larger images take the guess-write path
constexpr int kGwMaxWalk = 64;  // lanes a repair walk may re-derive before the image goes sequential
// Restart intervals on the guess-write path (round 6): an image whose intervals average at least
// kDriGwMin unstuffed bytes (ICX_DRI_GW: 0 never, 1 from kSubBytesSmall) has each interval cut into
// kint lanes of at most kSubBytes instead of one serial lane per interval (mode 3).
constexpr int kDriGwMin = 4096;
struct GwOut {
    uint64_t g0;     // first block start at or after the lane's start: pack_state(pos, b, 0)
    int32_t k;       // blocks the lane stored (slots 0 .. k-1)
    int32_t ds[3];   // lane-local DC sums over them (predictors relative to g0)
    int32_t err;     // slot of the first block whose decode failed (INT32_MAX: none)
    int32_t chunk0;  // first overflow chunk (pool block / kGwChunk), -1: none
    int32_t nrec;    // block-start records (RecState, b = 0: MCU starts) taken after g0
    int32_t over;    // the pool ran out: the image goes sequential
};
struct GcRec {
    int32_t chunk0;  // the count lane's blocks: a chain of pool chunks (-1: none)
    int32_t pad_;
    int32_t c;       // blocks it stored: the true path from the previous lane's exit to the splice
    int32_t m;       // guess record it spliced at; -1: none (the c blocks are the whole lane); -2: the
                     // lane was synchronised at its start (no count decode)
    int32_t cds[3];  // DC sums over the c blocks
    int32_t err;     // first of the c blocks whose decode failed (INT32_MAX: none)
};

// Device workspace for one group of images processed together (slot i = image i of the
// group). Capacities are per slot and cover any sampling NanoJPEG accepts at max_w x max_h.
// Absolute quantized DC per block: stored in the block itself (natural index 0, never an AC
// position) as int16; values outside int16 (only corrupt streams) store kDcEscape there and the
// exact int32 in GroupWs::dc. Keeps the DC inside the block's 128-byte line (no scattered stores).
constexpr int16_t kDcEscape = INT16_MIN;
__host__ __device__ inline int16_t dc_cell(int32_t dc) {
    return (dc > -32768 && dc <= 32767) ? (int16_t)dc : kDcEscape;
}

struct GroupWs {
    int slots = 0;
    int max_w = 0, max_h = 0;
    int64_t coef_cap = 0;    // blocks per slot
    int64_t plane_cap = 0;   // bytes per slot (all components' IDCT planes)
    int64_t tmp_cap = 0;     // bytes per ping-pong buffer per component per slot
    Desc* desc = nullptr;    // [slots]
    int16_t* ac = nullptr;   // [pool_cap + kGwChunk][64] coefficient pool: quantized blocks, zig-zag order
    int32_t* dc = nullptr;   // [pool_cap + kGwChunk] int32 DC of pool blocks whose cell holds kDcEscape
    uint8_t* planes = nullptr;  // [slots][plane_cap]
    uint8_t* tmp = nullptr;     // [slots][3 comps][2 buffers][tmp_cap]; aliases `ac` (tmp_own == false)
    bool tmp_own = false;       // tmp is an allocation of its own (ac too small to hold it)
    // parallel entropy decode
    int64_t ucap = 0;           // unstuffed bytes per slot on average: U is one pool of (slots + 2) * ucap
                                // bytes, each image's stream at SpecImg::uoff (k_spec_plan), so one
                                // image may take several slots' worth (a noisy q100 4:4:4 scan ~2 B/px)
    int64_t upool = 0;          // bytes of the U pool: (slots + 2) * ucap
    int64_t tiles_cap = 0;      // flat tile records for the whole group
    int64_t lanes_cap = 0;      // flat lane records for the whole group
    SpecImg* spec = nullptr;    // [slots]
    int32_t* tilepre = nullptr; // [slots+1]
    int32_t* wgpre = nullptr;   // [slots+1] 256-lane groups
    int32_t* wg2pre = nullptr;  // [slots+1] kWriteLanesBig-lane groups (write pass, large images)
    int32_t* totals = nullptr;  // [4]: tiles, 256-lane groups, big write groups
    TileRec* tiles = nullptr;
    int32_t* tile_obase = nullptr;
    uint8_t* U = nullptr;       // [slots][ucap]
    uint64_t* X = nullptr;      // [lanes_cap] exit states (guess pass; repaired in place)
    uint64_t* Y = nullptr;      // [lanes_cap] exit states re-derived by the count pass
    RecState* rec = nullptr;    // [lanes_cap][kRec]
    int32_t* nrec = nullptr;    // [lanes_cap]
    int32_t* guess_cnt = nullptr;  // [lanes_cap][4]: DC codes and DC sums over the whole guess lane
    int32_t* repair = nullptr;  // [slots][kMaxRepair] lanes whose chain needs a serial repair
    SubRec* sub = nullptr;      // [lanes_cap]
    int64_t rst_cap = 0;        // restart markers recorded per slot (>= MCUs per image)
    int64_t* rst = nullptr;     // [slots][rst_cap] (U byte index << 3) | marker number
    int32_t* tile_rbase = nullptr;  // [tiles_cap] restart markers before the tile (per image)
    LaneEntry* ent = nullptr;   // [lanes_cap]
    struct StepSet* steps = nullptr;  // [slots] step tables (icx_step.h), built per group
    int32_t* stats = nullptr;   // [4] path counters, accumulated over a batch call
    // coefficient pool (Desc::acbase / mapped) and the guess-write path's records
    int64_t pool_cap = 0;              // pool blocks (+ kGwChunk scratch blocks allocated past it)
    uint2* map = nullptr;              // [pool_cap] block n of a mapped image: {pool block, DC offset} at acbase + n
    int32_t* chunk_next = nullptr;     // [pool_cap / kGwChunk + 1] overflow chunk chains
    unsigned long long* pool_next = nullptr;  // [1] next free pool block (k_spec_plan sets it past the static regions)
    GwOut* gw = nullptr;               // [lanes_cap]
    GcRec* crec = nullptr;             // [lanes_cap]
    int2* clist = nullptr;             // [lanes_cap] per image, in its lane-record range: (image, lane) to count-decode
    int32_t* h_defer = nullptr;        // pinned [3]: images the last k_spec_plan deferred, gave restart-interval lanes, gave
                                       // interval-aligned guess-write lanes
    int32_t* h_layout = nullptr;       // pinned: the group has an image outside the fused 4:2:0 layout (k_parse)
    hipEvent_t ev_defer = nullptr;     // after round 0's k_spec_plan
};

// Where block n of an image lives in its group's coefficient pool: the pool block and the offset
// to add to its DC cell (Desc::acbase / mapped).
struct BlkLoc {
    int64_t blk;
    int32_t dcoff;
};
__device__ __forceinline__ BlkLoc blk_loc(const Desc& d, const uint2* map, int64_t n) {
    if (!d.mapped) return BlkLoc{d.acbase + n, 0};
    const uint2 e = map[d.acbase + n];
    return BlkLoc{(int64_t)e.x, (int32_t)e.y};
}
// A block's absolute quantized DC: its cell (or the int32 escape) plus the location's offset.
// (The escape load sits in a wave-uniform branch that valid streams never take: as a per-lane
// select its s_waitcnt vmcnt(0) landed after the join, in every block's path, where it waited
// for every load and store the wave had in flight.)
__device__ __forceinline__ int32_t blk_dc(int16_t cell, const int32_t* dcv, const BlkLoc& l) {
    int32_t v = cell;
    if (__any(cell == kDcEscape)) {
        const int32_t e = dcv[l.blk];
        v = cell == kDcEscape ? e : v;
    }
    return wadd(v, l.dcoff);
}
// A block location whose map entry is still in flight: the entry is loaded unconditionally (for an
// image written in place the slot is in bounds and ignored) and resolved where the location is
// used, so the load's wait lands there and not right after the load (blk_loc's branch did that).
struct BlkPend {
    uint2 e;
    int64_t n;  // acbase + block index
};
__device__ __forceinline__ BlkPend blk_pend(const Desc& d, const uint2* map, int64_t n) {
    return BlkPend{map[d.acbase + n], d.acbase + n};
}
__device__ __forceinline__ BlkLoc blk_resolve(const Desc& d, const BlkPend& q) {
#ifdef ICX_EXP_BACK_NOMAP
    return BlkLoc{q.n, 0};
#else
    return d.mapped ? BlkLoc{(int64_t)q.e.x, (int32_t)q.e.y} : BlkLoc{q.n, 0};
#endif
}


int64_t ws_coef_cap(int w, int h);
int64_t ws_plane_cap(int w, int h);
int64_t ws_tmp_cap(int w, int h);

// Stage hooks so the host can bracket each stage with HIP events.
enum Stage { kStParse = 0, kStUnstuff, kStEntropy, kStWrite, kStIdct, kStUpsample, kStConvert, kStCount };
extern const char* const kStageNames[kStCount];
struct StageHook {
    virtual void begin(Stage s, hipStream_t st) = 0;
    virtual void end(Stage s, hipStream_t st) = 0;
    virtual ~StageHook() = default;
};

// Enqueue the whole decode of `n` (<= ws.slots) images on `st`.
void launch_decode_group(const GroupWs& ws, int n, const uint8_t* d_data, const uint64_t* d_off,
                         const uint64_t* d_size, uint8_t* d_out, uint64_t out_stride, int32_t* d_status,
                         int32_t* d_dims, hipStream_t st, StageHook* hook);
// The same in two halves: front = parse, unstuff, entropy decode (latency-bound); back = IDCT,
// upsample, convert, statuses (HBM-bound). The batch scheduler overlaps one group's back with the
// next group's front on another stream.
// part: kFrontAll every entropy round; kFrontFirst parse + round 0 (ws.h_defer holds round 0's
// deferred-image count once ws.ev_defer has completed); kFrontRest the later rounds when that count
// is not 0 (the caller has waited for ws.ev_defer), then the sequential kernel.
enum { kFrontAll = 0, kFrontFirst = 1, kFrontRest = 2 };
void launch_decode_front(const GroupWs& ws, int n, const uint8_t* d_data, const uint64_t* d_off,
                         const uint64_t* d_size, uint64_t out_stride, hipStream_t st, StageHook* hook,
                         int part = kFrontAll);
// known_layout: the host may wait for ws.ev_defer and read ws.h_layout (k_parse) to skip the
// other samplings' kernels when the group has only fused-layout 4:2:0 images.
void launch_decode_back(const GroupWs& ws, int n, uint8_t* d_out, uint64_t out_stride, int32_t* d_status,
                        int32_t* d_dims, hipStream_t st, StageHook* hook, bool known_layout = false);
void launch_spec_entropy(const GroupWs& ws, int n, const uint8_t* d_data, const uint64_t* d_off, hipStream_t st,
                         StageHook* hook, int part = kFrontAll);
// piece: kRoundAll the whole round; kRoundHead up to its restart-interval write; kRoundTail that
// write and the round's end; kRoundTailNoDri the end alone (no image got restart-interval lanes);
// kRoundTailGw that write on a small grid (only guess-write DRI images, whose lanes fall back to it
// when they cannot decide the image).
enum { kRoundAll = 0, kRoundHead = 1, kRoundTail = 2, kRoundTailNoDri = 3, kRoundTailGw = 4 };
void launch_spec_round(const GroupWs& ws, int n, const uint8_t* d_data, const uint64_t* d_off, hipStream_t st,
                       StageHook* hook, int round, int last, int piece = kRoundAll);

// Per-image result record (icx_records.hip; include/icx.h icx_record): status, dims and the
// 64-bit weighted word sum of the decoded bytes.
struct Record {
    int32_t status, w, h, c;
    uint64_t checksum;
};
static_assert(sizeof(Record) == 24, "icx_record layout");
void launch_records(int n, const uint8_t* d_out, uint64_t out_stride, const int32_t* d_status, const int32_t* d_dims,
                    Record* d_rec, int max_w, int max_h, hipStream_t st);

// tiny_jpeg-exact encode on the GPU (icx_encode.hip); `out` receives the whole file.
bool tje_encode_gpu(hipStream_t st, int quality, int w, int h, int comps, const uint8_t* src,
                    std::vector<uint8_t>& out);
// C4 extension encoder (4:4:4 / 4:2:0, IJG quality 1..100; oracle/tje_oracle.c or_jpeg_encode).
struct EncWs;
EncWs* enc_ws_create();
void enc_ws_destroy(EncWs* ws);
int enc_ws_stage_times(EncWs* ws, const char** names, float* ms, int cap);
bool jpeg_encode_gpu(hipStream_t st, int quality, int subsampling, int w, int h, int comps, const uint8_t* src,
                     std::vector<uint8_t>& out);
int jpeg_encode_device(hipStream_t st, EncWs* ws, int quality, int subsampling, int w, int h, int comps,
                       const uint8_t* d_src, uint8_t* d_out, uint64_t cap, uint64_t* size);
int jpeg_encode_device_batch(hipStream_t st, EncWs* ws, int n, int quality, int subsampling, int w, int h, int comps,
                             const uint8_t* const* d_srcs, uint8_t* d_out, uint64_t stride, uint64_t* sizes,
                             int32_t* status);

// PNG encoder (icx_png.hip): png_encoder::saveToFile's colour choice and filters, GPU deflate.
struct PngWs;
PngWs* png_ws_create();
void png_ws_destroy(PngWs* ws);
int png_ws_stage_times(PngWs* ws, const char** names, float* ms, int cap);
int png_encode_device_batch(int k, hipStream_t* sts, PngWs** wss, int n, int w, int h, int d,
                            const uint8_t* const* d_srcs, uint8_t* d_out, uint64_t stride, uint64_t* sizes,
                            int32_t* status);
int png_encode_device(hipStream_t st, PngWs* ws, int w, int h, int d, const uint8_t* d_src, uint8_t* d_out,
                      uint64_t cap, uint64_t* size);
bool png_encode_gpu(hipStream_t st, int w, int h, int d, const uint8_t* src, std::vector<uint8_t>& out);

// Radiance .hdr decode (icx_hdr.hip; Image::readHdr, codecs.cpp:706-777). Status codes match
// include/icx.h ICX_HDR_*; kHdrPending is internal.
enum : int32_t {
    kHdrOk = 0, kHdrNotRadiance = 1, kHdrBadHeader = 2, kHdrMalformed = 3, kHdrTruncated = 4, kHdrTooLarge = 5,
    kHdrPending = 6
};
struct HdrDesc {
    int32_t status, w, h, rows;
    int64_t ds, size;      // pixel data start, file size
    int32_t has_marker;    // an aligned old-style run marker exists (k_hdr_scan)
    int32_t not_flat;      // some row is not a plain RGBE row at ds + 4*w*y (k_hdr_flatcheck)
    int32_t ncand, new_ok; // new-style scanline starts found; they chain over all rows (k_hdr_link)
    int32_t mode;          // 0 failed, 1 all rows plain, 2 all rows new-style, 3 per-row table (k_hdr_walk)
    int32_t pad_;
};
struct HdrWs {
    int max_images = 0, max_w = 0, max_h = 0;
    HdrDesc* desc = nullptr;   // [max_images]
    int32_t* cq = nullptr;     // [max_images][kHdrCandCap] new-style scanline starts (relative to ds)
    int32_t* ce = nullptr;     // [max_images][kHdrCandCap] their ends (relative), or -1/-2/-3
    int64_t* start = nullptr;  // [max_images][max_h] row start (byte offset in the file)
    uint8_t* kind = nullptr;   // [max_images][max_h] row kind (mode 3)
    uint8_t* planes = nullptr; // [max_images][max_h][4][max_w] RGBE planes of run-length coded rows
};
int hdr_probe(const uint8_t* data, int64_t size, int* w, int* h);
int64_t hdr_ws_bytes(int max_images, int max_w, int max_h);
bool hdr_ws_alloc(HdrWs& ws, int max_images, int max_w, int max_h);
void hdr_ws_free(HdrWs& ws);
void launch_hdr_decode(const HdrWs& ws, int n, const uint8_t* d_data, const uint64_t* d_off, const uint64_t* d_size,
                       float* d_out, uint64_t out_stride, int32_t* d_status, int32_t* d_dims, hipStream_t st,
                       StageHook* hook);

// ---- OpenEXR read (icx_exr.hip) ----
// tinyexr's LoadEXRFromMemory; returns its code (-100: HIP failure, err says which).
struct ExrWs;
ExrWs* exr_ws_create();
void exr_ws_destroy(ExrWs* w);
int exr_decode(hipStream_t st, ExrWs& ws, const uint8_t* data, size_t size, const uint8_t* d_file, float* d_out,
               size_t out_floats, float** out_rgba, int* width, int* height, std::string& err);
int exr_decode_batch(hipStream_t st, ExrWs& ws, int n, const uint8_t* const* data, const uint8_t* const* d_data,
                     const size_t* sizes, float* const* d_out, const size_t* out_floats, int32_t* codes, int32_t* widths,
                     int32_t* heights, std::string& err);
int exr_probe(const uint8_t* data, size_t size, int* width, int* height);

}  // namespace icx
