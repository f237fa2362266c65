// icx_api.cpp -- host side of libicx.so: the C ABI declared in include/icx.h.
//
// Contexts own a HIP stream and the NanoJPEG-style single-image state; batches own the
// device workspace of one image group. No CPU decode path exists: every decode runs the
// HIP kernels in icx_decode.hip, and a missing/unusable GPU is reported as an error.
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <string>
#include <vector>

#include "../../include/icx.h"
#include "icx_internal.h"
#include "icx_step.h"

using namespace icx;

struct icx_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // njDecode-style state (jpeg_dec.h:313-330 equivalent, per context)
    std::vector<uint8_t> nj_image;
    int nj_w = 0, nj_h = 0, nj_color = 0, nj_size = 0;
    icx_batch* single = nullptr;  // cached workspace for one-image calls
    // staging for one-image calls
    uint8_t* d_in = nullptr;
    size_t d_in_cap = 0;
    ExrWs* exr = nullptr;  // grow-only EXR read buffers (icx_exr.hip)
};

struct EventHook;

// Up to kMaxPipes decode pipelines per batch, each a workspace + a stream: consecutive groups of
// a call alternate between them, so one group's entropy kernels (latency/LDS-bound) run beside
// another group's IDCT/convert (memory-bound) instead of after them.
#ifndef ICX_MAX_PIPES  // (timing experiments: more pipelines)
#define ICX_MAX_PIPES 2
#endif
constexpr int kMaxPipes = ICX_MAX_PIPES;
struct icx_batch {
    icx_ctx* ctx = nullptr;
    int max_images = 0;
    int pipes = 1;
    GroupWs ws[kMaxPipes];
    hipStream_t pst[kMaxPipes] = {};  // pst[0] unused: pipe 0 runs on the caller's stream
    hipEvent_t fork = nullptr, join[kMaxPipes] = {};
    std::vector<hipEvent_t> front_done;  // per group of a call: its front half has run
    int min_groups = 1;                  // a call is cut into at least this many groups
    bool stagger = false;                // group g's front waits for group g-1's front (ICX_STAGGER=1; measured slower)
    uint8_t* d_hin = nullptr;  // staging for icx_jpeg_batch_decode_host
    size_t d_hin_cap = 0;
    hipEvent_t done = nullptr;      // recorded after the last decode call's work (path_stats waits on it)
    bool decoded = false;
    std::unique_ptr<EventHook> hook;
};

static std::string g_create_err;

static thread_local char g_msg[512];

#define ICX_HIP(ctx, call, ret)                                                             \
    do {                                                                                    \
        hipError_t e_ = (call);                                                             \
        if (e_ != hipSuccess) {                                                             \
            (void)hipGetLastError(); /* reported here: not left for the caller's next check */ \
            std::snprintf(g_msg, sizeof g_msg, "%s failed: %s", #call, hipGetErrorString(e_)); \
            if (ctx) (ctx)->err = g_msg;                                                    \
            return ret;                                                                     \
        }                                                                                   \
    } while (0)

// Brackets every pipeline stage with HIP events on the launch stream, and with a roctx range on
// the host (the launch side: `rocprofv3 --marker-trace` shows which stage enqueued which kernels).
// One roctx range per API call, around every stage's range.
struct RoctxRange {
    explicit RoctxRange(const char* m) { (void)roctxRangePushA(m); }
    ~RoctxRange() { (void)roctxRangePop(); }
};
static const char* const kRangeNames[kStCount] = {"icx:parse", "icx:unstuff", "icx:entropy", "icx:write",
                                                  "icx:idct", "icx:upsample", "icx:convert"};
struct EventHook : StageHook {
    struct Rec { Stage s; hipEvent_t a, b; };
    std::vector<Rec> recs;
    std::vector<hipEvent_t> pool;
    size_t used = 0;
    hipEvent_t get() {
        if (used == pool.size()) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            pool.push_back(e);
        }
        return pool[used++];
    }
    void reset() { recs.clear(); used = 0; }
    void begin(Stage s, hipStream_t st) override {
        (void)roctxRangePushA(kRangeNames[s]);
        hipEvent_t a = get(), b = get();
        if (!a || !b) return;
        (void)hipEventRecord(a, st);
        recs.push_back({s, a, b});
    }
    void end(Stage s, hipStream_t st) override {
        (void)roctxRangePop();
        for (auto it = recs.rbegin(); it != recs.rend(); ++it)
            if (it->s == s) { (void)hipEventRecord(it->b, st); return; }
    }
    ~EventHook() override {
        for (auto e : pool) (void)hipEventDestroy(e);
    }
};

extern "C" {

const char* icx_version(void) { return "icx 0.1.0 gfx950"; }

const char* icx_last_error(const icx_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_err.c_str(); }

icx_ctx* icx_create(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        g_create_err = "no HIP device available (libicx has no CPU decode path)";
        return nullptr;
    }
    if (device < 0 || device >= n) {
        g_create_err = "device ordinal out of range";
        return nullptr;
    }
    if (hipSetDevice(device) != hipSuccess) {
        g_create_err = "hipSetDevice failed";
        return nullptr;
    }
    auto* c = new icx_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        g_create_err = "hipStreamCreate failed";
        delete c;
        return nullptr;
    }
    return c;
}

void icx_batch_destroy(icx_batch* b);

void icx_destroy(icx_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->single) icx_batch_destroy(c->single);
    if (c->d_in) (void)hipFree(c->d_in);
    if (c->exr) exr_ws_destroy(c->exr);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

void icx_free(void* p) { std::free(p); }
int icx_ctx_device(const icx_ctx* c) { return c ? c->device : -1; }
void* icx_ctx_stream(const icx_ctx* c) { return c ? (void*)c->stream : nullptr; }

int icx_jpeg_probe(const uint8_t* jpeg, size_t size, int* w, int* h, int* ncomp) {
    if (w) *w = 0;
    if (h) *h = 0;
    if (ncomp) *ncomp = 0;
    if (!jpeg) return ICX_NO_JPEG;
    auto d = std::make_unique<Desc>();
    int st = parse_headers(jpeg, (int64_t)std::min<size_t>(size, 0x7FFFFFFF), *d);
    if (st != kPending) return st;
    if (w) *w = d->W;
    if (h) *h = d->H;
    if (ncomp) *ncomp = d->nc == 1 ? 1 : 3;
    return ICX_OK;
}

// ----------------------------------------------------------------------------- batches
// Bytes of one workspace slot (one image in flight) for max_w x max_h images; fills the caps.
static int64_t ws_per_slot(GroupWs& ws, int max_w, int max_h) {
    ws.max_w = max_w;
    ws.max_h = max_h;
    ws.coef_cap = ws_coef_cap(max_w, max_h);
    ws.plane_cap = ws_plane_cap(max_w, max_h);
    ws.tmp_cap = ws_tmp_cap(max_w, max_h);
    // unstuffed entropy bytes per slot: 2 B/px (ICX_UPOOL_BPP; q90 4:2:0 is ~0.4, a 4:4:4 q100 photo
    // 1.3-2.5). A group whose scans pass the pool defers the rest to further entropy rounds
    // (launch_spec_entropy), so this sizes the common case, not a limit.
    const int bpp = std::getenv("ICX_UPOOL_BPP") ? std::max(1, std::min(16, std::atoi(std::getenv("ICX_UPOOL_BPP")))) : 2;
    ws.ucap = ((int64_t)max_w * max_h * bpp + 4095) / 4096 * 4096;
    ws.rst_cap = ((int64_t)max_w / 8 + 1) * ((int64_t)max_h / 8 + 1);  // >= MCUs per image
    // decode lanes of kSubBytesSmall .. kSubBytes bytes (k_spec_plan picks per image)
    const int64_t tiles_per_slot = ws.ucap / kTileBytes + 2;
    const int64_t lanes_per_slot = ((ws.ucap + kSubBytesSmall - 1) / kSubBytesSmall + kLanes - 1) / kLanes * kLanes + kLanes;
    // coefficient pool: kPoolPerSlot x coef_cap blocks per slot (int16 block + int32 DC escape + map entry)
    // (the generic upsample's ping-pong planes, 6 x tmp_cap, live in the coefficient pool: ws_alloc_all)
    return ws.coef_cap * kPoolPerSlotX4 / 4 * (64 * 2 + 4 + 8) + ws.plane_cap + (int64_t)sizeof(Desc) + ws.ucap +
           (int64_t)sizeof(StepSet) +
           tiles_per_slot * 28 + ws.rst_cap * 8 +
           lanes_per_slot * (8 + 8 + 20 + 24 + 4 + 16 + (int64_t)sizeof(RecState) * kRec + (int64_t)sizeof(GwOut) +
                             (int64_t)sizeof(GcRec) + 8) + kMaxRepair * 4;
}

static void ws_free(GroupWs& ws) {
    if (ws.tmp_own && ws.tmp) (void)hipFree(ws.tmp);
    for (void* p : {(void*)ws.desc, (void*)ws.ac, (void*)ws.dc, (void*)ws.planes, (void*)ws.spec,
                    (void*)ws.tilepre, (void*)ws.wgpre, (void*)ws.wg2pre, (void*)ws.totals, (void*)ws.tiles,
                    (void*)ws.tile_obase, (void*)ws.U, (void*)ws.X, (void*)ws.sub, (void*)ws.rst, (void*)ws.tile_rbase,
                    (void*)ws.ent, (void*)ws.stats, (void*)ws.Y, (void*)ws.rec, (void*)ws.nrec, (void*)ws.guess_cnt,
                    (void*)ws.repair, (void*)ws.steps, (void*)ws.map, (void*)ws.chunk_next, (void*)ws.pool_next,
                    (void*)ws.gw, (void*)ws.crec, (void*)ws.clist})
        if (p) (void)hipFree(p);
    if (ws.h_defer) (void)hipHostFree(ws.h_defer);
    if (ws.h_layout) (void)hipHostFree(ws.h_layout);
    if (ws.ev_defer) (void)hipEventDestroy(ws.ev_defer);
    ws = GroupWs{};
}

static bool ws_alloc_all(icx_ctx* ctx, GroupWs& ws, int group, int max_w, int max_h);
// All or nothing: a failure part-way frees this workspace's buffers before returning.
static bool ws_alloc(icx_ctx* ctx, GroupWs& ws, int group, int max_w, int max_h) {
    if (ws_alloc_all(ctx, ws, group, max_w, max_h)) return true;
    ws_free(ws);
    return false;
}

static bool ws_alloc_all(icx_ctx* ctx, GroupWs& ws, int group, int max_w, int max_h) {
    (void)ws_per_slot(ws, max_w, max_h);
    const int64_t tiles_per_slot = ws.ucap / kTileBytes + 2;
    const int64_t lanes_per_slot = ((ws.ucap + kSubBytesSmall - 1) / kSubBytesSmall + kLanes - 1) / kLanes * kLanes + kLanes;
    ws.slots = group;
    // the U pool and the flat tile / lane records it bounds: two slots' worth beyond the group, so
    // even a one-image group takes a 3 B/px scan (k_spec_plan sends images past the pool to
    // the sequential kernel)
    ws.upool = (int64_t)(group + 2) * ws.ucap;
    ICX_HIP(ctx, hipMalloc(&ws.desc, sizeof(Desc) * group), false);
    // the coefficient pool (k_spec_plan places each image in it; the guess-write lanes' overflow
    // chunks and count blocks take its tail), + kGwChunk scratch blocks past pool_cap. The static
    // regions take 1.1 x each image's blocks; the tail, 2.5 (G + 2) - 1.1 G > 1.4 G image-blocks,
    // holds every block of every image in overflow chunks (a photo whose flat sky is a few lanes'
    // worth of bytes stores nearly all its blocks there) plus the count lanes' copies and the
    // chunks' rounding, so a conforming group never runs out of it.
    ws.pool_cap = (int64_t)(group + 2) * ws.coef_cap * kPoolPerSlotX4 / 4;
    ICX_HIP(ctx, hipMalloc(&ws.ac, (size_t)(ws.pool_cap + kGwChunk) * 64 * 2), false);
    ICX_HIP(ctx, hipMalloc(&ws.dc, (size_t)(ws.pool_cap + kGwChunk) * 4), false);
    ICX_HIP(ctx, hipMalloc(&ws.map, (size_t)ws.pool_cap * sizeof(uint2)), false);
    ICX_HIP(ctx, hipMalloc(&ws.chunk_next, (size_t)(ws.pool_cap / kGwChunk + 2) * 4), false);
    ICX_HIP(ctx, hipMalloc(&ws.pool_next, sizeof(unsigned long long)), false);
    ICX_HIP(ctx, hipMalloc(&ws.planes, (size_t)ws.plane_cap * group), false);
    // The generic upsample's ping-pong planes (exotic samplings only: k_upsample, k_convert) share
    // the coefficient pool's memory: launch_decode_back runs them after every kernel that reads the
    // group's coefficients (the pool holds >= 15 x the slot's MCU-padded pixels in bytes, the planes
    // 6 x (w + 8)(h + 8) <= 7.6 x), and the next group on this workspace writes the pool only after
    // that, in stream order. (A separate buffer only if the pool were ever too small.)
    if ((int64_t)(ws.pool_cap + kGwChunk) * 64 * 2 >= ws.tmp_cap * 6 * group) {
        ws.tmp = reinterpret_cast<uint8_t*>(ws.ac);
    } else {
        ICX_HIP(ctx, hipMalloc(&ws.tmp, (size_t)ws.tmp_cap * 6 * group), false);
        ws.tmp_own = true;
    }
    ws.tiles_cap = tiles_per_slot * (group + 2);
    ws.lanes_cap = lanes_per_slot * (group + 2);
    ICX_HIP(ctx, hipMalloc(&ws.spec, sizeof(SpecImg) * group), false);
    ICX_HIP(ctx, hipMalloc(&ws.tilepre, sizeof(int32_t) * (group + 1)), false);
    ICX_HIP(ctx, hipMalloc(&ws.wgpre, sizeof(int32_t) * (group + 1)), false);
    ICX_HIP(ctx, hipMalloc(&ws.wg2pre, sizeof(int32_t) * (group + 1)), false);
    ICX_HIP(ctx, hipMalloc(&ws.totals, sizeof(int32_t) * 4), false);
    ICX_HIP(ctx, hipMalloc(&ws.tiles, sizeof(TileRec) * ws.tiles_cap), false);
    ICX_HIP(ctx, hipMalloc(&ws.tile_obase, sizeof(int32_t) * ws.tiles_cap), false);
    // + slack: the entropy readers load whole 16-byte chunks (icx_spec_core.h Reader)
    ICX_HIP(ctx, hipMalloc(&ws.U, (size_t)ws.upool + 256), false);
    ICX_HIP(ctx, hipMalloc(&ws.X, sizeof(uint64_t) * ws.lanes_cap), false);
    ICX_HIP(ctx, hipMalloc(&ws.sub, sizeof(SubRec) * ws.lanes_cap), false);
    ICX_HIP(ctx, hipMalloc(&ws.rst, sizeof(int64_t) * ws.rst_cap * group), false);
    ICX_HIP(ctx, hipMalloc(&ws.tile_rbase, sizeof(int32_t) * ws.tiles_cap), false);
    ICX_HIP(ctx, hipMalloc(&ws.ent, sizeof(LaneEntry) * ws.lanes_cap), false);
    ICX_HIP(ctx, hipMalloc(&ws.stats, sizeof(int32_t) * 4), false);
    ICX_HIP(ctx, hipMalloc(&ws.Y, sizeof(uint64_t) * ws.lanes_cap), false);
    ICX_HIP(ctx, hipMalloc(&ws.rec, sizeof(RecState) * kRec * ws.lanes_cap), false);
    ICX_HIP(ctx, hipMalloc(&ws.nrec, sizeof(int32_t) * ws.lanes_cap), false);
    ICX_HIP(ctx, hipMalloc(&ws.guess_cnt, sizeof(int32_t) * 4 * ws.lanes_cap), false);
    ICX_HIP(ctx, hipMalloc(&ws.repair, sizeof(int32_t) * kMaxRepair * group), false);
    ICX_HIP(ctx, hipMalloc(&ws.steps, sizeof(StepSet) * group), false);
    ICX_HIP(ctx, hipMalloc(&ws.gw, sizeof(GwOut) * ws.lanes_cap), false);
    ICX_HIP(ctx, hipMalloc(&ws.crec, sizeof(GcRec) * ws.lanes_cap), false);
    ICX_HIP(ctx, hipMalloc(&ws.clist, sizeof(int2) * ws.lanes_cap), false);
    ICX_HIP(ctx, hipHostMalloc(&ws.h_defer, 3 * sizeof(int32_t), hipHostMallocDefault), false);
    ws.h_defer[0] = ws.h_defer[1] = ws.h_defer[2] = 0;
    ICX_HIP(ctx, hipHostMalloc(&ws.h_layout, sizeof(int32_t), hipHostMallocDefault), false);
    *ws.h_layout = 1;
    ICX_HIP(ctx, hipEventCreateWithFlags(&ws.ev_defer, hipEventDisableTiming), false);
    return true;
}

icx_batch* icx_batch_create(icx_ctx* ctx, int max_images, int max_w, int max_h, int group) {
    if (!ctx || max_images <= 0 || max_w <= 0 || max_h <= 0 || max_w > 65535 || max_h > 65535) {
        if (ctx) ctx->err = "icx_batch_create: bad arguments";
        return nullptr;
    }
    ICX_HIP(ctx, hipSetDevice(ctx->device), nullptr);
    // Every early return below (an allocation or stream/event creation failing part-way) frees
    // what was already created: the deleter is icx_batch_destroy, which skips null members.
    std::unique_ptr<icx_batch, void (*)(icx_batch*)> b(new icx_batch(), icx_batch_destroy);
    b->ctx = ctx;
    b->max_images = max_images;
    // pipelines: ICX_PIPES (1..2, default 2) when the batch holds at least two images
    int pipes = kMaxPipes;
    if (const char* e = std::getenv("ICX_PIPES")) pipes = std::max(1, std::min(kMaxPipes, std::atoi(e)));
    if (max_images < 2) pipes = 1;
    GroupWs probe;
    const int64_t per_slot = ws_per_slot(probe, max_w, max_h);
    if (group <= 0) {  // auto: up to 80% of the free HBM (288 GB per MI355X), at least one image
        // (C3's 512 images per GPU fit one group per pipeline at ~395 MB per 4096^2 slot: 2 groups
        // of 256 instead of 4 of 128, C3 +3%, C3 with restart markers +12%: its interval lanes take
        // as long for 256 images as for 128)
        size_t free_b = 0, total_b = 0;
        ICX_HIP(ctx, hipMemGetInfo(&free_b, &total_b), nullptr);
        const int64_t budget = (int64_t)(0.8 * (double)free_b);
        group = (int)std::max<int64_t>(1, std::min<int64_t>(max_images, budget / per_slot));
    }
    group = std::min(group, max_images);
    if (group < 2) pipes = 1;
    b->pipes = pipes;
    if (const char* e = std::getenv("ICX_GROUPS")) b->min_groups = std::max(1, std::atoi(e));
    if (const char* e = std::getenv("ICX_STAGGER")) b->stagger = std::atoi(e) != 0;
    for (int p = 0; p < pipes; ++p) {
        // `group` images in flight over all pipes: each workspace holds its share
        const int slots = (group + pipes - 1) / pipes;
        if (!ws_alloc(ctx, b->ws[p], slots, max_w, max_h)) return nullptr;
        if (p > 0) ICX_HIP(ctx, hipStreamCreateWithFlags(&b->pst[p], hipStreamNonBlocking), nullptr);
        ICX_HIP(ctx, hipEventCreateWithFlags(&b->join[p], hipEventDisableTiming), nullptr);
    }
    ICX_HIP(ctx, hipEventCreateWithFlags(&b->fork, hipEventDisableTiming), nullptr);
    ICX_HIP(ctx, hipEventCreateWithFlags(&b->done, hipEventDisableTiming), nullptr);
    b->hook = std::make_unique<EventHook>();
    return b.release();
}

void icx_batch_destroy(icx_batch* b) {
    if (!b) return;
    (void)hipSetDevice(b->ctx->device);
    for (int p = 0; p < kMaxPipes; ++p) {
        ws_free(b->ws[p]);
        if (b->pst[p]) (void)hipStreamDestroy(b->pst[p]);
        if (b->join[p]) (void)hipEventDestroy(b->join[p]);
    }
    if (b->fork) (void)hipEventDestroy(b->fork);
    if (b->done) (void)hipEventDestroy(b->done);
    for (auto e : b->front_done) (void)hipEventDestroy(e);
    if (b->d_hin) (void)hipFree(b->d_hin);
    delete b;
}

// How a call of n images is cut (equal-sized groups, see icx_jpeg_batch_decode): *per images a
// group (the last may hold fewer), returning the groups actually launched, ceil(n / per). Enough
// groups for the slots and at least ICX_GROUPS; and a multiple of the pipelines where rounding the
// count up still gives one (3 groups on 2 pipes run the third alone; 4 smaller ones keep both
// busy) -- only then, since a rounded-up count whose `per` launches fewer groups (n = 5 on slots
// of 2: 4 -> per 2 -> 3 groups) buys nothing.
static int batch_split(const icx_batch* b, int n, int* per_out) {
    const int slots = b->ws[0].slots;
    const int want = std::min(n, std::max((n + slots - 1) / slots, b->min_groups));
    int per = (n + want - 1) / want;
    int ng = (n + per - 1) / per;
    if (b->pipes > 1 && ng > 1 && ng % b->pipes) {
        const int up = (ng + b->pipes - 1) / b->pipes * b->pipes;
        if (up <= n) {
            const int per2 = (n + up - 1) / up;
            const int ng2 = (n + per2 - 1) / per2;
            if (ng2 % b->pipes == 0) {
                per = per2;
                ng = ng2;
            }
        }
    }
    *per_out = per;
    return ng;
}

int icx_batch_groups(const icx_batch* b, int n) {
    int per = 0;
    return b && n > 0 ? batch_split(b, n, &per) : 0;
}

int icx_jpeg_batch_decode(icx_batch* b, int n, const uint8_t* d_data, const uint64_t* d_off, const uint64_t* d_size,
                          uint8_t* d_out, uint64_t out_stride, int32_t* d_status, int32_t* d_dims, void* stream) {
    if (!b) return ICX_INTERNAL_ERR;
    icx_ctx* ctx = b->ctx;
    if (n < 0 || n > b->max_images) { ctx->err = "icx_jpeg_batch_decode: n exceeds batch capacity"; return ICX_INTERNAL_ERR; }
    if (n == 0) return ICX_OK;
    if (!d_data || !d_off || !d_size || !d_out || !d_status || !d_dims) { ctx->err = "null pointer"; return ICX_INTERNAL_ERR; }
    ICX_HIP(ctx, hipSetDevice(ctx->device), ICX_INTERNAL_ERR);
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    const RoctxRange range("icx_jpeg_batch_decode");
    b->hook->reset();
    for (int p = 0; p < b->pipes; ++p)
        ICX_HIP(ctx, hipMemsetAsync(b->ws[p].stats, 0, sizeof(int32_t) * 4, st), ICX_INTERNAL_ERR);
    // equal-sized groups (512 images on 361 slots -> 256 + 256, not 361 + 151): every kernel's
    // grid is sized by the work of its group, so a small tail group leaves the GPU half idle
    int per = 0;
    const int ng = batch_split(b, n, &per);
    const int used = std::min(b->pipes, ng);
    if (used > 1) {  // the other pipes start after the caller's prior work on `st`
        ICX_HIP(ctx, hipEventRecord(b->fork, st), ICX_INTERNAL_ERR);
        for (int p = 1; p < used; ++p) ICX_HIP(ctx, hipStreamWaitEvent(b->pst[p], b->fork, 0), ICX_INTERNAL_ERR);
    }
    // Software pipeline over the groups, alternating pipes: group g's front half (parse, unstuff,
    // entropy decode: latency-bound) starts when group g-1's front half is done, on the other
    // pipe's stream, so it runs beside group g-1's back half (IDCT, convert: HBM-bound) instead
    // of in lockstep with it.
    const bool stagger = b->stagger && used > 1;
    // Host waits (the deferred-image count and the layout flag read from pinned memory after
    // each group's plan) only when the call runs eagerly: under stream capture (hipGraph) a
    // host wait would invalidate the capture, so every entropy round and every layout's back
    // half is enqueued unconditionally (kFrontAll; empty rounds find no work). ICX_HOST_WAIT=0
    // forces that form without capture.
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    ICX_HIP(ctx, hipStreamIsCapturing(st, &cap), ICX_INTERNAL_ERR);
    const char* hw = std::getenv("ICX_HOST_WAIT");  // (read per call: tests vary it)
    const bool no_wait_env = hw && std::atoi(hw) == 0;
    const bool host_wait = !stagger && cap == hipStreamCaptureStatusNone && !no_wait_env;
    while (stagger && (int)b->front_done.size() < ng) {
        hipEvent_t e;
        ICX_HIP(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming), ICX_INTERNAL_ERR);
        b->front_done.push_back(e);
    }
    // Entropy round 0 of the first group on each pipe goes out first; then, per group, the later
    // rounds only while its previous round deferred an image (the host reads that count once the
    // round's k_spec_plan has run: the call returns after the last group's planning, not after the
    // decode), its back half, and round 0 of the group that follows on the same pipe.
    auto front0 = [&](int g) {
        const int g0 = g * per, p = g % used;
        launch_decode_front(b->ws[p], std::min(per, n - g0), d_data, d_off + g0, d_size + g0, out_stride,
                            p == 0 ? st : b->pst[p], b->hook.get(), host_wait ? kFrontFirst : kFrontAll);
    };
    for (int g = 0; g < std::min(used, ng); ++g) {
        if (stagger && g > 0) ICX_HIP(ctx, hipStreamWaitEvent(b->pst[g % used], b->front_done[g - 1], 0), ICX_INTERNAL_ERR);
        front0(g);
        if (stagger) ICX_HIP(ctx, hipEventRecord(b->front_done[g], g % used == 0 ? st : b->pst[g % used]), ICX_INTERNAL_ERR);
    }
    for (int g = 0; g < ng; ++g) {
        const int g0 = g * per, gn = std::min(per, n - g0), p = g % used;
        hipStream_t ps = p == 0 ? st : b->pst[p];
        if (host_wait) launch_decode_front(b->ws[p], gn, d_data, d_off + g0, d_size + g0, out_stride, ps, b->hook.get(),
                                           kFrontRest);
        launch_decode_back(b->ws[p], gn, d_out + (uint64_t)g0 * out_stride, out_stride, d_status + g0, d_dims + 3 * g0,
                           ps, b->hook.get(), host_wait);
        const int gnext = g + used;
        if (gnext < ng) {
            hipStream_t pn = gnext % used == 0 ? st : b->pst[gnext % used];
            if (stagger) ICX_HIP(ctx, hipStreamWaitEvent(pn, b->front_done[gnext - 1], 0), ICX_INTERNAL_ERR);
            front0(gnext);
            if (stagger) ICX_HIP(ctx, hipEventRecord(b->front_done[gnext], pn), ICX_INTERNAL_ERR);
        }
    }
    for (int p = 1; p < used; ++p) {  // the caller's stream waits for every pipe
        ICX_HIP(ctx, hipEventRecord(b->join[p], b->pst[p]), ICX_INTERNAL_ERR);
        ICX_HIP(ctx, hipStreamWaitEvent(st, b->join[p], 0), ICX_INTERNAL_ERR);
    }
    // owned by the batch: path_stats waits on this event, never on the caller's stream (which
    // the caller may destroy after the call)
    ICX_HIP(ctx, hipEventRecord(b->done, st), ICX_INTERNAL_ERR);
    b->decoded = true;
    ICX_HIP(ctx, hipGetLastError(), ICX_INTERNAL_ERR);
    return ICX_OK;
}

int icx_batch_path_stats(const icx_batch* b, int32_t* parallel, int32_t* fallback, int32_t* sequential) {
    if (!b) return ICX_INTERNAL_ERR;
    int32_t h[4] = {0, 0, 0, 0};
    // The decode ran on non-blocking streams, which the null stream does not order against:
    // wait for the batch's own event recorded after every pipe joined.
    ICX_HIP(b->ctx, hipSetDevice(b->ctx->device), ICX_INTERNAL_ERR);
    if (b->decoded) ICX_HIP(b->ctx, hipEventSynchronize(b->done), ICX_INTERNAL_ERR);
    for (int p = 0; p < b->pipes; ++p) {
        int32_t q[4];
        ICX_HIP(b->ctx, hipMemcpy(q, b->ws[p].stats, sizeof q, hipMemcpyDeviceToHost), ICX_INTERNAL_ERR);
        for (int k = 0; k < 4; ++k) h[k] += q[k];
    }
    if (parallel) *parallel = h[0];
    if (fallback) *fallback = h[1];
    if (sequential) *sequential = h[2];
    return ICX_OK;
}

int icx_batch_group(const icx_batch* b) { return b ? b->ws[0].slots : 0; }

int icx_batch_stage_times(const icx_batch* b, const char** names, float* ms, int cap) {
    if (!b) return 0;
    float acc[kStCount] = {0};
    for (auto& r : b->hook->recs) {
        float t = 0;
        if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&t, r.a, r.b) == hipSuccess) acc[r.s] += t;
        else (void)hipGetLastError();  // (not left for the caller's next check)
    }
    int k = 0;
    for (int s = 0; s < kStCount && k < cap; ++s, ++k) {
        if (names) names[k] = kStageNames[s];
        if (ms) ms[k] = acc[s];
    }
    return kStCount;
}

int icx_jpeg_batch_decode_host(icx_batch* b, int n, const uint8_t* const* jpegs, const size_t* sizes,
                               uint8_t* const* outs, uint64_t out_stride, int32_t* status, int32_t* dims) {
    if (!b) return ICX_INTERNAL_ERR;
    icx_ctx* ctx = b->ctx;
    if (n <= 0) return n == 0 ? ICX_OK : ICX_INTERNAL_ERR;
    ICX_HIP(ctx, hipSetDevice(ctx->device), ICX_INTERNAL_ERR);
    std::vector<uint64_t> off(n), sz(n);
    uint64_t total = 0;
    for (int i = 0; i < n; ++i) { off[i] = total; sz[i] = sizes[i]; total += (sizes[i] + 15) & ~uint64_t(15); }
    const size_t meta = (size_t)n * (8 + 8 + 4 + 12);
    const size_t need = total + meta + (size_t)n * out_stride + 256;
    if (need > b->d_hin_cap) {
        if (b->d_hin) (void)hipFree(b->d_hin);
        b->d_hin = nullptr;
        b->d_hin_cap = 0;
        ICX_HIP(ctx, hipMalloc(&b->d_hin, need), ICX_OUT_OF_MEM);
        b->d_hin_cap = need;
    }
    uint8_t* base = b->d_hin;
    uint8_t* d_data = base;
    uint64_t* d_off = reinterpret_cast<uint64_t*>(base + ((total + 15) & ~uint64_t(15)));
    uint64_t* d_sz = d_off + n;
    int32_t* d_st = reinterpret_cast<int32_t*>(d_sz + n);
    int32_t* d_dm = d_st + n;
    uint8_t* d_out = reinterpret_cast<uint8_t*>(((uintptr_t)(d_dm + 3 * n) + 255) & ~uintptr_t(255));
    hipStream_t st = ctx->stream;
    for (int i = 0; i < n; ++i)
        if (sz[i]) ICX_HIP(ctx, hipMemcpyAsync(d_data + off[i], jpegs[i], sz[i], hipMemcpyHostToDevice, st), ICX_INTERNAL_ERR);
    ICX_HIP(ctx, hipMemcpyAsync(d_off, off.data(), 8 * n, hipMemcpyHostToDevice, st), ICX_INTERNAL_ERR);
    ICX_HIP(ctx, hipMemcpyAsync(d_sz, sz.data(), 8 * n, hipMemcpyHostToDevice, st), ICX_INTERNAL_ERR);
    int rc = icx_jpeg_batch_decode(b, n, d_data, d_off, d_sz, d_out, out_stride, d_st, d_dm, st);
    if (rc) return rc;
    ICX_HIP(ctx, hipMemcpyAsync(status, d_st, 4 * n, hipMemcpyDeviceToHost, st), ICX_INTERNAL_ERR);
    ICX_HIP(ctx, hipMemcpyAsync(dims, d_dm, 12 * n, hipMemcpyDeviceToHost, st), ICX_INTERNAL_ERR);
    ICX_HIP(ctx, hipStreamSynchronize(st), ICX_INTERNAL_ERR);
    for (int i = 0; i < n; ++i) {
        const size_t bytes = (size_t)dims[3 * i] * dims[3 * i + 1] * dims[3 * i + 2];
        if (status[i] == ICX_OK && bytes)
            ICX_HIP(ctx, hipMemcpyAsync(outs[i], d_out + (uint64_t)i * out_stride, bytes, hipMemcpyDeviceToHost, st),
                    ICX_INTERNAL_ERR);
    }
    ICX_HIP(ctx, hipStreamSynchronize(st), ICX_INTERNAL_ERR);
    return ICX_OK;
}

// ------------------------------------------------------------------- one-image decode
// Image::readJpg's path (codecs.cpp:821-849): probe on the host for the allocation size,
// then the full GPU pipeline on a cached one-slot workspace.
static int decode_one(icx_ctx* ctx, const uint8_t* jpeg, size_t size, std::vector<uint8_t>& out, int& w, int& h,
                      int& color) {
    w = h = color = 0;
    out.clear();
    if (!ctx) return ICX_INTERNAL_ERR;
    int pw = 0, ph = 0, pc = 0;
    const int probe = icx_jpeg_probe(jpeg, size, &pw, &ph, &pc);
    if (probe != ICX_OK) return probe;  // header-level result is final (no entropy data reached)
    if (!ctx->single || ctx->single->ws[0].max_w < pw || ctx->single->ws[0].max_h < ph) {
        if (ctx->single) icx_batch_destroy(ctx->single);
        ctx->single = icx_batch_create(ctx, 1, std::max(pw, 1), std::max(ph, 1), 1);
        if (!ctx->single) return ICX_OUT_OF_MEM;
    }
    const uint8_t* in[1] = {jpeg};
    size_t sizes[1] = {std::min<size_t>(size, 0x7FFFFFFF)};
    out.resize(std::max<size_t>((size_t)pw * ph * 3, 1));
    uint8_t* outs[1] = {out.data()};
    int32_t st = 0, dims[3] = {0, 0, 0};
    int rc = icx_jpeg_batch_decode_host(ctx->single, 1, in, sizes, outs, out.size(), &st, dims);
    if (rc) return rc;
    if (st != ICX_OK) { out.clear(); return st; }
    w = dims[0];
    h = dims[1];
    color = dims[2] == 3;
    out.resize((size_t)w * h * dims[2]);
    return ICX_OK;
}

int icx_jpeg_decode(icx_ctx* ctx, const uint8_t* jpeg, size_t size, uint8_t** out, int* w, int* h, int* ncomp) {
    if (out) *out = nullptr;
    std::vector<uint8_t> buf;
    int W = 0, H = 0, color = 0;
    int rc = decode_one(ctx, jpeg, size, buf, W, H, color);
    if (w) *w = W;
    if (h) *h = H;
    if (ncomp) *ncomp = rc == ICX_OK ? (color ? 3 : 1) : 0;
    if (rc == ICX_OK && out && !buf.empty()) {
        *out = static_cast<uint8_t*>(std::malloc(buf.size()));
        if (!*out) return ICX_OUT_OF_MEM;
        std::memcpy(*out, buf.data(), buf.size());
    }
    return rc;
}

// ------------------------------------------------------- NanoJPEG-compatible state API
void icx_nj_init(icx_ctx* ctx) {
    if (!ctx) return;
    ctx->nj_image.clear();
    ctx->nj_w = ctx->nj_h = ctx->nj_color = ctx->nj_size = 0;
}
void icx_nj_done(icx_ctx* ctx) { icx_nj_init(ctx); }

int icx_nj_decode(icx_ctx* ctx, const void* jpeg, int size) {
    if (!ctx) return ICX_INTERNAL_ERR;
    icx_nj_init(ctx);  // njDecode starts with njDone (jpeg_dec.h:881)
    int W = 0, H = 0, color = 0;
    int rc = decode_one(ctx, static_cast<const uint8_t*>(jpeg), (size_t)(size & 0x7FFFFFFF), ctx->nj_image, W, H, color);
    if (rc == ICX_OK) {
        ctx->nj_w = W;
        ctx->nj_h = H;
        ctx->nj_color = color;
        ctx->nj_size = (int)ctx->nj_image.size();
    }
    return rc;
}
int icx_nj_get_width(const icx_ctx* ctx) { return ctx ? ctx->nj_w : 0; }
int icx_nj_get_height(const icx_ctx* ctx) { return ctx ? ctx->nj_h : 0; }
int icx_nj_is_color(const icx_ctx* ctx) { return ctx ? ctx->nj_color : 0; }
unsigned char* icx_nj_get_image(icx_ctx* ctx) {
    return (ctx && !ctx->nj_image.empty()) ? ctx->nj_image.data() : nullptr;
}
int icx_nj_get_image_size(const icx_ctx* ctx) { return ctx ? ctx->nj_size : 0; }

// ------------------------------------------------------------------ encode (tiny_jpeg)
int icx_tje_encode_with_func(icx_ctx* ctx, icx_write_func* func, void* context, int quality, int width, int height,
                             int num_components, const unsigned char* src) {
    if (!ctx || !func) return 0;
    if (quality < 1 || quality > 3) { ctx->err = "quality must be 1, 2 or 3"; return 0; }   // jpeg_enc.h:1223
    if (num_components != 3 && num_components != 4) { ctx->err = "num_components must be 3 or 4"; return 0; }  // :954
    if (width > 0xFFFF || height > 0xFFFF || width < 0 || height < 0) { ctx->err = "image too large"; return 0; }  // :958
    if ((int64_t)width * height > 0 && !src) { ctx->err = "null source"; return 0; }
    ICX_HIP(ctx, hipSetDevice(ctx->device), 0);
    std::vector<uint8_t> file;
    if (!tje_encode_gpu(ctx->stream, quality, width, height, num_components, src, file)) {
        ctx->err = "HIP failure in tje_encode_gpu";
        return 0;
    }
    // tje hands the sink buffered chunks of TJEI_BUFFER_SIZE-1 bytes (jpeg_enc.h:474-496)
    for (size_t o = 0; o < file.size(); o += 1023)
        func(context, file.data() + o, (int)std::min<size_t>(1023, file.size() - o));
    return 1;
}

static void file_sink(void* ctx, void* data, int size) { std::fwrite(data, (size_t)size, 1, (FILE*)ctx); }

int icx_tje_encode_to_file_at_quality(icx_ctx* ctx, const char* dest_path, int quality, int width, int height,
                                      int num_components, const unsigned char* src) {
    FILE* fd = std::fopen(dest_path, "wb");  // jpeg_enc.h:1194-1213
    if (!fd) { if (ctx) ctx->err = "could not open file for writing"; return 0; }
    int result = icx_tje_encode_with_func(ctx, file_sink, fd, quality, width, height, num_components, src);
    result |= 0 == std::fclose(fd);  // the reference's own (lossy) success rule, :1210
    return result;
}

int icx_tje_encode_to_file(icx_ctx* ctx, const char* dest_path, int width, int height, int num_components,
                           const unsigned char* src) {
    return icx_tje_encode_to_file_at_quality(ctx, dest_path, 3, width, height, num_components, src);  // :1177-1185
}

// ------------------------------------------------------------------ encode extension (C4)
static const char* enc_args_bad(int quality, int subsampling, int width, int height, int comps) {
    if (quality < 1 || quality > 100) return "quality must be 1..100";
    if (subsampling != 444 && subsampling != 420) return "subsampling must be 444 or 420";
    if (comps != 3 && comps != 4) return "num_components must be 3 or 4";
    if (width > 0xFFFF || height > 0xFFFF || width < 0 || height < 0) return "image too large";
    return nullptr;
}

int icx_jpeg_encode_with_func(icx_ctx* ctx, icx_write_func* func, void* context, int quality, int subsampling,
                              int width, int height, int num_components, const unsigned char* src) {
    if (!ctx || !func) return 0;
    if (const char* e = enc_args_bad(quality, subsampling, width, height, num_components)) { ctx->err = e; return 0; }
    if ((int64_t)width * height > 0 && !src) { ctx->err = "null source"; return 0; }
    ICX_HIP(ctx, hipSetDevice(ctx->device), 0);
    std::vector<uint8_t> file;
    if (!jpeg_encode_gpu(ctx->stream, quality, subsampling, width, height, num_components, src, file)) {
        ctx->err = "HIP failure in jpeg_encode_gpu";
        return 0;
    }
    for (size_t o = 0; o < file.size(); o += 1023)
        func(context, file.data() + o, (int)std::min<size_t>(1023, file.size() - o));
    return 1;
}

struct icx_encoder {
    icx_ctx* ctx = nullptr;
    EncWs* ws = nullptr;
};

icx_encoder* icx_encoder_create(icx_ctx* ctx) {
    if (!ctx) return nullptr;
    icx_encoder* e = new icx_encoder();
    e->ctx = ctx;
    e->ws = enc_ws_create();
    return e;
}

void icx_encoder_destroy(icx_encoder* enc) {
    if (!enc) return;
    (void)hipSetDevice(enc->ctx->device);
    enc_ws_destroy(enc->ws);
    delete enc;
}

int icx_encoder_stage_times(icx_encoder* enc, const char** names, float* ms, int cap) {
    if (!enc || cap <= 0) return 0;
    return enc_ws_stage_times(enc->ws, names, ms, cap);
}

int icx_jpeg_encode_device(icx_encoder* enc, int quality, int subsampling, int width, int height,
                           int num_components, const uint8_t* d_src, uint8_t* d_out, uint64_t out_cap,
                           uint64_t* out_size, void* hip_stream) {
    if (!enc || !out_size) return ICX_UNSUPPORTED;
    icx_ctx* ctx = enc->ctx;
    if (const char* e = enc_args_bad(quality, subsampling, width, height, num_components)) {
        ctx->err = e;
        return ICX_UNSUPPORTED;
    }
    if (((int64_t)width * height > 0 && !d_src) || (out_cap && !d_out)) { ctx->err = "null buffer"; return ICX_UNSUPPORTED; }
    ICX_HIP(ctx, hipSetDevice(ctx->device), ICX_INTERNAL_ERR);
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : ctx->stream;
    const int rc = jpeg_encode_device(st, enc->ws, quality, subsampling, width, height, num_components, d_src, d_out,
                                      out_cap, out_size);
    if (rc < 0) { ctx->err = "HIP failure in jpeg_encode_device"; return ICX_INTERNAL_ERR; }
    return rc == 0 ? ICX_OK : ICX_OUT_OF_MEM;
}

int icx_jpeg_encode_device_batch(icx_encoder* enc, int n, int quality, int subsampling, int width, int height,
                                 int num_components, const uint8_t* const* d_srcs, uint8_t* d_out, uint64_t out_stride,
                                 uint64_t* out_sizes, int32_t* status, void* hip_stream) {
    if (!enc || n < 0 || (n > 0 && (!d_srcs || !out_sizes || !status))) return ICX_UNSUPPORTED;
    icx_ctx* ctx = enc->ctx;
    if (const char* e = enc_args_bad(quality, subsampling, width, height, num_components)) {
        ctx->err = e;
        return ICX_UNSUPPORTED;
    }
    for (int i = 0; i < n; ++i)
        if ((int64_t)width * height > 0 && !d_srcs[i]) { ctx->err = "null buffer"; return ICX_UNSUPPORTED; }
    if (n > 0 && out_stride && !d_out) { ctx->err = "null buffer"; return ICX_UNSUPPORTED; }
    ICX_HIP(ctx, hipSetDevice(ctx->device), ICX_INTERNAL_ERR);
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : ctx->stream;
    std::vector<int32_t> rc(n > 0 ? n : 1);
    if (jpeg_encode_device_batch(st, enc->ws, n, quality, subsampling, width, height, num_components, d_srcs, d_out,
                                 out_stride, out_sizes, rc.data()) < 0) {
        ctx->err = "HIP failure in jpeg_encode_device_batch";
        return ICX_INTERNAL_ERR;
    }
    for (int i = 0; i < n; ++i) status[i] = rc[i] == 0 ? ICX_OK : ICX_OUT_OF_MEM;
    return ICX_OK;
}

// ------------------------------------------------------------------ PNG (png_encoder::saveToFile)
static const char* png_args_bad(int w, int h, int d) {
    if (d != 3 && d != 4) return "d must be 3 or 4";
    if (w <= 0 || h <= 0) return "empty image";
    if ((int64_t)w * h > (int64_t)1 << 31) return "image too large";
    return nullptr;
}

int icx_png_encode_with_func(icx_ctx* ctx, icx_write_func* func, void* context, const unsigned char* pixels, int width,
                             int height, int d) {
    if (!ctx || !func) return 0;
    if (const char* e = png_args_bad(width, height, d)) { ctx->err = e; return 0; }
    if (!pixels) { ctx->err = "null source"; return 0; }
    ICX_HIP(ctx, hipSetDevice(ctx->device), 0);
    std::vector<uint8_t> file;
    if (!png_encode_gpu(ctx->stream, width, height, d, pixels, file)) {
        ctx->err = "HIP failure in png_encode_gpu";
        return 0;
    }
    for (size_t o = 0; o < file.size(); o += 1023)
        func(context, file.data() + o, (int)std::min<size_t>(1023, file.size() - o));
    return 1;
}

int icx_png_save_to_file(icx_ctx* ctx, const char* path, const unsigned char* pixels, int width, int height, int d) {
    if (!ctx || !path) return ICX_UNSUPPORTED;
    FILE* fd = std::fopen(path, "wb");
    if (!fd) { ctx->err = "could not open file for writing"; return ICX_INTERNAL_ERR; }
    const int ok = icx_png_encode_with_func(ctx, file_sink, fd, pixels, width, height, d);
    const bool closed = std::fclose(fd) == 0;
    if (!ok) return png_args_bad(width, height, d) || !pixels ? ICX_UNSUPPORTED : ICX_INTERNAL_ERR;
    return closed ? ICX_OK : ICX_INTERNAL_ERR;
}

// Images the PNG batch entry keeps in flight (each with its own workspace and stream):
// ICX_PNG_INFLIGHT, 1..8.
constexpr int kPngInflightMax = 8;
struct icx_png_encoder {
    icx_ctx* ctx = nullptr;
    PngWs* ws = nullptr;
    PngWs* wsx[kPngInflightMax] = {};      // the batch entry's other workspaces + streams (created on use)
    hipStream_t stx[kPngInflightMax] = {};
    hipEvent_t fork = nullptr;
};

icx_png_encoder* icx_png_encoder_create(icx_ctx* ctx) {
    if (!ctx) return nullptr;
    icx_png_encoder* e = new icx_png_encoder();
    e->ctx = ctx;
    e->ws = png_ws_create();
    return e;
}

void icx_png_encoder_destroy(icx_png_encoder* enc) {
    if (!enc) return;
    (void)hipSetDevice(enc->ctx->device);
    png_ws_destroy(enc->ws);
    for (int j = 0; j < kPngInflightMax; ++j) {
        if (enc->wsx[j]) png_ws_destroy(enc->wsx[j]);
        if (enc->stx[j]) (void)hipStreamDestroy(enc->stx[j]);
    }
    if (enc->fork) (void)hipEventDestroy(enc->fork);
    delete enc;
}

int icx_png_encode_device(icx_png_encoder* enc, int width, int height, int d, const uint8_t* d_src, uint8_t* d_out,
                          uint64_t out_cap, uint64_t* out_size, void* hip_stream) {
    if (!enc || !out_size) return ICX_UNSUPPORTED;
    icx_ctx* ctx = enc->ctx;
    if (const char* e = png_args_bad(width, height, d)) { ctx->err = e; return ICX_UNSUPPORTED; }
    if (!d_src || (out_cap && !d_out)) { ctx->err = "null buffer"; return ICX_UNSUPPORTED; }
    ICX_HIP(ctx, hipSetDevice(ctx->device), ICX_INTERNAL_ERR);
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : ctx->stream;
    const int rc = png_encode_device(st, enc->ws, width, height, d, d_src, d_out, out_cap, out_size);
    if (rc < 0) { ctx->err = "HIP failure in png_encode_device"; return ICX_INTERNAL_ERR; }
    return rc == 0 ? ICX_OK : ICX_OUT_OF_MEM;
}

int icx_png_encode_device_batch(icx_png_encoder* enc, int n, int width, int height, int d, const uint8_t* const* d_srcs,
                                uint8_t* d_out, uint64_t out_stride, uint64_t* out_sizes, int32_t* status,
                                void* hip_stream) {
    if (!enc || n < 0 || (n > 0 && (!d_srcs || !out_sizes || !status))) return ICX_UNSUPPORTED;
    icx_ctx* ctx = enc->ctx;
    if (const char* e = png_args_bad(width, height, d)) { ctx->err = e; return ICX_UNSUPPORTED; }
    for (int i = 0; i < n; ++i)
        if (!d_srcs[i]) { ctx->err = "null buffer"; return ICX_UNSUPPORTED; }
    if (n > 0 && (!d_out || !out_stride)) { ctx->err = "null buffer"; return ICX_UNSUPPORTED; }
    if (n == 0) return ICX_OK;
    ICX_HIP(ctx, hipSetDevice(ctx->device), ICX_INTERNAL_ERR);
    const int k = [] {  // (read per call)
        const char* e = std::getenv("ICX_PNG_INFLIGHT");
        return e ? std::max(1, std::min(kPngInflightMax, std::atoi(e))) : kPngInflightMax;
    }();
    if (!enc->fork) ICX_HIP(ctx, hipEventCreateWithFlags(&enc->fork, hipEventDisableTiming), ICX_INTERNAL_ERR);
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : ctx->stream;
    // the other streams start after the caller's prior work on `st` (which may produce the inputs)
    ICX_HIP(ctx, hipEventRecord(enc->fork, st), ICX_INTERNAL_ERR);
    hipStream_t sts[kPngInflightMax];
    PngWs* wss[kPngInflightMax];
    sts[0] = st;
    wss[0] = enc->ws;
    for (int j = 1; j < k; ++j) {
        if (!enc->wsx[j]) enc->wsx[j] = png_ws_create();
        if (!enc->stx[j]) ICX_HIP(ctx, hipStreamCreateWithFlags(&enc->stx[j], hipStreamNonBlocking), ICX_INTERNAL_ERR);
        ICX_HIP(ctx, hipStreamWaitEvent(enc->stx[j], enc->fork, 0), ICX_INTERNAL_ERR);
        sts[j] = enc->stx[j];
        wss[j] = enc->wsx[j];
    }
    std::vector<int32_t> rc(n, -1);
    for (int i = 0; i < n; ++i) out_sizes[i] = 0;
    const int call = png_encode_device_batch(k, sts, wss, n, width, height, d, d_srcs, d_out, out_stride, out_sizes,
                                             rc.data());
    // every image gets its own status, also when another one failed: 0 OK, 1 its file did not fit
    // out_stride, -1 a HIP or host allocation failure in its own job
    for (int i = 0; i < n; ++i) {
        status[i] = rc[i] == 0 ? ICX_OK : rc[i] == 1 ? ICX_OUT_OF_MEM : ICX_INTERNAL_ERR;
        if (rc[i] < 0) out_sizes[i] = 0;
    }
    if (call < 0) {  // a stream failed: the whole call
        ctx->err = "HIP failure in png_encode_device_batch";
        return ICX_INTERNAL_ERR;
    }
    for (int i = 0; i < n; ++i)
        if (rc[i] < 0) { ctx->err = "png_encode_device_batch: an image's job failed (see status)"; break; }
    return ICX_OK;
}

int icx_png_encoder_stage_times(icx_png_encoder* enc, const char** names, float* ms, int cap) {
    if (!enc || cap <= 0) return 0;
    const int k = png_ws_stage_times(enc->ws, names, ms, cap);
    for (int j = 1; j < kPngInflightMax; ++j) {  // the batch entry's other workspaces: summed
        if (!enc->wsx[j] || !ms) continue;
        float m2[8] = {};
        const int k2 = png_ws_stage_times(enc->wsx[j], nullptr, m2, std::min(cap, 8));
        for (int i = 0; i < std::min(k, k2); ++i) ms[i] += m2[i];
    }
    return k;
}

// --------------------------------------------------------- Radiance .hdr (Image::readHdr)
struct icx_hdr_batch {
    icx_ctx* ctx = nullptr;
    HdrWs ws;
    std::unique_ptr<EventHook> hook;
};

int icx_hdr_probe(const uint8_t* data, size_t size, int* w, int* h) {
    int ww = 0, hh = 0;
    const int rc = data ? hdr_probe(data, (int64_t)size, &ww, &hh) : ICX_HDR_NOT_RADIANCE;
    if (w) *w = rc == ICX_HDR_OK ? ww : 0;
    if (h) *h = rc == ICX_HDR_OK ? hh : 0;
    return rc;
}

icx_hdr_batch* icx_hdr_batch_create(icx_ctx* ctx, int max_images, int max_w, int max_h) {
    if (!ctx || max_images <= 0 || max_w <= 0 || max_h <= 0) {
        if (ctx) ctx->err = "icx_hdr_batch_create: bad arguments";
        return nullptr;
    }
    ICX_HIP(ctx, hipSetDevice(ctx->device), nullptr);
    auto* b = new icx_hdr_batch();
    b->ctx = ctx;
    b->hook = std::make_unique<EventHook>();
    if (!hdr_ws_alloc(b->ws, max_images, max_w, max_h)) {
        hdr_ws_free(b->ws);
        delete b;
        ctx->err = "icx_hdr_batch_create: out of device memory";
        return nullptr;
    }
    return b;
}

void icx_hdr_batch_destroy(icx_hdr_batch* b) {
    if (!b) return;
    (void)hipSetDevice(b->ctx->device);
    hdr_ws_free(b->ws);
    delete b;
}

int icx_hdr_batch_decode(icx_hdr_batch* b, int n, const uint8_t* d_data, const uint64_t* d_off, const uint64_t* d_size,
                         float* d_out, uint64_t out_stride, int32_t* d_status, int32_t* d_dims, void* stream) {
    if (!b) return ICX_HDR_INTERNAL_ERR;
    icx_ctx* ctx = b->ctx;
    if (n < 0 || n > b->ws.max_images) { ctx->err = "icx_hdr_batch_decode: n exceeds batch capacity"; return ICX_HDR_INTERNAL_ERR; }
    if (n == 0) return ICX_HDR_OK;
    if (!d_data || !d_off || !d_size || !d_out || !d_status || !d_dims) { ctx->err = "null pointer"; return ICX_HDR_INTERNAL_ERR; }
    if (out_stride < 4ull * b->ws.max_w * b->ws.max_h) { ctx->err = "icx_hdr_batch_decode: out_stride too small"; return ICX_HDR_INTERNAL_ERR; }
    ICX_HIP(ctx, hipSetDevice(ctx->device), ICX_HDR_INTERNAL_ERR);
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    const RoctxRange range("icx_hdr_batch_decode");
    b->hook->reset();
    launch_hdr_decode(b->ws, n, d_data, d_off, d_size, d_out, out_stride, d_status, d_dims, st, b->hook.get());
    ICX_HIP(ctx, hipGetLastError(), ICX_HDR_INTERNAL_ERR);
    return ICX_HDR_OK;
}

int icx_hdr_batch_stage_times(const icx_hdr_batch* b, const char** names, float* ms, int cap) {
    if (!b) return 0;
    static const Stage order[4] = {kStParse, kStUnstuff, kStEntropy, kStConvert};
    static const char* const label[4] = {"parse", "locate", "unpack", "convert"};
    float acc[kStCount] = {0};
    for (auto& r : b->hook->recs) {
        float t = 0;
        if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&t, r.a, r.b) == hipSuccess) acc[r.s] += t;
    }
    for (int k = 0; k < 4 && k < cap; ++k) {
        if (names) names[k] = label[k];
        if (ms) ms[k] = acc[order[k]];
    }
    return 4;
}

int icx_hdr_decode(icx_ctx* ctx, const uint8_t* data, size_t size, float** out, int* w, int* h, int* rows) {
    if (out) *out = nullptr;
    if (w) *w = 0;
    if (h) *h = 0;
    if (rows) *rows = 0;
    if (!ctx || !out) return ICX_HDR_INTERNAL_ERR;
    int ww = 0, hh = 0;
    const int prc = icx_hdr_probe(data, size, &ww, &hh);
    if (prc != ICX_HDR_OK) return prc;  // header errors need no device work
    ICX_HIP(ctx, hipSetDevice(ctx->device), ICX_HDR_INTERNAL_ERR);
    icx_hdr_batch* b = icx_hdr_batch_create(ctx, 1, ww, hh);
    if (!b) return ICX_HDR_INTERNAL_ERR;
    const uint64_t nout = 4ull * ww * hh;
    uint8_t* d_in = nullptr;
    float* d_out = nullptr;
    uint64_t* d_meta = nullptr;
    int32_t* d_res = nullptr;
    int rc = ICX_HDR_INTERNAL_ERR;
    const uint64_t meta[2] = {0, (uint64_t)size};
    int32_t res[4] = {0, 0, 0, 0};
    hipStream_t st = ctx->stream;
    if (hipMalloc(&d_in, size + 16) == hipSuccess && hipMalloc(&d_out, nout * 4) == hipSuccess &&
        hipMalloc(&d_meta, 16) == hipSuccess && hipMalloc(&d_res, 16) == hipSuccess &&
        hipMemcpyAsync(d_in, data, size, hipMemcpyHostToDevice, st) == hipSuccess &&
        hipMemcpyAsync(d_meta, meta, 16, hipMemcpyHostToDevice, st) == hipSuccess &&
        icx_hdr_batch_decode(b, 1, d_in, d_meta, d_meta + 1, d_out, nout, d_res, d_res + 1, st) == ICX_HDR_OK &&
        hipMemcpyAsync(res, d_res, 16, hipMemcpyDeviceToHost, st) == hipSuccess && hipStreamSynchronize(st) == hipSuccess) {
        rc = res[0];
        float* hostp = (float*)std::malloc(nout * 4);
        if (hostp && hipMemcpy(hostp, d_out, nout * 4, hipMemcpyDeviceToHost) == hipSuccess) {
            *out = hostp;
            if (w) *w = res[1];
            if (h) *h = res[2];
            if (rows) *rows = res[3];
        } else {
            std::free(hostp);
            ctx->err = "icx_hdr_decode: host allocation or copy failed";
            rc = ICX_HDR_INTERNAL_ERR;
        }
    } else if (ctx->err.empty()) {
        ctx->err = "icx_hdr_decode: HIP failure";
    }
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    (void)hipFree(d_meta);
    (void)hipFree(d_res);
    icx_hdr_batch_destroy(b);
    return rc;
}

// --------------------------------------------------------- OpenEXR (Image::readExr)
int icx_exr_probe(const uint8_t* data, size_t size, int* w, int* h) {
    if (w) *w = 0;
    if (h) *h = 0;
    if (!data) return ICX_EXR_INVALID_ARGUMENT;
    try {  // (nothing may cross the C ABI: a host allocation failure is an internal error)
        return exr_probe(data, size, w, h);
    } catch (const std::exception&) {
        return ICX_EXR_INTERNAL_ERR;
    }
}

int icx_exr_decode(icx_ctx* ctx, const uint8_t* data, size_t size, float** out, int* w, int* h) {
    if (out) *out = nullptr;
    if (w) *w = 0;
    if (h) *h = 0;
    if (!ctx) return ICX_EXR_INTERNAL_ERR;
    if (!data || !out) return ICX_EXR_INVALID_ARGUMENT;  // LoadEXRFromMemory's NULL checks (:6648-6651)
    ICX_HIP(ctx, hipSetDevice(ctx->device), ICX_EXR_INTERNAL_ERR);
    const RoctxRange range("icx_exr_decode");
    int ww = 0, hh = 0;
    std::string err;
    int rc;
    try {  // (nothing may cross the C ABI: a host allocation failure is an internal error)
        if (!ctx->exr) ctx->exr = exr_ws_create();
        rc = exr_decode(ctx->stream, *ctx->exr, data, size, nullptr, nullptr, 0, out, &ww, &hh, err);
    } catch (const std::exception& e) {
        err = std::string("icx_exr_decode: ") + e.what();
        rc = ICX_EXR_INTERNAL_ERR;
    }
    if (rc == ICX_EXR_INTERNAL_ERR) ctx->err = err.empty() ? "icx_exr_decode: HIP failure" : err;
    if (rc == ICX_EXR_SUCCESS) {
        if (w) *w = ww;
        if (h) *h = hh;
    }
    return rc;
}

int icx_exr_decode_device_batch(icx_ctx* ctx, int n, const uint8_t* const* data, const uint8_t* const* d_data,
                                const size_t* sizes, float* const* d_out, const size_t* out_floats, int32_t* codes,
                                int32_t* widths, int32_t* heights) {
    if (!ctx) return ICX_EXR_INTERNAL_ERR;
    if (n < 0 || (n > 0 && (!data || !d_data || !sizes || !d_out || !out_floats || !codes || !widths || !heights)))
        return ICX_EXR_INVALID_ARGUMENT;
    for (int i = 0; i < n; ++i)
        if (!data[i] || !d_data[i] || !d_out[i] || (reinterpret_cast<uintptr_t>(d_data[i]) & 15)) {
            ctx->err = "icx_exr_decode_device_batch: d_data[i] must be non-null and 16-byte aligned";
            return ICX_EXR_INVALID_ARGUMENT;
        }
    if (n == 0) return ICX_EXR_SUCCESS;
    ICX_HIP(ctx, hipSetDevice(ctx->device), ICX_EXR_INTERNAL_ERR);
    const RoctxRange range("icx_exr_decode_device_batch");
    std::string err;
    int rc;
    try {
        if (!ctx->exr) ctx->exr = exr_ws_create();
        rc = exr_decode_batch(ctx->stream, *ctx->exr, n, data, d_data, sizes, d_out, out_floats, codes, widths, heights, err);
    } catch (const std::exception& e) {
        err = std::string("icx_exr_decode_device_batch: ") + e.what();
        rc = ICX_EXR_INTERNAL_ERR;
    }
    if (rc != 0) {
        ctx->err = err.empty() ? "icx_exr_decode_device_batch: HIP failure" : err;
        return ICX_EXR_INTERNAL_ERR;
    }
    return ICX_EXR_SUCCESS;
}

int icx_exr_decode_device(icx_ctx* ctx, const uint8_t* data, const uint8_t* d_data, size_t size, float* d_out,
                          size_t out_floats, int* w, int* h) {
    if (w) *w = 0;
    if (h) *h = 0;
    if (!ctx) return ICX_EXR_INTERNAL_ERR;
    if (!data || !d_data || !d_out || (reinterpret_cast<uintptr_t>(d_data) & 15)) {
        ctx->err = "icx_exr_decode_device: d_data must be non-null and 16-byte aligned";
        return ICX_EXR_INVALID_ARGUMENT;
    }
    ICX_HIP(ctx, hipSetDevice(ctx->device), ICX_EXR_INTERNAL_ERR);
    const RoctxRange range("icx_exr_decode_device");
    int ww = 0, hh = 0;
    std::string err;
    int rc;
    try {
        if (!ctx->exr) ctx->exr = exr_ws_create();
        rc = exr_decode(ctx->stream, *ctx->exr, data, size, d_data, d_out, out_floats, nullptr, &ww, &hh, err);
    } catch (const std::exception& e) {
        err = std::string("icx_exr_decode_device: ") + e.what();
        rc = ICX_EXR_INTERNAL_ERR;
    }
    if (rc == ICX_EXR_INTERNAL_ERR) ctx->err = err.empty() ? "icx_exr_decode_device: HIP failure" : err;
    if (rc == ICX_EXR_SUCCESS) {
        if (w) *w = ww;
        if (h) *h = hh;
    }
    return rc;
}

}  // extern "C"
