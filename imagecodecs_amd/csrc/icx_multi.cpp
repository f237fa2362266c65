// icx_multi.cpp -- multi-GPU batch decode for C/C++ callers of libicx.so.
//
// Images are independent, so a batch is sharded by image: a greedy longest-first split by
// compressed size (decode time follows the entropy-coded bytes), one host thread per device, each
// with its own icx context, batch workspace and stream. Every device decodes its shard and
// computes the per-image records {status, w, h, ncomp, checksum64} (icx_records.hip). The final
// gather of those 24-byte records goes over RCCL (xGMI between the GPUs of a node): one
// communicator per device from ncclCommInitAll, every device's records padded to the largest
// shard and all-gathered in one grouped ncclAllGather, then read from the first device -- the
// same exchange the multi-process path makes (imagecodecs_amd/shard.py). With one device, a
// device listed twice (RCCL needs distinct GPUs: a one-GPU lease tests the sharding this way) or
// no RCCL, the records come back per device through host memory. The caller's pixels are copied
// to its host buffers by each device.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "../../include/icx.h"
#include "icx_internal.h"

using namespace icx;

namespace {
struct Dev {
    int device = 0;
    icx_ctx* ctx = nullptr;
    icx_batch* batch = nullptr;
    int cap_images = 0;
    // device staging, grown on demand
    uint8_t* d_buf = nullptr;
    size_t d_cap = 0;
    Record* d_rec = nullptr;  // the last shard's records on the device (RCCL gather)
    Record* d_all = nullptr;  // the gather's receive buffer
    std::string err;
};
}  // namespace

// RCCL, loaded at run time (librccl.so of the ROCm install): the library links no collective
// library, so a process that never builds a multi-device batch does not load it.
struct Rccl {
    void* so = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    bool load() {
        so = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (!so) so = dlopen("/opt/rocm/lib/librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (!so) return false;
        init_all = reinterpret_cast<decltype(init_all)>(dlsym(so, "ncclCommInitAll"));
        all_gather = reinterpret_cast<decltype(all_gather)>(dlsym(so, "ncclAllGather"));
        group_start = reinterpret_cast<decltype(group_start)>(dlsym(so, "ncclGroupStart"));
        group_end = reinterpret_cast<decltype(group_end)>(dlsym(so, "ncclGroupEnd"));
        destroy = reinterpret_cast<decltype(destroy)>(dlsym(so, "ncclCommDestroy"));
        error_string = reinterpret_cast<decltype(error_string)>(dlsym(so, "ncclGetErrorString"));
        return init_all && all_gather && group_start && group_end && destroy && error_string;
    }
};

struct icx_multi {
    std::vector<Dev> devs;
    int max_w = 0, max_h = 0;
    std::string err;
    Rccl rccl;
    std::vector<ncclComm_t> comms;  // empty: records gathered through host memory
    std::string gather_note, gather_desc;
};

extern "C" {

icx_multi* icx_multi_create(const int* devices, int ndev, int max_width, int max_height) {
    if (!devices || ndev <= 0 || max_width <= 0 || max_height <= 0) return nullptr;
    auto* m = new icx_multi();
    m->max_w = max_width;
    m->max_h = max_height;
    for (int k = 0; k < ndev; ++k) {
        Dev d;
        d.device = devices[k];
        d.ctx = icx_create(devices[k]);
        if (!d.ctx) {
            for (auto& e : m->devs) icx_destroy(e.ctx);
            delete m;
            return nullptr;
        }
        m->devs.push_back(d);
    }
    // RCCL communicators over distinct devices (ICX_MULTI_RCCL=0: always the host gather)
    std::vector<int> dl(devices, devices + ndev), sorted = dl;
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    const char* env = std::getenv("ICX_MULTI_RCCL");
    if (ndev < 2) m->gather_note = "one device";
    else if (!distinct) m->gather_note = "a device listed twice (RCCL needs distinct GPUs)";
    else if (env && std::atoi(env) == 0) m->gather_note = "ICX_MULTI_RCCL=0";
    else if (!m->rccl.load()) m->gather_note = "librccl.so not loadable";
    else {
        m->comms.assign(ndev, nullptr);
        const ncclResult_t r = m->rccl.init_all(m->comms.data(), ndev, dl.data());
        if (r != ncclSuccess) {
            m->gather_note = std::string("ncclCommInitAll: ") + m->rccl.error_string(r);
            m->comms.clear();
        } else {
            m->gather_note = "rccl";
        }
    }
    m->gather_desc = m->comms.empty() ? "host (" + m->gather_note + ")" : "rccl";
    return m;
}

void icx_multi_destroy(icx_multi* m) {
    if (!m) return;
    for (ncclComm_t c : m->comms)
        if (c) (void)m->rccl.destroy(c);
    for (auto& d : m->devs) {
        (void)hipSetDevice(d.device);
        if (d.d_buf) (void)hipFree(d.d_buf);
        if (d.batch) icx_batch_destroy(d.batch);
        icx_destroy(d.ctx);
    }
    delete m;
}

const char* icx_multi_last_error(const icx_multi* m) { return m ? m->err.c_str() : ""; }

int icx_multi_shard(const size_t* sizes, int n, int ndev, int32_t* shard_of) {
    if (n < 0 || ndev <= 0 || (n > 0 && (!sizes || !shard_of))) return ICX_INTERNAL_ERR;
    std::vector<int> order(n);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return sizes[a] > sizes[b]; });
    std::vector<uint64_t> load(ndev, 0);
    for (int i : order) {
        const int r = (int)(std::min_element(load.begin(), load.end()) - load.begin());  // lowest index on ties
        shard_of[i] = r;
        load[r] += sizes[i];
    }
    return ICX_OK;
}

// One device's shard: stage the files, decode, records, copy pixels back; its records go to
// `records` (the host gather; the shard reads them anyway to pick its pixel copies) and, for the
// RCCL gather, stay in d.d_rec, padded to `pad` entries.
static int run_shard(icx_multi* m, Dev& d, const std::vector<int>& idx, const uint8_t* const* jpegs,
                     const size_t* sizes, uint8_t* const* outs, uint64_t out_stride, icx_record* records, int pad) {
    const int n = (int)idx.size();
    d.d_rec = nullptr;
    if (n == 0 && pad == 0) return ICX_OK;
    if (hipSetDevice(d.device) != hipSuccess) { d.err = "hipSetDevice failed"; return ICX_INTERNAL_ERR; }
    if (n > 0 && (!d.batch || d.cap_images < n)) {
        if (d.batch) icx_batch_destroy(d.batch);
        d.batch = icx_batch_create(d.ctx, n, m->max_w, m->max_h, 0);
        d.cap_images = d.batch ? n : 0;
        if (!d.batch) { d.err = std::string("icx_batch_create: ") + icx_last_error(d.ctx); return ICX_OUT_OF_MEM; }
    }
    std::vector<uint64_t> off(n), sz(n);
    uint64_t total = 0;
    for (int k = 0; k < n; ++k) {
        off[k] = total;
        sz[k] = sizes[idx[k]];
        total += (sz[k] + 15) & ~uint64_t(15);
    }
    const uint64_t stride_al = (out_stride + 255) & ~uint64_t(255);
    const int nr = std::max(n, pad);  // record slots: the shard, padded for the gather
    const size_t meta = (size_t)n * (8 + 8 + 4 + 12) + (size_t)nr * sizeof(icx_record) * (1 + m->devs.size()) + 1024;
    const size_t need = total + meta + (size_t)n * stride_al + 256;
    if (need > d.d_cap) {
        if (d.d_buf) (void)hipFree(d.d_buf);
        d.d_buf = nullptr;
        d.d_cap = 0;
        if (hipMalloc(&d.d_buf, need) != hipSuccess) { d.err = "hipMalloc of the shard staging failed"; return ICX_OUT_OF_MEM; }
        d.d_cap = need;
    }
    uint8_t* base = d.d_buf;
    auto align = [](uintptr_t p, uintptr_t a) { return (p + a - 1) & ~(a - 1); };
    uint8_t* d_data = base;
    uint64_t* d_off = reinterpret_cast<uint64_t*>(align((uintptr_t)(base + total), 16));
    uint64_t* d_sz = d_off + n;
    int32_t* d_st = reinterpret_cast<int32_t*>(d_sz + n);
    int32_t* d_dm = d_st + n;
    Record* d_rec = reinterpret_cast<Record*>(align((uintptr_t)(d_dm + 3 * n), 16));
    d.d_all = d_rec + nr;  // (the RCCL gather's receive buffer: nr records per device)
    uint8_t* d_out = reinterpret_cast<uint8_t*>(align((uintptr_t)(d.d_all + nr * m->devs.size()), 256));
    hipStream_t st = nullptr;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) { d.err = "hipStreamCreate failed"; return ICX_INTERNAL_ERR; }
    int rc = ICX_OK;
    auto chk = [&](hipError_t e, const char* what) {
        if (e != hipSuccess && rc == ICX_OK) {
            d.err = std::string(what) + ": " + hipGetErrorString(e);
            rc = ICX_INTERNAL_ERR;
        }
        return rc == ICX_OK;
    };
    for (int k = 0; k < n && rc == ICX_OK; ++k)
        if (sz[k]) chk(hipMemcpyAsync(d_data + off[k], jpegs[idx[k]], sz[k], hipMemcpyHostToDevice, st), "H2D");
    if (n > 0) {
        chk(hipMemcpyAsync(d_off, off.data(), 8 * n, hipMemcpyHostToDevice, st), "H2D offsets");
        chk(hipMemcpyAsync(d_sz, sz.data(), 8 * n, hipMemcpyHostToDevice, st), "H2D sizes");
    }
    if (rc == ICX_OK && n > 0) {
        rc = icx_jpeg_batch_decode(d.batch, n, d_data, d_off, d_sz, d_out, stride_al, d_st, d_dm, st);
        if (rc != ICX_OK) d.err = icx_last_error(d.ctx);
    }
    if (rc == ICX_OK && pad > n) chk(hipMemsetAsync(d_rec + n, 0, sizeof(Record) * (pad - n), st), "record padding");
    if (rc == ICX_OK && n > 0) {
        launch_records(n, d_out, stride_al, d_st, d_dm, d_rec, m->max_w, m->max_h, st);
        chk(hipGetLastError(), "k_records launch");
    }
    std::vector<Record> rec(n);
    if (rc == ICX_OK && n > 0) chk(hipMemcpyAsync(rec.data(), d_rec, sizeof(Record) * n, hipMemcpyDeviceToHost, st), "D2H records");
    if (rc == ICX_OK) chk(hipStreamSynchronize(st), "decode");
    for (int k = 0; k < n && rc == ICX_OK; ++k) {
        Record& r = rec[k];
        uint64_t bytes = (uint64_t)r.w * r.h * r.c;
        if (r.status == ICX_OK && bytes > out_stride) {
            // decoded into the 256-aligned staging stride, but the caller's buffer holds less:
            // NanoJPEG's allocation failure, as icx_jpeg_batch_decode reports an image past its
            // out_stride (never a truncated copy under an OK status)
            r = Record{};
            r.status = ICX_OUT_OF_MEM;
            bytes = 0;
        }
        std::memcpy(&records[idx[k]], &r, sizeof r);  // (also with RCCL: the fallback if its gather fails)
        if (outs && outs[idx[k]] && r.status == ICX_OK && bytes)
            chk(hipMemcpyAsync(outs[idx[k]], d_out + (uint64_t)k * stride_al, std::min<uint64_t>(bytes, out_stride),
                               hipMemcpyDeviceToHost, st), "D2H pixels");
    }
    if (rc == ICX_OK) chk(hipStreamSynchronize(st), "D2H");
    (void)hipStreamDestroy(st);
    if (rc == ICX_OK && pad > 0) d.d_rec = d_rec;
    return rc;
}

// The records of every shard (d.d_rec, `pad` each) all-gathered over RCCL, read from the first
// device; the out_stride rule run_shard applies on the host gather applied here too.
static int rccl_gather(icx_multi* m, const std::vector<std::vector<int>>& idx, int pad, uint64_t out_stride,
                       icx_record* records) {
    const int nd = (int)m->devs.size();
    std::vector<hipStream_t> sts(nd, nullptr);
    int rc = ICX_OK;
    for (int k = 0; k < nd && rc == ICX_OK; ++k) {
        if (hipSetDevice(m->devs[k].device) != hipSuccess ||
            hipStreamCreateWithFlags(&sts[k], hipStreamNonBlocking) != hipSuccess) rc = ICX_INTERNAL_ERR;
    }
    if (rc == ICX_OK) {
        ncclResult_t r = m->rccl.group_start();
        for (int k = 0; k < nd && r == ncclSuccess; ++k)
            r = m->rccl.all_gather(m->devs[k].d_rec, m->devs[k].d_all, sizeof(Record) * (size_t)pad, ncclUint8,
                                   m->comms[k], sts[k]);
        const ncclResult_t e = m->rccl.group_end();
        if (r == ncclSuccess) r = e;
        if (r != ncclSuccess) {
            m->err = std::string("ncclAllGather: ") + m->rccl.error_string(r);
            rc = ICX_INTERNAL_ERR;
        }
    }
    std::vector<Record> all((size_t)nd * pad);
    if (rc == ICX_OK) {
        (void)hipSetDevice(m->devs[0].device);
        if (hipMemcpyAsync(all.data(), m->devs[0].d_all, sizeof(Record) * all.size(), hipMemcpyDeviceToHost, sts[0]) !=
            hipSuccess) rc = ICX_INTERNAL_ERR;
    }
    for (int k = 0; k < nd; ++k) {
        if (!sts[k]) continue;
        (void)hipSetDevice(m->devs[k].device);
        if (hipStreamSynchronize(sts[k]) != hipSuccess && rc == ICX_OK) rc = ICX_INTERNAL_ERR;
        (void)hipStreamDestroy(sts[k]);
    }
    if (rc != ICX_OK) {
        if (m->err.empty()) m->err = "RCCL records gather failed";
        return rc;
    }
    for (int k = 0; k < nd; ++k)
        for (size_t j = 0; j < idx[k].size(); ++j) {
            Record r = all[(size_t)k * pad + j];
            if (r.status == ICX_OK && (uint64_t)r.w * r.h * r.c > out_stride) {
                r = Record{};
                r.status = ICX_OUT_OF_MEM;
            }
            std::memcpy(&records[idx[k][j]], &r, sizeof r);
        }
    return ICX_OK;
}

int icx_multi_decode_host(icx_multi* m, int n, const uint8_t* const* jpegs, const size_t* sizes, uint8_t* const* outs,
                          uint64_t out_stride, icx_record* records, int32_t* shard_of) {
    if (!m) return ICX_INTERNAL_ERR;
    if (n < 0 || (n > 0 && (!jpegs || !sizes || !records))) { m->err = "icx_multi_decode_host: bad arguments"; return ICX_INTERNAL_ERR; }
    if (n == 0) return ICX_OK;
    const int nd = (int)m->devs.size();
    std::vector<int32_t> owner(n);
    icx_multi_shard(sizes, n, nd, owner.data());
    if (shard_of) std::memcpy(shard_of, owner.data(), sizeof(int32_t) * n);
    std::vector<std::vector<int>> idx(nd);
    for (int i = 0; i < n; ++i) idx[owner[i]].push_back(i);
    size_t pad = 0;  // RCCL gather: every device's records padded to the largest shard
    for (const auto& v : idx) pad = std::max(pad, v.size());
    if (m->comms.empty()) pad = 0;
    std::vector<int> rc(nd, ICX_OK);
    std::vector<std::thread> th;
    for (int k = 0; k < nd; ++k)
        th.emplace_back([&, k] { rc[k] = run_shard(m, m->devs[k], idx[k], jpegs, sizes, outs, out_stride, records, (int)pad); });
    for (auto& t : th) t.join();
    for (int k = 0; k < nd; ++k)
        if (rc[k] != ICX_OK) {
            m->err = "device " + std::to_string(m->devs[k].device) + ": " + m->devs[k].err;
            return rc[k];
        }
    if (!pad) return ICX_OK;
    // The decode and the pixel copies succeeded and `records` already holds every shard's records
    // (run_shard): a failed RCCL gather falls back to them and says why, rather than
    // failing a call whose results are all there.
    std::vector<icx_record> via_rccl(records, records + n);
    if (rccl_gather(m, idx, (int)pad, out_stride, via_rccl.data()) == ICX_OK) {
        std::memcpy(records, via_rccl.data(), sizeof(icx_record) * n);
        m->gather_desc = "rccl";
    } else {
        m->gather_desc = "host (RCCL gather failed: " + m->err + ")";
        m->err.clear();
    }
    return ICX_OK;
}

const char* icx_multi_gather(const icx_multi* m) { return m ? m->gather_desc.c_str() : ""; }

int icx_jpeg_records(icx_ctx* ctx, int n, const uint8_t* d_out, uint64_t out_stride, const int32_t* d_status,
                     const int32_t* d_dims, int max_width, int max_height, icx_record* d_records, void* stream) {
    if (!ctx || n < 0 || (n > 0 && (!d_out || !d_status || !d_dims || !d_records))) return ICX_INTERNAL_ERR;
    if (n == 0) return ICX_OK;
    if (hipSetDevice(icx_ctx_device(ctx)) != hipSuccess) return ICX_INTERNAL_ERR;
    hipStream_t st = stream ? (hipStream_t)stream : (hipStream_t)icx_ctx_stream(ctx);
    launch_records(n, d_out, out_stride, d_status, d_dims, reinterpret_cast<Record*>(d_records), max_width, max_height, st);
    return hipGetLastError() == hipSuccess ? ICX_OK : ICX_INTERNAL_ERR;
}

uint64_t icx_checksum64(const uint8_t* data, size_t size) {
    uint64_t acc = 0;
    const size_t nw = (size + 3) / 4;
    for (size_t k = 0; k < nw; ++k) {
        uint32_t w = 0;
        for (int b = 0; b < 4; ++b)
            if (4 * k + b < size) w |= (uint32_t)data[4 * k + b] << (8 * b);
        acc += (uint64_t)w * (2 * (uint64_t)k + 1);
    }
    return acc;
}

}  // extern "C"
