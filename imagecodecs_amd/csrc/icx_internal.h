// icx_internal.h -- declarations shared by the host API (icx_api.cpp) and the kernel
// launchers (icx_decode.hip). Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "icx_jpeg.h"

namespace icx {

// Device workspace for one group of images processed together (slot i = image i of the
// group). Capacities are per slot and cover any sampling NanoJPEG accepts at max_w x max_h.
struct GroupWs {
    int slots = 0;
    int max_w = 0, max_h = 0;
    int64_t coef_cap = 0;    // blocks per slot
    int64_t plane_cap = 0;   // bytes per slot (all components' IDCT planes)
    int64_t tmp_cap = 0;     // bytes per ping-pong buffer per component per slot
    Desc* desc = nullptr;    // [slots]
    int16_t* ac = nullptr;   // [slots][coef_cap][64] quantized coefficients, natural order
    int32_t* dc = nullptr;   // [slots][coef_cap] absolute quantized DC per block
    uint8_t* planes = nullptr;  // [slots][plane_cap]
    uint8_t* tmp = nullptr;     // [slots][3 comps][2 buffers][tmp_cap]
};

int64_t ws_coef_cap(int w, int h);
int64_t ws_plane_cap(int w, int h);
int64_t ws_tmp_cap(int w, int h);

// Stage hooks so the host can bracket each stage with HIP events.
enum Stage { kStParse = 0, kStEntropy, kStIdct, kStUpsample, kStConvert, kStCount };
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

// tiny_jpeg-exact encode on the GPU (icx_encode.hip); `out` receives the whole file.
bool tje_encode_gpu(hipStream_t st, int quality, int w, int h, int comps, const uint8_t* src,
                    std::vector<uint8_t>& out);

}  // namespace icx
