/*
 * icx.h -- C ABI of libicx.so, the MI355X-native JPEG codec behind ImageCodecs' codecs.h.
 *
 * Plain pointers and sizes only (no torch / HIP types in signatures). Every function is
 * extern "C", never throws, and is reentrant per icx_ctx. Each entry point names the
 * reference interface it replaces (paths relative to the jstrom2002/ImageCodecs tree):
 *
 *   NanoJPEG (jpeg_dec.h:117-171): njInit/njDecode/njGetWidth/njGetHeight/njIsColor/
 *       njGetImage/njGetImageSize/njDone  -> icx_nj_* below, with the decoder state held
 *       in an icx_ctx instead of NanoJPEG's process-global `nj` (jpeg_dec.h:332).
 *   tiny_jpeg (jpeg_enc.h:114-160): tje_encode_to_file/_at_quality/tje_encode_with_func
 *       -> icx_tje_* below (same quality 1..3 contract and byte stream).
 *   Image::readJpg (codecs.cpp:821-849) -> icx_jpeg_decode (one call, host in/host out).
 *   Batch decode (new) -> icx_jpeg_batch_* (device-resident in and out).
 *
 * Result codes are NanoJPEG's nj_result_t values (jpeg_dec.h:117-125).
 */
#ifndef ICX_H
#define ICX_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum icx_result {
    ICX_OK = 0,              /* NJ_OK            */
    ICX_NO_JPEG = 1,         /* NJ_NO_JPEG       */
    ICX_UNSUPPORTED = 2,     /* NJ_UNSUPPORTED   */
    ICX_OUT_OF_MEM = 3,      /* NJ_OUT_OF_MEM    */
    ICX_INTERNAL_ERR = 4,    /* NJ_INTERNAL_ERR  */
    ICX_SYNTAX_ERROR = 5     /* NJ_SYNTAX_ERROR  */
};

typedef struct icx_ctx icx_ctx;

/* ---- context ------------------------------------------------------------------- */
/* One context per (device, HIP stream). `device` is a HIP device ordinal. Returns NULL
 * if the device cannot be opened (see icx_last_error(NULL)). */
icx_ctx* icx_create(int device);
void icx_destroy(icx_ctx* ctx);
/* Last error message for this context (or the last icx_create failure when ctx==NULL). */
const char* icx_last_error(const icx_ctx* ctx);
/* Library version string, e.g. "icx 0.1.0 gfx950". */
const char* icx_version(void);

/* ---- header probe (host only; no device work) ------------------------------------ */
/* Parses markers up to the first SOS exactly as njDecode does (jpeg_dec.h:880-903).
 * Returns ICX_OK when the stream is well-formed up to the entropy-coded data (decode may
 * still fail later) and fills width/height/ncomp (ncomp: 1 gray, 3 colour); otherwise the
 * code njDecode would return. */
int icx_jpeg_probe(const uint8_t* jpeg, size_t size, int* width, int* height, int* ncomp);

/* ---- NanoJPEG-compatible stateful API (jpeg_dec.h:130-171) ------------------------- */
/* njInit (jpeg_dec.h:130) / njDone (:171): reset the context's decoder state. */
void icx_nj_init(icx_ctx* ctx);
void icx_nj_done(icx_ctx* ctx);
/* njDecode (jpeg_dec.h:138): decodes on the GPU; returns an icx_result. */
int icx_nj_decode(icx_ctx* ctx, const void* jpeg, int size);
int icx_nj_get_width(const icx_ctx* ctx);         /* njGetWidth     (:142) */
int icx_nj_get_height(const icx_ctx* ctx);        /* njGetHeight    (:146) */
int icx_nj_is_color(const icx_ctx* ctx);          /* njIsColor      (:151) */
unsigned char* icx_nj_get_image(icx_ctx* ctx);    /* njGetImage     (:160) host memory owned by ctx */
int icx_nj_get_image_size(const icx_ctx* ctx);    /* njGetImageSize (:165) */

/* ---- one-shot decode (Image::readJpg, codecs.cpp:821-849) ------------------------- */
/* Decodes on the GPU; *out receives a malloc()'d W*H*ncomp buffer (free with icx_free).
 * ncomp is 3 for colour and 1 for gray (the reference adapter's d=3-for-gray over-read,
 * codecs.cpp:840-844, is not reproduced). */
int icx_jpeg_decode(icx_ctx* ctx, const uint8_t* jpeg, size_t size, uint8_t** out, int* width,
                    int* height, int* ncomp);
void icx_free(void* p);

/* ---- batch decode, device-resident (the throughput path) ------------------------- */
typedef struct icx_batch icx_batch;

/* Workspace for up to `max_images` images per call, each at most max_width x max_height
 * (any sampling NanoJPEG accepts). At most `group` images (0 = auto: 80% of free HBM) are in
 * flight at once, split over up to two decode pipelines (a workspace and a HIP stream each;
 * env ICX_PIPES=1 keeps one): consecutive groups alternate between the pipelines so their
 * kernels overlap, and the call's stream waits for both. Returns NULL on allocation failure. */
icx_batch* icx_batch_create(icx_ctx* ctx, int max_images, int max_width, int max_height, int group);
void icx_batch_destroy(icx_batch* b);

/* Decode n images. All pointers are DEVICE pointers on the context's device:
 *   d_data      concatenated JPEG files; image i is d_data[d_offsets[i] .. + d_sizes[i])
 *   d_out       output; image i is written at d_out + i*out_stride, packed W*H*ncomp bytes
 *   d_status    n int32 icx_result codes (per image; one bad image never fails the batch)
 *   d_dims      n*3 int32 {width, height, ncomp} (ncomp 3 colour / 1 gray; 0s on error)
 * An image larger than the batch limits, or whose pixels exceed out_stride, gets
 * ICX_OUT_OF_MEM. Work is enqueued on `stream` (a hipStream_t; NULL = the context's
 * stream). The call does not wait for the decode, but when the stream is not capturing it does
 * wait on the host for each group's entropy planning, and so for all work enqueued on `stream`
 * before the call (it reads how many images a group's planning deferred to a further entropy
 * round, and enqueues that round only when there are any): do not make `stream` wait on an
 * event the caller records only after this call. Under stream capture (hipStreamBeginCapture,
 * e.g. to build a hipGraph of the decode) the call never waits: every entropy round and every
 * layout's back half is enqueued unconditionally (rounds with nothing to do find no work), so the
 * captured graph is complete; ICX_HOST_WAIT=0 selects that form without capture. Returns ICX_OK
 * or a call-level error. */
int icx_jpeg_batch_decode(icx_batch* b, int n, const uint8_t* d_data, const uint64_t* d_offsets,
                          const uint64_t* d_sizes, uint8_t* d_out, uint64_t out_stride,
                          int32_t* d_status, int32_t* d_dims, void* stream);

/* Host-buffer convenience: copies inputs to the device, decodes, copies results back.
 * outs[i] must hold out_stride bytes. */
int icx_jpeg_batch_decode_host(icx_batch* b, int n, const uint8_t* const* jpegs, const size_t* sizes,
                               uint8_t* const* outs, uint64_t out_stride, int32_t* status, int32_t* dims);

/* Images per workspace group (each kernel of the pipeline launches once per group). */
int icx_batch_group(const icx_batch* b); /* images per group (one pipeline's workspace) */
int icx_batch_groups(const icx_batch* b, int n); /* groups (launches of each per-group kernel) a call of n images takes */

/* Per-stage timings (ms) of the most recent batch call, measured with HIP events on the
 * stream the kernels ran on. Fills up to `cap` entries; returns the number of stages. */
int icx_batch_stage_times(const icx_batch* b, const char** names, float* ms, int cap);

/* Which entropy path the images of the most recent batch call took: the parallel
 * self-synchronising decoder, the parallel decoder falling back to the sequential one
 * (unverified chain), or the sequential decoder only (restart intervals, exotic sampling).
 * Synchronizes with the device. */
int icx_batch_path_stats(const icx_batch* b, int32_t* parallel, int32_t* fallback, int32_t* sequential);

/* ---- per-image result records and multi-GPU decode ------------- */
/* The record each device computes for every image it decoded; ranks (or devices) exchange
 * these 24 bytes per image instead of pixels. checksum = sum of the decoded bytes' little-
 * endian 32-bit words w_k (last one zero-padded) times (2k + 1), mod 2^64 (icx_checksum64). */
typedef struct icx_record {
    int32_t status, width, height, ncomp; /* icx_result; dims as d_dims (0s on error) */
    uint64_t checksum;                    /* 0 for a failed image */
} icx_record;

/* Records of a batch call's outputs (device pointers, enqueued on `stream`, NULL = the
 * context's stream): d_status / d_dims / d_out as icx_jpeg_batch_decode wrote them. */
int icx_jpeg_records(icx_ctx* ctx, int n, const uint8_t* d_out, uint64_t out_stride, const int32_t* d_status,
                     const int32_t* d_dims, int max_width, int max_height, icx_record* d_records, void* stream);
/* The same checksum on the host (a reference for tests and callers). */
uint64_t icx_checksum64(const uint8_t* data, size_t size);
int icx_ctx_device(const icx_ctx* ctx);   /* the context's HIP device ordinal */
void* icx_ctx_stream(const icx_ctx* ctx); /* the context's hipStream_t */

/* Multi-GPU batch decode in one process: the batch is split over `ndev` devices by
 * compressed size (greedy longest-first, icx_multi_shard), one host thread per device decodes
 * its shard with its own context, workspace and stream, and computes its per-image records on
 * the device. The records are gathered over RCCL (one communicator per device, ncclCommInitAll;
 * one grouped ncclAllGather of every shard's records padded to the largest shard) when the
 * devices are distinct and librccl.so loads, else through host memory (ICX_MULTI_RCCL=0 forces
 * that); each device copies its images' pixels to the caller's host buffers. Every image of
 * every device may be up to max_width x max_height. */
typedef struct icx_multi icx_multi;
icx_multi* icx_multi_create(const int* devices, int ndev, int max_width, int max_height);
void icx_multi_destroy(icx_multi* m);
/* outs[i] (may be NULL, or outs itself NULL: records only) receives image i's packed pixels,
 * at most out_stride bytes; records[i] its record; shard_of[i] (optional) the index into
 * `devices` that decoded it. Returns ICX_OK or the first device's call-level error. */
int icx_multi_decode_host(icx_multi* m, int n, const uint8_t* const* jpegs, const size_t* sizes,
                          uint8_t* const* outs, uint64_t out_stride, icx_record* records, int32_t* shard_of);
const char* icx_multi_last_error(const icx_multi* m);
/* How the records are gathered: "rccl", or "host (<reason>)". */
const char* icx_multi_gather(const icx_multi* m);
/* The split: shard_of[i] in [0, ndev) for n images of the given compressed sizes. */
int icx_multi_shard(const size_t* sizes, int n, int ndev, int32_t* shard_of);

/* ---- encode (tiny_jpeg, jpeg_enc.h:114-160) --------------------------------------- */
typedef void icx_write_func(void* context, void* data, int size); /* = tje_write_func */

/* tje_encode_with_func (jpeg_enc.h:154): quality 1..3, comps 3 (RGB) or 4 (RGBA);
 * returns 1 on success, 0 on error. The byte stream is identical to tiny_jpeg's. */
int icx_tje_encode_with_func(icx_ctx* ctx, icx_write_func* func, void* context, int quality,
                             int width, int height, int num_components, const unsigned char* src);
/* tje_encode_to_file_at_quality (jpeg_enc.h:137) / tje_encode_to_file (:114, quality 3). */
int icx_tje_encode_to_file_at_quality(icx_ctx* ctx, const char* dest_path, int quality, int width,
                                      int height, int num_components, const unsigned char* src);
int icx_tje_encode_to_file(icx_ctx* ctx, const char* dest_path, int width, int height,
                           int num_components, const unsigned char* src);

/* ---- encode extension (IJG quality 1..100, 4:4:4 or 4:2:0) ----------
 * tiny_jpeg only offers quality 1..3 at 4:4:4 (jpeg_enc.h:1223-1256). The extension keeps its
 * entropy coder and float AAN DCT (jpeg_enc.h:980-1100) and adds IJG-scaled tables (luma =
 * tiny_jpeg's, chroma = JPEG spec K.2) and 2x2-mean 4:2:0 chroma. The byte stream is defined by
 * oracle/tje_oracle.c or_jpeg_encode and decodes with NanoJPEG. */
/* Host image -> file bytes through `func`; returns 1 on success, 0 on error. */
int icx_jpeg_encode_with_func(icx_ctx* ctx, icx_write_func* func, void* context, int quality,
                              int subsampling, int width, int height, int num_components,
                              const unsigned char* src);

typedef struct icx_encoder icx_encoder;
/* Reusable device workspace for device-resident encodes on ctx's device. */
icx_encoder* icx_encoder_create(icx_ctx* ctx);
void icx_encoder_destroy(icx_encoder* enc);
/* Device image d_src (width*height*num_components bytes) -> whole JPEG file at d_out.
 * Synchronous on `hip_stream` (NULL = the context's stream). *out_size receives the file size.
 * Returns ICX_OK, ICX_OUT_OF_MEM when out_cap < *out_size (nothing written),
 * ICX_UNSUPPORTED for bad arguments, ICX_INTERNAL_ERR on a HIP failure. */
int icx_jpeg_encode_device(icx_encoder* enc, int quality, int subsampling, int width, int height,
                           int num_components, const uint8_t* d_src, uint8_t* d_out, uint64_t out_cap,
                           uint64_t* out_size, void* hip_stream);
/* A batch of n device images of one geometry and setting (d_srcs: host array of device
 * pointers) -> JPEG files at d_out + i*out_stride; out_sizes[i] and status[i] (ICX_OK, or
 * ICX_OUT_OF_MEM when out_stride < out_sizes[i]: nothing written) on the host. Images alternate
 * between two workspaces on two streams (hip_stream and an internal one), so each image's host
 * wait overlaps the next image's kernels. Synchronous; returns ICX_OK, ICX_UNSUPPORTED or
 * ICX_INTERNAL_ERR. Replaces a loop of icx_jpeg_encode_device calls (same bytes). */
int icx_jpeg_encode_device_batch(icx_encoder* enc, int n, int quality, int subsampling, int width, int height,
                                 int num_components, const uint8_t* const* d_srcs, uint8_t* d_out,
                                 uint64_t out_stride, uint64_t* out_sizes, int32_t* status, void* hip_stream);
/* Per-stage GPU time (HIP events) of the encodes since the previous call, summed: units
 * (DCT+quantise), count, scan, emit, stuff. Returns the number of stages filled (<= cap). */
int icx_encoder_stage_times(icx_encoder* enc, const char** names, float* ms, int cap);

/* ---- PNG encode (png_encoder::saveToFile, png_encoder.h:7 / png_encoder.cpp:4474-4486) ------
 * d = 3 (RGB8) or 4 (RGBA8) like saveToFile. lodepng's automatic colour type (palette / grey /
 * grey+alpha / RGB / RGBA, tRNS key) and its MINSUM filter bytes are reproduced exactly; the IDAT
 * is our GPU deflate (valid zlib, inflates to lodepng's filtered stream; bytes differ). */
/* Host image -> PNG bytes through `func` (<= 1023-byte chunks); returns 1 on success, 0 on error. */
int icx_png_encode_with_func(icx_ctx* ctx, icx_write_func* func, void* context, const unsigned char* pixels,
                             int width, int height, int d);
/* png_encoder::saveToFile: returns ICX_OK or an error code (the reference returns nothing). */
int icx_png_save_to_file(icx_ctx* ctx, const char* path, const unsigned char* pixels, int width, int height,
                         int d);

typedef struct icx_png_encoder icx_png_encoder;
icx_png_encoder* icx_png_encoder_create(icx_ctx* ctx);
void icx_png_encoder_destroy(icx_png_encoder* enc);
/* Device image d_src (width*height*d bytes) -> whole PNG file at d_out; synchronous on
 * hip_stream (NULL = the context's stream). Returns ICX_OK, ICX_OUT_OF_MEM when out_cap <
 * *out_size (nothing written), ICX_UNSUPPORTED for bad arguments, ICX_INTERNAL_ERR on a HIP
 * failure. */
int icx_png_encode_device(icx_png_encoder* enc, int width, int height, int d, const uint8_t* d_src,
                          uint8_t* d_out, uint64_t out_cap, uint64_t* out_size, void* hip_stream);
/* n images (width x height x d each, at d_srcs[i] on the context's device) into d_out + i *
 * out_stride; out_sizes[i] = file size (or the bytes needed), status[i] = ICX_OK, ICX_OUT_OF_MEM
 * (the slot is too small) or ICX_INTERNAL_ERR (that image's own job failed: every other image still
 * gets its status and size). Returns ICX_INTERNAL_ERR only when a stream failed. The batch form
 * of png_encoder::saveToFile for device-resident images: several images in flight
 * (ICX_PNG_INFLIGHT, default 8), each on its own workspace and stream. The host reads back one
 * thing per image, its colour statistics (the colour mode and palette are chosen on the host);
 * the file layout, IDAT length, Adler-32, CRC-32 and IEND are computed and written on the device,
 * and every image's size is read once, after the last image. Returns when every file is
 * written. */
int icx_png_encode_device_batch(icx_png_encoder* enc, int n, int width, int height, int d,
                                const uint8_t* const* d_srcs, uint8_t* d_out, uint64_t out_stride,
                                uint64_t* out_sizes, int32_t* status, void* hip_stream);
/* Milliseconds per stage summed over the icx_png_encode_device calls since the previous read
 * ("stats", "filter", "lz77", "huff", "emit", "crc"; HIP events on the launch stream). Returns
 * the number of stages. */
int icx_png_encoder_stage_times(icx_png_encoder* enc, const char** names, float* ms, int cap);

/* ---- Radiance .hdr read (Image::readHdr, codecs.cpp:706-777) -----------------------------------
 * Output as readHdr returns it (d = 4, Type::FLOAT): 4 floats per pixel, rows in file order,
 * R, G, B = convertComponent(E - 128, v) = v * 2^(E - 136) (codecs.cpp:610-615; exact, so the
 * GPU result equals the reference's bit for bit) and the fourth float = E (:624).
 * Where the reference's behaviour is undefined (runs past the scanline, a run on a scanline's first
 * pixel, a header without an empty line, a partial resolution line) the result is MALFORMED or
 * BAD_HEADER; rows after a scanline the reference stops at (it leaves them uninitialised,
 * :765-769) are zero and counted out of *rows. */
enum icx_hdr_result {
    ICX_HDR_OK = 0,            /* all rows decoded                                   */
    ICX_HDR_NOT_RADIANCE = 1,  /* "Invalid file format": no "#?RADIANCE" (:717-720)  */
    ICX_HDR_BAD_HEADER = 2,    /* header / resolution line not as readHdr parses it   */
    ICX_HDR_MALFORMED = 3,     /* run-length data the reference cannot decode (UB)     */
    ICX_HDR_TRUNCATED = 4,     /* the file ends first: rows < height                   */
    ICX_HDR_TOO_LARGE = 5,     /* larger than the batch workspace                      */
    ICX_HDR_INTERNAL_ERR = -1  /* HIP failure (see icx_last_error)                     */
};
/* Header only (host): width/height of a well-formed header, else the error code. */
int icx_hdr_probe(const uint8_t* data, size_t size, int* width, int* height);
/* One image, host in / host out: *out receives a malloc()'d width*height*4 float buffer (free
 * with icx_free); *rows = decoded rows. */
int icx_hdr_decode(icx_ctx* ctx, const uint8_t* data, size_t size, float** out, int* width, int* height,
                   int* rows);
/* Device-resident batch: image i = d_data[d_offsets[i] .. + d_sizes[i]), output floats at
 * d_out + i*out_stride (out_stride >= 4*width*height of every image), per-image status in
 * d_status[i] and {width, height, rows} in d_dims[3i..]. Asynchronous on hip_stream (NULL = the
 * context's stream). Returns ICX_HDR_OK or ICX_HDR_INTERNAL_ERR. */
typedef struct icx_hdr_batch icx_hdr_batch;
icx_hdr_batch* icx_hdr_batch_create(icx_ctx* ctx, int max_images, int max_width, int max_height);
void icx_hdr_batch_destroy(icx_hdr_batch* b);
int icx_hdr_batch_decode(icx_hdr_batch* b, int n, const uint8_t* d_data, const uint64_t* d_offsets,
                         const uint64_t* d_sizes, float* d_out, uint64_t out_stride, int32_t* d_status,
                         int32_t* d_dims, void* hip_stream);
/* Milliseconds per stage of the last icx_hdr_batch_decode ("parse", "locate", "unpack",
 * "convert"; synchronises). Returns the number of stages. */
int icx_hdr_batch_stage_times(const icx_hdr_batch* b, const char** names, float* ms, int cap);

/* ---- OpenEXR read (Image::readExr, codecs.cpp:464-493 -> tinyexr LoadEXRFromMemory, tinyexr.h:6645) ----
 * Output as LoadEXRFromMemory returns it: width*height*4 floats (R, G, B, A by channel name; a
 * one-channel image repeats its channel in all four; no A channel -> 1.0), data-window rows in
 * tinyexr's order. HALF samples are converted bit for bit (half_to_float), FLOAT copied, UINT
 * sample bits copied unconverted (tinyexr reads them through its float** view).
 * Scope: single-part scanline or tiled files, NONE / RLE / ZIPS / ZIP / PIZ compression (the
 * reference builds tinyexr with TINYEXR_USE_PIZ 1, tinyexr.h:126-128); mip- and rip-mapped tiled
 * files decode every level's tiles as DecodeChunk does (a failure in any level fails the read) and
 * return level 0; a broken offset table is reconstructed from the chunk headers
 * (ReconstructTileOffsets, where the multi-part and deep version bits change the chunk walk;
 * LoadEXRFromMemory does not reject them, only LoadEXR does, tinyexr.h:6268-6270). Pixels no
 * chunk wrote (tinyexr leaves them uninitialised) are 0. */
enum icx_exr_result {
    ICX_EXR_SUCCESS = 0,                /* TINYEXR_SUCCESS                          */
    ICX_EXR_INVALID_MAGIC_NUMBER = -1,  /* TINYEXR_ERROR_INVALID_MAGIC_NUMBER       */
    ICX_EXR_INVALID_EXR_VERSION = -2,   /* TINYEXR_ERROR_INVALID_EXR_VERSION        */
    ICX_EXR_INVALID_ARGUMENT = -3,      /* TINYEXR_ERROR_INVALID_ARGUMENT           */
    ICX_EXR_INVALID_DATA = -4,          /* TINYEXR_ERROR_INVALID_DATA               */
    ICX_EXR_UNSUPPORTED_FORMAT = -8,    /* TINYEXR_ERROR_UNSUPPORTED_FORMAT         */
    ICX_EXR_INVALID_HEADER = -9,        /* TINYEXR_ERROR_INVALID_HEADER             */
    ICX_EXR_UNSUPPORTED_FEATURE = -10,  /* TINYEXR_ERROR_UNSUPPORTED_FEATURE        */
    ICX_EXR_INTERNAL_ERR = -100         /* HIP failure (see icx_last_error)         */
};
/* Header, offset table and chunk headers only (host): the data window size, or the error code
 * LoadEXRFromMemory would return before decoding pixels. */
int icx_exr_probe(const uint8_t* data, size_t size, int* width, int* height);
/* One image, host in / host out: *out_rgba receives a malloc()'d width*height*4 float buffer
 * (free with icx_free). Returns an icx_exr_result. */
int icx_exr_decode(icx_ctx* ctx, const uint8_t* data, size_t size, float** out_rgba, int* width, int* height);
/* The same read with the file already resident on the device (batch pipelines, benchmarks): the
 * header and offset table are planned from the host copy `data`; the kernels read the device copy
 * `d_data` (the same `size` bytes followed by 16 zero bytes; 16-byte aligned, since the chunk
 * readers load 16-byte words: a misaligned pointer is ICX_EXR_INVALID_ARGUMENT) and write
 * width*height*4 floats to
 * `d_out` (room for `out_floats`; too little -> ICX_EXR_INTERNAL_ERR). Synchronises with the
 * context's stream; returns an icx_exr_result. */
int icx_exr_decode_device(icx_ctx* ctx, const uint8_t* data, const uint8_t* d_data, size_t size, float* d_out,
                          size_t out_floats, int* width, int* height);
/* n such reads in one call: every file is planned on the host, then the compressed chunks of all
 * n files are decompressed by one launch (a workgroup per chunk) before each file is converted --
 * one 2048^2 ZIP file has 128 chunks, a batch keeps thousands in flight. codes[i] gets file i's
 * icx_exr_result, widths[i] / heights[i] its size (0 when it fails). Returns ICX_EXR_SUCCESS when
 * the call ran (per-file results in codes), ICX_EXR_INVALID_ARGUMENT for a null pointer, or
 * ICX_EXR_INTERNAL_ERR (HIP failure, an output buffer too small; see icx_last_error). */
int icx_exr_decode_device_batch(icx_ctx* ctx, int n, const uint8_t* const* data, const uint8_t* const* d_data,
                                const size_t* sizes, float* const* d_out, const size_t* out_floats, int32_t* codes,
                                int32_t* widths, int32_t* heights);

#ifdef __cplusplus
}
#endif
#endif /* ICX_H */
