/*
 * oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference algorithms on the ImageCodecs JPEG hot path,
 * used exclusively as the parity checker by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg.  The product (imagecodecs_amd / libicx.so) never
 * includes, links or calls anything declared here.
 *
 *  or_nj_decode   restates NanoJPEG 1.3.5   (/root/reference/jpeg_dec.h:258-916)
 *  or_tje_encode  restates tiny_jpeg        (/root/reference/jpeg_enc.h:172-1271)
 *
 * Pinned against the reference itself (oracle/_ref, built from the reference
 * sources in place) by tests/test_oracle.py and the vectors in tests/golden/.
 * Built with -O2 -ffp-contract=off.
 */
#ifndef ICX_ORACLE_H
#define ICX_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* nj_result_t values (jpeg_dec.h:117-125) */
enum { OR_OK = 0, OR_NO_JPEG, OR_UNSUPPORTED, OR_OUT_OF_MEM, OR_INTERNAL_ERR, OR_SYNTAX_ERROR };

/* Optional per-stage trace, filled when non-NULL (for stage-level parity). */
typedef struct {
    int32_t nblocks;          /* blocks decoded, in bitstream order              */
    int16_t* coef;            /* nblocks*64 quantized coefs, natural order; [0] unused */
    int32_t* dc;              /* nblocks absolute (predicted) quantized DC values */
    int32_t cap_blocks;       /* capacity of coef/dc in blocks                    */
} or_trace;

/* Decode `size` bytes of JPEG. Returns an nj_result_t code. On OR_OK, *out is a
 * malloc'd W*H*ncomp buffer (NULL when that product is 0), ncomp in {0,1,3}. */
int or_nj_decode(const uint8_t* jpeg, int64_t size, uint8_t** out, int* w, int* h,
                 int* ncomp, or_trace* trace);

/* tiny_jpeg-equivalent encode: quality 1..3, comps 3 or 4. Returns 1 on success
 * (and *out malloc'd, *outlen bytes), 0 on error -- tje_encode_with_func's contract. */
int or_tje_encode(int quality, int w, int h, int comps, const uint8_t* src,
                  uint8_t** out, int64_t* outlen);

/* C4 extension (defined in tje_oracle.c, no reference exists): IJG quality 1..100,
 * subsampling 444 or 420, comps 3 or 4. Same return contract as or_tje_encode. */
int or_jpeg_encode(int quality, int subsampling, int w, int h, int comps, const uint8_t* src,
                   uint8_t** out, int64_t* outlen);

/* PNG path (png_oracle.c): lodepng's colour-mode choice and filtered IDAT stream for
 * png_encoder::saveToFile input (d = 3 RGB8, d = 4 RGBA8). colortype/bitdepth as in IHDR. */
typedef struct {
    int colortype, bitdepth;
    int npal;
    uint8_t pal[256 * 4];
    int key_defined, key_r, key_g, key_b;
} or_png_mode;
int or_png_choose(const uint8_t* px, int w, int h, int d, or_png_mode* m);
int64_t or_png_linebytes(int w, const or_png_mode* m);
int64_t or_png_filtered_size(int w, int h, const or_png_mode* m);
/* Filtered stream h*(1+linebytes) into out; 1 on success. */
int or_png_filter(const uint8_t* px, int w, int h, int d, const or_png_mode* m, uint8_t* out);
/* Whole PNG with the IDAT deflated by the system zlib at `zlevel` (size proxy, CPU baseline). */
int or_png_encode(const uint8_t* px, int w, int h, int d, int zlevel, uint8_t** out, int64_t* size);

/* Radiance .hdr reader (hdr_oracle.c; Image::readHdr, codecs.cpp:706-777). Result codes: */
enum { OR_HDR_OK = 0, OR_HDR_NOT_RADIANCE = 1, OR_HDR_BAD_HEADER = 2, OR_HDR_MALFORMED = 3, OR_HDR_TRUNCATED = 4 };
int or_hdr_header(const uint8_t* data, int64_t size, int* w, int* h, int64_t* data_start);
/* *out: malloc'd w*h*4 floats (R, G, B, E per pixel; rows past *rows are 0). */
int or_hdr_decode(const uint8_t* data, int64_t size, float** out, int* w, int* h, int* rows);

void or_free(void* p);

#ifdef __cplusplus
}
#endif
#endif
