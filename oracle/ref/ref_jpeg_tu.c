/*
 * TEST INFRASTRUCTURE ONLY -- never linked into the product (imagecodecs_amd).
 *
 * Implementation translation unit for the reference's own header-only JPEG
 * codecs, compiled IN PLACE from /root/reference (nothing is copied):
 *   - NanoJPEG 1.3.5   /root/reference/jpeg_dec.h   (njInit/njDecode/... :117-171)
 *   - tiny_jpeg        /root/reference/jpeg_enc.h   (tje_encode_with_func :154-160)
 * Build: oracle/Makefile target `ref` -> oracle/_ref/libref_jpeg.so (gitignored,
 * built only in the container where /root/reference exists).
 *
 * The thin exports below give ctypes a buffer-in/buffer-out surface; they add no
 * arithmetic of their own.
 */
#define TJE_IMPLEMENTATION
#include "jpeg_enc.h"
#include "jpeg_dec.h"

#include <stdlib.h>
#include <string.h>

/* Decode with the reference NanoJPEG. Returns nj_result_t. On success copies
 * njGetImageSize() bytes to `out` if `cap` suffices (else returns -1). */
int ref_nj_decode(const unsigned char* jpeg, int size, int* w, int* h, int* ncomp,
                  unsigned char* out, long long cap) {
    njInit();
    int r = (int)njDecode(jpeg, size);
    if (r == 0) {
        *w = njGetWidth();
        *h = njGetHeight();
        *ncomp = njIsColor() ? 3 : 1;
        long long n = njGetImageSize();
        if (n > cap) { njDone(); return -1; }
        if (n > 0) memcpy(out, njGetImage(), (size_t)n);
    }
    njDone();
    return r;
}

typedef struct { unsigned char* buf; long long len, cap; int overflow; } ref_sink;

static void ref_sink_write(void* ctx, void* data, int size) {
    ref_sink* s = (ref_sink*)ctx;
    if (s->len + size > s->cap) { s->overflow = 1; return; }
    memcpy(s->buf + s->len, data, (size_t)size);
    s->len += size;
}

/* Encode with the reference tiny_jpeg. Returns tje's result (1 ok / 0 error),
 * -1 if `cap` was too small. *outlen receives the byte count. */
int ref_tje_encode(int quality, int w, int h, int comps, const unsigned char* src,
                   unsigned char* out, long long cap, long long* outlen) {
    ref_sink s = { out, 0, cap, 0 };
    int r = tje_encode_with_func(ref_sink_write, &s, quality, w, h, comps, src);
    *outlen = s.len;
    return s.overflow ? -1 : r;
}
