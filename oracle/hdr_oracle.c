/* hdr_oracle.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of ImageCodecs' Radiance .hdr reader
 * (Image::readHdr, codecs.cpp:706-777, with decrunchHDR :662-703, oldDecrunchHDR :630-660,
 * workOnRGBE :617-628, convertComponent :610-615). Only tests/ and bench.py's cpu_baseline leg use
 * it, as the checker; libicx never links it.
 *
 * Parity: the reference file codecs.cpp does not compile on Linux (MSVC-only constructs, missing
 * codec libraries), so this restatement is pinned only by the reference's fixture
 * data/test.hdr (tests/golden/test.hdr, a flat RGBE file) and by construction ("parity unpinned"
 * beyond that).
 *
 * The reader is emulated over a memory buffer with stdio semantics: getc() past the end returns
 * EOF (stored as 0xFF where the reference stores it into an unsigned char) and sets the EOF flag;
 * the one fseek(-1, SEEK_CUR) (:671) moves back and clears it.
 *
 * Where the reference has undefined behaviour this restatement stops with OR_HDR_MALFORMED:
 *  - a run or literal that would write past the scanline (:686-698, :646-650),
 *  - a non-empty old-style run on the first pixel of a scanline (reads scanline[-1], :647),
 *  - a run count E << rshift with rshift >= 32 (over-wide shift, :645); counts that overflow int
 *    are past the scanline anyway.
 * The header loops never end on a file without "\n\n" (:727-734); here that is OR_HDR_BAD_HEADER,
 * as are a resolution line sscanf cannot fully parse (:745-748 reads w uninitialised when only
 * h matches) and non-positive sizes. Rows the reference leaves uninitialised after a failed
 * scanline (:765-769) are zero here; *rows says how many were decoded.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct {
    const uint8_t* d;
    int64_t n, pos;
    int eof;
} hr_file;

static int hr_getc(hr_file* f) {
    if (f->pos >= f->n) { f->eof = 1; return -1; }
    return f->d[f->pos++];
}

/* convertComponent (codecs.cpp:610-615): (val / 256.0f) * (float)pow(2, expo) */
static float hr_component(int expo, int val) {
    const float v = val / 256.0f;
    const float d = (float)pow(2.0, (double)expo);
    return v * d;
}

/* oldDecrunchHDR (codecs.cpp:630-660) on scan[first .. first+len). */
static int hr_old(hr_file* f, uint8_t* scan, int first, int len, int* malformed) {
    int rshift = 0, x = first;
    while (len > 0) {
        uint8_t px[4];
        for (int k = 0; k < 4; ++k) px[k] = (uint8_t)hr_getc(f);
        if (f->eof) return 0;
        memcpy(scan + 4 * x, px, 4);
        if (px[0] == 1 && px[1] == 1 && px[2] == 1) {
            if (rshift >= 32) { *malformed = 1; return 0; }
            const int64_t cnt = (int64_t)px[3] << rshift;
            if (cnt > len || (cnt > 0 && x == 0)) { *malformed = 1; return 0; }
            for (int64_t i = cnt; i > 0; i--) {
                memcpy(scan + 4 * x, scan + 4 * (x - 1), 4);
                x++;
                len--;
            }
            rshift += 8;
        } else {
            x++;
            len--;
            rshift = 0;
        }
    }
    return 1;
}

/* decrunchHDR (codecs.cpp:662-703) */
static int hr_decrunch(hr_file* f, uint8_t* scan, int len, int* malformed) {
    if (len < 8 || len > 0x7fff) return hr_old(f, scan, 0, len, malformed);
    int i = hr_getc(f);
    if (i != 2) {  /* fseek(file, -1, SEEK_CUR): back one byte, EOF flag cleared */
        f->pos -= 1;
        f->eof = 0;
        return hr_old(f, scan, 0, len, malformed);
    }
    const uint8_t g = (uint8_t)hr_getc(f), b = (uint8_t)hr_getc(f);
    i = hr_getc(f);
    if (g != 2 || (b & 128)) {
        scan[0] = 2;
        scan[1] = g;
        scan[2] = b;
        scan[3] = (uint8_t)i;
        return hr_old(f, scan, 1, len - 1, malformed);
    }
    for (int c = 0; c < 4; c++) {
        for (int j = 0; j < len;) {
            int code = (uint8_t)hr_getc(f);
            if (f->eof) return 0; /* the reference returns false after this scanline (:702) */
            if (code > 128) {
                code &= 127;
                const uint8_t val = (uint8_t)hr_getc(f);
                if (f->eof) return 0;
                if (j + code > len) { *malformed = 1; return 0; }
                while (code--) scan[4 * (j++) + c] = val;
            } else {
                if (j + code > len) { *malformed = 1; return 0; }
                while (code--) {
                    scan[4 * (j++) + c] = (uint8_t)hr_getc(f);
                    if (f->eof) return 0;
                }
            }
        }
    }
    return f->eof ? 0 : 1;
}

/* Header walk of readHdr (codecs.cpp:713-750). Returns OR_HDR_OK and the data start. */
int or_hdr_header(const uint8_t* data, int64_t size, int* w, int* h, int64_t* data_start) {
    if (size < 10 || memcmp(data, "#?RADIANCE", 10) != 0) return OR_HDR_NOT_RADIANCE;
    hr_file f = {data, size, 11, 0}; /* fread 10 bytes, fseek(+1) (:716, :722) */
    char c = 0, oldc;
    for (;;) { /* header lines up to an empty line (:727-734) */
        oldc = c;
        const int g = hr_getc(&f);
        if (g < 0) return OR_HDR_BAD_HEADER;
        c = (char)g;
        if (c == 0xa && oldc == 0xa) break;
    }
    char reso[256];
    int n = 0;
    for (;;) { /* resolution line (:737-743) */
        const int g = hr_getc(&f);
        if (g < 0 || n >= (int)sizeof(reso) - 1) return OR_HDR_BAD_HEADER;
        reso[n++] = (char)g;
        if (g == 0xa) break;
    }
    reso[n] = 0;
    /* sscanf(reso, "-Y %ld +X %ld", &h, &w) (:745) */
    long hh = 0, ww = 0;
    const char* p = reso;
    if (p[0] != '-' || p[1] != 'Y') return OR_HDR_BAD_HEADER;
    p += 2;
    char* e;
    hh = strtol(p, &e, 10);
    if (e == p) return OR_HDR_BAD_HEADER;
    p = e;
    while (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r' || *p == '\v' || *p == '\f') ++p;
    if (p[0] != '+' || p[1] != 'X') return OR_HDR_BAD_HEADER;
    p += 2;
    ww = strtol(p, &e, 10);
    if (e == p) return OR_HDR_BAD_HEADER;
    if (hh <= 0 || ww <= 0 || hh > (1L << 20) || ww > (1L << 20) || hh * ww > (1L << 30)) return OR_HDR_BAD_HEADER;
    *w = (int)ww;
    *h = (int)hh;
    *data_start = f.pos;
    return OR_HDR_OK;
}

/* Image::readHdr (codecs.cpp:706-777): *out = malloc'd w*h*4 floats (rows past *rows are 0).
 * Returns OR_HDR_OK (all rows), OR_HDR_TRUNCATED (fewer rows; the reference reports nothing),
 * OR_HDR_MALFORMED, or a header error. */
int or_hdr_decode(const uint8_t* data, int64_t size, float** out, int* w, int* h, int* rows) {
    int64_t ds = 0;
    *out = NULL;
    *rows = 0;
    int rc = or_hdr_header(data, size, w, h, &ds);
    if (rc != OR_HDR_OK) return rc;
    const int W = *w, H = *h;
    float* px = (float*)calloc((size_t)W * H * 4, sizeof(float));
    uint8_t* scan = (uint8_t*)malloc((size_t)W * 4);
    if (!px || !scan) { free(px); free(scan); return OR_HDR_BAD_HEADER; }
    hr_file f = {data, size, ds, 0};
    int malformed = 0, y = 0;
    for (; y < H; ++y) { /* the reference loops y = h-1 .. 0 but fills rows in file order (:765-776) */
        if (!hr_decrunch(&f, scan, W, &malformed)) break;
        float* row = px + (size_t)y * W * 4;
        for (int x = 0; x < W; ++x) { /* workOnRGBE (:617-628) */
            const int expo = scan[4 * x + 3] - 128;
            row[4 * x + 0] = hr_component(expo, scan[4 * x + 0]);
            row[4 * x + 1] = hr_component(expo, scan[4 * x + 1]);
            row[4 * x + 2] = hr_component(expo, scan[4 * x + 2]);
            row[4 * x + 3] = (float)scan[4 * x + 3];
        }
    }
    free(scan);
    *out = px;
    *rows = y;
    if (malformed) return OR_HDR_MALFORMED;
    return y == H ? OR_HDR_OK : OR_HDR_TRUNCATED;
}
