/*
 * tje_oracle.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement of tiny_jpeg's encoder (/root/reference/jpeg_enc.h), the path
 * behind ImageCodecs::Image::writeJpg (codecs.cpp:851-854).  Float arithmetic is
 * kept in the reference's evaluation order; this file MUST be compiled with
 * -ffp-contract=off so no multiply-add is fused.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* Annex K tables as tiny_jpeg ships them (jpeg_enc.h:265-368). */
static const uint8_t kLumaQ[64] = {
    16, 11, 10, 16, 24, 40, 51, 61,   12, 12, 14, 19, 26, 58, 60, 55,
    14, 13, 16, 24, 40, 57, 69, 56,   14, 17, 22, 29, 51, 87, 80, 62,
    18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99 };
static const uint8_t kChromaQPaper[64] = {
    16, 12, 14, 14, 18, 24, 49, 72,   11, 10, 16, 24, 40, 51, 61, 12,
    13, 17, 22, 35, 64, 92, 14, 16,   22, 37, 55, 78, 95, 19, 24, 29,
    56, 64, 87, 98, 26, 40, 51, 68,   81, 103, 112, 58, 57, 87, 109, 104,
    121, 100, 60, 69, 80, 103, 113, 120, 103, 55, 56, 62, 77, 92, 101, 99 };
static const uint8_t kDcLumaBits[16] = { 0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0 };
static const uint8_t kDcChromaBits[16] = { 0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0 };
static const uint8_t kDcVals[12] = { 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11 };
static const uint8_t kAcLumaBits[16] = { 0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d };
static const uint8_t kAcLumaVals[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07,
    0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xA1, 0x08, 0x23, 0x42, 0xB1, 0xC1, 0x15, 0x52, 0xD1, 0xF0,
    0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0A, 0x16, 0x17, 0x18, 0x19, 0x1A, 0x25, 0x26, 0x27, 0x28,
    0x29, 0x2A, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3A, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49,
    0x4A, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5A, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69,
    0x6A, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7A, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89,
    0x8A, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9A, 0xA2, 0xA3, 0xA4, 0xA5, 0xA6, 0xA7,
    0xA8, 0xA9, 0xAA, 0xB2, 0xB3, 0xB4, 0xB5, 0xB6, 0xB7, 0xB8, 0xB9, 0xBA, 0xC2, 0xC3, 0xC4, 0xC5,
    0xC6, 0xC7, 0xC8, 0xC9, 0xCA, 0xD2, 0xD3, 0xD4, 0xD5, 0xD6, 0xD7, 0xD8, 0xD9, 0xDA, 0xE1, 0xE2,
    0xE3, 0xE4, 0xE5, 0xE6, 0xE7, 0xE8, 0xE9, 0xEA, 0xF1, 0xF2, 0xF3, 0xF4, 0xF5, 0xF6, 0xF7, 0xF8,
    0xF9, 0xFA };
static const uint8_t kAcChromaBits[16] = { 0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77 };
static const uint8_t kAcChromaVals[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71,
    0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xA1, 0xB1, 0xC1, 0x09, 0x23, 0x33, 0x52, 0xF0,
    0x15, 0x62, 0x72, 0xD1, 0x0A, 0x16, 0x24, 0x34, 0xE1, 0x25, 0xF1, 0x17, 0x18, 0x19, 0x1A, 0x26,
    0x27, 0x28, 0x29, 0x2A, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3A, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48,
    0x49, 0x4A, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5A, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68,
    0x69, 0x6A, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7A, 0x82, 0x83, 0x84, 0x85, 0x86, 0x87,
    0x88, 0x89, 0x8A, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9A, 0xA2, 0xA3, 0xA4, 0xA5,
    0xA6, 0xA7, 0xA8, 0xA9, 0xAA, 0xB2, 0xB3, 0xB4, 0xB5, 0xB6, 0xB7, 0xB8, 0xB9, 0xBA, 0xC2, 0xC3,
    0xC4, 0xC5, 0xC6, 0xC7, 0xC8, 0xC9, 0xCA, 0xD2, 0xD3, 0xD4, 0xD5, 0xD6, 0xD7, 0xD8, 0xD9, 0xDA,
    0xE2, 0xE3, 0xE4, 0xE5, 0xE6, 0xE7, 0xE8, 0xE9, 0xEA, 0xF2, 0xF3, 0xF4, 0xF5, 0xF6, 0xF7, 0xF8,
    0xF9, 0xFA };

/* zig-zag index of each natural position (jpeg_enc.h:376-386) */
static const uint8_t kZigOf[64] = {
     0,  1,  5,  6, 14, 15, 27, 28,   2,  4,  7, 13, 16, 26, 29, 42,
     3,  8, 12, 17, 25, 30, 41, 43,   9, 11, 18, 24, 31, 40, 44, 53,
    10, 19, 23, 32, 39, 45, 52, 54,  20, 22, 33, 38, 46, 51, 55, 60,
    21, 34, 37, 47, 50, 56, 59, 61,  35, 36, 48, 49, 57, 58, 62, 63 };

typedef struct { uint16_t code[256]; uint8_t len[256]; } huff_enc;

/* JPEG C.2 code generation (jpeg_enc.h:546-592, 907-946) */
static void build_huff(huff_enc* t, const uint8_t* bits, const uint8_t* vals) {
    memset(t, 0, sizeof(*t));
    uint16_t code = 0;
    int k = 0;
    for (int L = 1; L <= 16; ++L) {
        for (int i = 0; i < bits[L - 1]; ++i, ++k) {
            t->code[vals[k]] = code++;
            t->len[vals[k]] = (uint8_t)L;
        }
        code = (uint16_t)(code << 1);
    }
}

typedef struct {
    uint8_t* buf;
    int64_t len, cap;
    int oom;
    uint32_t acc;   /* bitbuffer  (jpeg_enc.h:1090) */
    uint32_t fill;  /* location   (jpeg_enc.h:1091) */
} sink;

static void put(sink* s, const void* p, int64_t n) {
    if (s->oom) return;
    if (s->len + n > s->cap) {
        int64_t nc = s->cap ? s->cap * 2 : 4096;
        while (nc < s->len + n) nc *= 2;
        uint8_t* nb = (uint8_t*)realloc(s->buf, (size_t)nc);
        if (!nb) { s->oom = 1; return; }
        s->buf = nb;
        s->cap = nc;
    }
    memcpy(s->buf + s->len, p, (size_t)n);
    s->len += n;
}
static void put_u8(sink* s, int v) { uint8_t b = (uint8_t)v; put(s, &b, 1); }
static void put_be16(sink* s, int v) { put_u8(s, v >> 8); put_u8(s, v & 0xFF); }

/* MSB-first bit packer with FF->FF00 stuffing (tjei_write_bits, jpeg_enc.h:613-643) */
static void put_bits(sink* s, int nbits, uint32_t bits) {
    uint32_t nf = s->fill + (uint32_t)nbits;
    s->acc |= bits << (32 - nf);
    s->fill = nf;
    while (s->fill >= 8) {
        uint8_t c = (uint8_t)(s->acc >> 24);
        put_u8(s, c);
        if (c == 0xFF) put_u8(s, 0);
        s->acc <<= 8;
        s->fill -= 8;
    }
}

/* magnitude category + low bits (tjei_calculate_variable_length_int, :598-610) */
static void vli(int v, int* nbits, uint32_t* bits) {
    int mag = v < 0 ? -v : v;
    if (v < 0) --v;
    int n = 1;
    while (mag >>= 1) ++n;
    *nbits = n;
    *bits = (uint32_t)v & ((1u << n) - 1u);
}

/* AAN float forward DCT (tjei_fdct, jpeg_enc.h:656-763), rows then columns */
static void fdct8(float* p, int step) {
    float t0 = p[0] + p[7 * step], t7 = p[0] - p[7 * step];
    float t1 = p[step] + p[6 * step], t6 = p[step] - p[6 * step];
    float t2 = p[2 * step] + p[5 * step], t5 = p[2 * step] - p[5 * step];
    float t3 = p[3 * step] + p[4 * step], t4 = p[3 * step] - p[4 * step];
    float e10 = t0 + t3, e13 = t0 - t3, e11 = t1 + t2, e12 = t1 - t2;
    p[0] = e10 + e11;
    p[4 * step] = e10 - e11;
    float z1 = (e12 + e13) * ((float)0.707106781);
    p[2 * step] = e13 + z1;
    p[6 * step] = e13 - z1;
    float o10 = t4 + t5, o11 = t5 + t6, o12 = t6 + t7;
    float z5 = (o10 - o12) * ((float)0.382683433);
    float z2 = ((float)0.541196100) * o10 + z5;
    float z4 = ((float)1.306562965) * o12 + z5;
    float z3 = o11 * ((float)0.707106781);
    float z11 = t7 + z3, z13 = t7 - z3;
    p[5 * step] = z13 + z2;
    p[3 * step] = z13 - z2;
    p[step] = z11 + z4;
    p[7 * step] = z11 - z4;
}

/* one data unit (tjei_encode_and_write_MCU, jpeg_enc.h:786-889) */
static void encode_unit(sink* s, const float* in, const float* pq, const huff_enc* dc,
                        const huff_enc* ac, int* pred) {
    float f[64];
    memcpy(f, in, sizeof(f));
    for (int r = 0; r < 8; ++r) fdct8(f + 8 * r, 1);
    for (int c = 0; c < 8; ++c) fdct8(f + c, 8);
    int zz[64];
    for (int i = 0; i < 64; ++i) {
        float v = f[i];
        v *= pq[i];
        v = floorf(v + 1024 + 0.5f);
        v -= 1024;
        zz[kZigOf[i]] = (int)v;
    }
    int nb;
    uint32_t bits;
    int diff = zz[0] - *pred;
    *pred = zz[0];
    if (diff) {
        vli(diff, &nb, &bits);
        put_bits(s, dc->len[nb], dc->code[nb]);
        put_bits(s, nb, bits);
    } else {
        put_bits(s, dc->len[0], dc->code[0]);
    }
    int last = 0;
    for (int i = 63; i > 0; --i)
        if (zz[i]) { last = i; break; }
    for (int i = 1; i <= last; ++i) {
        int run = 0;
        while (zz[i] == 0) {
            ++run;
            ++i;
            if (run == 16) { put_bits(s, ac->len[0xF0], ac->code[0xF0]); run = 0; }
        }
        vli(zz[i], &nb, &bits);
        int sym = (run << 4) | nb;
        put_bits(s, ac->len[sym], ac->code[sym]);
        put_bits(s, nb, bits);
    }
    if (last != 63) put_bits(s, ac->len[0], ac->code[0]);
}

static void put_dht(sink* s, int cls_id, const uint8_t* bits, const uint8_t* vals) {
    int n = 0;
    for (int i = 0; i < 16; ++i) n += bits[i];
    put_be16(s, 0xFFC4);
    put_be16(s, 2 + 1 + 16 + n);
    put_u8(s, cls_id);
    put(s, bits, 16);
    put(s, vals, n);
}

int or_tje_encode(int quality, int w, int h, int comps, const uint8_t* src, uint8_t** out,
                  int64_t* outlen) {
    *out = NULL;
    *outlen = 0;
    if (quality < 1 || quality > 3) return 0;         /* :1223-1226 */
    if (comps != 3 && comps != 4) return 0;           /* :954-956 */
    if (w > 0xFFFF || h > 0xFFFF) return 0;           /* :958-960 */
    uint8_t ql[64], qc[64];
    for (int i = 0; i < 64; ++i) {                    /* :1231-1256 */
        if (quality == 3) { ql[i] = qc[i] = 1; continue; }
        int div = quality == 2 ? 10 : 1;
        ql[i] = (uint8_t)(kLumaQ[i] / div);
        if (!ql[i]) ql[i] = 1;
        qc[i] = (uint8_t)(kChromaQPaper[i] / div);
        if (!qc[i]) qc[i] = 1;
    }
    static const float aan[8] = { 1.0f, 1.387039845f, 1.306562965f, 1.175875602f,
                                  1.0f, 0.785694958f, 0.541196100f, 0.275899379f };
    float pl[64], pc[64];                             /* :980-986 */
    for (int y = 0; y < 8; ++y)
        for (int x = 0; x < 8; ++x) {
            int i = y * 8 + x;
            pl[i] = 1.0f / (8 * aan[x] * aan[y] * ql[kZigOf[i]]);
            pc[i] = 1.0f / (8 * aan[x] * aan[y] * qc[kZigOf[i]]);
        }
    huff_enc hdl, hal, hdc, hac;
    build_huff(&hdl, kDcLumaBits, kDcVals);
    build_huff(&hal, kAcLumaBits, kAcLumaVals);
    build_huff(&hdc, kDcChromaBits, kDcVals);
    build_huff(&hac, kAcChromaBits, kAcChromaVals);

    sink s;
    memset(&s, 0, sizeof(s));
    /* SOI + APP0/JFIF 1.02, 96 dpi (:989-1005) */
    static const uint8_t jfif[] = { 0xFF, 0xD8, 0xFF, 0xE0, 0x00, 0x10, 'J', 'F', 'I', 'F', 0,
                                    0x01, 0x02, 0x01, 0x00, 0x60, 0x00, 0x60, 0x00, 0x00 };
    put(&s, jfif, sizeof(jfif));
    static const char com[] = "Created by Tiny JPEG Encoder"; /* :409, 1006-1014 */
    put_be16(&s, 0xFFFE);
    put_be16(&s, 2 + (int)sizeof(com) - 1);
    put(&s, com, (int64_t)sizeof(com) - 1);
    put_be16(&s, 0xFFDB); put_be16(&s, 0x43); put_u8(&s, 0); put(&s, ql, 64);   /* :498-509 */
    put_be16(&s, 0xFFDB); put_be16(&s, 0x43); put_u8(&s, 1); put(&s, qc, 64);
    put_be16(&s, 0xFFC0); put_be16(&s, 17); put_u8(&s, 8);                          /* :1020-1045 */
    put_be16(&s, h); put_be16(&s, w); put_u8(&s, 3);
    for (int i = 0; i < 3; ++i) { put_u8(&s, i + 1); put_u8(&s, 0x11); put_u8(&s, i ? 1 : 0); }
    put_dht(&s, 0x00, kDcLumaBits, kDcVals);                                      /* :1047-1050 */
    put_dht(&s, 0x10, kAcLumaBits, kAcLumaVals);
    put_dht(&s, 0x01, kDcChromaBits, kDcVals);
    put_dht(&s, 0x11, kAcChromaBits, kAcChromaVals);
    put_be16(&s, 0xFFDA); put_be16(&s, 12); put_u8(&s, 3);                         /* :1052-1077 */
    put_u8(&s, 1); put_u8(&s, 0x00); put_u8(&s, 2); put_u8(&s, 0x11); put_u8(&s, 3); put_u8(&s, 0x11);
    put_u8(&s, 0); put_u8(&s, 63); put_u8(&s, 0);

    float Y[64], U[64], V[64];
    int py = 0, pu = 0, pv = 0;
    for (int by = 0; by < h; by += 8)                                              /* :1094-1158 */
        for (int bx = 0; bx < w; bx += 8) {
            for (int oy = 0; oy < 8; ++oy) {
                int row = by + oy < h ? by + oy : h - 1;
                for (int ox = 0; ox < 8; ++ox) {
                    int col = bx + ox < w ? bx + ox : w - 1;
                    const uint8_t* p = src + ((int64_t)row * w + col) * comps;
                    uint8_t r = p[0], g = p[1], b = p[2];
                    int k = oy * 8 + ox;
                    Y[k] = 0.299f * r + 0.587f * g + 0.114f * b - 128;
                    U[k] = -0.1687f * r - 0.3313f * g + 0.5f * b;
                    V[k] = 0.5f * r - 0.4187f * g - 0.0813f * b;
                }
            }
            encode_unit(&s, Y, pl, &hdl, &hal, &py);
            encode_unit(&s, U, pc, &hdc, &hac, &pu);
            encode_unit(&s, V, pc, &hdc, &hac, &pv);
        }
    if (s.fill > 0 && s.fill < 8) put_bits(&s, (int)(8 - s.fill), 0);             /* :1161-1165 */
    put_be16(&s, 0xFFD9);
    if (s.oom) { free(s.buf); return 0; }
    *out = s.buf;
    *outlen = s.len;
    return 1;
}

/* ------------------------------------------------------------------------------------------
 * C4 extension: baseline JPEG with 4:2:0 (or 4:4:4) sampling and IJG
 * quality scaling. tiny_jpeg has neither, so there is no reference to restate: THIS FUNCTION
 * IS THE DEFINITION of the extension, and the GPU encoder (icx_jpeg_encode*) must reproduce its
 * bytes exactly. It keeps tiny_jpeg's arithmetic everywhere it overlaps:
 *   - per-pixel float RGB->YCbCr with the same expressions (jpeg_enc.h:1118-1120), edge clamp
 *     of rows/cols to the image (:1106-1111);
 *   - 4:2:0: each chroma sample is ((c(x,y) + c(x+1,y)) + (c(x,y+1) + c(x+1,y+1))) * 0.25f of the
 *     per-pixel values, with the same edge clamp;
 *   - AAN float FDCT, pq = 1/(8*aan[x]*aan[y]*q), floorf(v*pq + 1024 + 0.5f) - 1024;
 *   - Annex K Huffman tables, MSB-first emit with FF00 stuffing, zero-bit final pad, DC
 *     predictors never reset.
 * Quantization: the JPEG spec K.1 / K.2 tables (natural order) scaled as IJG libjpeg does
 * (q < 50 ? 5000/q : 200 - 2q; (t*scale + 50)/100 clamped to 1..255), written to DQT in
 * zig-zag order. MCU 16x16 for 4:2:0 (Y0 Y1 Y2 Y3 Cb Cr), 8x8 for 4:4:4.
 * ---------------------------------------------------------------------------------------- */
static const uint8_t kK2Chroma[64] = {  /* JPEG spec table K.2, natural order */
    17, 18, 24, 47, 99, 99, 99, 99,   18, 21, 26, 66, 99, 99, 99, 99,
    24, 26, 56, 99, 99, 99, 99, 99,   47, 66, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99,   99, 99, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99,   99, 99, 99, 99, 99, 99, 99, 99 };

static void ijg_table(const uint8_t* base, int q, uint8_t* out) {
    const int scale = q < 50 ? 5000 / q : 200 - 2 * q;
    for (int i = 0; i < 64; ++i) {
        int v = (base[i] * scale + 50) / 100;
        out[i] = (uint8_t)(v < 1 ? 1 : v > 255 ? 255 : v);
    }
}

int or_jpeg_encode(int quality, int subsampling, int w, int h, int comps, const uint8_t* src,
                   uint8_t** out, int64_t* outlen) {
    *out = NULL;
    *outlen = 0;
    if (quality < 1 || quality > 100) return 0;
    if (subsampling != 444 && subsampling != 420) return 0;
    if (comps != 3 && comps != 4) return 0;
    if (w > 0xFFFF || h > 0xFFFF) return 0;
    uint8_t ql[64], qc[64];   /* natural order */
    ijg_table(kLumaQ, quality, ql);      /* kLumaQ is table K.1 in natural order */
    ijg_table(kK2Chroma, quality, qc);
    static const float aan[8] = { 1.0f, 1.387039845f, 1.306562965f, 1.175875602f,
                                  1.0f, 0.785694958f, 0.541196100f, 0.275899379f };
    float pl[64], pc[64];
    for (int y = 0; y < 8; ++y)
        for (int x = 0; x < 8; ++x) {
            int i = y * 8 + x;
            pl[i] = 1.0f / (8 * aan[x] * aan[y] * ql[i]);
            pc[i] = 1.0f / (8 * aan[x] * aan[y] * qc[i]);
        }
    huff_enc hdl, hal, hdc, hac;
    build_huff(&hdl, kDcLumaBits, kDcVals);
    build_huff(&hal, kAcLumaBits, kAcLumaVals);
    build_huff(&hdc, kDcChromaBits, kDcVals);
    build_huff(&hac, kAcChromaBits, kAcChromaVals);

    sink s;
    memset(&s, 0, sizeof(s));
    static const uint8_t jfif[] = { 0xFF, 0xD8, 0xFF, 0xE0, 0x00, 0x10, 'J', 'F', 'I', 'F', 0,
                                    0x01, 0x02, 0x01, 0x00, 0x60, 0x00, 0x60, 0x00, 0x00 };
    put(&s, jfif, sizeof(jfif));
    static const char com[] = "icx JPEG encoder";
    put_be16(&s, 0xFFFE);
    put_be16(&s, 2 + (int)sizeof(com) - 1);
    put(&s, com, (int64_t)sizeof(com) - 1);
    uint8_t zq[64];
    for (int k = 0; k < 64; ++k) zq[kZigOf[k]] = ql[k];   /* DQT holds zig-zag order */
    put_be16(&s, 0xFFDB); put_be16(&s, 0x43); put_u8(&s, 0); put(&s, zq, 64);
    for (int k = 0; k < 64; ++k) zq[kZigOf[k]] = qc[k];
    put_be16(&s, 0xFFDB); put_be16(&s, 0x43); put_u8(&s, 1); put(&s, zq, 64);
    put_be16(&s, 0xFFC0); put_be16(&s, 17); put_u8(&s, 8);
    put_be16(&s, h); put_be16(&s, w); put_u8(&s, 3);
    for (int i = 0; i < 3; ++i) {
        put_u8(&s, i + 1);
        put_u8(&s, i == 0 && subsampling == 420 ? 0x22 : 0x11);
        put_u8(&s, i ? 1 : 0);
    }
    put_dht(&s, 0x00, kDcLumaBits, kDcVals);
    put_dht(&s, 0x10, kAcLumaBits, kAcLumaVals);
    put_dht(&s, 0x01, kDcChromaBits, kDcVals);
    put_dht(&s, 0x11, kAcChromaBits, kAcChromaVals);
    put_be16(&s, 0xFFDA); put_be16(&s, 12); put_u8(&s, 3);
    put_u8(&s, 1); put_u8(&s, 0x00); put_u8(&s, 2); put_u8(&s, 0x11); put_u8(&s, 3); put_u8(&s, 0x11);
    put_u8(&s, 0); put_u8(&s, 63); put_u8(&s, 0);

    const int ms = subsampling == 420 ? 16 : 8;
    float blk[64];
    int py = 0, pu = 0, pv = 0;
#define PIX(X, Y) (src + ((int64_t)((Y) < h ? (Y) : h - 1) * w + ((X) < w ? (X) : w - 1)) * comps)
    for (int my = 0; my < h; my += ms)
        for (int mx = 0; mx < w; mx += ms) {
            for (int sb = 0; sb < (ms == 16 ? 4 : 1); ++sb) {       /* luma blocks, raster order */
                const int bx = mx + (sb & 1) * 8, by = my + (sb >> 1) * 8;
                for (int oy = 0; oy < 8; ++oy)
                    for (int ox = 0; ox < 8; ++ox) {
                        const uint8_t* p = PIX(bx + ox, by + oy);
                        const uint8_t r = p[0], g = p[1], b = p[2];
                        blk[oy * 8 + ox] = 0.299f * r + 0.587f * g + 0.114f * b - 128;
                    }
                encode_unit(&s, blk, pl, &hdl, &hal, &py);
            }
            for (int c = 1; c <= 2; ++c) {
                for (int oy = 0; oy < 8; ++oy)
                    for (int ox = 0; ox < 8; ++ox) {
                        float v;
                        if (ms == 8) {
                            const uint8_t* p = PIX(mx + ox, my + oy);
                            const uint8_t r = p[0], g = p[1], b = p[2];
                            v = c == 1 ? -0.1687f * r - 0.3313f * g + 0.5f * b : 0.5f * r - 0.4187f * g - 0.0813f * b;
                        } else {
                            float q4[4];
                            for (int d = 0; d < 4; ++d) {
                                const uint8_t* p = PIX(mx + 2 * ox + (d & 1), my + 2 * oy + (d >> 1));
                                const uint8_t r = p[0], g = p[1], b = p[2];
                                q4[d] = c == 1 ? -0.1687f * r - 0.3313f * g + 0.5f * b
                                               : 0.5f * r - 0.4187f * g - 0.0813f * b;
                            }
                            v = ((q4[0] + q4[1]) + (q4[2] + q4[3])) * 0.25f;
                        }
                        blk[oy * 8 + ox] = v;
                    }
                encode_unit(&s, blk, pc, &hdc, &hac, c == 1 ? &pu : &pv);
            }
        }
#undef PIX
    if (s.fill > 0 && s.fill < 8) put_bits(&s, (int)(8 - s.fill), 0);
    put_be16(&s, 0xFFD9);
    if (s.oom) { free(s.buf); return 0; }
    *out = s.buf;
    *outlen = s.len;
    return 1;
}
