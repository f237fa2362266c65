/*
 * synth.c -- synthetic test/bench input generator (tools/, not product, not oracle).
 *
 * 1. synth_rgb: deterministic synthetic photo-like images (SURVEY.md §8(d) recipe):
 *    per channel fx,fy ~ U(0.005,0.05), phase ~ U(0,2pi),
 *    v = 128 + 70 sin(x fx + phase) cos(y fy) + N(0,12), clipped to u8.
 *    PRNG: splitmix64; the N(0,12) term uses an Irwin-Hall (sum of 4 uniform bytes)
 *    approximation so a 4096^2 image generates in well under a second.
 * 2. synth_jpeg: a plain baseline JPEG encoder (JFIF, IJG quality scaling of the
 *    Annex K tables, Annex K Huffman tables, gray / 4:4:4 / 4:2:2 / 4:2:0 / 4:4:0 /
 *    4:1:1, optional DRI + RSTn).  It only has to produce valid baseline streams;
 *    decode parity is always judged against the NanoJPEG oracle on its output.
 */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static uint64_t sm64(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double unif(uint64_t* s) { return (double)(sm64(s) >> 11) * (1.0 / 9007199254740992.0); }

int synth_rgb(uint64_t seed, int w, int h, int comps, uint8_t* out) {
    if (w <= 0 || h <= 0 || comps < 1 || comps > 4) return 0;
    uint64_t s = seed * 0x2545F4914F6CDD1Dull + 1234567ull;
    double fx[4], fy[4], ph[4];
    for (int c = 0; c < comps; ++c) {
        fx[c] = 0.005 + 0.045 * unif(&s);
        fy[c] = 0.005 + 0.045 * unif(&s);
        ph[c] = 6.283185307179586 * unif(&s);
    }
    float* sx = (float*)malloc(sizeof(float) * (size_t)w * comps);
    float* cy = (float*)malloc(sizeof(float) * (size_t)h * comps);
    if (!sx || !cy) { free(sx); free(cy); return 0; }
    for (int c = 0; c < comps; ++c) {
        for (int x = 0; x < w; ++x) sx[c * w + x] = (float)(70.0 * sin(x * fx[c] + ph[c]));
        for (int y = 0; y < h; ++y) cy[c * h + y] = (float)cos(y * fy[c]);
    }
    const float kNoise = 12.0f / 147.7996f; /* std of a sum of 4 U{0..255} */
    for (int y = 0; y < h; ++y) {
        uint8_t* row = out + (int64_t)y * w * comps;
        uint64_t r = 0;
        int have = 0;
        for (int x = 0; x < w; ++x)
            for (int c = 0; c < comps; ++c) {
                if (!have) { r = sm64(&s); have = 2; }
                int sum = (int)(r & 255) + (int)((r >> 8) & 255) + (int)((r >> 16) & 255) + (int)((r >> 24) & 255);
                r >>= 32;
                --have;
                float v = 128.0f + sx[c * w + x] * cy[c * h + y] + (float)(sum - 510) * kNoise;
                int iv = (int)lrintf(v);
                row[x * comps + c] = (uint8_t)(iv < 0 ? 0 : iv > 255 ? 255 : iv);
            }
    }
    free(sx);
    free(cy);
    return 1;
}

/* ---------------------------------------------------------------- encoder --- */
static const uint8_t kStdLuma[64] = {
    16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55, 14, 13, 16, 24, 40, 57,
    69, 56, 14, 17, 22, 29, 51, 87, 80, 62, 18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64,
    81, 104, 113, 92, 49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99 };
static const uint8_t kStdChroma[64] = {
    17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99, 24, 26, 56, 99, 99, 99,
    99, 99, 47, 66, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99 };
/* natural position of zig-zag index k */
static const uint8_t kNat[64] = {
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63 };
static const uint8_t kBitsDcL[16] = { 0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0 };
static const uint8_t kBitsDcC[16] = { 0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0 };
static const uint8_t kValDc[12] = { 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11 };
static const uint8_t kBitsAcL[16] = { 0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d };
static const uint8_t kValAcL[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22, 0x71,
    0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72,
    0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37,
    0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59,
    0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3,
    0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
    0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
    0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa };
static const uint8_t kBitsAcC[16] = { 0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77 };
static const uint8_t kValAcC[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13, 0x22,
    0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1,
    0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36,
    0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58,
    0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a,
    0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba,
    0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
    0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa };

typedef struct { uint16_t code[256]; uint8_t len[256]; } henc;
static void mk_henc(henc* t, const uint8_t* bits, const uint8_t* vals) {
    memset(t, 0, sizeof(*t));
    unsigned code = 0;
    int k = 0;
    for (int L = 1; L <= 16; ++L) {
        for (int i = 0; i < bits[L - 1]; ++i, ++k) { t->code[vals[k]] = (uint16_t)code++; t->len[vals[k]] = (uint8_t)L; }
        code <<= 1;
    }
}

typedef struct {
    uint8_t* p;
    int64_t n, cap;
    int full;
    uint64_t acc;
    int nacc;
} wbuf;
static void wb(wbuf* w, int v) {
    if (w->n >= w->cap) { w->full = 1; return; }
    w->p[w->n++] = (uint8_t)v;
}
static void wb16(wbuf* w, int v) { wb(w, v >> 8); wb(w, v & 255); }
static void wbits(wbuf* w, unsigned bits, int n) {
    w->acc = (w->acc << n) | (bits & ((1u << n) - 1u));
    w->nacc += n;
    while (w->nacc >= 8) {
        int b = (int)((w->acc >> (w->nacc - 8)) & 255);
        wb(w, b);
        if (b == 0xFF) wb(w, 0);
        w->nacc -= 8;
    }
}
static void wflush1(wbuf* w) { /* pad with 1-bits to a byte boundary */
    if (w->nacc & 7) wbits(w, 0x7F, 8 - (w->nacc & 7));
    w->nacc = 0;
    w->acc = 0;
}

static float gCos[8][8];
/* filled once when the library loads, so concurrent synth_jpeg calls (thread pools) only read it */
__attribute__((constructor)) static void init_cos_table(void) {
    for (int u = 0; u < 8; ++u)
        for (int x = 0; x < 8; ++x)
            gCos[u][x] = (float)((u ? 0.5 : 0.5 / sqrt(2.0)) * cos((2 * x + 1) * u * 3.14159265358979323846 / 16.0));
}
static void init_cos(void) {}

static void code_block(wbuf* w, const float* px, const uint16_t* q, const henc* dc, const henc* ac, int* pred) {
    float tmp[64], co[64];
    for (int y = 0; y < 8; ++y)
        for (int u = 0; u < 8; ++u) {
            float s = 0;
            for (int x = 0; x < 8; ++x) s += gCos[u][x] * px[y * 8 + x];
            tmp[y * 8 + u] = s;
        }
    for (int v = 0; v < 8; ++v)
        for (int u = 0; u < 8; ++u) {
            float s = 0;
            for (int y = 0; y < 8; ++y) s += gCos[v][y] * tmp[y * 8 + u];
            co[v * 8 + u] = s;
        }
    int z[64];
    for (int k = 0; k < 64; ++k) z[k] = (int)lrintf(co[kNat[k]] / q[k]);
    int d = z[0] - *pred;
    *pred = z[0];
    int ad = d < 0 ? -d : d, nb = 0;
    while (ad) { ++nb; ad >>= 1; }
    wbits(w, dc->code[nb], dc->len[nb]);
    if (nb) wbits(w, (unsigned)(d < 0 ? d - 1 : d), nb);
    int run = 0;
    for (int k = 1; k < 64; ++k) {
        int v = z[k];
        if (!v) { ++run; continue; }
        while (run > 15) { wbits(w, ac->code[0xF0], ac->len[0xF0]); run -= 16; }
        int av = v < 0 ? -v : v;
        nb = 0;
        while (av) { ++nb; av >>= 1; }
        if (nb > 10) { nb = 10; v = v < 0 ? -1023 : 1023; }
        int sym = (run << 4) | nb;
        wbits(w, ac->code[sym], ac->len[sym]);
        wbits(w, (unsigned)(v < 0 ? v - 1 : v), nb);
        run = 0;
    }
    if (run) wbits(w, ac->code[0], ac->len[0]);
}

/* sampling: 0 -> grayscale; otherwise Y factors (H<<4|V) in {0x11,0x21,0x22,0x12,0x41}
 * with 1x1 chroma. quality 1..100 (IJG scaling). restart: DRI interval in MCUs (0 = none).
 * Returns bytes written, or -1 if `cap` is too small / bad arguments. */
int64_t synth_jpeg(const uint8_t* px, int w, int h, int comps_in, int sampling, int quality,
                   int restart, uint8_t* out, int64_t cap) {
    if (w <= 0 || h <= 0 || w > 65535 || h > 65535 || comps_in < 1) return -1;
    init_cos();
    int nc = sampling ? 3 : 1;
    int hs = sampling ? sampling >> 4 : 1, vs = sampling ? sampling & 15 : 1;
    if (quality < 1) quality = 1;
    if (quality > 100) quality = 100;
    int scale = quality < 50 ? 5000 / quality : 200 - 2 * quality;
    uint8_t qz[2][64];
    uint16_t qk[2][64];
    for (int k = 0; k < 64; ++k) {
        int a = (kStdLuma[kNat[k]] * scale + 50) / 100, b = (kStdChroma[kNat[k]] * scale + 50) / 100;
        a = a < 1 ? 1 : a > 255 ? 255 : a;
        b = b < 1 ? 1 : b > 255 ? 255 : b;
        qz[0][k] = (uint8_t)a; qz[1][k] = (uint8_t)b;
        qk[0][k] = (uint16_t)a; qk[1][k] = (uint16_t)b;
    }
    henc hdl, hal, hdc, hac;
    mk_henc(&hdl, kBitsDcL, kValDc);
    mk_henc(&hal, kBitsAcL, kValAcL);
    mk_henc(&hdc, kBitsDcC, kValDc);
    mk_henc(&hac, kBitsAcC, kValAcC);
    wbuf W = { out, 0, cap, 0, 0, 0 };
    static const uint8_t app0[] = { 0xFF, 0xD8, 0xFF, 0xE0, 0, 16, 'J', 'F', 'I', 'F', 0, 1, 1, 0, 0, 1, 0, 1, 0, 0 };
    for (size_t i = 0; i < sizeof(app0); ++i) wb(&W, app0[i]);
    for (int t = 0; t < (nc == 3 ? 2 : 1); ++t) {
        wb16(&W, 0xFFDB); wb16(&W, 67); wb(&W, t);
        for (int k = 0; k < 64; ++k) wb(&W, qz[t][k]);
    }
    wb16(&W, 0xFFC0); wb16(&W, 8 + 3 * nc); wb(&W, 8); wb16(&W, h); wb16(&W, w); wb(&W, nc);
    for (int c = 0; c < nc; ++c) { wb(&W, c + 1); wb(&W, c ? 0x11 : (hs << 4 | vs)); wb(&W, c ? 1 : 0); }
    const uint8_t* hb[4] = { kBitsDcL, kBitsAcL, kBitsDcC, kBitsAcC };
    const uint8_t* hv[4] = { kValDc, kValAcL, kValDc, kValAcC };
    const int hid[4] = { 0x00, 0x10, 0x01, 0x11 };
    for (int t = 0; t < (nc == 3 ? 4 : 2); ++t) {
        int n = 0;
        for (int i = 0; i < 16; ++i) n += hb[t][i];
        wb16(&W, 0xFFC4); wb16(&W, 19 + n); wb(&W, hid[t]);
        for (int i = 0; i < 16; ++i) wb(&W, hb[t][i]);
        for (int i = 0; i < n; ++i) wb(&W, hv[t][i]);
    }
    if (restart > 0) { wb16(&W, 0xFFDD); wb16(&W, 4); wb16(&W, restart); }
    wb16(&W, 0xFFDA); wb16(&W, 6 + 2 * nc); wb(&W, nc);
    for (int c = 0; c < nc; ++c) { wb(&W, c + 1); wb(&W, c ? 0x11 : 0x00); }
    wb(&W, 0); wb(&W, 63); wb(&W, 0);

    int mbw = (w + 8 * hs - 1) / (8 * hs), mbh = (h + 8 * vs - 1) / (8 * vs);
    int pred[3] = { 0, 0, 0 };
    int left = restart, rst = 0;
    float blk[64];
    for (int my = 0; my < mbh; ++my)
        for (int mx = 0; mx < mbw; ++mx) {
            for (int c = 0; c < nc; ++c) {
                int ch = c ? 1 : hs, cv = c ? 1 : vs;
                for (int by = 0; by < cv; ++by)
                    for (int bx = 0; bx < ch; ++bx) {
                        for (int y = 0; y < 8; ++y)
                            for (int x = 0; x < 8; ++x) {
                                /* sample position in full-res pixels; chroma averages hs x vs */
                                float acc = 0;
                                int fx = c ? hs : 1, fy = c ? vs : 1;
                                int x0 = (mx * ch + bx) * 8 + x, y0 = (my * cv + by) * 8 + y;
                                for (int sy = 0; sy < fy; ++sy)
                                    for (int sx = 0; sx < fx; ++sx) {
                                        int X = x0 * fx + sx, Y = y0 * fy + sy;
                                        if (X >= w) X = w - 1;
                                        if (Y >= h) Y = h - 1;
                                        const uint8_t* p = px + ((int64_t)Y * w + X) * comps_in;
                                        float r = p[0], g = comps_in >= 3 ? p[1] : p[0], b = comps_in >= 3 ? p[2] : p[0];
                                        float v;
                                        if (nc == 1) v = comps_in >= 3 ? 0.299f * r + 0.587f * g + 0.114f * b : r;
                                        else if (c == 0) v = 0.299f * r + 0.587f * g + 0.114f * b;
                                        else if (c == 1) v = -0.168736f * r - 0.331264f * g + 0.5f * b + 128.0f;
                                        else v = 0.5f * r - 0.418688f * g - 0.081312f * b + 128.0f;
                                        acc += v;
                                    }
                                blk[y * 8 + x] = acc / (fx * fy) - 128.0f;
                            }
                        code_block(&W, blk, qk[c ? 1 : 0], c ? &hdc : &hdl, c ? &hac : &hal, &pred[c]);
                    }
            }
            int last = (mx + 1 == mbw) && (my + 1 == mbh);
            if (restart > 0 && !last && --left == 0) {
                wflush1(&W);
                wb(&W, 0xFF); wb(&W, 0xD0 + rst);
                rst = (rst + 1) & 7;
                left = restart;
                pred[0] = pred[1] = pred[2] = 0;
            }
        }
    wflush1(&W);
    wb16(&W, 0xFFD9);
    return W.full ? -1 : W.n;
}

/* ---------------------------------------------------------------- Radiance .hdr (RGBE) inputs
 * synth_rgbe: smooth RGBE pixels with noise (mantissas 128..255, exponents around 128) and a band of
 * constant rows so that run-length coding has runs to find. Never emits R=G=B=1 (an old-style run
 * marker). hdr_encode writes the header the reference reader expects (codecs.cpp:713-750) and the
 * pixel data as mode 0: new-style per-component RLE (Radiance RGBE_WriteBytes_RLE scheme),
 * mode 1: flat RGBE (what Image::writeHdr writes, codecs.cpp:779-817), mode 2: old-style RLE
 * (repeated pixels as (1,1,1,count) markers, count < 256). */
int synth_rgbe(uint64_t seed, int w, int h, uint8_t* out) {
    if (w <= 0 || h <= 0) return 0;
    uint64_t s = seed * 0x9E3779B97F4A7C15ull + 12345;
    const double fx = 0.002 + 0.01 * unif(&s), fy = 0.002 + 0.01 * unif(&s), ph = 6.283 * unif(&s);
    const int band0 = h / 3, band1 = band0 + h / 10;
    for (int y = 0; y < h; ++y) {
        for (int x = 0; x < w; ++x) {
            uint8_t* p = out + ((size_t)y * w + x) * 4;
            if (y >= band0 && y < band1) { p[0] = 200; p[1] = 150; p[2] = 180; p[3] = 129; continue; }
            const double v = sin(x * fx + ph) * cos(y * fy);
            const int e = 128 + (int)floor(2.5 * v);
            for (int c = 0; c < 3; ++c) {
                int m = 128 + (int)(60 + 55 * sin(x * fx * (c + 1) + y * fy + c) + 10 * (unif(&s) - 0.5));
                p[c] = (uint8_t)(m < 128 ? 128 : (m > 255 ? 255 : m));
            }
            p[3] = (uint8_t)e;
        }
    }
    return 1;
}

static int64_t hdr_put(uint8_t* out, int64_t n, int64_t cap, int v) {
    if (n < cap) out[n] = (uint8_t)v;
    return n + 1;
}

/* one component of one scanline, Radiance's RLE scheme (runs >= 4, literals <= 128) */
static int64_t hdr_rle_comp(const uint8_t* px, int w, int c, uint8_t* out, int64_t n, int64_t cap) {
    int cur = 0;
#define D(i) px[4 * (i) + c]
    while (cur < w) {
        int beg = cur, run = 0, old_run = 0;
        while (run < 4 && beg < w) {
            beg += run;
            old_run = run;
            run = 1;
            while (beg + run < w && run < 127 && D(beg) == D(beg + run)) run++;
        }
        if (old_run > 1 && old_run == beg - cur) {
            n = hdr_put(out, n, cap, 128 + old_run);
            n = hdr_put(out, n, cap, D(cur));
            cur = beg;
        }
        while (cur < beg) {
            int k = beg - cur;
            if (k > 128) k = 128;
            n = hdr_put(out, n, cap, k);
            for (int i = 0; i < k; ++i) n = hdr_put(out, n, cap, D(cur + i));
            cur += k;
        }
        if (run >= 4) {
            n = hdr_put(out, n, cap, 128 + run);
            n = hdr_put(out, n, cap, D(beg));
            cur += run;
        }
    }
#undef D
    return n;
}

int64_t hdr_encode(const uint8_t* rgbe, int w, int h, int mode, uint8_t* out, int64_t cap) {
    char hdr[128];
    const int hl = snprintf(hdr, sizeof hdr, "#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y %d +X %d\n", h, w);
    int64_t n = 0;
    for (int i = 0; i < hl; ++i) n = hdr_put(out, n, cap, hdr[i]);
    for (int y = 0; y < h; ++y) {
        const uint8_t* px = rgbe + (size_t)y * w * 4;
        if (mode == 0 && w >= 8 && w <= 0x7fff) {
            n = hdr_put(out, n, cap, 2);
            n = hdr_put(out, n, cap, 2);
            n = hdr_put(out, n, cap, w >> 8);
            n = hdr_put(out, n, cap, w & 255);
            for (int c = 0; c < 4; ++c) n = hdr_rle_comp(px, w, c, out, n, cap);
        } else if (mode == 2) {
            int x = 0;
            while (x < w) {
                for (int k = 0; k < 4; ++k) n = hdr_put(out, n, cap, px[4 * x + k]);
                int r = 0;
                while (x + 1 + r < w && r < 255 && !memcmp(px + 4 * x, px + 4 * (x + 1 + r), 4)) r++;
                if (r >= 2) {
                    n = hdr_put(out, n, cap, 1);
                    n = hdr_put(out, n, cap, 1);
                    n = hdr_put(out, n, cap, 1);
                    n = hdr_put(out, n, cap, r);
                    x += 1 + r;
                } else {
                    x += 1;
                }
            }
        } else {
            for (int i = 0; i < w * 4; ++i) n = hdr_put(out, n, cap, px[i]);
        }
    }
    return n <= cap ? n : -n;
}
